// Probe of the gfx950 fp64 pipes the Cholesky / contraction kernels live on:
// dependent latencies (v_fma_f64, v_rcp_f64, ds_bpermute, v_readlane) and how
// v_mfma_f64_16x16x4_f64 shares a SIMD with fp64 VALU work, from the same
// wave and from a second wave on the SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o fp64_pipe_probe fp64_pipe_probe.hip && ./fp64_pipe_probe
// Cycles are s_memtime deltas per wave (median over waves), one workgroup per
// CU, so each SIMD holds the stated number of waves.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef double v4d __attribute__((ext_vector_type(4)));

constexpr int ITERS = 2048;

__device__ __forceinline__ long long stamp() { return (long long)__builtin_amdgcn_s_memtime(); }

// kind: 0 fma chain, 1 rcp chain, 2 bpermute chain, 3 readlane chain
template <int KIND>
__global__ __launch_bounds__(256) void k_latency(double seed, double* sink, long long* cyc) {
  double x = seed + threadIdx.x * 1e-3;
  const long long t0 = stamp();
  for (int i = 0; i < ITERS; ++i) {
    if constexpr (KIND == 0) x = fma(x, 0.999999, 1e-9);
    if constexpr (KIND == 1) x = __builtin_amdgcn_rcp(x);
    if constexpr (KIND == 2) x = __shfl(x, (threadIdx.x + 1) & 63);
    if constexpr (KIND == 3) {
      const int lo = __builtin_amdgcn_readlane(__double2loint(x), 5);
      const int hi = __builtin_amdgcn_readlane(__double2hiint(x), 5);
      x = __hiloint2double(hi, lo) * 0.999999;
    }
  }
  const long long t1 = stamp();
  sink[blockIdx.x * 256 + threadIdx.x] = x;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

// NM independent MFMA accumulators and NV independent fp64 FMA chains per
// iteration, in one wave (ROLE = 0), or split over two waves on the SIMD:
// waves 0-3 run the MFMAs, waves 4-7 the FMAs (ROLE = 1, 512 threads).
template <int NM, int NV, int ROLE>
__global__ __launch_bounds__(512) void k_mix(double seed, double* sink, long long* cyc) {
  const int wave = threadIdx.x >> 6;
  const bool do_m = ROLE == 0 || wave < 4;
  const bool do_v = ROLE == 0 || wave >= 4;
  v4d acc[NM > 0 ? NM : 1];
  double x[NV > 0 ? NV : 1];
  const double a = seed + threadIdx.x * 1e-6, b = seed - threadIdx.x * 1e-6;
  for (int j = 0; j < (NM > 0 ? NM : 1); ++j) acc[j] = v4d{a, b, a, b};
  for (int j = 0; j < (NV > 0 ? NV : 1); ++j) x[j] = a + j;
  const long long t0 = stamp();
  for (int i = 0; i < ITERS; ++i) {
    if (do_m) {
#pragma unroll
      for (int j = 0; j < NM; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
    }
    if (do_v) {
#pragma unroll
      for (int j = 0; j < NV; ++j) x[j] = fma(x[j], 0.999999, 1e-9);
    }
  }
  const long long t1 = stamp();
  double s = 0;
  for (int j = 0; j < NM; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  for (int j = 0; j < NV; ++j) s += x[j];
  sink[blockIdx.x * 512 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

static double median(std::vector<long long> v) {
  std::sort(v.begin(), v.end());
  return (double)v[v.size() / 2];
}

template <typename K>
static void run(const char* name, K kern, int threads, int per_iter_div, double* sink, long long* cyc, int waves_sel) {
  const int nblk = 256;
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(threads), 0, 0, 1.0, sink, cyc);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(threads), 0, 0, 1.0, sink, cyc);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const int wpb = threads / 64;
  std::vector<long long> h(nblk * wpb);
  (void)hipMemcpy(h.data(), cyc, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
  std::vector<long long> a, b;
  for (int i = 0; i < nblk; ++i)
    for (int w = 0; w < wpb; ++w) (w < 4 ? a : b).push_back(h[i * wpb + w]);
  printf("%-34s cyc/iter waves0-3 %7.2f", name, median(a) / ITERS / per_iter_div);
  if (!b.empty()) printf("  waves4-7 %7.2f", median(b) / ITERS / per_iter_div);
  printf("  wall %.3f ms\n", ms);
  (void)waves_sel;
}

int main() {
  double* sink;
  long long* cyc;
  (void)hipMalloc(&sink, 256 * 512 * sizeof(double));
  (void)hipMalloc(&cyc, 256 * 8 * sizeof(long long));
  run("lat v_fma_f64", k_latency<0>, 256, 1, sink, cyc, 0);
  run("lat v_rcp_f64", k_latency<1>, 256, 1, sink, cyc, 0);
  run("lat ds_bpermute (f64)", k_latency<2>, 256, 1, sink, cyc, 0);
  run("lat readlane x2 + mul", k_latency<3>, 256, 1, sink, cyc, 0);
  run("mfma dep chain (1 acc)", k_mix<1, 0, 0>, 256, 1, sink, cyc, 0);
  run("mfma 4 acc (per mfma)", k_mix<4, 0, 0>, 256, 4, sink, cyc, 0);
  run("mfma 8 acc (per mfma)", k_mix<8, 0, 0>, 256, 8, sink, cyc, 0);
  run("fma 8 chains (per fma)", k_mix<0, 8, 0>, 256, 8, sink, cyc, 0);
  run("fma 16 chains (per fma)", k_mix<0, 16, 0>, 256, 16, sink, cyc, 0);
  run("1w: 4 mfma + 4 fma (per iter)", k_mix<4, 4, 0>, 256, 1, sink, cyc, 0);
  run("1w: 4 mfma + 8 fma (per iter)", k_mix<4, 8, 0>, 256, 1, sink, cyc, 0);
  run("1w: 4 mfma + 16 fma (per iter)", k_mix<4, 16, 0>, 256, 1, sink, cyc, 0);
  run("1w: 4 mfma + 32 fma (per iter)", k_mix<4, 32, 0>, 256, 1, sink, cyc, 0);
  run("2w: 4 mfma | 8 fma (per iter)", k_mix<4, 8, 1>, 512, 1, sink, cyc, 0);
  run("2w: 4 mfma | 16 fma (per iter)", k_mix<4, 16, 1>, 512, 1, sink, cyc, 0);
  run("2w: 4 mfma | 32 fma (per iter)", k_mix<4, 32, 1>, 512, 1, sink, cyc, 0);
  run("2w: 4 mfma | 64 fma (per iter)", k_mix<4, 64, 1>, 512, 1, sink, cyc, 0);
  run("2w: 4 mfma | 0 fma (per iter)", k_mix<4, 0, 1>, 512, 1, sink, cyc, 0);
  run("2w: 0 mfma | 32 fma (per iter)", k_mix<0, 32, 1>, 512, 1, sink, cyc, 0);
  printf("PROBE_DONE\n");
  return 0;
}
