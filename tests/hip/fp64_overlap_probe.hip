// Which instruction classes share a gfx950 SIMD with v_mfma_f64_16x16x4_f64
// issued by another wave: waves 0-3 of each 512-thread workgroup run op A,
// waves 4-7 run op B (two waves per SIMD), each NA / NB independent chains
// per iteration.  Cycles per iteration (s_memtime, median over waves) of each
// side, alone and together.
//   hipcc --offload-arch=gfx950 -O3 -o fp64_overlap_probe fp64_overlap_probe.hip && ./fp64_overlap_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef double v4d __attribute__((ext_vector_type(4)));
constexpr int ITERS = 1024;

enum { NONE = 0, MFMA = 1, FMA = 2, BPERM = 3, IADD = 4, DPP = 5, RLANE = 6, DSREAD = 7 };

template <int OP, int N>
__device__ __forceinline__ void work(v4d* acc, double* x, int* ix, double a, double b, const double* lds) {
  if constexpr (OP == MFMA) {
#pragma unroll
    for (int j = 0; j < N; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
  } else if constexpr (OP == FMA) {
#pragma unroll
    for (int j = 0; j < N; ++j) x[j] = fma(x[j], 0.999999, 1e-9);
  } else if constexpr (OP == BPERM) {
#pragma unroll
    for (int j = 0; j < N; ++j) ix[j] = __builtin_amdgcn_ds_bpermute(((threadIdx.x + j + 1) & 63) << 2, ix[j]);
  } else if constexpr (OP == IADD) {
#pragma unroll
    for (int j = 0; j < N; ++j) ix[j] = ix[j] * 3 + 1;
  } else if constexpr (OP == DPP) {
#pragma unroll
    for (int j = 0; j < N; ++j) ix[j] = __builtin_amdgcn_update_dpp(0, ix[j], 0x153, 0xf, 0xf, false) + 1;
  } else if constexpr (OP == RLANE) {
#pragma unroll
    for (int j = 0; j < N; ++j) ix[j] = __builtin_amdgcn_readlane(ix[j], 3) + 1;
  } else if constexpr (OP == DSREAD) {
#pragma unroll
    for (int j = 0; j < N; ++j) x[j] += lds[(threadIdx.x & 15) + 16 * ((j + ix[0]) & 7)];
  }
}

template <int OA, int NA, int OB, int NB>
__global__ __launch_bounds__(512) void k_pair(double seed, double* sink, long long* cyc) {
  __shared__ double lds[128];
  if (threadIdx.x < 128) lds[threadIdx.x] = seed + threadIdx.x;
  __syncthreads();
  const int wave = threadIdx.x >> 6;
  v4d acc[8];
  double x[16];
  int ix[16];
  const double a = seed + threadIdx.x * 1e-6, b = seed - threadIdx.x * 1e-6;
  for (int j = 0; j < 8; ++j) acc[j] = v4d{a, b, a, b};
  for (int j = 0; j < 16; ++j) { x[j] = a + j; ix[j] = threadIdx.x + j; }
  const long long t0 = (long long)__builtin_amdgcn_s_memtime();
  if (wave < 4) {
    for (int i = 0; i < ITERS; ++i) work<OA, NA>(acc, x, ix, a, b, lds);
  } else {
    for (int i = 0; i < ITERS; ++i) work<OB, NB>(acc, x, ix, a, b, lds);
  }
  const long long t1 = (long long)__builtin_amdgcn_s_memtime();
  double s = 0;
  for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][3];
  for (int j = 0; j < 16; ++j) s += x[j] + ix[j];
  sink[blockIdx.x * 512 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
}

static double med(std::vector<long long> v) {
  std::sort(v.begin(), v.end());
  return (double)v[v.size() / 2];
}

template <typename K>
static void run(const char* name, K kern, double* sink, long long* cyc) {
  hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, 1.0, sink, cyc);
  (void)hipDeviceSynchronize();
  hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, 1.0, sink, cyc);
  (void)hipDeviceSynchronize();
  std::vector<long long> h(256 * 8);
  (void)hipMemcpy(h.data(), cyc, h.size() * sizeof(long long), hipMemcpyDeviceToHost);
  std::vector<long long> a, b;
  for (int i = 0; i < 256; ++i)
    for (int w = 0; w < 8; ++w) (w < 4 ? a : b).push_back(h[i * 8 + w]);
  printf("%-40s A %8.2f   B %8.2f  cyc/iter\n", name, med(a) / ITERS, med(b) / ITERS);
}

#define RUN(OA, NA, OB, NB) run(#OA "x" #NA " | " #OB "x" #NB, k_pair<OA, NA, OB, NB>, sink, cyc)

int main() {
  double* sink;
  long long* cyc;
  (void)hipMalloc(&sink, 256 * 512 * sizeof(double));
  (void)hipMalloc(&cyc, 256 * 8 * sizeof(long long));
  RUN(MFMA, 4, NONE, 0);
  RUN(NONE, 0, BPERM, 8);
  RUN(MFMA, 4, BPERM, 8);
  RUN(NONE, 0, DSREAD, 8);
  RUN(MFMA, 4, DSREAD, 8);
  RUN(NONE, 0, IADD, 16);
  RUN(MFMA, 4, IADD, 16);
  RUN(NONE, 0, DPP, 16);
  RUN(MFMA, 4, DPP, 16);
  RUN(NONE, 0, RLANE, 16);
  RUN(MFMA, 4, RLANE, 16);
  RUN(NONE, 0, FMA, 16);
  RUN(MFMA, 4, FMA, 16);
  RUN(FMA, 16, BPERM, 8);
  RUN(FMA, 16, IADD, 16);
  RUN(FMA, 16, DSREAD, 8);
  RUN(FMA, 16, FMA, 16);
  RUN(BPERM, 8, BPERM, 8);
  printf("OVERLAP_DONE\n");
  return 0;
}
