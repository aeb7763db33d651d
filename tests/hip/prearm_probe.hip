// Probe (dev only, not part of the library): what a sampler call would save
// if the latency kernel were launched ahead of the call and released by a
// doorbell in coherent pinned host memory ("pre-armed"), against a launch per
// call.  The kernel is the trivial one of theta_stage_probe.hip (read 182
// theta values from pinned memory, write their sum to pinned memory, the
// host spins on it).  Per call: launch-per-call round trip; pre-armed: the
// doorbell-to-result time and the whole call including arming the next
// kernel.  Every poll loop is bounded (the kernel leaves after 20 ms without
// a request or when the stop flag is set; the host gives up after 1 s).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(2); } } while (0)

struct Bell {
  unsigned long long seq;
  unsigned int stop;
  unsigned int pad;
};

__global__ void read_kernel(const double* th, int n, double* out) {
  __shared__ double s[256];
  const int t = threadIdx.x;
  s[t] = t < n ? th[t] : 0.0;
  __syncthreads();
  if (t == 0) {
    double acc = 0.0;
    for (int i = 0; i < n; ++i) acc += s[i];
    out[0] = acc;
  }
}

__global__ void armed_read_kernel(const Bell* bell, unsigned long long want, const double* th, int n, double* out) {
  __shared__ double s[256];
  __shared__ int go;
  const int t = threadIdx.x;
  if (t == 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    int g = 0;
    for (;;) {
      if (__hip_atomic_load(&bell->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
      if (__hip_atomic_load(&bell->seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) == want) {
        g = 1;
        break;
      }
      if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) break;     // 20 ms
      __builtin_amdgcn_s_sleep(1);
    }
    go = g;
  }
  __syncthreads();
  if (!go) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  s[t] = t < n ? th[t] : 0.0;
  __syncthreads();
  if (t == 0) {
    double acc = 0.0;
    for (int i = 0; i < n; ++i) acc += s[i];
    out[0] = acc;
  }
}

static bool spin(volatile double* o, double want) {
  const auto t0 = std::chrono::steady_clock::now();
  for (long i = 0;; ++i) {
    if (*o == want) return true;
    if ((i & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) return false;
  }
}

int main() {
  const int n = 182, reps = 3000;
  const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
  double *h_th, *h_out, *d_th, *d_out;
  Bell *h_bell, *d_bell;
  CK(hipHostMalloc((void**)&h_th, 4096, fl));
  CK(hipHostMalloc((void**)&h_out, 64, fl));
  CK(hipHostMalloc((void**)&h_bell, 64, fl));
  CK(hipHostGetDevicePointer((void**)&d_th, h_th, 0));
  CK(hipHostGetDevicePointer((void**)&d_out, h_out, 0));
  CK(hipHostGetDevicePointer((void**)&d_bell, h_bell, 0));
  h_bell->seq = 0;
  h_bell->stop = 0;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  volatile double* th = h_th;
  volatile double* out = h_out;
  std::vector<double> a, b, c;
  // launch per call
  for (int r = 0; r < reps; ++r) {
    const double base = 1.0 + r;
    for (int i = 0; i < n; ++i) th[i] = base;
    *out = -1.0;
    const auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(read_kernel, dim3(1), dim3(256), 0, st, d_th, n, d_out);
    if (!spin(out, base * n)) { printf("launch path: no result\n"); return 3; }
    a.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  CK(hipStreamSynchronize(st));
  // pre-armed
  unsigned long long want = 1;
  hipLaunchKernelGGL(armed_read_kernel, dim3(1), dim3(256), 0, st, d_bell, want, d_th, n, d_out);
  for (int r = 0; r < reps; ++r) {
    const double base = 1.0 + r;
    for (int i = 0; i < n; ++i) th[i] = base;
    *out = -1.0;
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(&h_bell->seq, want, __ATOMIC_RELEASE);
    if (!spin(out, base * n)) { printf("armed path: no result at %d\n", r); h_bell->stop = 1; (void)hipStreamSynchronize(st); return 3; }
    const auto t1 = std::chrono::steady_clock::now();
    ++want;
    hipLaunchKernelGGL(armed_read_kernel, dim3(1), dim3(256), 0, st, d_bell, want, d_th, n, d_out);
    const auto t2 = std::chrono::steady_clock::now();
    b.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    c.push_back(std::chrono::duration<double, std::micro>(t2 - t0).count());
  }
  __atomic_store_n(&h_bell->stop, 1u, __ATOMIC_RELEASE);
  CK(hipStreamSynchronize(st));
  for (auto* v : {&a, &b, &c}) std::sort(v->begin(), v->end());
  printf("{\"launch_per_call_us\": %.2f, \"armed_doorbell_to_result_us\": %.2f, \"armed_call_incl_rearm_us\": %.2f, "
         "\"p10\": [%.2f, %.2f, %.2f]}\n", a[reps / 2], b[reps / 2], c[reps / 2], a[reps / 10], b[reps / 10], c[reps / 10]);
  return 0;
}
