// Probe (dev only, not part of the library): where should a one-proposal
// call put theta?  The latency kernel reads theta from coherent pinned host
// memory; its stamps show ~6 k cycles before theta is staged (a PCIe read
// round trip).  This measures, per staging kind, (1) whether the host can
// store to it, (2) the in-kernel latency of the first dependent read and
// (3) the host round trip of a call: host writes 182 doubles, launches a
// 1-workgroup kernel that sums them and writes the sum to pinned memory,
// host spins on it.  Kinds: pinned coherent host memory (the current
// staging), fine-grained device memory, uncached device memory.
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(2); } } while (0)

__global__ void read_kernel(const double* th, int n, volatile double* out, long long* cyc) {
  __shared__ double s[256];
  const int t = threadIdx.x;
  const long long t0 = (long long)__builtin_amdgcn_s_memtime();
  double v = t < n ? th[t] : 0.0;
  s[t] = v;
  __syncthreads();
  const long long t1 = (long long)__builtin_amdgcn_s_memtime();
  if (t == 0) {
    double acc = 0.0;
    for (int i = 0; i < n; ++i) acc += s[i];
    out[0] = acc;
    cyc[0] = t1 - t0;
  }
}

static bool host_can_touch(double* p) {
  const pid_t pid = fork();
  if (pid == 0) {
    volatile double* q = p;
    q[0] = 1.0;
    const double r = q[0];
    _exit(r == 1.0 ? 0 : 3);
  }
  int st = 0;
  waitpid(pid, &st, 0);
  return WIFEXITED(st) && WEXITSTATUS(st) == 0;
}

int main() {
  const int n = 182, reps = 2000;
  double* h_out;
  CK(hipHostMalloc((void**)&h_out, 64, hipHostMallocMapped | hipHostMallocCoherent));
  double* d_out;
  CK(hipHostGetDevicePointer((void**)&d_out, h_out, 0));
  long long* d_cyc;
  CK(hipMalloc((void**)&d_cyc, 64));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  struct Kind { const char* name; int k; };
  const Kind kinds[] = {{"pinned_coherent", 0}, {"pinned_noncoherent", 1}, {"device_finegrained", 2}, {"device_uncached", 3}};
  for (const Kind& K : kinds) {
    double* host = nullptr;   // host-side pointer
    double* dev = nullptr;    // kernel-side pointer
    if (K.k == 0 || K.k == 1) {
      CK(hipHostMalloc((void**)&host, 4096, hipHostMallocMapped | (K.k == 0 ? hipHostMallocCoherent : hipHostMallocNonCoherent)));
      CK(hipHostGetDevicePointer((void**)&dev, host, 0));
    } else {
      hipError_t e = hipExtMallocWithFlags((void**)&dev, 4096, K.k == 2 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached);
      if (e != hipSuccess) { printf("%s: alloc failed %s\n", K.name, hipGetErrorString(e)); continue; }
      host = dev;
      if (!host_can_touch(host)) { printf("%s: host cannot store to it\n", K.name); continue; }
    }
    std::vector<double> ts;
    std::vector<long long> cs;
    for (int r = 0; r < reps; ++r) {
      const double base = 1.0 + r;
      for (int i = 0; i < n; ++i) ((volatile double*)host)[i] = base;
      ((volatile double*)h_out)[0] = -1.0;
      const auto t0 = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(read_kernel, dim3(1), dim3(256), 0, st, dev, n, d_out, d_cyc);
      while (((volatile double*)h_out)[0] != base * n) {}
      const auto t1 = std::chrono::steady_clock::now();
      ts.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      CK(hipStreamSynchronize(st));
      long long c;
      CK(hipMemcpy(&c, d_cyc, sizeof c, hipMemcpyDeviceToHost));
      cs.push_back(c);
    }
    std::sort(ts.begin(), ts.end());
    std::sort(cs.begin(), cs.end());
    printf("%s: call round trip median %.2f us (p10 %.2f); in-kernel read+stage median %lld cycles\n", K.name,
           ts[reps / 2], ts[reps / 10], cs[reps / 2]);
  }
  return 0;
}
