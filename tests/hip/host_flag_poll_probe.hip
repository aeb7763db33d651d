// Probe (dev only, not part of the library): can a running kernel see a flag
// the host writes into coherent pinned host memory, and how fast?  Written for
// the round-4 persistent latency server experiment (measured
// slower than a launch per call, removed).  Result (MI355X): a system-scope
// atomic load, a volatile load and a fenced relaxed load all see the flag
// within one poll (~1.4 us per poll, a PCIe round trip); a nontemporal load
// never does.  One
// wave polls a host flag with one of several load forms until it reads 1 or
// 50 ms of the 100 MHz real-time counter pass (every poll loop is bounded);
// the host sets the flag 2 ms after the launch.  Prints, per form and
// allocation kind, whether the flag was seen and after how long.
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(2); } } while (0)

__global__ void poll_kernel(unsigned int* flag, int form, unsigned long long* out) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned long long n = 0, t = t0;
  unsigned int v = 0;
  while (t - t0 < 5000000ull) {            // 50 ms
    ++n;
    if (form == 0) {
      v = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (form == 1) {
      v = *(volatile unsigned int*)flag;
    } else if (form == 2) {
      v = __builtin_nontemporal_load(flag);
    } else if (form == 3) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      v = __hip_atomic_fetch_add(flag, 0u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (v == 1u) break;
    __builtin_amdgcn_s_sleep(1);
    t = __builtin_amdgcn_s_memrealtime();
  }
  out[0] = v;
  out[1] = __builtin_amdgcn_s_memrealtime() - t0;
  out[2] = n;
}

int main(int argc, char** argv) {
  const int maxform = argc > 1 ? atoi(argv[1]) : 3;      // (form 4, a PCIe atomic, only on request)
  const char* kinds[] = {"coherent", "coherent|mapped|portable", "noncoherent|mapped"};
  const unsigned flags[] = {hipHostMallocCoherent, hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable,
                            hipHostMallocNonCoherent | hipHostMallocMapped};
  unsigned long long* out;
  CK(hipHostMalloc((void**)&out, 64, hipHostMallocCoherent | hipHostMallocMapped));
  for (int kd = 0; kd < 3; ++kd) {
    unsigned int* flag;
    CK(hipHostMalloc((void**)&flag, 4096, flags[kd]));
    unsigned int* dflag;
    CK(hipHostGetDevicePointer((void**)&dflag, flag, 0));
    for (int form = 0; form <= maxform; ++form) {
      __atomic_store_n(flag, 0u, __ATOMIC_RELEASE);
      out[0] = out[1] = out[2] = 0;
      hipLaunchKernelGGL(poll_kernel, dim3(1), dim3(64), 0, 0, dflag, form, out);
      std::this_thread::sleep_for(std::chrono::milliseconds(2));
      __atomic_store_n(flag, 1u, __ATOMIC_RELEASE);
      CK(hipDeviceSynchronize());
      printf("{\"kind\": \"%s\", \"form\": %d, \"seen\": %llu, \"us_in_kernel\": %.1f, \"polls\": %llu}\n", kinds[kd],
             form, out[0], out[1] / 100.0, out[2]);
      fflush(stdout);
    }
    CK(hipHostFree(flag));
  }
  CK(hipHostFree(out));
  return 0;
}
