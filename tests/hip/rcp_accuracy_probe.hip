// Accuracy of the gfx950 v_rcp_f64 / v_rsq_f64 estimates (before Newton
// refinement), over log-uniform positive doubles 1e-300..1e300 and the
// mantissa range of one binade.  Prints the max relative error in units of
// 2^-52 and its log2.
//   hipcc --offload-arch=gfx950 -O3 -o rcp_accuracy_probe rcp_accuracy_probe.hip && ./rcp_accuracy_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k(const double* x, double* r, double* s, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  r[i] = __builtin_amdgcn_rcp(x[i]);
  s[i] = __builtin_amdgcn_rsq(x[i]);
}

int main() {
  const int n = 1 << 22;
  std::vector<double> x(n), r(n), s(n);
  unsigned long long st = 88172645463325252ull;
  for (int i = 0; i < n; ++i) {
    st ^= st << 13; st ^= st >> 7; st ^= st << 17;
    const double u = (st >> 11) * (1.0 / 9007199254740992.0);
    x[i] = (i & 1) ? std::exp((u - 0.5) * 2 * 690.0) : 1.0 + u;
  }
  double *dx, *dr, *ds;
  (void)hipMalloc(&dx, n * 8); (void)hipMalloc(&dr, n * 8); (void)hipMalloc(&ds, n * 8);
  (void)hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dr, ds, n);
  (void)hipMemcpy(r.data(), dr, n * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(s.data(), ds, n * 8, hipMemcpyDeviceToHost);
  long double er = 0, es = 0;
  for (int i = 0; i < n; ++i) {
    const long double xr = 1.0L / (long double)x[i], xs = 1.0L / sqrtl((long double)x[i]);
    er = fmaxl(er, fabsl((r[i] - xr) / xr));
    es = fmaxl(es, fabsl((s[i] - xs) / xs));
  }
  printf("v_rcp_f64 max rel err %.3Le = %.2Lf ulp(2^-52) = 2^%.2Lf\n", er, er / 2.220446049250313e-16L, log2l(er));
  printf("v_rsq_f64 max rel err %.3Le = %.2Lf ulp(2^-52) = 2^%.2Lf\n", es, es / 2.220446049250313e-16L, log2l(es));
  printf("RCP_PROBE_DONE\n");
  return 0;
}
