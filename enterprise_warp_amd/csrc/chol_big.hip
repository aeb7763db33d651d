// chol_big.hip — left-looking wide-basis factorisation chol_big_kernel<NB 10..16>.
#include "ewarp_dev.h"

namespace ewh_dev {
namespace {

template <int NB>
void launch_chol_big(const CholJob* jobs, int B, long long u0, long long n, int b_off, const double* theta, int ldth,
                     double* units, double* scr, long long cap, hipStream_t st) {
  for (long long o = 0; o < n; o += cap)   // one scratch slot per workgroup of a launch
    hipLaunchKernelGGL(HIP_KERNEL_NAME(chol_big_kernel<NB>), dim3((unsigned)std::min(cap, n - o)), dim3(64), 0, st,
                       jobs, B, u0 + o, b_off, theta, ldth, units, scr);
}

}  // namespace

int launch_chol_big_nb(int nb, const CholJob* jobs, int B, long long u0, long long n, int b_off,
                       const double* theta, int ldth, double* units, double* scr, long long cap, hipStream_t st) {
  switch (nb) {
    case 10: launch_chol_big<10>(jobs, B, u0, n, b_off, theta, ldth, units, scr, cap, st); return 0;
    case 11: launch_chol_big<11>(jobs, B, u0, n, b_off, theta, ldth, units, scr, cap, st); return 0;
    case 12: launch_chol_big<12>(jobs, B, u0, n, b_off, theta, ldth, units, scr, cap, st); return 0;
    case 13: launch_chol_big<13>(jobs, B, u0, n, b_off, theta, ldth, units, scr, cap, st); return 0;
    case 14: launch_chol_big<14>(jobs, B, u0, n, b_off, theta, ldth, units, scr, cap, st); return 0;
    case 15: launch_chol_big<15>(jobs, B, u0, n, b_off, theta, ldth, units, scr, cap, st); return 0;
    case 16: launch_chol_big<16>(jobs, B, u0, n, b_off, theta, ldth, units, scr, cap, st); return 0;
    default: return set_err(EWH_E_UNSUPPORTED, "basis too wide (> 255 reduced columns)");
  }
}

}  // namespace ewh_dev
