// chol_partial.hip — chol_mfma_kernel<..., KEEP>: per-pulsar partial
// factorisation for the correlated common process (see ewarp_hip.hip).
#include "ewarp_dev.h"

namespace ewh_dev {
namespace {

template <int NB, int KEEP>
int launch_partial(const CholJob* jobs, int B, long long u0, long long n, int b_off, const double* theta, int ldth,
                   double* units, double* keep_out, int keep_bs, hipStream_t st) {
  if constexpr (NB - KEEP >= Split<NB>::H && NB - KEEP >= 0) {
    hipLaunchKernelGGL(HIP_KERNEL_NAME(chol_mfma_kernel<NB, default_waves(NB), PANEL_2L, false, KEEP>),
                       dim3((unsigned)n), dim3(64), 0, st, jobs, B, u0, b_off, theta, ldth, units, keep_out, 0,
                       keep_bs);
    return 0;
  } else {
    return set_err(EWH_E_UNSUPPORTED, "common: reduced basis too narrow for the kept common block");
  }
}

}  // namespace

int launch_partial_nb(int nb, int keep, const CholJob* jobs, int B, long long u0, long long n, int b_off,
                      const double* theta, int ldth, double* units, double* keep_out, int keep_bs, hipStream_t st) {
#define EWH_PART(NBV)                                                                                             \
  case NBV:                                                                                                       \
    return keep == 1 ? launch_partial<NBV, 1>(jobs, B, u0, n, b_off, theta, ldth, units, keep_out, keep_bs, st)   \
                     : launch_partial<NBV, 2>(jobs, B, u0, n, b_off, theta, ldth, units, keep_out, keep_bs, st);
  switch (nb) {
    EWH_PART(2)
    EWH_PART(3)
    EWH_PART(4)
    EWH_PART(5)
    EWH_PART(6)
    EWH_PART(7)
    EWH_PART(8)
    EWH_PART(9)
    default: return set_err(EWH_E_UNSUPPORTED, "common: unsupported reduced width");
  }
#undef EWH_PART
}


}  // namespace ewh_dev
