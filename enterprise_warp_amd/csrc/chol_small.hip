// chol_small.hip — register-resident factorisation chol_mfma_kernel<NB <= 9>
// and (dev library only, -DEWH_DEV) its A/B variants (see ewarp_dev.h,
// ewh_set_kernel_mode).
#include "ewarp_dev.h"

namespace ewh_dev {
namespace {

template <int NB, int ALG = PANEL_2L, bool STAMP = false, int W = default_waves(NB), bool FULL = false>
void launch_chol_mfma(const CholJob* jobs, int B, long long u0, long long n, int b_off, const double* theta, int ldth,
                      double* units, hipStream_t st) {
  hipLaunchKernelGGL(HIP_KERNEL_NAME(chol_mfma_kernel<NB, W, ALG, STAMP, 0, FULL>), dim3((unsigned)n),
                     dim3(64), 0, st, jobs, B, u0, b_off, theta, ldth, units, nullptr, 0, 0);
}

}  // namespace

#ifdef EWH_DEV
// (23: the latency kernel with every wait forced to run out, LAT_VAR_STALL;
// 24, 25: latency-kernel variants, chol_lat.hip LAT_VAR_BARRIER / LAT_VAR_R3;
// 26: one wave per SIMD, whole triangle resident, plain right-looking order;
// 28: the C5 row update + panel with one tile per workgroup, one block row
// per pass (round 3); 30: the TwoSum contraction up to 10 blocks;
// 31: the C5 row update one block row per pass, two tiles per workgroup;
// 32: the C5 pair kernel with each U_pj slab loaded at the top of its step)
bool variant_built(int mode) {
  return mode == 15 || mode == 16 || mode == 17 || mode == 19 || mode == 21 || mode == 22 || mode == 23 ||
         mode == 24 || mode == 25 || mode == 26 || mode == 28 || mode == 30 || mode == 31 || mode == 32;
}
// phase stamps of kernel mode 21 (g_stamps: STAMP_UNITS x STAMP_N)
extern "C" int ewh_dev_stamps(long long* out, long long n) {
  if (n > (long long)STAMP_UNITS * STAMP_N) n = (long long)STAMP_UNITS * STAMP_N;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), (size_t)n * sizeof(long long)) == hipSuccess ? 0 : -1;
}
#else
bool variant_built(int) { return false; }
#endif

int launch_chol_small(int mode, int nb, const CholJob* jobs, int B, long long u0, long long n, int b_off,
                      const double* theta, int ldth, double* units, hipStream_t st) {
#ifdef EWH_DEV
  // A/B variants (NB = 8, the C3 reduced width)
  if (nb == 8) {
    switch (mode) {
      case 17: launch_chol_mfma<8, PANEL_1L>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // round-2 one-level panel
      case 21: launch_chol_mfma<8, PANEL_2L, true>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // default + phase stamps
      case 26: launch_chol_mfma<8, PANEL_2L, false, 1, true>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // W = 1, FULL
      default: break;
    }
  }
#endif
  if (mode == 1) return 1;
  // default: the two-level LDL^T panel (ewarp_dev.h PANEL_2L)
  switch (nb) {
    case 1: launch_chol_mfma<1>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;
    case 2: launch_chol_mfma<2>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;
    case 3: launch_chol_mfma<3>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;
    case 4: launch_chol_mfma<4>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;
    case 5: launch_chol_mfma<5>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;
    case 6: launch_chol_mfma<6>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;
    case 7: launch_chol_mfma<7>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;
    case 8: launch_chol_mfma<8>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;
    case 9: launch_chol_mfma<9>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;
    default: return 1;
  }
}

}  // namespace ewh_dev
