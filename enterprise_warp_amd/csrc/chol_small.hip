// chol_small.hip — register-resident factorisation chol_mfma_kernel<NB <= 9>
// and (dev library only, -DEWH_DEV) its A/B variants (see ewarp_dev.h,
// ewh_set_kernel_mode).
#include "ewarp_dev.h"

namespace ewh_dev {
namespace {

template <int NB, int FULL = 0, int W = default_waves(NB), int ALG = 0>
void launch_chol_mfma(const CholJob* jobs, int B, long long u0, long long n, int b_off, const double* theta, int ldth,
                      double* units, hipStream_t st) {
  hipLaunchKernelGGL(HIP_KERNEL_NAME(chol_mfma_kernel<NB, FULL, W, ALG, 0>), dim3((unsigned)n), dim3(64), 0, st, jobs,
                     B, u0, b_off, theta, ldth, units, nullptr, 0, 0);
}

}  // namespace

#ifdef EWH_DEV
bool ab_variants_built() { return true; }
// phase stamps of kernel mode 21 (g_stamps: STAMP_UNITS x STAMP_N)
extern "C" int ewh_dev_stamps(long long* out, long long n) {
  if (n > (long long)STAMP_UNITS * STAMP_N) n = (long long)STAMP_UNITS * STAMP_N;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), (size_t)n * sizeof(long long)) == hipSuccess ? 0 : -1;
}
#else
bool ab_variants_built() { return false; }
#endif

int launch_chol_small(int mode, int nb, const CholJob* jobs, int B, long long u0, long long n, int b_off,
                      const double* theta, int ldth, double* units, hipStream_t st) {
#ifdef EWH_DEV
  // A/B variants (NB = 8, the C3 reduced width)
  if (nb == 8 && mode >= 3) {
    switch (mode) {
#ifdef EWH_DEV_ALL   // round-1/2 panel experiments: make dev DEVALL=1
      case 3: launch_chol_mfma<8, 1, 1, 3>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // 1 wave/SIMD
      case 4: launch_chol_mfma<8, 0, 2, 1>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // LDL, looped
      case 5: launch_chol_mfma<8, 1, 2, 1>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // LDL, bpermute u_i
      case 6: launch_chol_mfma<8, 0, 2, 2>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // LDL, LDS bcast
      case 8: launch_chol_mfma<8, 1, 2, 4>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // DPP, exec-masked pivot row
      case 9: launch_chol_mfma<8, 1, 2, 3>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // unblocked DPP panel (ALG 3)
      case 10: launch_chol_mfma<8, 1, 2, 5>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // blocked panel, rcp / rsqrt + 2 Newton
      case 11: launch_chol_mfma<8, 1, 2, 6>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // + row scales by rsqrt_fast (spills)
      case 12: launch_chol_mfma<8, 1, 2, 7>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // default without the packed row scales
      case 13: launch_chol_mfma<8, 1, 2, 9>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // phase split H = 3, every row scale packed
      case 14: launch_chol_mfma<8, 1, 2, 10>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // ALG 8 + lookahead (trailing MFMAs inside the next panel)
#endif
      case 17: launch_chol_mfma<8, 1, 2, 8>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // ALG 8: DPP mov + fma pairs (the round-1 default)
      case 18: launch_chol_mfma<8, 1, 2, 12>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // + replicated pivot rows (no bpermute in the chain)
      case 22: launch_chol_mfma<8, 1, 2, 16>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // ALG 11 + raised priority in the pivots
      case 23: launch_chol_mfma<8, 1, 2, 17>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // + in the phi prologue
      case 24: launch_chol_mfma<8, 1, 2, 11>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // ALG 11 without the early block-row-0 load
      case 25: launch_chol_mfma<8, 1, 2, 19>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // diagnostic: no spectra (wrong values)
      case 26: launch_chol_mfma<8, 1, 2, 20>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // default (ALG0 18) + phase stamps
      case 27: launch_chol_mfma<8, 1, 2, 21>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // default + A22 blocks loaded during phase 1
      case 28: launch_chol_mfma<8, 1, 2, 18>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // default without the pad-pivot skip
      case 29: launch_chol_mfma<8, 1, 2, 22>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // default without the spectrum dedupe
      case 30: launch_chol_mfma<8, 1, 2, 24>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // default + A22's first block row loaded before the last phase-1 panel
      case 21: launch_chol_mfma<8, 1, 2, 15>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // ALG 11 + phase stamps
      case 20: launch_chol_mfma<8, 1, 2, 14>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // ALG 11 + staggered first generation
      case 19: launch_chol_mfma<8, 1, 2, 13>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // + issue order pinned by sched barriers
      default: break;
    }
  }
#endif
  if (mode == 1) return 1;
  // default: LDL^T panel; up to NB = 8 the steps are unrolled and the panel is
  // blocked (ALG 11: diagonal block by VALU, each pivot's row and E = L^-T
  // updates one fused v_fmac_f64_dpp per register -- bit-identical to ALG 8,
  // the DPP-mov + fma form --, the rest of the block row by MFMA with L^-1;
  // quotients by one cubic correction of the rcp estimate; phase-3 row scales
  // packed; block row 0 loaded before the spectra; the last panel's pad
  // pivots skipped; each distinct spectrum formed once: ALG0 23); mode 2:
  // the round-1 Cholesky panel (looped) as the A/B baseline
  const bool base = mode == 2;
#define EWH_CHOL_CASE(NBV)                                                                                   \
  case NBV:                                                                                                  \
    if (base) launch_chol_mfma<NBV, 0, default_waves(NBV), 0>(jobs, B, u0, n, b_off, theta, ldth, units, st); \
    else launch_chol_mfma<NBV, (NBV <= 8), default_waves(NBV), (NBV <= 8 ? 23 : 1)>(jobs, B, u0, n, b_off, theta, ldth, units, st); \
    return 0;
  switch (nb) {
    EWH_CHOL_CASE(1)
    EWH_CHOL_CASE(2)
    EWH_CHOL_CASE(3)
    EWH_CHOL_CASE(4)
    EWH_CHOL_CASE(5)
    EWH_CHOL_CASE(6)
    EWH_CHOL_CASE(7)
    EWH_CHOL_CASE(8)
    EWH_CHOL_CASE(9)
    default: return 1;
  }
#undef EWH_CHOL_CASE
}

}  // namespace ewh_dev
