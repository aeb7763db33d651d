// contract.hip — instantiations of the contraction kernels (see ewarp_dev.h);
// bases past 16 blocks: contract_wide.hip.
#include "ewarp_dev.h"

namespace ewh_dev {
namespace {

template <int NB>
void launch_contract(const PsrDev& P, const double* w, const double* beta, const double* s, const double* fac,
                     double* G, int nb_samples, hipStream_t st) {
  const size_t lds = (size_t)(CT_ROWS * 16 * NB + CT_ROWS) * sizeof(double);
  hipLaunchKernelGGL(HIP_KERNEL_NAME(contract_mfma_kernel<NB>), dim3(nb_samples), dim3(256), lds, st, P, w, beta, s,
                     fac, G);
}

int dispatch_contract(int nb, const PsrDev& P, const double* w, const double* beta, const double* s,
                      const double* fac, double* G, int nb_samples, hipStream_t st, double* Glo) {
  if (nb > 16) return launch_contract_wide(nb, P, w, beta, s, fac, G, nb_samples, st, Glo);   // (contract_wide.hip)
  switch (nb) {
    case 1: launch_contract<1>(P, w, beta, s, fac, G, nb_samples, st); break;
    case 2: launch_contract<2>(P, w, beta, s, fac, G, nb_samples, st); break;
    case 3: launch_contract<3>(P, w, beta, s, fac, G, nb_samples, st); break;
    case 4: launch_contract<4>(P, w, beta, s, fac, G, nb_samples, st); break;
    case 5: launch_contract<5>(P, w, beta, s, fac, G, nb_samples, st); break;
    case 6: launch_contract<6>(P, w, beta, s, fac, G, nb_samples, st); break;
    case 7: launch_contract<7>(P, w, beta, s, fac, G, nb_samples, st); break;
    case 8: launch_contract<8>(P, w, beta, s, fac, G, nb_samples, st); break;
    case 9: launch_contract<9>(P, w, beta, s, fac, G, nb_samples, st); break;
    case 10: launch_contract<10>(P, w, beta, s, fac, G, nb_samples, st); break;
    case 11: launch_contract<11>(P, w, beta, s, fac, G, nb_samples, st); break;
    case 12: launch_contract<12>(P, w, beta, s, fac, G, nb_samples, st); break;
    case 13: launch_contract<13>(P, w, beta, s, fac, G, nb_samples, st); break;
    case 14: launch_contract<14>(P, w, beta, s, fac, G, nb_samples, st); break;
    case 15: launch_contract<15>(P, w, beta, s, fac, G, nb_samples, st); break;
    case 16: launch_contract<16>(P, w, beta, s, fac, G, nb_samples, st); break;
    default: return set_err(EWH_E_UNSUPPORTED, "basis too wide for the contraction kernel (> 255 columns)");
  }
  return 0;
}

constexpr size_t contract2_lds(int nb) { return (size_t)(2 * CT_ROWS * 16 * nb + 6 * CT_ROWS) * sizeof(double); }

// waves per sample: 4, or 8 where measured faster (fewer accumulators per
// wave: more waves per SIMD to hide the k-steps' LDS latency)
constexpr int contract2_default_waves(int nb) { return nb >= 9 || contract2_comp(nb) == CT_TWOSUM ? 8 : 4; }
// the run remainder on the last waves (ct_run_start) where the accumulator is
// single (NB <= 9: C2's ECORR model); the blocked NB >= 10 kernel keeps the
// round-4 order -- with the remainder moved its spill grew 12 -> 28 B/lane
constexpr bool contract2_late(int nb) { return nb <= 9; }

template <int NB>
int launch_contract2(int waves, const PsrDev& P, const double* w, const double* beta, double* s, long long s_stride,
                     double* G, int nb_samples, hipStream_t st, const double* rho) {
  // (the dynamic-LDS attribute is set per device by set_contract_attributes)
  constexpr int CP = contract2_comp(NB);
#ifdef EWH_DEV
  if constexpr (NB <= 10) {
    if (waves == 30) {   // (dev A/B: TwoSum accumulation)
      hipLaunchKernelGGL(HIP_KERNEL_NAME(contract2_kernel<NB, 8, CT_TWOSUM>), dim3(nb_samples), dim3(512),
                         contract2_lds(NB), st, P, w, beta, s, s_stride, G, nullptr);
      return 0;
    }
    if (waves == 38 || waves == 39) {   // (dev A/B: blocked accumulation, 4 / 8 waves)
      if (waves == 39)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(contract2_kernel<NB, 8, CT_BLOCKED, contract2_late(NB)>), dim3(nb_samples),
                           dim3(512), contract2_lds(NB), st, P, w, beta, s, s_stride, G, nullptr);
      else
        hipLaunchKernelGGL(HIP_KERNEL_NAME(contract2_kernel<NB, 4, CT_BLOCKED, contract2_late(NB)>), dim3(nb_samples),
                           dim3(256), contract2_lds(NB), st, P, w, beta, s, s_stride, G, nullptr);
      return 0;
    }
  }
  if (waves == 35) {     // (dev A/B: the extra blocks on the first waves, round 4-5a)
    if (contract2_default_waves(NB) == 8)
      hipLaunchKernelGGL(HIP_KERNEL_NAME(contract2_kernel<NB, 8, CP, false>), dim3(nb_samples), dim3(512),
                         contract2_lds(NB), st, P, w, beta, s, s_stride, G, nullptr);
    else
      hipLaunchKernelGGL(HIP_KERNEL_NAME(contract2_kernel<NB, 4, CP, false>), dim3(nb_samples), dim3(256),
                         contract2_lds(NB), st, P, w, beta, s, s_stride, G, nullptr);
    return 0;
  }
#endif
  if (waves == 0 || waves == 30) waves = contract2_default_waves(NB);
  constexpr bool LT = contract2_late(NB);
  if constexpr (NB >= 2) {
    if (rho) {   // the r-separated contraction (run_white decides; no ECORR, m <= 16 (NB - 1))
      if (waves == 8)
        hipLaunchKernelGGL(HIP_KERNEL_NAME(contract2_kernel<NB, 8, CP, LT, true>), dim3(nb_samples), dim3(512),
                           contract2_lds(NB), st, P, w, beta, s, s_stride, G, rho);
      else
        hipLaunchKernelGGL(HIP_KERNEL_NAME(contract2_kernel<NB, 4, CP, LT, true>), dim3(nb_samples), dim3(256),
                           contract2_lds(NB), st, P, w, beta, s, s_stride, G, rho);
      return 0;
    }
  }
  if (waves == 8)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(contract2_kernel<NB, 8, CP, LT>), dim3(nb_samples), dim3(512),
                       contract2_lds(NB), st, P, w, beta, s, s_stride, G, nullptr);
  else
    hipLaunchKernelGGL(HIP_KERNEL_NAME(contract2_kernel<NB, 4, CP, LT>), dim3(nb_samples), dim3(256),
                       contract2_lds(NB), st, P, w, beta, s, s_stride, G, nullptr);
  return 0;
}

int dispatch_contract2(int nb, int waves, const PsrDev& P, const double* w, const double* beta, double* s,
                       long long s_stride, double* G, int nb_samples, hipStream_t st, const double* rho) {
  int rc = 1;
  static_for<1, CONTRACT2_NB_MAX + 1>([&](auto N) {
    if (nb == decltype(N)::value)
      rc = launch_contract2<decltype(N)::value>(waves, P, w, beta, s, s_stride, G, nb_samples, st, rho);
  });
  if (rc == 1) return set_err(EWH_E_UNSUPPORTED, "basis too wide for the pipelined contraction (> 207 columns)");
  return rc;
}

template <int NB>
int set_attr2() {
  constexpr int CP = contract2_comp(NB);
  constexpr bool LT = contract2_late(NB);
  EWH_HIP(hipFuncSetAttribute((const void*)contract2_kernel<NB, 4, CP, LT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)contract2_lds(NB)));
  EWH_HIP(hipFuncSetAttribute((const void*)contract2_kernel<NB, 8, CP, LT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)contract2_lds(NB)));
  if constexpr (NB >= 2) {
    EWH_HIP(hipFuncSetAttribute((const void*)contract2_kernel<NB, 4, CP, LT, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)contract2_lds(NB)));
    EWH_HIP(hipFuncSetAttribute((const void*)contract2_kernel<NB, 8, CP, LT, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)contract2_lds(NB)));
  }
#ifdef EWH_DEV
  if constexpr (NB <= 10) {
    EWH_HIP(hipFuncSetAttribute((const void*)contract2_kernel<NB, 8, CT_TWOSUM>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)contract2_lds(NB)));
    EWH_HIP(hipFuncSetAttribute((const void*)contract2_kernel<NB, 4, CT_BLOCKED, contract2_late(NB)>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)contract2_lds(NB)));
    EWH_HIP(hipFuncSetAttribute((const void*)contract2_kernel<NB, 8, CT_BLOCKED, contract2_late(NB)>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)contract2_lds(NB)));
  }
  EWH_HIP(hipFuncSetAttribute((const void*)contract2_kernel<NB, 4, CP, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)contract2_lds(NB)));
  EWH_HIP(hipFuncSetAttribute((const void*)contract2_kernel<NB, 8, CP, false>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)contract2_lds(NB)));
#endif
  return 0;
}

template <int NB>
int set_attr1() {
  const size_t lds = (size_t)(CT_ROWS * 16 * NB + CT_ROWS) * sizeof(double);
  EWH_HIP(hipFuncSetAttribute((const void*)contract_mfma_kernel<NB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds));
  return 0;
}

}  // namespace

// dynamic-LDS limits of every contraction instantiation on the current device
int set_contract_attributes() {
  int rc = 0;
  static_for<1, CONTRACT2_NB_MAX + 1>([&](auto N) {
    if (!rc) rc = set_attr2<decltype(N)::value>();
  });
  static_for<1, 17>([&](auto N) {
    if (!rc) rc = set_attr1<decltype(N)::value>();
  });
  return rc;
}

int launch_contract_nb(int nb, const PsrDev& P, const double* w, const double* beta, const double* s,
                       const double* fac, double* G, int nb_samples, hipStream_t st, double* Glo) {
  return dispatch_contract(nb, P, w, beta, s, fac, G, nb_samples, st, Glo);
}

int launch_contract2_nb(int nb, int waves, const PsrDev& P, const double* w, const double* beta, double* s,
                        long long s_stride, double* G, int nb_samples, hipStream_t st, const double* rho) {
  return dispatch_contract2(nb, waves, P, w, beta, s, s_stride, G, nb_samples, st, rho);
}

}  // namespace ewh_dev
