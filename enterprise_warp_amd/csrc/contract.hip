// contract.hip — instantiations of the contraction kernels (see ewarp_dev.h).
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

// Any width (NB > 16, up to WIDE_NB_MAX): the contraction of
// contract_mfma_kernel with NB a runtime value.  Grid (groups, samples): the
// workgroup of group x owns the upper 16x16 blocks [32 x, 32 x + 32) (8 per
// wave, blocks w + 4 sl); TOA tiles of WT_ROWS rows, every column, are staged
// in LDS and shared by the four waves; pass 0 the TOA rows (weights w), pass 1
// the epoch rows (the epoch sums s, weights -beta).  Each workgroup streams
// the whole basis: for these rare wide bases the re-read is the price of
// holding 8 accumulators per wave.  Compensated as contract2_kernel: each
// group of WT_GROUP tiles is summed into a fresh accumulator, added into
// hi + lo by TwoSum; G = hi (rounded) and, when Glo is given, Glo = the
// remainder (the double-double input of chol_dd_kernel).
constexpr int WT_ROWS = 16;
constexpr int WT_GROUP = 4;
constexpr int WSL = 8;
constexpr size_t contract_wide_lds(int ld) { return (size_t)(WT_ROWS * ld + WT_ROWS) * sizeof(double); }

__global__ __launch_bounds__(256) void contract_wide_kernel(PsrDev P, const double* __restrict__ w,
                                                            const double* __restrict__ beta,
                                                            const double* __restrict__ s,
                                                            const double* __restrict__ fac, double* __restrict__ G,
                                                            double* __restrict__ Glo) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int LD = P.ld, NB = LD >> 4, NBLK = NB * (NB + 1) / 2;
  double* tile = smem;                     // WT_ROWS x LD
  double* wt = smem + WT_ROWS * LD;        // WT_ROWS weights
  const int bl = blockIdx.y;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;
  int bi[WSL], bj[WSL];
  bool valid[WSL];
#pragma unroll
  for (int sl = 0; sl < WSL; ++sl) {
    int blk = 4 * WSL * blockIdx.x + wave + 4 * sl;
    valid[sl] = blk < NBLK;
    int i = 0;
    while (blk >= NB - i && i < NB - 1) { blk -= NB - i; ++i; }
    bi[sl] = i;
    bj[sl] = i + blk;
  }
  v4d acc[WSL], hi[WSL], lo[WSL];
#pragma unroll
  for (int sl = 0; sl < WSL; ++sl) {
    acc[sl] = v4d{0.0, 0.0, 0.0, 0.0};
    hi[sl] = acc[sl];
    lo[sl] = acc[sl];
  }
  auto flush = [&]() {
#pragma unroll
    for (int sl = 0; sl < WSL; ++sl)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const dd t = dd_two_sum(hi[sl][r], acc[sl][r]);
        hi[sl][r] = t.hi;
        lo[sl][r] += t.lo;
        acc[sl][r] = 0.0;
      }
  };
  for (int pass = 0; pass < 2; ++pass) {
    const int nrows = pass == 0 ? P.n_toa : P.n_epoch;
    const double* src = pass == 0 ? P.T : s + (long long)bl * P.n_epoch * LD;
    const double* wsrc = pass == 0 ? w + (long long)bl * P.n_toa : beta + (long long)bl * P.n_epoch;
    const double wsign = pass == 0 ? 1.0 : -1.0;
    for (int t0 = 0; t0 < nrows; t0 += WT_ROWS) {
      const int rows = min(WT_ROWS, nrows - t0);
      for (int idx = threadIdx.x; idx < WT_ROWS * LD; idx += 256) {
        const int r = idx / LD, cc = idx - r * LD;
        double v = r < rows ? src[(long long)(t0 + r) * LD + cc] : 0.0;
        if (pass == 0 && P.n_bgroup) {   // theta-dependent chromatic columns: scale per TOA
          const int g = P.col_bgroup[cc];
          if (g >= 0 && r < rows) v *= fac[((long long)bl * P.n_bgroup + g) * P.n_toa + t0 + r];
        }
        tile[idx] = v;
      }
      if (threadIdx.x < WT_ROWS) wt[threadIdx.x] = (int)threadIdx.x < rows ? wsign * wsrc[t0 + threadIdx.x] : 0.0;
      __syncthreads();
#pragma unroll
      for (int kk = 0; kk < WT_ROWS / 4; ++kk) {
        const int row = 4 * kk + q;
        const double wr = wt[row];
        const double* trow = tile + row * LD + c;
#pragma unroll
        for (int sl = 0; sl < WSL; ++sl) {
          if (valid[sl]) {
            const double a = wr * trow[16 * bi[sl]];
            const double b = trow[16 * bj[sl]];
            acc[sl] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[sl], 0, 0, 0);
          }
        }
      }
      if ((t0 / WT_ROWS) % WT_GROUP == WT_GROUP - 1 || t0 + WT_ROWS >= nrows) flush();
      __syncthreads();
    }
  }
  double* out = G + (long long)bl * LD * LD;
  double* outl = Glo ? Glo + (long long)bl * LD * LD : nullptr;
#pragma unroll
  for (int sl = 0; sl < WSL; ++sl) {
    if (!valid[sl]) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * bi[sl] + q + 4 * r, col = 16 * bj[sl] + c;
      dd v = dd_fast(hi[sl][r], lo[sl][r]);
      if (row == col && row >= P.m && row < LD - 1) v = {1.0, 0.0};
      out[(long long)row * LD + col] = v.hi;
      out[(long long)col * LD + row] = v.hi;
      if (outl) {
        outl[(long long)row * LD + col] = v.lo;
        outl[(long long)col * LD + row] = v.lo;
      }
    }
  }
}

int dispatch_contract(int nb, const PsrDev& P, const double* w, const double* beta, const double* s,
                      const double* fac, double* G, int nb_samples, hipStream_t st, double* Glo) {
  if (nb > 16) {
    if (nb > WIDE_NB_MAX) return set_err(EWH_E_UNSUPPORTED, "basis wider than 1023 columns");
    const int nblk = nb * (nb + 1) / 2;
    hipLaunchKernelGGL(contract_wide_kernel, dim3((nblk + 4 * WSL - 1) / (4 * WSL), nb_samples), dim3(256),
                       contract_wide_lds(16 * nb), st, P, w, beta, s, fac, G, Glo);
    return 0;
  }
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
constexpr int contract2_default_waves(int nb) { return nb >= 9 ? 8 : 4; }

template <int NB>
int launch_contract2(int waves, const PsrDev& P, const double* w, const double* beta, double* s, long long s_stride,
                     double* G, int nb_samples, hipStream_t st) {
  // (the dynamic-LDS attribute is set per device by set_contract_attributes)
  constexpr int CP = contract2_comp(NB);
#ifdef EWH_DEV
  if constexpr (NB <= 10) {
    if (waves == 30) {   // (dev A/B: TwoSum accumulation)
      hipLaunchKernelGGL(HIP_KERNEL_NAME(contract2_kernel<NB, 8, CT_TWOSUM>), dim3(nb_samples), dim3(512),
                         contract2_lds(NB), st, P, w, beta, s, s_stride, G);
      return 0;
    }
  }
#endif
  if (waves == 0 || waves == 30) waves = contract2_default_waves(NB);
  if (waves == 8)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(contract2_kernel<NB, 8, CP>), dim3(nb_samples), dim3(512), contract2_lds(NB),
                       st, P, w, beta, s, s_stride, G);
  else
    hipLaunchKernelGGL(HIP_KERNEL_NAME(contract2_kernel<NB, 4, CP>), dim3(nb_samples), dim3(256), contract2_lds(NB),
                       st, P, w, beta, s, s_stride, G);
  return 0;
}

int dispatch_contract2(int nb, int waves, const PsrDev& P, const double* w, const double* beta, double* s,
                       long long s_stride, double* G, int nb_samples, hipStream_t st) {
  int rc = 1;
  static_for<1, CONTRACT2_NB_MAX + 1>([&](auto N) {
    if (nb == decltype(N)::value) rc = launch_contract2<decltype(N)::value>(waves, P, w, beta, s, s_stride, G, nb_samples, st);
  });
  if (rc == 1) return set_err(EWH_E_UNSUPPORTED, "basis too wide for the pipelined contraction (> 207 columns)");
  return rc;
}

template <int NB>
int set_attr2() {
  constexpr int CP = contract2_comp(NB);
  EWH_HIP(hipFuncSetAttribute((const void*)contract2_kernel<NB, 4, CP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)contract2_lds(NB)));
  EWH_HIP(hipFuncSetAttribute((const void*)contract2_kernel<NB, 8, CP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)contract2_lds(NB)));
#ifdef EWH_DEV
  if constexpr (NB <= 10)
    EWH_HIP(hipFuncSetAttribute((const void*)contract2_kernel<NB, 8, CT_TWOSUM>,
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
  if (!rc && hipFuncSetAttribute((const void*)contract_wide_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)contract_wide_lds(WIDE_LD_MAX)) != hipSuccess)
    rc = set_err(EWH_E_HIP, "hipFuncSetAttribute(contract_wide_kernel) failed");
  return rc;
}

int launch_contract_nb(int nb, const PsrDev& P, const double* w, const double* beta, const double* s,
                       const double* fac, double* G, int nb_samples, hipStream_t st, double* Glo) {
  return dispatch_contract(nb, P, w, beta, s, fac, G, nb_samples, st, Glo);
}

int launch_contract2_nb(int nb, int waves, const PsrDev& P, const double* w, const double* beta, double* s,
                        long long s_stride, double* G, int nb_samples, hipStream_t st) {
  return dispatch_contract2(nb, waves, P, w, beta, s, s_stride, G, nb_samples, st);
}

}  // namespace ewh_dev
