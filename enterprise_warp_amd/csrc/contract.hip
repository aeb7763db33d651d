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

// Any width (NB > 16, up to WIDE_NB_MAX): the per-sample contraction with NB
// a runtime value -- the ECORR term after contract_xr_kernel (epochs_only:
// G_b -= sum_e beta_e s_e s_e^T, continuing from its G_hi / G_lo), or both
// terms where the basis depends on theta (chromatic index sampled: pass 0
// scales those columns per TOA by fac).  Grid (workgroups, samples): the upper
// triangle is cut into super-blocks of 2 block rows x 4 block columns
// (SB row R: rows 2R, 2R + 1; SB column C: columns 4C .. 4C + 3; blocks below
// the diagonal skipped), one per wave, four per workgroup in row-major SB
// order.  Per k-step (4 rows) a lane loads its two row operands and four
// column operands straight from L2 (the row data -- T or the epoch sums s_b --
// is read by every wave of every workgroup of the sample: L1 / L2 resident),
// one step ahead: 6 loads and 2 weight multiplies for 8 MFMAs (round 4:
// blocks dealt round-robin, 16 LDS reads + 8 multiplies per 8 MFMAs, a 16-row
// LDS tile staged by scalar loads with an integer division per element:
// 0.066 of the fp64 peak on 372 columns).  Compensated as contract2: groups
// of WT_GROUP rows summed by the MFMAs into fresh accumulators, added into
// hi + lo by TwoSum; G = hi (rounded) and, when Glo is given, Glo = the
// remainder (the double-double input of chol_dd_kernel).
constexpr int WT_GROUP = 128;
// EWARP_CONTRACT_WIDE_ONLY=1: both terms by this kernel (no contract_xr_kernel; A/B)
bool contract_wide_only() {
  static const bool v = [] {
    const char* e = getenv("EWARP_CONTRACT_WIDE_ONLY");
    return e && e[0] == '1';
  }();
  return v;
}

// super-blocks of an NB-block upper triangle, row-major: count / decode
__host__ __device__ inline int sb_cols(int nb) { return (nb + 3) / 4; }
__host__ __device__ inline int sb_count(int nb) {
  int n = 0;
  for (int R = 0; 2 * R < nb; ++R) n += sb_cols(nb) - (2 * R) / 4;
  return n;
}

__global__ __launch_bounds__(256) void contract_wide_kernel(PsrDev P, const double* __restrict__ w,
                                                            const double* __restrict__ beta,
                                                            const double* __restrict__ s,
                                                            const double* __restrict__ fac, double* __restrict__ G,
                                                            double* __restrict__ Glo, int epochs_only) {
  const int LD = P.ld, NB = LD >> 4;
  const int bl = blockIdx.y;
  const int lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;
  // this wave's super-block (uniform)
  int sb = __builtin_amdgcn_readfirstlane(4 * (int)blockIdx.x + (int)(threadIdx.x >> 6));
  if (sb >= sb_count(NB)) return;          // (no barrier in this kernel)
  int R = 0;
  while (sb >= sb_cols(NB) - (2 * R) / 4) {
    sb -= sb_cols(NB) - (2 * R) / 4;
    ++R;
  }
  const int C = (2 * R) / 4 + sb;
  const int i0 = 2 * R, j0 = 4 * C;
  bool valid[2][4];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int k = 0; k < 4; ++k) valid[x][k] = i0 + x < NB && j0 + k < NB && i0 + x <= j0 + k;
  v4d acc[2][4], hi[2][4], lo[2][4];
  double* gout = G + (long long)bl * LD * LD;
  double* glo = Glo ? Glo + (long long)bl * LD * LD : nullptr;
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc[x][k] = hi[x][k] = lo[x][k] = v4d{0.0, 0.0, 0.0, 0.0};
      if (epochs_only && valid[x][k]) {    // the TOA term from contract_xr_kernel: continue its sum
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long long o = (long long)(16 * (i0 + x) + q + 4 * r) * LD + 16 * (j0 + k) + c;
          hi[x][k][r] = gout[o];
          lo[x][k][r] = glo ? glo[o] : 0.0;
        }
      }
    }
  auto flush = [&]() {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double a = hi[x][k][r], b = acc[x][k][r];
          const double sum = a + b, bp = sum - a;
          lo[x][k][r] += (a - (sum - bp)) + (b - bp);
          hi[x][k][r] = sum;
          acc[x][k][r] = 0.0;
        }
  };
  // clamped column indices (a column past NB reads column 0; its block is invalid)
  int ca[2], cb[4], ga[2], gb[4];
#pragma unroll
  for (int x = 0; x < 2; ++x) ca[x] = (i0 + x < NB ? 16 * (i0 + x) : 0) + c;
#pragma unroll
  for (int k = 0; k < 4; ++k) cb[k] = (j0 + k < NB ? 16 * (j0 + k) : 0) + c;
#pragma unroll
  for (int x = 0; x < 2; ++x) ga[x] = P.n_bgroup ? P.col_bgroup[ca[x]] : -1;
#pragma unroll
  for (int k = 0; k < 4; ++k) gb[k] = P.n_bgroup ? P.col_bgroup[cb[k]] : -1;
  for (int pass = epochs_only ? 1 : 0; pass < 2; ++pass) {
    const int nrows = pass == 0 ? P.n_toa : P.n_epoch;
    if (nrows == 0) continue;
    const double* src = pass == 0 ? P.T : s + (long long)bl * P.n_epoch * LD;
    const double* wsrc = pass == 0 ? w + (long long)bl * P.n_toa : beta + (long long)bl * P.n_epoch;
    const double wsign = pass == 0 ? 1.0 : -1.0;
    const double* fb = (pass == 0 && P.n_bgroup) ? fac + (long long)bl * P.n_bgroup * P.n_toa : nullptr;
    // operands of k-step t0 (rows t0 + q), rows past nrows read as zero weight
    double na[2], nbv[4], nw;
    auto load = [&](int t0) {
      const int row = t0 + q;
      const bool in = row < nrows;
      const double* rp = src + (long long)(in ? row : 0) * LD;
#pragma unroll
      for (int x = 0; x < 2; ++x) na[x] = rp[ca[x]];
#pragma unroll
      for (int k = 0; k < 4; ++k) nbv[k] = rp[cb[k]];
      nw = in ? wsign * wsrc[row] : 0.0;
      if (fb && in) {
#pragma unroll
        for (int x = 0; x < 2; ++x)
          if (ga[x] >= 0) na[x] *= fb[(long long)ga[x] * P.n_toa + row];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (gb[k] >= 0) nbv[k] *= fb[(long long)gb[k] * P.n_toa + row];
      }
    };
    load(0);
    for (int t0 = 0; t0 < nrows; t0 += 4) {
      double a[2] = {nw * na[0], nw * na[1]}, b[4] = {nbv[0], nbv[1], nbv[2], nbv[3]};
      if (t0 + 4 < nrows) load(t0 + 4);
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (valid[x][k]) acc[x][k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[x], b[k], acc[x][k], 0, 0, 0);
      if (((t0 + 4) % WT_GROUP) == 0 || t0 + 4 >= nrows) flush();
    }
  }
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (!valid[x][k]) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * (i0 + x) + q + 4 * r, col = 16 * (j0 + k) + c;
        dd v = dd_fast(hi[x][k][r], lo[x][k][r]);
        if (row == col && row >= P.m && row < LD - 1) v = {1.0, 0.0};
        gout[(long long)row * LD + col] = v.hi;
        gout[(long long)col * LD + row] = v.hi;
        if (glo) {
          glo[(long long)row * LD + col] = v.lo;
          glo[(long long)col * LD + row] = v.lo;
        }
      }
    }
}

// The TOA term of a wide basis (NB > 16, no theta-dependent columns) as ONE
// GEMM over the batch instead of a Gram per sample:
//   G_b[a][c] = sum_t w_bt T[t][a] T[t][c]  (b: sample, a <= c: columns)
// is (samples x TOAs) W times the (TOAs x column pairs) Khatri-Rao product
// X[t][(a, c)] = T[t][a] T[t][c], which is never stored: MFMA m = 16 samples,
// n = the 16 columns c of block j, k = 4 TOA rows, and for a column a of
// block i the B operand T[t][a] T[t][c] is one multiply of the lane's T[t][c]
// by T[t][a] broadcast from lane a of its 16-lane row (row_newbcast).  The
// basis is then read once per (block pair, 32 samples) instead of once per
// (block group, sample): 48 MB per sample instead of ~300 MB for 384 columns
// x 10k TOAs, and the operands of 8 MFMAs cost 4 LDS reads and 4 multiplies.
// Workgroup: one upper block pair (i, j) x XR_S = 32 samples, 4 waves; wave V
// owns columns a = 16 i + 4 V .. + 3 (x 16 columns c x 2 sample groups = 8
// accumulators).  Rows in tiles of XR_R = 64 (w and the two column blocks of
// T staged in LDS, the next tile prefetched into registers); compensated like
// contract2: each XR_GROUP = 128 rows summed by the MFMAs into fresh
// accumulators, added into hi + lo by TwoSum.  The ECORR term follows in
// contract_wide_kernel (epochs_only), which continues from G_hi / G_lo.
constexpr int XR_S = 32;
constexpr int XR_R = 64;
constexpr int XR_GROUP_TILES = 2;
constexpr int XR_WLD = XR_R + 4;                // padded row of the staged w tile (LDS banks)

template <int V>
__device__ __forceinline__ void contract_xr_body(const PsrDev& P, const double* __restrict__ w, int nsamp, int bi,
                                                 int bj, int s0, double* __restrict__ G, double* __restrict__ Glo,
                                                 double* wl, double* tl) {
  const int tid = threadIdx.x, lane = tid & 63, q = lane >> 4, c = lane & 15;
  const int LD = P.ld, n = P.n_toa;
  v4d acc[2][4], hi[2][4], lo[2][4];
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int x = 0; x < 4; ++x) acc[g][x] = hi[g][x] = lo[g][x] = v4d{0.0, 0.0, 0.0, 0.0};
  // staging: thread tid loads w[s0 + tid / 8][t0 + 8 (tid % 8) ..] and
  // T[t0 + tid / 4][16 blk + 8 ((tid / 2) % 2) ..] for blk = (i, j)[tid % 2]
  const int ws = tid >> 3, wr0 = (tid & 7) * 8;
  const int tr = tid >> 2, tb = tid & 1, tc0 = ((tid >> 1) & 1) * 8;
  const double* wrow = w + (long long)(s0 + ws) * n;
  const bool wok = s0 + ws < nsamp;
  const double* tcol = P.T + 16 * (tb ? bj : bi) + tc0;
  double wv[8], tv[8];
  auto fetch = [&](int t0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) wv[k] = (wok && t0 + wr0 + k < n) ? wrow[t0 + wr0 + k] : 0.0;
    // (T_aug carries CT_ROWS zero rows past n_toa; rows past those read 0)
#pragma unroll
    for (int k = 0; k < 8; ++k) tv[k] = t0 + tr < n ? tcol[(long long)(t0 + tr) * LD + k] : 0.0;
  };
  auto stage = [&]() {
#pragma unroll
    for (int k = 0; k < 8; ++k) wl[ws * XR_WLD + wr0 + k] = wv[k];
#pragma unroll
    for (int k = 0; k < 8; ++k) tl[tr * 32 + 16 * tb + tc0 + k] = tv[k];
  };
  auto flush = [&]() {
#pragma unroll
    for (int g = 0; g < 2; ++g)
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double a = hi[g][x][r], b = acc[g][x][r];
          const double sum = a + b, bp = sum - a;
          lo[g][x][r] += (a - (sum - bp)) + (b - bp);
          hi[g][x][r] = sum;
          acc[g][x][r] = 0.0;
        }
  };
  const int ntile = (n + XR_R - 1) / XR_R;
  fetch(0);
  stage();
  __syncthreads();
  for (int it = 0; it < ntile; ++it) {
    if (it + 1 < ntile) fetch((it + 1) * XR_R);
#pragma unroll 4
    for (int kk = 0; kk < XR_R / 4; ++kk) {
      const int row = 4 * kk + q;
      const double a0 = wl[c * XR_WLD + row], a1 = wl[(16 + c) * XR_WLD + row];
      const double ti = tl[row * 32 + c], tj = tl[row * 32 + 16 + c];
      static_for<0, 4>([&](auto X) {
        constexpr int x = decltype(X)::value;
        const double bx = tj * row_newbcast<4 * V + x>(ti);
        acc[0][x] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, bx, acc[0][x], 0, 0, 0);
        acc[1][x] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, bx, acc[1][x], 0, 0, 0);
      });
    }
    if ((it % XR_GROUP_TILES) == XR_GROUP_TILES - 1 || it + 1 == ntile) flush();
    __syncthreads();
    if (it + 1 < ntile) {
      stage();
      __syncthreads();
    }
  }
  // D layout: lane (q, c), register r -> sample s0 + 16 g + q + 4 r, entry
  // (16 bi + 4 V + x, 16 bj + c); the mirror too off the diagonal blocks; pad
  // columns (m .. LD - 2) get a unit diagonal
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int sb = s0 + 16 * g + q + 4 * r;
      if (sb >= nsamp) continue;
      double* out = G + (long long)sb * LD * LD;
      double* outl = Glo ? Glo + (long long)sb * LD * LD : nullptr;
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int row = 16 * bi + 4 * V + x, col = 16 * bj + c;
        dd v = dd_fast(hi[g][x][r], lo[g][x][r]);
        if (row == col && row >= P.m && row < LD - 1) v = {1.0, 0.0};
        out[(long long)row * LD + col] = v.hi;
        if (outl) outl[(long long)row * LD + col] = v.lo;
        if (bi != bj) {
          out[(long long)col * LD + row] = v.hi;
          if (outl) outl[(long long)col * LD + row] = v.lo;
        }
      }
    }
}

__global__ __launch_bounds__(256) void contract_xr_kernel(PsrDev P, const double* __restrict__ w, int nsamp,
                                                          double* __restrict__ G, double* __restrict__ Glo) {
  __shared__ double wl[XR_S * XR_WLD];
  __shared__ double tl[XR_R * 32];
  const int NB = P.ld >> 4, npair = NB * (NB + 1) / 2;
  // XCD-contiguous: the workgroups resident on one XCD share a sample group
  // (its w tile) and stream the same T rows through that XCD's L2
  const long long L = xcd_unit(blockIdx.x, gridDim.x);
  const int sg = (int)(L / npair), pr = (int)(L % npair);
  int bi = 0, rem = pr;
  while (rem >= NB - bi) {
    rem -= NB - bi;
    ++bi;
  }
  const int bj = bi + rem;
  const int wv = threadIdx.x >> 6;
  static_for<0, 4>([&](auto V) {
    if (wv == decltype(V)::value)
      contract_xr_body<decltype(V)::value>(P, w, nsamp, bi, bj, sg * XR_S, G, Glo, wl, tl);
  });
}

int dispatch_contract(int nb, const PsrDev& P, const double* w, const double* beta, const double* s,
                      const double* fac, double* G, int nb_samples, hipStream_t st, double* Glo) {
  if (nb > 16) {
    if (nb > WIDE_NB_MAX) return set_err(EWH_E_UNSUPPORTED, "basis wider than 1023 columns");
    const int nblk = nb * (nb + 1) / 2;
    // no theta-dependent columns: the TOA term as one GEMM over the batch,
    // then the ECORR term per sample onto it (or nothing, without epochs)
    const bool xr = P.n_bgroup == 0 && !contract_wide_only();
    if (xr) {
      const unsigned groups = (unsigned)((nb_samples + XR_S - 1) / XR_S);
      hipLaunchKernelGGL(contract_xr_kernel, dim3(groups * (unsigned)nblk), dim3(256), 0, st, P, w, nb_samples, G, Glo);
      if (P.n_epoch == 0) return 0;
    }
    hipLaunchKernelGGL(contract_wide_kernel, dim3((sb_count(nb) + 3) / 4, nb_samples), dim3(256), 0, st, P, w, beta,
                       s, fac, G, Glo, xr ? 1 : 0);
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
