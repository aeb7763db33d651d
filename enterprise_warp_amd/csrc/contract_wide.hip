// contract_wide.hip — the varying-white-noise contraction of bases past 16
// blocks (X_<n>_nfreqs models, enterprise_models.py:148-167, :436-468):
// contract_xr_kernel (the TOA term as one GEMM over the batch) and
// contract_wide_kernel (per sample: the ECORR term, or both terms where the
// basis depends on theta).  Its own translation unit: built with the MFMAs in
// the VGPR form (Makefile UFLAGS_contract_wide).
#include "ewarp_dev.h"

#include <cstdlib>

namespace ewh_dev {
namespace {

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

// CHROM: pass 0 scales the theta-dependent columns per TOA (fac); without it
// the kernel carries no per-column group state (registers)
template <bool CHROM>
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
  int ca[2], cb[4], ga[2] = {-1, -1}, gb[4] = {-1, -1, -1, -1};
#pragma unroll
  for (int x = 0; x < 2; ++x) ca[x] = (i0 + x < NB ? 16 * (i0 + x) : 0) + c;
#pragma unroll
  for (int k = 0; k < 4; ++k) cb[k] = (j0 + k < NB ? 16 * (j0 + k) : 0) + c;
  if constexpr (CHROM) {
#pragma unroll
    for (int x = 0; x < 2; ++x) ga[x] = P.col_bgroup[ca[x]];
#pragma unroll
    for (int k = 0; k < 4; ++k) gb[k] = P.col_bgroup[cb[k]];
  }
  for (int pass = epochs_only ? 1 : 0; pass < 2; ++pass) {
    const int nrows = pass == 0 ? P.n_toa : P.n_epoch;
    if (nrows == 0) continue;
    const double* src = pass == 0 ? P.T : s + (long long)bl * P.n_epoch * LD;
    const double* wsrc = pass == 0 ? w + (long long)bl * P.n_toa : beta + (long long)bl * P.n_epoch;
    const double wsign = pass == 0 ? 1.0 : -1.0;
    const double* fb = (CHROM && pass == 0) ? fac + (long long)bl * P.n_bgroup * P.n_toa : nullptr;
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
      if (CHROM && fb && in) {
#pragma unroll
        for (int x = 0; x < 2; ++x)
          if (ga[x] >= 0) na[x] *= fb[(long long)ga[x] * P.n_toa + row];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (gb[k] >= 0) nbv[k] *= fb[(long long)gb[k] * P.n_toa + row];
      }
    };
    load(0);
    for (int g0 = 0; g0 < nrows; g0 += WT_GROUP) {
      const int g1 = min(g0 + WT_GROUP, nrows);
      for (int t0 = g0; t0 < g1; t0 += 4) {
        double a[2] = {nw * na[0], nw * na[1]}, b[4] = {nbv[0], nbv[1], nbv[2], nbv[3]};
        if (t0 + 4 < nrows) load(t0 + 4);
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (valid[x][k]) acc[x][k] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[x], b[k], acc[x][k], 0, 0, 0);
      }
      flush();
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
// accumulators), operands loaded one k-step ahead from L1 / L2 (no LDS, no
// barrier: a first form staged 64-row tiles of w and T in LDS with a register
// prefetch of the next tile, which pushed the accumulators through
// v_accvgpr_read / write around every MFMA -- 0.46 of peak); compensated like
// contract2: each XR_GROUP = 128 rows summed by the MFMAs into fresh
// accumulators, added into hi + lo by TwoSum.  The ECORR term follows in
// contract_wide_kernel (epochs_only), which continues from G_hi / G_lo.
constexpr int XR_S = 32;
constexpr int XR_GROUP = 128;                   // rows per compensated group

template <int V>
__device__ __forceinline__ void contract_xr_body(const PsrDev& P, const double* __restrict__ w, int nsamp, int bi,
                                                 int bj, int s0, double* __restrict__ G, double* __restrict__ Glo) {
  const int lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;
  const int LD = P.ld, n = P.n_toa;
  v4d acc[2][4], hi[2][4], lo[2][4];
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int x = 0; x < 4; ++x) acc[g][x] = hi[g][x] = lo[g][x] = v4d{0.0, 0.0, 0.0, 0.0};
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
  // operands straight from L1 / L2, one k-step ahead (the four waves of the
  // workgroup read the same w rows and T columns: L1 hits for three of
  // them).  Rows past n: T row n (zero padding), w of row n - 1 (finite);
  // samples past nsamp: the last sample (finite, never written).
  const double* w0 = w + (long long)min(s0 + c, nsamp - 1) * n;
  const double* w1 = w + (long long)min(s0 + 16 + c, nsamp - 1) * n;
  const double* ti_p = P.T + 16 * bi + c;
  const double* tj_p = P.T + 16 * bj + c;
  double na0, na1, nti, ntj;
  auto load = [&](int t0) {            // (the last k-steps: rows clamped)
    const int row = t0 + q;
    const int rw = min(row, n - 1), rt = min(row, n);
    na0 = w0[rw];
    na1 = w1[rw];
    nti = ti_p[(long long)rt * LD];
    ntj = tj_p[(long long)rt * LD];
  };
  // Every other k-step (rows t0 + q < n): wave-uniform bases w + t0 and
  // T + t0 LD plus per-lane 32-bit byte offsets fixed for the whole loop, so
  // the loads take the SGPR-base form and a step costs no VALU address
  // arithmetic (round 5h: the clamped 64-bit form above spent ~20 VALU per
  // 8 MFMAs on addresses -- PMC 5.4 VALU per MFMA, 0.70 MFMA-busy).  w_off
  // is the caller's guarantee (nsamp n 8 < 4 GB).
  const unsigned wo0 = (unsigned)((min(s0 + c, nsamp - 1) * (long long)n + q) * 8);
  const unsigned wo1 = (unsigned)((min(s0 + 16 + c, nsamp - 1) * (long long)n + q) * 8);
  const unsigned toi = (unsigned)((q * LD + 16 * bi + c) * 8), toj = (unsigned)((q * LD + 16 * bj + c) * 8);
  auto load_fast = [&](int t) {
    const char* wb = (const char*)(w + t);
    const char* tb = (const char*)(P.T + (long long)t * LD);
    na0 = *(const double*)(wb + wo0);
    na1 = *(const double*)(wb + wo1);
    nti = *(const double*)(tb + toi);
    ntj = *(const double*)(tb + toj);
  };
  if (n >= 4) load_fast(0); else load(0);
  // (the flush outside the k-step loop: the accumulators stay in the MFMA's
  // registers for a whole group instead of moving around every MFMA)
  for (int g0 = 0; g0 < n; g0 += XR_GROUP) {
    const int g1 = min(g0 + XR_GROUP, n);
    for (int t0 = g0; t0 < g1; t0 += 4) {
      const double a0 = na0, a1 = na1, ti = nti, tj = ntj;
      if (t0 + 8 <= n)
        load_fast(t0 + 4);
      else if (t0 + 4 < n)
        load(t0 + 4);
      static_for<0, 4>([&](auto X) {
        constexpr int x = decltype(X)::value;
        const double bx = tj * row_newbcast<4 * V + x>(ti);
        acc[0][x] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, bx, acc[0][x], 0, 0, 0);
        acc[1][x] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, bx, acc[1][x], 0, 0, 0);
      });
    }
    flush();
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
  const int NB = P.ld >> 4, npair = NB * (NB + 1) / 2;
  // XCD-contiguous: the workgroups resident on one XCD share a sample group
  // (its w rows) and stream the same T rows through that XCD's L2
  const long long L = xcd_unit(blockIdx.x, gridDim.x);
  const int sg = (int)(L / npair), pr = (int)(L % npair);
  // (debug build: the sample group and the block pair inside the launch)
  EWH_DCHECK(sg * XR_S < nsamp && NB <= WIDE_NB_MAX && (long long)nsamp * P.n_toa * 8 < (1LL << 32),
             "contract_xr: sample group / 32-bit weight offsets in range");
  int bi = 0, rem = pr;
  while (rem >= NB - bi) {
    rem -= NB - bi;
    ++bi;
  }
  const int bj = bi + rem;
  const int wv = threadIdx.x >> 6;
  static_for<0, 4>([&](auto V) {
    if (wv == decltype(V)::value) contract_xr_body<decltype(V)::value>(P, w, nsamp, bi, bj, sg * XR_S, G, Glo);
  });
}

}  // namespace

int launch_contract_wide(int nb, const PsrDev& P, const double* w, const double* beta, const double* s,
                         const double* fac, double* G, int nb_samples, hipStream_t st, double* Glo) {
  if (nb > WIDE_NB_MAX) return set_err(EWH_E_UNSUPPORTED, "basis wider than 1023 columns");
  const int nblk = nb * (nb + 1) / 2;
  // no theta-dependent columns: the TOA term as one GEMM over the batch,
  // then the ECORR term per sample onto it (or nothing, without epochs)
  // (the batch GEMM addresses the chunk's weights with 32-bit byte offsets)
  const bool xr = P.n_bgroup == 0 && !contract_wide_only() && (long long)nb_samples * P.n_toa * 8 < (1LL << 32);
  if (xr) {
    const unsigned groups = (unsigned)((nb_samples + XR_S - 1) / XR_S);
    hipLaunchKernelGGL(contract_xr_kernel, dim3(groups * (unsigned)nblk), dim3(256), 0, st, P, w, nb_samples, G, Glo);
    if (P.n_epoch == 0) return 0;
  }
  if (P.n_bgroup)
    hipLaunchKernelGGL(contract_wide_kernel<true>, dim3((sb_count(nb) + 3) / 4, nb_samples), dim3(256), 0, st, P, w,
                       beta, s, fac, G, Glo, xr ? 1 : 0);
  else
    hipLaunchKernelGGL(contract_wide_kernel<false>, dim3((sb_count(nb) + 3) / 4, nb_samples), dim3(256), 0, st, P, w,
                       beta, s, fac, G, Glo, xr ? 1 : 0);
  return 0;
}

}  // namespace ewh_dev
