// ewarp_hip.hip — MI355X (gfx950) PTA log-likelihood engine.
//
// Implements include/ewarp_hip.h.  The arithmetic restates the enterprise
// likelihood that enterprise_warp drives (signal_base.PTA built at
// enterprise_warp.py:502, called at bilby_warp.py:35):
//
//   lnL = sum_p [ -1/2 (r^T N^-1 r + log|N|)
//                 + 1/2 (d^T Sigma^-1 d - log|Sigma| - log|phi|) ],
//   Sigma = T^T N^-1 T + diag(1/phi),  d = T^T N^-1 r.
//
// Device formulation:
//  * The residual vector is appended to the basis as its LAST column
//    (T_aug = [T | pad | r]), so one contraction G = T_aug^T N^-1 T_aug gives
//    T^T N^-1 T, d and r^T N^-1 r together, and one Cholesky of
//    G + diag(1/phi, 0) gives, in its last pivot, q = r^T N^-1 r - d^T Sigma^-1 d.
//    lnL_p = -1/2 log|N| - 1/2 q - sum_j log U_jj - 1/2 sum_j log phi_j.
//  * White noise fixed: G and the elimination of the theta-independent
//    leading (timing-model, phi = 1e40) block are computed once at create; per
//    sample only the reduced (m - n_tm + 1)^2 factorisation runs.
//  * Kernels: wn_weights (N, ECORR Sherman-Morrison terms), epoch_sums,
//    contract_mfma (fp64 MFMA T^T N^-1 T with LDS-staged TOA tiles),
//    schur (fixed-WN lead elimination), chol_mfma (one wave per
//    (pulsar, sample): 16x16 blocks register-resident in MFMA C/D layout,
//    panel rows by VALU + cross-lane shuffles, trailing update by
//    v_mfma_f64_16x16x4_f64), chol_lds (general fallback, matrix in LDS),
//    reduce_units (sum over pulsars in pulsar order).
#include "ewarp_dev.h"
#include "ewarp_desc.h"

#include <atomic>
#include <chrono>
#include <map>
#include <mutex>

namespace ewh_dev {

thread_local std::string g_err;

int set_err(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// ----------------------------------------------------------------------------
// white noise: w_t = 1/N_t, ECORR beta_e, -1/2 log|N|     ([ent] ShermanMorrison)
// grid: one 256-thread block per sample of the chunk
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void wn_weights_kernel(PsrDev P, const double* __restrict__ theta,
                                                         int ldth, int b0, double* __restrict__ w,
                                                         double* __restrict__ beta,
                                                         double* __restrict__ Kb, double* __restrict__ fac,
                                                         double* __restrict__ rho) {
  __shared__ double red[4];
  const int bl = blockIdx.x;
  const double* th = theta + (long long)(b0 + bl) * ldth;
  double* wr = w + (long long)bl * P.n_toa;
  // theta-dependent chromatic basis: fac[t][g] = (1400/nu_t)^idx_g
  for (int g = 0; g < P.n_bgroup; ++g) {
    const double idx = pref_val(P.bgroup[g], th);
    double* fr = fac + ((long long)bl * P.n_bgroup + g) * P.n_toa;
    for (int t = threadIdx.x; t < P.n_toa; t += 256) fr[t] = exp(idx * P.ln_chrom[t]);
  }
  double acc = 0.0;
  for (int t = threadIdx.x; t < P.n_toa; t += 256) {
    const double ef = pref_val(P.slots[P.efac_slot[t]], th);
    double D = ef * ef * P.sig2[t];                       // MeasurementNoise
    const int qs = P.equad_slot[t];
    if (qs >= 0) D += pow(10.0, 2.0 * pref_val(P.slots[qs], th));  // TNEquadNoise
    wr[t] = 1.0 / D;
    acc += log(D);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < P.n_epoch; e += 256) {   // EcorrKernelNoise
    double s = 0.0;
    for (int t = P.ep_start[e]; t < P.ep_stop[e]; ++t) s += wr[t];
    const double J = pow(10.0, 2.0 * pref_val(P.slots[P.ep_slot[e]], th));
    const double be = 1.0 / (s + 1.0 / J);
    beta[(long long)bl * P.n_epoch + e] = be;
    acc += log(J) - log(be);
  }
  acc = block_sum256(acc, red);
  if (threadIdx.x == 0) Kb[bl] = -0.5 * acc;
  if (rho) {
    // r^T W r (no ECORR: the r-separated contraction, contract2 RSEP): r is
    // T_aug's last column; per thread a strided partial sum, then the tree
    double q = 0.0;
    for (int t = threadIdx.x; t < P.n_toa; t += 256) {
      const double r = P.T[(long long)t * P.ld + P.ld - 1];
      q = fma(wr[t] * r, r, q);
    }
    q = block_sum256(q, red);
    if (threadIdx.x == 0) rho[bl] = q;
  }
}

// s[bl][e][:] = sum_{t in epoch e} w_t T_aug[t][:]
__global__ __launch_bounds__(256) void epoch_sums_kernel(PsrDev P, const double* __restrict__ w,
                                                         const double* __restrict__ fac,
                                                         double* __restrict__ s) {
  const int e = blockIdx.x, bl = blockIdx.y;
  const double* wr = w + (long long)bl * P.n_toa;
  double* out = s + ((long long)bl * P.n_epoch + e) * P.ld;
  const int t0 = P.ep_start[e], t1 = P.ep_stop[e];
  for (int c = threadIdx.x; c < P.ld; c += 256) {
    const int g = P.n_bgroup ? P.col_bgroup[c] : -1;
    const double* fr = g >= 0 ? fac + ((long long)bl * P.n_bgroup + g) * P.n_toa : nullptr;
    double a = 0.0;
    for (int t = t0; t < t1; ++t) {
      const double x = P.T[(long long)t * P.ld + c];
      a += wr[t] * (g >= 0 ? x * fr[t] : x);
    }
    out[c] = a;
  }
}

// The same for ES_S samples per workgroup (round 5, the varying-white-noise
// wide path: the per-(epoch, sample) kernel above re-read the epoch's T rows
// from L2 / MALL for every sample -- 1.0 ms per 256 samples at 384 columns x
// 10k TOAs, 8 % of the w372 batch): the epoch's rows of each column are read
// once into registers (ES_R at a time), the group's weights staged in LDS
// (epochs up to ES_RMAX TOAs; longer ones, and theta-dependent bases, keep
// the kernel above).  s[b][e][c] = sum_t w_bt T[t][c], the terms in TOA
// order by fma.
constexpr int ES_S = 32, ES_R = 16, ES_RMAX = 128;
__global__ __launch_bounds__(256) void epoch_sums_multi_kernel(PsrDev P, const double* __restrict__ w, int nsamp,
                                                               double* __restrict__ s) {
  __shared__ double ws[ES_S * ES_RMAX];
  const int e = blockIdx.x, s0 = blockIdx.y * ES_S;
  const int t0 = P.ep_start[e], nr = P.ep_stop[e] - t0;
  const int ns = min(ES_S, nsamp - s0);
  for (int i = threadIdx.x; i < ES_S * nr; i += 256) {
    const int sl = i / nr, r = i - sl * nr;
    ws[sl * ES_RMAX + r] = sl < ns ? w[(long long)(s0 + sl) * P.n_toa + t0 + r] : 0.0;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < P.ld; c += 256) {
    double acc[ES_S];
#pragma unroll
    for (int sl = 0; sl < ES_S; ++sl) acc[sl] = 0.0;
    for (int r0 = 0; r0 < nr; r0 += ES_R) {
      double tv[ES_R];
#pragma unroll
      for (int r = 0; r < ES_R; ++r) tv[r] = r0 + r < nr ? P.T[(long long)(t0 + r0 + r) * P.ld + c] : 0.0;
      const int rn = min(ES_R, nr - r0);
#pragma unroll
      for (int sl = 0; sl < ES_S; ++sl) {
        const double* wl = ws + sl * ES_RMAX + r0;
#pragma unroll
        for (int r = 0; r < ES_R; ++r)
          if (r < rn) acc[sl] = fma(wl[r], tv[r], acc[sl]);
      }
    }
#pragma unroll
    for (int sl = 0; sl < ES_S; ++sl)
      if (sl < ns) s[((long long)(s0 + sl) * P.n_epoch + e) * P.ld + c] = acc[sl];
  }
}

// ----------------------------------------------------------------------------
// The double-double Gram G = X^T W X - sum_e beta_e s_e s_e^T of one pulsar,
// X = T_aug = X_hi + X_lo: X_hi the projected basis the fp64 kernels read
// (P.T), X_lo its projection residual (PsrHost::d_Tlo, round 6: X_hi + X_lo =
// T - M C to double-double, create_ctx), so the Gram is that of the exactly
// projected basis -- an exact reparametrisation of enterprise's -- and the
// projection's fp64 rounding (a basis perturbation of O(eps |M C|), up to
// ~1e-14 of the projected column's own size) stays out.  Every w_t X_ta X_tb
// is summed in double-double (Dot2, Ogita-Rump-Oishi 2005: TwoProd by fma,
// TwoSum): w X_a,hi is itself split by TwoProd, so each hi x hi term is exact
// with only w_t = 1/N_t rounded once (a relative perturbation of N_t by <=
// 2^-53, benign: it keeps G a Gram); the cross terms w (X_a,hi X_b,lo +
// X_a,lo X_b,hi) are added to the low part in fp64.  The ECORR epoch sums
// s_e = sum over the epoch of w_t (X_hi + X_lo)_t are formed here in fp64
// (<= 16-32 TOAs).  Rounds 2-5 summed the Gram of the rounded projected basis:
// on ill-conditioned prior draws that left the device's double-double twin
// ~16x strict from the CPU double-double value on C3 and made C4 units
// indefinite (tests/test_gpu_parity.py::test_headline_matches_dd_at_scale,
// test_c4_bench_inf_sets_at_scale).  One workgroup per upper 16x16 block,
// thread (ty, tx) -> entry (16 bi + ty, 16 bj + tx); 32-row chunks staged in
// LDS.  Writes G_hi / G_lo of block (bi, bj) (both triangles).
__device__ __forceinline__ void gram_dd_block(const PsrDev& P, const double* __restrict__ Xlo,
                                              const double* __restrict__ w, const double* __restrict__ beta, int bi,
                                              int bj, double* __restrict__ G, double* __restrict__ Glo,
                                              double (*Ta)[17], double (*Tb)[17], double (*Ua)[17], double (*Ub)[17],
                                              double* wv) {
#pragma clang fp contract(off)
  const int LD = P.ld;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  dd acc = {0.0, 0.0};
  for (int pass = 0; pass < 2; ++pass) {     // TOA rows (w), then epoch rows (-beta)
    const int nrows = pass == 0 ? P.n_toa : P.n_epoch;
    for (int t0 = 0; t0 < nrows; t0 += 32) {
      for (int idx = threadIdx.x; idx < 1024; idx += 256) {
        const int r = idx >> 5, c = idx & 31, cc = c & 15;
        const int col = 16 * (c < 16 ? bi : bj) + cc;
        double v = 0.0, vl = 0.0;
        if (t0 + r < nrows) {
          if (pass == 0) {
            const long long o = (long long)(t0 + r) * LD + col;
            v = P.T[o];
            vl = Xlo ? Xlo[o] : 0.0;
          } else {
            // s_e[col] = sum over the epoch's rows of w_t X_t,col in
            // double-double (round 6; fp64 until then -- a relative rounding
            // of the rank-one ECORR term, i.e. of G itself)
            for (int t = P.ep_start[t0 + r]; t < P.ep_stop[t0 + r]; ++t) {
              const long long o = (long long)t * LD + col;
              const double p = w[t] * P.T[o];
              const double pe = fma(w[t], P.T[o], -p);
              const double sum = v + p, bp = sum - v;
              vl += ((v - (sum - bp)) + (p - bp)) + pe + (Xlo ? w[t] * Xlo[o] : 0.0);
              v = sum;
            }
          }
        }
        if (c < 16) {
          Ta[r][cc] = v;
          Ua[r][cc] = vl;
        } else {
          Tb[r][cc] = v;
          Ub[r][cc] = vl;
        }
      }
      if (threadIdx.x < 32)
        wv[threadIdx.x] = t0 + (int)threadIdx.x < nrows ? (pass == 0 ? w[t0 + threadIdx.x] : -beta[t0 + threadIdx.x])
                                                        : 0.0;
      __syncthreads();
      // the tile's 32 terms by Dot2 into a fresh (hi, lo), then added to the
      // running total in double-double (round 6: one Dot2 over all rows had an
      // error bound of gamma_n^2 sum |terms| -- ~5e-24 of it at 20k TOAs; now
      // gamma_32^2 per tile and 2^-106 per tile fold)
      double hi = 0.0, lo = 0.0;
      for (int r = 0; r < 32; ++r) {
        const double wa = wv[r], ta = Ta[r][ty], yv = Tb[r][tx];
        const double x = wa * ta;
        const double xe = fma(wa, ta, -x);          // TwoProd: w X_a = x + xe exactly
        const double pr = x * yv;
        const double pe = fma(x, yv, -pr);          // TwoProd: x X_b = pr + pe exactly
        const double sum = hi + pr;                 // TwoSum: hi + pr = sum + se exactly
        const double bp = sum - hi;
        const double se = (hi - (sum - bp)) + (pr - bp);
        hi = sum;
        // + the low parts' cross terms (X_lo, or the epoch sums' low parts)
        lo += se + fma(xe, yv, pe) + wa * fma(ta, Ub[r][tx], Ua[r][ty] * yv);
      }
      acc = dd_add_ieee(acc, dd_two_sum(hi, lo));
      __syncthreads();
    }
  }
  const int row = 16 * bi + ty, col = 16 * bj + tx;
  if (row > col) return;      // diagonal block: the upper entry's thread writes both (exactly symmetric)
  dd v = acc;
  if (row == col && row >= P.m && row < LD - 1) v = {1.0, 0.0};   // unit pads, as the contraction kernels
  G[(long long)row * LD + col] = v.hi;
  G[(long long)col * LD + row] = v.hi;
  Glo[(long long)row * LD + col] = v.lo;
  Glo[(long long)col * LD + row] = v.lo;
}

__device__ __forceinline__ void upper_block(int blk, int nb, int& bi, int& bj) {
  bi = 0;
  while (blk >= nb - bi) { blk -= nb - bi; ++bi; }
  bj = bi + blk;
}

// fixed white noise, one-off (ewh_create / ewh_set_fixed_white): the cached
// Gram for the double-double timing-model elimination (schur_kernel).  One
// fp64 MFMA accumulator over 20k TOAs had moved prior-draw lnL by up to 7e-2
// on C3 through the ill-conditioned elimination (round 2,
// tests/test_gpu_parity.py::test_c3_bench_workload_prior_draws).  (Chromatic
// `vary` bases never take this path: their basis is theta-dependent, so white
// noise is not cached.)
__global__ __launch_bounds__(256) void gram_dd_kernel(PsrDev P, const double* __restrict__ Xlo,
                                                      const double* __restrict__ w,
                                                      const double* __restrict__ beta, double* __restrict__ G,
                                                      double* __restrict__ Glo) {
  __shared__ double Ta[32][17], Tb[32][17], Ua[32][17], Ub[32][17], wv[32];
  int bi, bj;
  upper_block(blockIdx.x, P.nb, bi, bj);
  gram_dd_block(P, Xlo, w, beta, bi, bj, G, Glo, Ta, Tb, Ua, Ub, wv);
}

// Round 6: the same Gram for the varying-white-noise units whose fp64
// factorisation failed (a pivot <= 0: an -inf term), listed by the failure
// scan (verify_units_kernel on the unit terms alone).  The exact Sigma of a
// full-rank basis is positive definite, so such an -inf is a rounding failure
// of the fp64 Gram or factorisation; the unit is refactored by chol_dd_kernel
// on this G_hi + G_lo (tests/test_gpu_parity.py::
// test_c4_bench_inf_sets_at_scale).  Grid (upper blocks, list slots): slot y
// takes list entries y, y + gridDim.y, ...; unit u -> sample b = u % B, row
// j = b - b_off of the chunk's per-sample weights / beta and of G (stride
// ld^2).
__global__ __launch_bounds__(256) void gram_dd_units_kernel(PsrDev P, const double* __restrict__ Xlo,
                                                            const double* __restrict__ w,
                                                            const double* __restrict__ beta,
                                                            const int* __restrict__ list,
                                                            const int* __restrict__ count, int B, int b_off,
                                                            double* __restrict__ G, double* __restrict__ Glo) {
  __shared__ double Ta[32][17], Tb[32][17], Ua[32][17], Ub[32][17], wv[32];
  int bi, bj;
  upper_block(blockIdx.x, P.nb, bi, bj);
  const int cnt = *count;
  const long long LD2 = (long long)P.ld * P.ld;
  for (int y = blockIdx.y; y < cnt; y += gridDim.y) {
    const int jb = list[y] % B - b_off;
    gram_dd_block(P, Xlo, w + (long long)jb * P.n_toa, beta + (long long)jb * P.n_epoch, bi, bj, G + jb * LD2,
                  Glo + jb * LD2, Ta, Tb, Ua, Ub, wv);
  }
}

// ----------------------------------------------------------------------------
// fixed white noise: eliminate the leading constant-phi (timing-model) block
// of G = Ghi + Glo once, in double-double (Cholesky, row k scaled by
// 1/sqrt(pivot)); write the reduced matrix S (fx_ld x fx_ld, r last, rounded
// to fp64) and K.  The elimination cancels most of the low-frequency Fourier
// columns' Gram (they are close to the span of the spin-down columns), so it
// runs on the double-double Gram.  One 256-thread block per
// pulsar; Ghi / Glo are modified in place.
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void schur_kernel(double* Ghi, double* Glo, int ld, int m, int nlead,
                                                    const int* __restrict__ col_ptr,
                                                    const DSpec* __restrict__ spec,
                                                    double Kb, double* S, int fx_ld, int nloc, int gstart,
                                                    int ncommon, double* Kout, int* fail_out, double* Slo) {
#pragma clang fp contract(off)   // (double-double elimination: ewarp_dev.h)
  __shared__ double rh[256 * 4], rl[256 * 4];
  __shared__ double red[4];
  double lphi = 0.0;
  for (int a = threadIdx.x; a < nlead; a += 256) {
    double ph = 0.0;
    for (int e = col_ptr[a]; e < col_ptr[a + 1]; ++e) ph += spec_phi(spec[e], nullptr);
    const dd v = dd_add({Ghi[(long long)a * ld + a], Glo[(long long)a * ld + a]}, {1.0 / ph, 0.0});
    Ghi[(long long)a * ld + a] = v.hi;
    Glo[(long long)a * ld + a] = v.lo;
    lphi += log(ph);
  }
  lphi = block_sum256(lphi, red);
  __syncthreads();
  double logdet = 0.0;
  int ok = 1;
  for (int k = 0; k < nlead; ++k) {
    const dd piv = {Ghi[(long long)k * ld + k], Glo[(long long)k * ld + k]};
    ok &= piv.hi > 0.0;
    const dd d = dd_sqrt(piv);
    logdet += log(d.hi) + d.lo / d.hi;
    __syncthreads();
    for (int j = k + 1 + threadIdx.x; j < ld; j += 256) {
      const dd x = dd_div({Ghi[(long long)k * ld + j], Glo[(long long)k * ld + j]}, d);
      rh[j] = x.hi;
      rl[j] = x.lo;
    }
    __syncthreads();
    for (int i = k + 1; i < ld; ++i) {
      const dd ri = {rh[i], rl[i]};
      for (int j = k + 1 + threadIdx.x; j < ld; j += 256) {
        const dd v = dd_add({Ghi[(long long)i * ld + j], Glo[(long long)i * ld + j]}, dd_mul({-ri.hi, -ri.lo}, {rh[j], rl[j]}));
        Ghi[(long long)i * ld + j] = v.hi;
        Glo[(long long)i * ld + j] = v.lo;
      }
    }
    __syncthreads();
  }
  // reduced index a -> G column: own columns a < nloc -> nlead + a; common
  // columns gstart <= a < gstart + ncommon -> nlead + nloc + (a - gstart);
  // a == fx_ld - 1 -> r (ld - 1); else an identity pad
  auto gmap = [&](int a) {
    if (a < nloc) return nlead + a;
    if (a >= gstart && a < gstart + ncommon) return nlead + nloc + (a - gstart);
    return a == fx_ld - 1 ? ld - 1 : -1;
  };
  for (int idx = threadIdx.x; idx < fx_ld * fx_ld; idx += 256) {
    const int a = idx / fx_ld, bcol = idx % fx_ld;
    const int ga = gmap(a);
    const int gb = gmap(bcol);
    dd v = {(a == bcol) ? 1.0 : 0.0, 0.0};
    if (ga >= 0 && gb >= 0) v = dd_two_sum(Ghi[(long long)ga * ld + gb], Glo[(long long)ga * ld + gb]);
    S[idx] = v.hi;
    if (Slo) Slo[idx] = v.lo;     // (the double-double factorisation's input, chol_dd_kernel)
  }
  if (threadIdx.x == 0) {
    *Kout = Kb - logdet - 0.5 * lphi;
    *fail_out = ok ? 0 : 1;
  }
}

// ----------------------------------------------------------------------------
// batched Cholesky, general fallback: one 256-thread block per unit, the
// (compacted) matrix as a packed lower triangle in LDS.
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void chol_lds_kernel(const CholJob* __restrict__ jobs, int B,
                                                       long long u0, int b_off,
                                                       const double* __restrict__ theta, int ldth,
                                                       double* __restrict__ out_units) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  __shared__ double red[4];
  const long long u = u0 + blockIdx.x;
  const int p = (int)(u / B), b = (int)(u % B);
  const CholJob J = jobs[p];
  const int mr = J.mreal, ma = mr + 1, ld = J.ld;
  double* L = sm;                               // ma(ma+1)/2
  double* col = sm + (long long)ma * (ma + 1) / 2;
  const double* A = J.mats + (long long)(b - b_off) * J.mstride;
  const double* th = theta + (long long)b * ldth;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int i = wave; i < ma; i += 4) {
    const int gi = i < mr ? i : ld - 1;
    const int base = i * (i + 1) / 2;
    for (int j = lane; j <= i; j += 64) L[base + j] = A[(long long)gi * ld + (j < mr ? j : ld - 1)];
  }
  __syncthreads();
  LogAcc lphi;
  for (int a = threadIdx.x; a < mr; a += 256) {
    double ph = 0.0;
    for (int e = J.col_ptr[a]; e < J.col_ptr[a + 1]; ++e) ph += spec_phi(J.spec[e], th);
    L[a * (a + 1) / 2 + a] += 1.0 / ph;
    lphi.add(ph);
  }
  const double lphi_sum = block_sum256(lphi.value(), red);
  __syncthreads();
  LogAcc ldet;                                  // sum of log pivots = 2 sum log U_jj
  bool ok = true;
  for (int k = 0; k < ma - 1; ++k) {
    const double piv = L[k * (k + 1) / 2 + k];
    ok = ok && (piv > 0.0);
    ldet.add(piv);
    const double rinv = rsqrt_nr(piv);
    for (int i = k + 1 + threadIdx.x; i < ma; i += 256) col[i] = L[i * (i + 1) / 2 + k] * rinv;
    __syncthreads();
    for (int i = k + 1 + wave; i < ma; i += 4) {
      const double ci = col[i];
      const int base = i * (i + 1) / 2;
      for (int j = k + 1 + lane; j <= i; j += 64) L[base + j] = fma(-ci, col[j], L[base + j]);
    }
    __syncthreads();
  }
  const double qv = L[(ma - 1) * ma / 2 + ma - 1];
  if (threadIdx.x == 0) {
    double lnl = J.K[(long long)(b - b_off) * J.kstride] - 0.5 * qv - 0.5 * ldet.value() - 0.5 * lphi_sum;
    if (!ok || J.fail) lnl = -INFINITY;
    out_units[(long long)p * B + b] = lnl;
  }
}

// M_g^-1 and log|M_g| by in-place Gauss-Jordan (SPD: no pivoting needed).
// grid (n_c, Bc), 256 threads, dynamic LDS (P (P+1) + 3 P) doubles.
// grid.x runs over the distinct M_g (sin / cos columns of one frequency share
// it): slot blockIdx.x stands for common column uniq[blockIdx.x].
__global__ __launch_bounds__(256) void common_minv_kernel(const CommonPsr* __restrict__ cps, int P,
                                                          const double* __restrict__ orf,
                                                          const DSpec* __restrict__ cspec, int nc,
                                                          const int* __restrict__ uniq,
                                                          const double* __restrict__ theta, int ldth, int b0,
                                                          double* __restrict__ minv, double* __restrict__ mlog) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int LDP = P + 1;
  double* M = sm;
  double* colk = sm + P * LDP;
  double* rowk = colk + P;
  double* own = rowk + P;
  const int slot = blockIdx.x, g = uniq[slot], bl = blockIdx.y;
  const double* th = theta + (long long)(b0 + bl) * ldth;
  const double pc = spec_phi(cspec[g], th);
  for (int a = threadIdx.x; a < P; a += 256) {
    const CommonPsr c = cps[a];
    double v = 0.0;
    for (int e = c.colptr[c.gstart + g]; e < c.colptr[c.gstart + g + 1]; ++e) v += spec_phi(c.spec[e], th);
    own[a] = v;
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < P * P; idx += 256) {
    const int i = idx / P, j = idx - i * P;
    M[i * LDP + j] = orf[idx] * pc + (i == j ? own[i] : 0.0);
  }
  __syncthreads();
  double lsum = 0.0;
  bool ok = true;
  for (int k = 0; k < P; ++k) {
    const double piv = M[k * LDP + k];
    ok = ok && (piv > 0.0);
    lsum += log(piv);
    const double pinv = 1.0 / piv;
    for (int i = threadIdx.x; i < P; i += 256) {
      colk[i] = M[i * LDP + k];
      rowk[i] = M[k * LDP + i] * pinv;
    }
    __syncthreads();
    for (int idx = threadIdx.x; idx < P * P; idx += 256) {
      const int i = idx / P, j = idx - i * P;
      double v;
      if (i == k) v = (j == k) ? pinv : rowk[j];
      else if (j == k) v = -colk[i] * pinv;
      else v = M[i * LDP + j] - colk[i] * rowk[j];
      M[i * LDP + j] = v;
    }
    __syncthreads();
  }
  double* out = minv + ((long long)bl * nc + slot) * P * P;
  for (int idx = threadIdx.x; idx < P * P; idx += 256) {
    const int i = idx / P, j = idx - i * P;
    out[idx] = M[i * LDP + j];
  }
  if (threadIdx.x == 0) mlog[(long long)bl * nc + slot] = ok ? lsum : __builtin_nan("");
}

// The same inverse for P <= MINV_PMAX with M held in registers: 8 waves, wave
// w owns rows i = w + 8 r (r < MINV_PMAX / 8), lane l columns j = l + 64 cc
// (cc < 2).  Per pivot k the owners of column k and row k publish them to LDS
// (double buffered by pivot parity: one barrier per pivot) and every thread
// updates its elements in place.  The pivot loop is unrolled over the row
// register r (k = 8 r + w_k), so row k's register and column k's half are
// compile-time indices (the round-3 form, 4 waves with a runtime register
// select and 338 registers at one wave per SIMD, took 6.7 ms per C5 batch of
// 512; the same arithmetic in the same order: bit-identical).
constexpr int MINV_PMAX = 128;
// sample chunks up to this size factor Sigma_c right-looking (corr_finish):
// C5 right- vs left-looking per chunk, ms (profiles/r04g/xover_B*.log):
// B = 4 1.67 / 3.21, 8 2.62 / 3.53, 12 3.65 / 4.01, 16 4.72 / 4.59
constexpr int CORR_RIGHT_LOOKING_MAX = 12;

__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) void common_minv_reg_kernel(const CommonPsr* __restrict__ cps, int P,
                                                              const double* __restrict__ orf,
                                                              const DSpec* __restrict__ cspec, int nc,
                                                              const int* __restrict__ uniq,
                                                              const double* __restrict__ theta, int ldth, int b0,
                                                              double* __restrict__ minv, double* __restrict__ mlog) {
  constexpr int NW = 8, RW = MINV_PMAX / NW;     // waves; rows per wave
  __shared__ double own[MINV_PMAX];
  __shared__ double colk[2][MINV_PMAX], rowk[2][MINV_PMAX];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int slot = blockIdx.x, g = uniq[slot], bl = blockIdx.y;
  const double* th = theta + (long long)(b0 + bl) * ldth;
  const double pc = spec_phi(cspec[g], th);
  for (int a = tid; a < P; a += 64 * NW) {
    const CommonPsr c = cps[a];
    double v = 0.0;
    for (int e = c.colptr[c.gstart + g]; e < c.colptr[c.gstart + g + 1]; ++e) v += spec_phi(c.spec[e], th);
    own[a] = v;
  }
  __syncthreads();
  double m[RW][2];
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const int i = w + NW * r;
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int j = lane + 64 * cc;
      m[r][cc] = (i < P && j < P) ? orf[i * P + j] * pc + (i == j ? own[i] : 0.0) : 0.0;
    }
  }
  LogAcc lacc;
  bool ok = true;
  static_for<0, RW>([&](auto R) {
    constexpr int r = decltype(R)::value;
    constexpr int cc = (NW * r) >= 64 ? 1 : 0;     // column k = NW r + wk lies in half cc
#pragma unroll 1
    for (int wk = 0; wk < NW; ++wk) {
      const int k = NW * r + wk;
      if (k >= P) break;
      const int buf = k & 1;
      const bool colown = lane == (k & 63);
      if (colown) {                                  // column k: one lane per wave
#pragma unroll
        for (int r2 = 0; r2 < RW; ++r2) colk[buf][w + NW * r2] = m[r2][cc];
      }
      if (w == wk) {                                 // row k: this wave, register r
        rowk[buf][lane] = m[r][0];
        rowk[buf][lane + 64] = m[r][1];
      }
      __syncthreads();
      const double piv = rowk[buf][k];
      ok = ok && (piv > 0.0);
      lacc.add(piv);
      const double pinv = 1.0 / piv;
      const double rj0 = rowk[buf][lane] * pinv, rj1 = rowk[buf][lane + 64] * pinv;
      double ci[RW];                                 // (all reads first: one LDS wait)
#pragma unroll
      for (int r2 = 0; r2 < RW; ++r2) ci[r2] = colk[buf][w + NW * r2];
#pragma unroll
      for (int r2 = 0; r2 < RW; ++r2) {
        const double u0 = fma(-ci[r2], rj0, m[r2][0]), u1 = fma(-ci[r2], rj1, m[r2][1]);
        const double cv = -ci[r2] * pinv;            // column k: -M[i][k] / piv (a select, no branch)
        m[r2][0] = (cc == 0 && colown) ? cv : u0;
        m[r2][1] = (cc == 1 && colown) ? cv : u1;
      }
      if (w == wk) {                                 // row k: M[k][j] / piv, the pivot 1 / piv
        m[r][0] = rj0;
        m[r][1] = rj1;
        if (colown) m[r][cc] = pinv;
      }
    }
  });
  double* out = minv + ((long long)bl * nc + slot) * P * P;
  int o0 = w * P + lane;              // (formed here: addresses carried from the loads spill)
  asm volatile("" : "+v"(o0));
#pragma unroll
  for (int r = 0; r < RW; ++r) {
    const int i = w + NW * r;
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int j = lane + 64 * cc;
      if (i < P && j < P) out[o0 + NW * r * P + 64 * cc] = m[r][cc];
    }
  }
  if (tid == 0) mlog[(long long)bl * nc + slot] = ok ? lacc.value() : __builtin_nan("");
}

// Dense Sigma_c (Np x Np, row-major) of sample bl, one row per wave (four
// per workgroup): rows/cols (a, g) -> a nc + g; r at Np - 1; pad rows/cols
// identity.  keep: pulsar-major kept blocks, Bk samples per pulsar; this chunk
// starts at sample b0 (pulsar a's block of sample bl at keep[(a Bk + b0 + bl)
// KD^2]).  Column j -> (pulsar, common column) by a float reciprocal (exact:
// (j + 1/2) / nc is at least 1/(2 nc) from an integer) instead of an integer
// division per element.
__device__ __forceinline__ int div_nc(int j, float rnc) { return (int)(((float)j + 0.5f) * rnc); }

__global__ __launch_bounds__(256) void common_assemble_kernel(const double* __restrict__ keep, int KD, int P, int nc,
                                                              long long Bk, int b0,
                                                              const double* __restrict__ minv,
                                                              const int* __restrict__ rep, int Np,
                                                              double* __restrict__ mats, double* __restrict__ cldet,
                                                              double* __restrict__ cq, int* __restrict__ cfail) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const int i = 4 * blockIdx.x + (threadIdx.x >> 6), lane = threadIdx.x & 63, bl = blockIdx.y;
  if (blockIdx.x == 0 && threadIdx.x == 0) {   // the factorisation's per-sample accumulators (no memset launches)
    cldet[bl] = 0.0;
    cq[bl] = 0.0;
    cfail[bl] = 0;
  }
  if (i >= Np) return;
  const int N = P * nc;
  const float rnc = 1.0f / (float)nc;
  const long long ps = Bk * KD * KD;                                // pulsar stride
  double* row = mats + ((long long)bl * Np + i) * Np;
  const double* kb = keep + (long long)(b0 + bl) * KD * KD;
  const double* mb = minv + (long long)bl * nc * P * P;
  // only the upper tiles (64-column tiles at or right of the diagonal tile)
  // are ever read by the factorisation: the rest of the row is not written.
  // Two columns per lane, one 16-byte store (Np and the tile starts are
  // multiples of 64: every pair is aligned and inside the row).
  const int j0 = (i / DCB) * DCB;
  if (i < N) {
    const int a = div_nc(i, rnc), g = i - a * nc;
    const double* ka = kb + (long long)a * ps + g * KD;            // row g of pulsar a's kept square
    const double* mg = mb + (long long)rep[g] * P * P + (long long)a * P;  // row a of M_g^-1
    auto val = [&](int j) {
      double v = 0.0;
      if (j < N) {
        const int bb = div_nc(j, rnc), h = j - bb * nc;
        if (bb == a) v = ka[h];
        if (h == g) v += mg[bb];
      } else if (j == Np - 1) {
        v = ka[KD - 1];
      }
      return v;
    };
    for (int j = j0 + 2 * lane; j < Np; j += 128) {
      const d2 v = {val(j), val(j + 1)};
      __builtin_nontemporal_store(v, (d2*)(row + j));
    }
  } else if (i == Np - 1) {
    for (int j = j0 + lane; j < Np; j += 64) {
      double v = 0.0;
      if (j < N) {
        const int bb = div_nc(j, rnc), h = j - bb * nc;
        v = kb[(long long)bb * ps + (KD - 1) * KD + h];
      } else if (j == Np - 1) {
        for (int a = 0; a < P; ++a) v += kb[(long long)a * ps + KD * KD - 1];
      }
      __builtin_nontemporal_store(v, row + j);
    }
  } else {
    for (int j = j0 + 2 * lane; j < Np; j += 128) {
      const d2 v = {(j == i) ? 1.0 : 0.0, (j + 1 == i) ? 1.0 : 0.0};
      __builtin_nontemporal_store(v, (d2*)(row + j));
    }
  }
}

// Diagonal 64 x 64 block k of every sample: Cholesky A_kk = L L^T in LDS,
// log-det accumulation, W = L^-1 (forward substitution, one column per
// thread) to wbuf.  The last pivot of the last block is r: stored as q.
__global__ __launch_bounds__(256) void dchol_diag_kernel(double* __restrict__ mats, int Np, int k,
                                                         double* __restrict__ wbuf, double* __restrict__ ldet,
                                                         double* __restrict__ qout, int* __restrict__ fail) {
  __shared__ double L[DCB][DCB + 1];
  __shared__ double Wl[DCB][DCB + 1];
  __shared__ double qlast;
  const int bl = blockIdx.x, t = threadIdx.x;
  const double* A = mats + (long long)bl * Np * Np + (long long)(DCB * k) * Np + DCB * k;
  for (int idx = t; idx < DCB * DCB; idx += 256) L[idx / DCB][idx % DCB] = A[(long long)(idx / DCB) * Np + idx % DCB];
  __syncthreads();
  const bool last = (k == Np / DCB - 1);
  const int npiv = last ? DCB - 1 : DCB;
  double lsum = 0.0;
  bool ok = true;
  for (int j = 0; j < npiv; ++j) {
    const double piv = L[j][j];
    ok = ok && (piv > 0.0);
    lsum += log(piv);
    const double rd = 1.0 / sqrt(piv);
    __syncthreads();
    for (int i = j + 1 + t; i < DCB; i += 256) L[i][j] *= rd;
    if (t == 0) L[j][j] = sqrt(piv);
    __syncthreads();
    for (int idx = t; idx < (DCB - j - 1) * (DCB - j - 1); idx += 256) {
      const int i = j + 1 + idx / (DCB - j - 1), l = j + 1 + idx % (DCB - j - 1);
      if (l <= i) L[i][l] -= L[i][j] * L[l][j];
    }
    __syncthreads();
  }
  if (last) {
    if (t == 0) {
      qlast = L[DCB - 1][DCB - 1];          // q = rho - d'^T Sigma^-1 d'
      L[DCB - 1][DCB - 1] = 1.0;            // W's r row is unused
    }
    __syncthreads();
  }
  // W = L^-1 by forward elimination on [L | I], all threads: step k scales row
  // k of W by 1/L_kk, then eliminates column k from the rows below
  for (int idx = t; idx < DCB * DCB; idx += 256) Wl[idx / DCB][idx % DCB] = (idx / DCB == idx % DCB) ? 1.0 : 0.0;
  __syncthreads();
  for (int k2 = 0; k2 < DCB; ++k2) {
    const double rk = 1.0 / L[k2][k2];
    if (t <= k2) Wl[k2][t] *= rk;
    __syncthreads();
    for (int idx = t; idx < (DCB - 1 - k2) * (k2 + 1); idx += 256) {
      const int i = k2 + 1 + idx / (k2 + 1), cc = idx % (k2 + 1);
      Wl[i][cc] -= L[i][k2] * Wl[k2][cc];
    }
    __syncthreads();
  }
  double* W = wbuf + (long long)bl * DCB * DCB;
  for (int idx = t; idx < DCB * DCB; idx += 256) W[idx] = Wl[idx / DCB][idx % DCB];
  if (t == 0) {
    ldet[bl] += lsum;
    if (!ok) fail[bl] = 1;
    if (last) qout[bl] = qlast;
  }
}

// ---- register-resident diagonal block + panel (the default) -------------
// wbuf per sample (DW doubles): slots of 256 doubles in the MFMA C/D lane
// layout (lane l holds 4 consecutive doubles: register r <-> row (l>>4) + 4r,
// column l&15) -- E_s = L_ss^-T of the 16-row sub-blocks s = 0..3 (slots
// 0-3), their row scales D_s^-1/2 (4-7), the scaled factor blocks U_st,
// s < t (8-13: 01 02 03 12 13 23).
constexpr int DW_SLOTS = 14;
__host__ __device__ constexpr int dw_u(int s, int t) { return 8 + (s == 0 ? t - 1 : s == 1 ? t + 1 : 5); }

struct DiagHook : NoHook {
  double* W;
  int bb;
  __device__ __forceinline__ void on_e(const v4d& E) const { *(v4d*)(W + bb * 256) = E; }
  __device__ __forceinline__ void on_scale(int r, double rs) const { W[(4 + bb) * 256 + r] = rs; }
};

// One wave per sample: the 64 x 64 diagonal block k of Sigma_c factored in
// registers by the blocked LDL^T panel of chol_mfma_kernel (NB = 4, no
// residual column except in the LAST block, whose last pivot is
// q_c = rho - d'^T Sigma_c^-1 d'); log-det and positivity accumulated; E_s,
// D_s^-1/2 and U_st written for dchol_panel_reg_kernel.
// (body shared with dchol_update_diag_kernel: one wave, sample bl)
template <bool LAST>
__device__ __forceinline__ void diag_reg_body(double* __restrict__ mats, int Np, int k, double* __restrict__ wbuf,
                                              double* __restrict__ ldet, double* __restrict__ qout,
                                              int* __restrict__ fail, int bl, int lane) {
  const int q = lane >> 4, c = lane & 15;
  const double* A = mats + (long long)bl * Np * Np + (long long)(DCB * k) * Np + DCB * k;
  double* W = wbuf + (long long)bl * DW_SLOTS * 256 + lane * 4;
  constexpr auto id = [](int i, int j) { return i * 4 - i * (i - 1) / 2 + (j - i); };
  v4d U[10];
  static_for<0, 4>([&](auto I) {
    constexpr int i = decltype(I)::value;
    static_for<i, 4>([&](auto J) {
      constexpr int j = decltype(J)::value;
      static_for<0, 4>([&](auto R) {
        constexpr int r = decltype(R)::value;
        U[id(i, j)][r] = A[(long long)(16 * i + q + 4 * r) * Np + 16 * j + c];
      });
    });
  });
  LogAcc ld;
  bool ok = true;
  static_for<0, 4>([&](auto BBc) {
    constexpr int bb = decltype(BBc)::value;
    DiagHook hk;
    hk.W = W;
    hk.bb = bb;
    panel_ldl_row<4, PANEL_2L, LAST, false>(BBc, [&](auto JJ) -> v4d& { return U[id(bb, decltype(JJ)::value)]; }, q,
                                            c, ld, ok, hk);
    static_for<bb + 1, 4>([&](auto II) {
      constexpr int i = decltype(II)::value;
      static_for<i, 4>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        syrk_update(U[id(i, j)], U[id(bb, i)], U[id(bb, j)]);
      });
    });
  });
  if constexpr (!LAST) {
    static_for<0, 4>([&](auto SS) {
      constexpr int s0 = decltype(SS)::value;
      static_for<s0 + 1, 4>([&](auto TT) {
        constexpr int t0 = decltype(TT)::value;
        *(v4d*)(W + dw_u(s0, t0) * 256) = U[id(s0, t0)];
      });
    });
  }
  const double ldv = wave_sum(ld.value());
  const bool ok_all = __all(ok);
  double qv = 0.0;
  if constexpr (LAST) qv = readlane_d(U[id(3, 3)][3], 63);
  if (lane == 0) {
    ldet[bl] += ldv;
    if (!ok_all) fail[bl] = 1;
    if (LAST) qout[bl] = qv;
  }
}

template <bool LAST>
__global__ __launch_bounds__(64) void dchol_diag_reg_kernel(double* __restrict__ mats, int Np, int k,
                                                            double* __restrict__ wbuf, double* __restrict__ ldet,
                                                            double* __restrict__ qout, int* __restrict__ fail) {
  diag_reg_body<LAST>(mats, Np, k, wbuf, ldet, qout, fail, blockIdx.x, threadIdx.x);
}

// U_kj = L_kk^-1 A_kj (scaled) for the tiles j > k: one wave per (16-column
// strip, tile, sample), the strip's four 16 x 16 blocks in registers, the
// block forward substitution by fp64 MFMA with the operands of wbuf.
__global__ __launch_bounds__(64) void dchol_panel_reg_kernel(double* __restrict__ mats, int Np, int k,
                                                             const double* __restrict__ wbuf) {
  const int strip = blockIdx.x & 3, jt = blockIdx.x >> 2, bl = blockIdx.y;
  const int lane = threadIdx.x, q = lane >> 4, c = lane & 15;
  const int j = k + 1 + jt;
  double* T = mats + (long long)bl * Np * Np + (long long)(DCB * k) * Np + DCB * j + 16 * strip;
  const double* W = wbuf + (long long)bl * DW_SLOTS * 256 + lane * 4;
  v4d a[4];
  static_for<0, 4>([&](auto SS) {
    constexpr int s0 = decltype(SS)::value;
    static_for<0, 4>([&](auto R) {
      constexpr int r = decltype(R)::value;
      a[s0][r] = T[(long long)(16 * s0 + q + 4 * r) * Np + c];
    });
  });
  static_for<0, 4>([&](auto SS) {
    constexpr int s0 = decltype(SS)::value;
    static_for<0, s0>([&](auto TT) {
      constexpr int t0 = decltype(TT)::value;
      syrk_update(a[s0], *(const v4d*)(W + dw_u(t0, s0) * 256), a[t0]);
    });
    const v4d E = *(const v4d*)(W + s0 * 256);
    const v4d rs = *(const v4d*)(W + (4 + s0) * 256);
    v4d acc = {0.0, 0.0, 0.0, 0.0};
    static_for<0, 4>([&](auto S2) {
      constexpr int sk = decltype(S2)::value;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(E[sk], a[s0][sk], acc, 0, 0, 0);
    });
    static_for<0, 4>([&](auto R) {
      constexpr int r = decltype(R)::value;
      a[s0][r] = acc[r] * rs[r];
    });
  });
  static_for<0, 4>([&](auto SS) {
    constexpr int s0 = decltype(SS)::value;
    static_for<0, 4>([&](auto R) {
      constexpr int r = decltype(R)::value;
      T[(long long)(16 * s0 + q + 4 * r) * Np + c] = a[s0][r];
    });
  });
}

// stage a 64 x 64 tile (row stride ld, 16-byte aligned rows) into LDS
// [64][64 + 1] with 256 threads: all eight 16-byte loads of a thread issued
// before its first LDS write (a rolled loop waited on each load in turn --
// 16 dependent global round trips per tile, most of the right-looking update
// kernel's time at B = 1)
typedef double v2d __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void stage64(double (*dst)[DCB + 1], const double* src, long long ld) {
  constexpr int NIT = DCB * DCB / 2 / 256;
  v2d v[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int p = threadIdx.x + 256 * it;
    v[it] = *(const v2d*)(src + (long long)(p >> 5) * ld + 2 * (p & 31));
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int p = threadIdx.x + 256 * it;
    dst[p >> 5][2 * (p & 31)] = v[it][0];
    dst[p >> 5][2 * (p & 31) + 1] = v[it][1];
  }
}

// Panel: U_kj = W A_kj for the blocks j > k of every sample (in place).
// grid (nb - k - 1, Bc); 4 waves, wave w -> rows 16w..16w+15, 4 column blocks.
__global__ __launch_bounds__(256) void dchol_panel_kernel(double* __restrict__ mats, int Np, int k,
                                                          const double* __restrict__ wbuf) {
  __shared__ double Ws[DCB][DCB + 1];
  __shared__ double As[DCB][DCB + 1];
  const int j = k + 1 + blockIdx.x, bl = blockIdx.y;
  double* Akj = mats + (long long)bl * Np * Np + (long long)(DCB * k) * Np + DCB * j;
  stage64(Ws, wbuf + (long long)bl * DCB * DCB, DCB);
  stage64(As, Akj, Np);
  __syncthreads();
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;
  v4d acc[4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
  for (int ts = 0; ts < DCB / 4; ++ts) {
    const double a = Ws[16 * w + c][4 * ts + q];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) acc[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, As[4 * ts + q][16 * jb + c], acc[jb], 0, 0, 0);
  }
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int r = 0; r < 4; ++r) Akj[(long long)(16 * w + q + 4 * r) * Np + 16 * jb + c] = acc[jb][r];
}

// Trailing update A_ij -= U_ki^T U_kj, k < i <= j, every sample.
// grid (T(k), Bc) with T(k) = m (m + 1) / 2, m = nb - k - 1.
__device__ __forceinline__ void update_tile_body(double* __restrict__ mats, int Np, int k) {
  __shared__ double Ui[DCB][DCB + 1];
  __shared__ double Uj[DCB][DCB + 1];
  const int nb = Np / DCB, m = nb - k - 1;
  int tix = blockIdx.x, ii = 0;
  while (tix >= m - ii) { tix -= m - ii; ++ii; }
  const int i = k + 1 + ii, j = i + tix;
  const int bl = blockIdx.y;
  double* base = mats + (long long)bl * Np * Np;
  stage64(Ui, base + (long long)(DCB * k) * Np + DCB * i, Np);
  stage64(Uj, base + (long long)(DCB * k) * Np + DCB * j, Np);
  double* Aij = base + (long long)(DCB * i) * Np + DCB * j;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;
  v4d acc[4];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[jb][r] = Aij[(long long)(16 * w + q + 4 * r) * Np + 16 * jb + c];
  __syncthreads();
#pragma unroll
  for (int ts = 0; ts < DCB / 4; ++ts) {
    const double a = -Ui[4 * ts + q][16 * w + c];
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) acc[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Uj[4 * ts + q][16 * jb + c], acc[jb], 0, 0, 0);
  }
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int r = 0; r < 4; ++r) Aij[(long long)(16 * w + q + 4 * r) * Np + 16 * jb + c] = acc[jb][r];
}

__global__ __launch_bounds__(256) void dchol_update_kernel(double* __restrict__ mats, int Np, int k) {
  update_tile_body(mats, Np, k);
}

// The trailing update of step k with the diagonal block k + 1 factored in
// the same launch: workgroup 0 of each sample owns tile (k + 1, k + 1);
// after storing it, its first wave runs the diagonal factorisation of
// dchol_diag_reg_kernel on it (same values, same code: bit-identical) while
// the other workgroups are still updating their tiles -- one launch and one
// dependent gap fewer per block row of the one-proposal schedule.  Nothing
// else reads the block-(k + 1) operands in wbuf before the next panel.
template <bool LAST>
__global__ __launch_bounds__(256) void dchol_update_diag_kernel(double* __restrict__ mats, int Np, int k,
                                                                double* __restrict__ wbuf, double* __restrict__ ldet,
                                                                double* __restrict__ qout, int* __restrict__ fail) {
  update_tile_body(mats, Np, k);
  if (blockIdx.x != 0) return;
  __syncthreads();   // the tile's rows stored by every wave of the workgroup
  if (threadIdx.x < 64) diag_reg_body<LAST>(mats, Np, k + 1, wbuf, ldet, qout, fail, blockIdx.y, threadIdx.x);
}

// Row-oriented (left-looking) update, the default: before block row i is
// factored, A_ij -= sum_{p < i} U_pi^T U_pj for every j >= i.  One workgroup
// per (j, sample) keeps its 64 x 64 tile in registers across all p (K = 64 i),
// staging U_pi / U_pj through LDS with the next pair prefetched into
// registers: each tile is read and written once per factorisation instead of
// once per panel step (the right-looking dchol_update_kernel above).
__global__ __launch_bounds__(256) void dchol_rowupdate_kernel(double* __restrict__ mats, int Np, int i) {
  __shared__ double Ui[DCB][DCB + 1];
  __shared__ double Uj[DCB][DCB + 1];
  const int j = i + blockIdx.x, bl = blockIdx.y, t = threadIdx.x;
  double* base = mats + (long long)bl * Np * Np;
  double* Aij = base + (long long)(DCB * i) * Np + DCB * j;
  const int w = t >> 6, lane = t & 63, q = lane >> 4, c = lane & 15;
  v4d acc[4];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[jb][r] = Aij[(long long)(16 * w + q + 4 * r) * Np + 16 * jb + c];
  double pf[32];
  auto gload = [&](int p) {
    const double* rp = base + (long long)(DCB * p) * Np;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int idx = t + 256 * r, row = idx >> 6, col = idx & 63;
      pf[r] = rp[(long long)row * Np + DCB * i + col];
      pf[16 + r] = rp[(long long)row * Np + DCB * j + col];
    }
  };
  gload(0);
  for (int p = 0; p < i; ++p) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int idx = t + 256 * r, row = idx >> 6, col = idx & 63;
      Ui[row][col] = pf[r];
      Uj[row][col] = pf[16 + r];
    }
    __syncthreads();
    if (p + 1 < i) gload(p + 1);
#pragma unroll
    for (int ts = 0; ts < DCB / 4; ++ts) {
      const double a = -Ui[4 * ts + q][16 * w + c];
#pragma unroll
      for (int jb = 0; jb < 4; ++jb)
        acc[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, Uj[4 * ts + q][16 * jb + c], acc[jb], 0, 0, 0);
    }
  }
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int r = 0; r < 4; ++r) Aij[(long long)(16 * w + q + 4 * r) * Np + 16 * jb + c] = acc[jb][r];
}

// The same row update with more waves per CU (the default): only U_pj is
// staged through LDS (one 64 x 64 tile, 33 KB: four workgroups fit a CU
// instead of two); each wave reads its A operand -- the 64 x 16 column slab
// of U_pi it multiplies, 16 doubles per lane -- straight from global memory
// into registers, prefetched one step ahead together with the U_pj tile; the
// minus sign is the MFMA neg modifier.  Same sums in the same order as
// dchol_rowupdate_kernel: bit-identical.  p0 > 0: only the rows p0 <= p < i
// (the rest already applied by dchol_rowpair_kernel).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4)))
void dchol_rowupdate2_kernel(double* __restrict__ mats, int Np, int i, int p0) {
  __shared__ double Uj[DCB][DCB + 1];
  const int j = i + blockIdx.x, bl = blockIdx.y, t = threadIdx.x;
  const int w = t >> 6, lane = t & 63, q = lane >> 4, c = lane & 15;
  // accesses as the sample's uniform base + 32-bit byte offsets (see
  // dchol_rowpair_kernel)
  char* cb = (char*)(mats + (long long)bl * Np * Np);
  auto at = [&](unsigned off) -> double& { return *(double*)(cb + off); };
  const unsigned rowb = 8u * (unsigned)Np;
  const unsigned toff = (unsigned)(DCB * i + 16 * w + q) * rowb + 8u * (unsigned)(DCB * j + c);
  v4d acc[4];
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[jb][r] = at(toff + (unsigned)(4 * r) * rowb + 8u * (unsigned)(16 * jb));
  // A slab of U_pi (column block 16w..16w+15, all 64 rows) in registers, U_pj
  // staged through LDS (prefetched one step ahead into registers)
  const unsigned aoff = (unsigned)q * rowb + 8u * (unsigned)(DCB * i + 16 * w + c);
  const unsigned boff = (unsigned)(t >> 6) * rowb + 8u * (unsigned)(DCB * j + (t & 63));
  double pb[16];
  auto bload = [&](int p) {
    unsigned o = boff + (unsigned)(DCB * p) * rowb;
    asm volatile("" : "+v"(o));
#pragma unroll
    for (int r = 0; r < 16; ++r) pb[r] = at(o + (unsigned)(4 * r) * rowb);
  };
  // the A slab of the next step is loaded into the registers of this one as
  // they die (a[0..7] after the MFMAs of ts = 7, a[8..15] after ts = 15), as
  // in dchol_rowpair_kernel<PIPE>; loads unconditional (the last step reloads
  // its own rows) so the waitcnt pass sees one path
  if (p0 < i) {
    double a[16];
    auto ahalf = [&](int p, int h) {
      unsigned o = aoff + (unsigned)(DCB * p) * rowb;
      asm volatile("" : "+v"(o));
#pragma unroll
      for (int ts = 8 * h; ts < 8 * h + 8; ++ts) a[ts] = at(o + (unsigned)(4 * ts) * rowb);
    };
    bload(p0);
    ahalf(p0, 0);
    ahalf(p0, 1);
    for (int p = p0; p < i; ++p) {
      const int pn = min(p + 1, i - 1);
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 16; ++r) Uj[(t >> 6) + 4 * r][t & 63] = pb[r];
      __syncthreads();
      bload(pn);
      static_for<0, 2>([&](auto H) {
        constexpr int h = decltype(H)::value;
#pragma unroll
        for (int ts = 8 * h; ts < 8 * h + 8; ++ts) {
#pragma unroll
          for (int jb = 0; jb < 4; ++jb)
            acc[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ts], Uj[4 * ts + q][16 * jb + c], acc[jb], 0, 0, 1);
        }
        asm volatile("" ::: "memory");
        ahalf(pn, h);
        asm volatile("" ::: "memory");
      });
    }
  }
  unsigned toff2 = toff;
  asm volatile("" : "+v"(toff2));
#pragma unroll
  for (int jb = 0; jb < 4; ++jb)
#pragma unroll
    for (int r = 0; r < 4; ++r) at(toff2 + (unsigned)(4 * r) * rowb + 8u * (unsigned)(16 * jb)) = acc[jb][r];
}

// Row update + panel in one pass for the tiles j > k of block row k (after
// dchol_diag_reg_kernel has factored tile (k, k)): wave w owns the 16-column
// strip w of tile (k, j) over all 64 rows, so after accumulating
// A_kj - sum_p U_pk^T U_pj it applies the block forward substitution of
// dchol_panel_reg_kernel to its own registers and writes U_kj once (no
// round trip of the updated tile through HBM, one launch less per block row).
// U_pk is staged through LDS (shared by the four waves), each wave's U_pj
// slab comes from global memory into registers.  Same sums, same order as
// dchol_rowupdate2_kernel + dchol_panel_reg_kernel: bit-identical.
// TPW = 2 (the default since round 4): two tiles (k, j), (k, j + 1) per
// 8-wave workgroup sharing one LDS copy of U_pk -- per p the workgroup reads
// 96 KB (U_pk + two U_pj) for two tiles instead of 64 KB for one; C5 at
// B = 512: 91.3 vs 95.8 ms per batch, bit-identical (scripts/c5_ab.py).
// TPW = 1: the round-3 form (dev kernel mode 28).  p0 > 0: only the rows
// p0 <= p < k (dchol_rowpair_kernel applied the others; p0 = k: the panel
// alone).
template <int TPW>
__global__ __launch_bounds__(256 * TPW) __attribute__((amdgpu_waves_per_eu(TPW == 1 ? 3 : 4, TPW == 1 ? 3 : 4)))
void dchol_rowpanel_kernel(double* __restrict__ mats, int Np, int k, int p0, const double* __restrict__ wbuf) {
  constexpr int NT = 256 * TPW, RW = 64 / (NT / 64);   // threads; U_pk rows staged per thread
  __shared__ double Uk[DCB][DCB + 1];
  const int t = threadIdx.x, wave = t >> 6, tile = wave >> 2, w = wave & 3;
  const int j = k + 1 + TPW * blockIdx.x + tile, bl = blockIdx.y;
  const bool live = j < Np / DCB;                  // (the last workgroup of an odd row: one tile)
  double* base = mats + (long long)bl * Np * Np;
  double* Akj = base + (long long)(DCB * k) * Np + DCB * (live ? j : k + 1);
  const int lane = t & 63, q = lane >> 4, c = lane & 15;
  v4d acc[4];
#pragma unroll
  for (int s0 = 0; s0 < 4; ++s0)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[s0][r] = live ? Akj[(long long)(16 * s0 + q + 4 * r) * Np + 16 * w + c] : 0.0;
  const double* bcol = base + DCB * (live ? j : k + 1) + 16 * w + c + (long long)q * Np;
  const double* acol = base + DCB * k + (t & 63) + (long long)(t >> 6) * Np;
  double pa[RW];
  auto aload = [&](int p) {
    const double* rp = acol + (long long)(DCB * p) * Np;
#pragma unroll
    for (int r = 0; r < RW; ++r) pa[r] = rp[(long long)((NT / 64) * r) * Np];
  };
  if (p0 < k) aload(p0);
  for (int p = p0; p < k; ++p) {
    double b[16];
    const double* bp = bcol + (long long)(DCB * p) * Np;
#pragma unroll
    for (int ts = 0; ts < 16; ++ts) b[ts] = bp[(long long)(4 * ts) * Np];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RW; ++r) Uk[(t >> 6) + (NT / 64) * r][t & 63] = pa[r];
    __syncthreads();
    // (measured round 4: forcing a true one-step-ahead prefetch here -- an
    // unconditional load pinned by an empty asm -- ran C5 at 89.9 instead of
    // 83.6 ms; as written the compiler issues it with the next step's loads)
    if (p + 1 < k) aload(p + 1);
#pragma unroll
    for (int ts = 0; ts < DCB / 4; ++ts) {
#pragma unroll
      for (int s0 = 0; s0 < 4; ++s0)
        acc[s0] = __builtin_amdgcn_mfma_f64_16x16x4f64(Uk[4 * ts + q][16 * s0 + c], b[ts], acc[s0], 0, 0, 1);
    }
  }
  if (!live) return;
  // the panel: U_kj = L_kk^-1 A_kj on this strip (dchol_panel_reg_kernel)
  const double* W = wbuf + (long long)bl * DW_SLOTS * 256 + lane * 4;
  static_for<0, 4>([&](auto SS) {
    constexpr int s0 = decltype(SS)::value;
    static_for<0, s0>([&](auto TT) {
      constexpr int t0 = decltype(TT)::value;
      syrk_update(acc[s0], *(const v4d*)(W + dw_u(t0, s0) * 256), acc[t0]);
    });
    const v4d E = *(const v4d*)(W + s0 * 256);
    const v4d rs = *(const v4d*)(W + (4 + s0) * 256);
    v4d v = {0.0, 0.0, 0.0, 0.0};
    static_for<0, 4>([&](auto S2) {
      constexpr int sk = decltype(S2)::value;
      v = __builtin_amdgcn_mfma_f64_16x16x4f64(E[sk], acc[s0][sk], v, 0, 0, 0);
    });
    static_for<0, 4>([&](auto R) {
      constexpr int r = decltype(R)::value;
      acc[s0][r] = v[r] * rs[r];
    });
  });
#pragma unroll
  for (int s0 = 0; s0 < 4; ++s0)
#pragma unroll
    for (int r = 0; r < 4; ++r) Akj[(long long)(16 * s0 + q + 4 * r) * Np + 16 * w + c] = acc[s0][r];
}

// The row update of two block rows at once -- a 128-row block row for the
// update, whose cost is streaming the finished rows U_pj from HBM: tiles
// (k, j) and (k + 1, j) for j > k take the updates of every row p < k, the
// U_pj tile streamed once for both (twice the MFMA work per HBM byte of
// dchol_rowpanel_kernel), U_pk and U_p,k+1 (adjacent; shared by every
// workgroup of the sample, from L2) staged through LDS.  8 waves per column
// tile j: wave w updates strip w & 3 (16 columns, all 64 rows) of tile
// (k + (w >> 2), j); the two waves of a strip read the same U_pj slab (the
// second read from L1 / L2).  Launched after dchol_diag_reg_kernel has
// factored tile (k, k): the row-k waves finish with the panel (U_kj written
// once, as dchol_rowpanel_kernel), the row-(k + 1) accumulators go back to
// HBM and row k + 1 takes its last update p = k in dchol_rowpanel_kernel
// (p0 = k) -- per tile the same MFMAs on the same operands in the same order
// as the one-row schedule, the accumulator stored and reloaded exactly in
// between: bit-identical (dev kernel mode 31 runs the one-row schedule).
// PIPE (the default): the next step's U_pj slab is loaded into the registers
// of the current one as they die -- b[0..7] after the MFMAs of ts = 7,
// b[8..15] after ts = 15 -- so no step starts on a cold load and no register
// is added (the loads pinned in place by empty asm statements).  C5 at
// B = 512: 80.7 vs 83.6 ms (!PIPE, the slab loaded at the top of its step:
// dev kernel mode 32), bit-identical.
// (Measured and dropped: one more workgroup per sample pre-updating the next
// pair's diagonal tile over p < k, which cut the diagonal-tile row update
// from 69 to 17 us per launch but lengthened the pair launches by more --
// m + 1 instead of m workgroups per sample, and late pairs have m ~ 1-3:
// 81.3 vs 79.7 ms per C5 batch.)
template <bool PIPE>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4)))
void dchol_rowpair_kernel(double* __restrict__ mats, int Np, int k, const double* __restrict__ wbuf) {
  __shared__ double Uk[2][DCB][DCB + 1];
  const int t = threadIdx.x, wave = t >> 6, rt = wave >> 2, w = wave & 3;
  const int j = k + 1 + blockIdx.x, bl = blockIdx.y;
  const int lane = t & 63, q = lane >> 4, c = lane & 15;
  // every access as the sample's (uniform) base + a 32-bit byte offset (a
  // sample's matrix is < 4 GB); the offsets pass through an empty asm where
  // the compiler would otherwise keep one register per load live across the
  // loop (which spills)
  char* cb = (char*)(mats + (long long)bl * Np * Np);
  auto at = [&](unsigned off) -> double& { return *(double*)(cb + off); };
  const unsigned rowb = 8u * (unsigned)Np;                       // bytes per row
  // this lane's element (q, c) of strip w of tile (k + rt, j)
  const unsigned toff = (unsigned)(DCB * (k + rt) + q) * rowb + 8u * (unsigned)(DCB * j + 16 * w + c);
  v4d acc[4];
#pragma unroll
  for (int s0 = 0; s0 < 4; ++s0)
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[s0][r] = at(toff + (unsigned)(16 * s0 + 4 * r) * rowb);
  const unsigned boff = (unsigned)q * rowb + 8u * (unsigned)(DCB * j + 16 * w + c);
  // staging: thread t holds column (t & 127) of the 128-column pair, rows
  // (t >> 7) + 4 r
  const int scol = t & 127, srow = t >> 7, stile = scol >> 6, scc = scol & 63;
  const unsigned aoff = 8u * (unsigned)(DCB * k + scol) + (unsigned)srow * rowb;
  double pa[16];
  auto aload = [&](int p) {
    unsigned o = aoff + (unsigned)(DCB * p) * rowb;
    asm volatile("" : "+v"(o));
#pragma unroll
    for (int r = 0; r < 16; ++r) pa[r] = at(o + (unsigned)(4 * r) * rowb);
  };
  if constexpr (!PIPE) {
    if (k > 0) aload(0);
    for (int p = 0; p < k; ++p) {
      double b[16];
      unsigned o = boff + (unsigned)(DCB * p) * rowb;
      asm volatile("" : "+v"(o));
#pragma unroll
      for (int ts = 0; ts < 16; ++ts) b[ts] = at(o + (unsigned)(4 * ts) * rowb);
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 16; ++r) Uk[stile][srow + 4 * r][scc] = pa[r];
      __syncthreads();
      // (measured round 4: forcing a true one-step-ahead prefetch here -- an
      // unconditional load pinned by an empty asm -- ran C5 at 89.9 instead of
      // 83.6 ms; as written the compiler issues it with the next step's loads)
      if (p + 1 < k) aload(p + 1);
#pragma unroll
      for (int ts = 0; ts < DCB / 4; ++ts) {
#pragma unroll
        for (int s0 = 0; s0 < 4; ++s0)
          acc[s0] = __builtin_amdgcn_mfma_f64_16x16x4f64(Uk[rt][4 * ts + q][16 * s0 + c], b[ts], acc[s0], 0, 0, 1);
      }
    }
  } else if (k > 0) {
    double b[16];
    auto bhalf = [&](int p, int h) {           // b[8 h .. 8 h + 7] of step p
      unsigned o = boff + (unsigned)(DCB * p) * rowb;
      asm volatile("" : "+v"(o));
#pragma unroll
      for (int ts = 8 * h; ts < 8 * h + 8; ++ts) b[ts] = at(o + (unsigned)(4 * ts) * rowb);
    };
    aload(0);
    bhalf(0, 0);
    bhalf(0, 1);
    for (int p = 0; p < k; ++p) {
      const int pn = min(p + 1, k - 1);          // (unconditional loads: one waitcnt path)
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 16; ++r) Uk[stile][srow + 4 * r][scc] = pa[r];
      __syncthreads();
      aload(pn);
      static_for<0, 2>([&](auto H) {
        constexpr int h = decltype(H)::value;
#pragma unroll
        for (int ts = 8 * h; ts < 8 * h + 8; ++ts) {
#pragma unroll
          for (int s0 = 0; s0 < 4; ++s0)
            acc[s0] = __builtin_amdgcn_mfma_f64_16x16x4f64(Uk[rt][4 * ts + q][16 * s0 + c], b[ts], acc[s0], 0, 0, 1);
        }
        asm volatile("" ::: "memory");
        bhalf(pn, h);
        asm volatile("" ::: "memory");
      });
    }
  }
  if (rt == 0) {
    // row k is complete: its panel U_kj = L_kk^-1 A_kj on this strip, with the
    // operands dchol_diag_reg_kernel left in wbuf (as dchol_rowpanel_kernel)
    const double* W = wbuf + (long long)bl * DW_SLOTS * 256 + lane * 4;
    static_for<0, 4>([&](auto SS) {
      constexpr int s0 = decltype(SS)::value;
      static_for<0, s0>([&](auto TT) {
        constexpr int t0 = decltype(TT)::value;
        syrk_update(acc[s0], *(const v4d*)(W + dw_u(t0, s0) * 256), acc[t0]);
      });
      const v4d E = *(const v4d*)(W + s0 * 256);
      const v4d rs = *(const v4d*)(W + (4 + s0) * 256);
      v4d v = {0.0, 0.0, 0.0, 0.0};
      static_for<0, 4>([&](auto S2) {
        constexpr int sk = decltype(S2)::value;
        v = __builtin_amdgcn_mfma_f64_16x16x4f64(E[sk], acc[s0][sk], v, 0, 0, 0);
      });
      static_for<0, 4>([&](auto R) {
        constexpr int r = decltype(R)::value;
        acc[s0][r] = v[r] * rs[r];
      });
    });
  }
  unsigned toff2 = toff;
  asm volatile("" : "+v"(toff2));
#pragma unroll
  for (int s0 = 0; s0 < 4; ++s0)
#pragma unroll
    for (int r = 0; r < 4; ++r) at(toff2 + (unsigned)(16 * s0 + 4 * r) * rowb) = acc[s0][r];
}

// ----------------------------------------------------------------------------
// optimal statistic (EWH_COMMON_OPTSTAT handles; ewh_optstat)
// From pulsar a's kept block K (its common columns G after eliminating the
// rest, phi^-1 on every column): (Sigma^-1)_GG = K_GG^-1 and
// (Sigma^-1 d)_G = K_GG^-1 K_Gr, so with D = diag(phi^-1)_G
//   X = D K_GG^-1 K_Gr,  Z = D - D K_GG^-1 D
// (F^T P^-1 r and F^T P^-1 F by Woodbury: TNT = Sigma - Phi^-1).  Stored
// pre-scaled by phihat^1/2: x^ = phihat^1/2 X, W = phihat^1/2 Z phihat^1/2, so
// that per pair top = x^_a . x^_b and bot = tr(Z_a phihat Z_b phihat) = <W_a, W_b>.
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(64) void os_xz_kernel(const double* __restrict__ keep, int KD, int P, int nc,
                                                   const CommonPsr* __restrict__ cps,
                                                   const double* __restrict__ theta, int ldth,
                                                   const double* __restrict__ phihat, double* __restrict__ xh,
                                                   double* __restrict__ wh) {
  __shared__ double M[32][33];
  __shared__ double colk[32], rowk[32], dv[32], kr[32], sq[32];
  const int a = blockIdx.x, bl = blockIdx.y, t = threadIdx.x;
  const double* K = keep + ((long long)a * gridDim.y + bl) * KD * KD;     // pulsar-major, B = gridDim.y
  const double* th = theta + (long long)bl * ldth;
  for (int idx = t; idx < nc * nc; idx += 64) M[idx / nc][idx % nc] = K[(idx / nc) * KD + idx % nc];
  if (t < nc) {
    kr[t] = K[t * KD + KD - 1];
    const CommonPsr c = cps[a];
    double ph = 0.0;
    for (int e = c.colptr[c.gstart + t]; e < c.colptr[c.gstart + t + 1]; ++e) ph += spec_phi(c.spec[e], th);
    dv[t] = 1.0 / ph;
    sq[t] = sqrt(phihat[(long long)bl * nc + t]);
  }
  __syncthreads();
  for (int k = 0; k < nc; ++k) {        // Gauss-Jordan inverse of K_GG (SPD)
    const double pinv = 1.0 / M[k][k];
    if (t < nc) {
      colk[t] = M[t][k];
      rowk[t] = M[k][t] * pinv;
    }
    __syncthreads();
    for (int idx = t; idx < nc * nc; idx += 64) {
      const int i = idx / nc, j = idx % nc;
      double v;
      if (i == k) v = (j == k) ? pinv : rowk[j];
      else if (j == k) v = -colk[i] * pinv;
      else v = M[i][j] - colk[i] * rowk[j];
      M[i][j] = v;
    }
    __syncthreads();
  }
  double* xo = xh + ((long long)bl * P + a) * nc;
  double* wo = wh + ((long long)bl * P + a) * nc * nc;
  if (t < nc) {
    double v = 0.0;
    for (int h = 0; h < nc; ++h) v += M[t][h] * kr[h];
    xo[t] = sq[t] * dv[t] * v;
  }
  for (int idx = t; idx < nc * nc; idx += 64) {
    const int g = idx / nc, h = idx % nc;
    const double z = (g == h ? dv[g] : 0.0) - dv[g] * M[g][h] * dv[h];
    wo[idx] = sq[g] * z * sq[h];
  }
}

// rho_ab, sig_ab for b > a: one wave per pair (lanes over the nc^2 entries).
__global__ __launch_bounds__(256) void os_pairs_kernel(const double* __restrict__ xh, const double* __restrict__ wh,
                                                       int P, int nc, double* __restrict__ rho,
                                                       double* __restrict__ sig) {
  const int a = blockIdx.x, bl = blockIdx.y, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const double* xa = xh + ((long long)bl * P + a) * nc;
  const double* wa = wh + ((long long)bl * P + a) * nc * nc;
  for (int b = a + 1 + w; b < P; b += 4) {
    const double* xb = xh + ((long long)bl * P + b) * nc;
    const double* wb = wh + ((long long)bl * P + b) * nc * nc;
    double top = 0.0, bot = 0.0;
    for (int g = lane; g < nc; g += 64) top += xa[g] * xb[g];
    for (int idx = lane; idx < nc * nc; idx += 64) bot += wa[idx] * wb[idx];
    top = wave_sum(top);
    bot = wave_sum(bot);
    if (lane == 0) {
      rho[((long long)bl * P + a) * P + b] = top / bot;
      sig[((long long)bl * P + a) * P + b] = 1.0 / sqrt(bot);
    }
  }
}

// OS = sum rho Gamma / sig^2 / sum Gamma^2 / sig^2 per draw (pairs in order).
__global__ void os_final_kernel(const double* __restrict__ rho, const double* __restrict__ sig,
                                const double* __restrict__ orf, int P, int B, double* __restrict__ os,
                                double* __restrict__ os_sig) {
  const int bl = blockIdx.x * blockDim.x + threadIdx.x;
  if (bl >= B) return;
  double num = 0.0, den = 0.0;
  for (int a = 0; a < P; ++a)
    for (int b = a + 1; b < P; ++b) {
      const double s = sig[((long long)bl * P + a) * P + b], r = rho[((long long)bl * P + a) * P + b];
      const double g = orf[a * P + b];
      num += r * g / (s * s);
      den += g * g / (s * s);
    }
  os[bl] = num / den;
  os_sig[bl] = 1.0 / sqrt(den);
}

// Global term of sample b: units[P * B + b] = -1/2 (log|Sigma_c| + q_c + sum_g log|M_g|).
__global__ void common_final_kernel(const double* __restrict__ ldet, const double* __restrict__ qv,
                                    const int* __restrict__ fail, const double* __restrict__ mlog,
                                    const int* __restrict__ rep, int nc, int Bc, int b0, int P, int B,
                                    double* __restrict__ units) {
  const int bl = blockIdx.x * blockDim.x + threadIdx.x;
  if (bl >= Bc) return;
  double ml = 0.0;
  for (int g = 0; g < nc; ++g) ml += mlog[(long long)bl * nc + rep[g]];
  double v = -0.5 * (ldet[bl] + qv[bl] + ml);
  if (fail[bl] || !(qv[bl] == qv[bl]) || !(ml == ml)) v = -INFINITY;
  units[(long long)P * B + b0 + bl] = v;
}

// out[b] = sum_p units[p * B + b], pulsars in order.
// fl(hi + 2 lo) of a double-double matrix: the reversed verify pass's input
// (chol_wide_kernel forms the same value per load where it is not cached)
__global__ void rev_input_kernel(const double* __restrict__ hi, const double* __restrict__ lo, double* __restrict__ out,
                                 long long n) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = hi[i] + 2.0 * lo[i];
}

__global__ void reduce_units_kernel(const double* __restrict__ units, int P, int B, double* __restrict__ out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double s = 0.0;
  for (int p = 0; p < P; ++p) s += units[(long long)p * B + b];
  out[b] = s;
}

// Multi-context handle, theta staging: segment s of the table (5 ints: row_lo,
// row_hi, ncol, column-list offset, payload offset; the column lists follow
// the nseg records) scatters its packed rows x columns payload into the
// full-layout theta [B x np] of this device.  Columns and rows outside the
// segments are never read by the context's units (stage_theta_range sets them
// to NaN first).
__global__ __launch_bounds__(256) void expand_theta_kernel(const double* __restrict__ stage,
                                                           const int* __restrict__ seg, int nseg, int np,
                                                           double* __restrict__ theta) {
  const int* rec = seg + 5 * blockIdx.x;
  const int r0 = rec[0], nr = rec[1] - rec[0], nc = rec[2];
  const int* cols = seg + 5 * nseg + rec[3];
  const double* src = stage + rec[4];
  for (int idx = threadIdx.x; idx < nr * nc; idx += 256) {
    const int r = idx / nc, j = idx - r * nc;
    theta[(long long)(r0 + r) * np + cols[j]] = src[idx];
  }
}

// Multi-context handle: out[b] = sum_i part[i * B + b], the contexts' partial
// sums (each over its unit range, pulsars in order) in context order.
__global__ void fold_partials_kernel(const double* __restrict__ part, int nd, int B, double* __restrict__ out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double s = 0.0;
  for (int i = 0; i < nd; ++i) s += part[(long long)i * B + b];
  out[b] = s;
}

}  // namespace ewh_dev

using namespace ewh_dev;

// ----------------------------------------------------------------------------
// host side
// ----------------------------------------------------------------------------
namespace {

constexpr size_t LDS_MAX = 160 * 1024;

struct PsrHost {
  int n_toa = 0, m = 0, nlead = 0, ld = 0, nb = 0, n_epoch = 0;
  int max_epoch = 0;               // TOAs of the longest ECORR epoch
  int fx_m = 0, fx_ld = 0, fx_nb = 0;
  int ncommon = 0, nloc = 0, gstart = 0;   // correlated layout of the reduced matrix
  // correlated common process with varying white noise: T_aug is laid out
  // [lead | own | pad to 16 | common | pad | r] -- common column g at
  // gstart_v + g, so the partial factorisation keeps whole blocks; the pads
  // inside take phi = 1 (CONST entries); mreal_v = gstart_v columns take phi^-1
  int gstart_v = 0;
  PsrDev dev{};
  int* d_colptr = nullptr;        // varying CSR (m+1)
  DSpec* d_spec = nullptr;
  int* d_fx_colptr = nullptr;     // fixed CSR (fx_m+1), entries re-indexed
  DSpec* d_fx_spec = nullptr;
  int* d_fx_rep = nullptr;        // fixed columns -> first column with the same spectrum
  int* d_fx_ulist = nullptr;      // the distinct-spectrum columns
  int fx_nu = 0;
  URec* d_fx_urec = nullptr;      // the distinct spectra with their entries inline (NULL: > URec::NE entries)
  std::vector<int> fx_tidx;       // theta entries the records read (their indices point here); empty: the whole row
  int* d_fx_urep = nullptr;       // fixed columns -> distinct-spectrum record (-1: no entry)
  double* d_S = nullptr;          // fx_ld^2
  double* d_Slo = nullptr;        // fx_ld^2, the low part of S (dd_path pulsars only)
  double* d_Srev = nullptr;       // fx_ld^2, fl(S + 2 S_lo): the reversed verify pass's input (with d_Slo)
  // the projection residual X_lo of T_aug (round 6; the layout of dev.T,
  // zero outside the projected columns): dev.T + d_Tlo = T - M C to double-
  // double, read by the double-double Grams (gram_dd_block).  NULL for
  // pulsars with a theta-dependent basis (n_bgroup > 0) or the correlated
  // varying-WN layout
  double* d_Tlo = nullptr;
  bool has_theta_white = false;
  int n_slot = 0;
  ewh_pref* d_slots = nullptr;    // device copy of the white-noise slot table (PsrDev::slots)
  std::vector<ewh_pref> slots;    // host copy (ewh_set_fixed_white updates the constants)
};

}  // namespace

struct DevCtx {
  int device = 0;
  int n_cu = 256;              // compute units (hipDeviceAttributeMultiprocessorCount)
  int P = 0, n_param = 0;
  bool white_fixed = false;
  int kernel_mode = 0;
  bool stage_spectra = true;   // register kernels read the staged spectrum records (dev mode 19: the CSR path)
  hipStream_t stream = nullptr;
  std::vector<PsrHost> psr;
  std::vector<void*> allocs;
  CholJob* d_jobs_fixed = nullptr;
  CholJob* d_jobs_var = nullptr;
  double* d_fxK = nullptr;
  int* d_fxfail = nullptr;
  // per-call scratch
  double* d_units = nullptr;
  size_t units_cap = 0;
  double* d_theta = nullptr;
  double* d_out = nullptr;
  size_t io_cap = 0;
  // varying-WN scratch
  double *d_w = nullptr, *d_beta = nullptr, *d_s = nullptr, *d_G = nullptr, *d_Kb = nullptr, *d_fac = nullptr;
  double* d_rho = nullptr;       // r^T W r per sample (the r-separated contraction)
  long long s_stride = 0;     // doubles per sample in d_s (epoch rows padded to whole tiles)
  double* d_bigscr = nullptr; // chol_big_kernel: per-workgroup U blocks
  long long bigscr_cap = 0;   // workgroups per launch it holds
  int bigscr_nb = 0;
  long long scr_budget = 0;      // bytes for each of the wide / dd scratches (scratch_budget)
  double* d_widescr = nullptr;   // chol_wide_kernel: per-workgroup U blocks
  long long widescr_len = 0;     // doubles
  double* d_ddscr = nullptr;     // chol_dd_kernel: per-workgroup hi / lo matrices
  long long ddscr_len = 0;       // doubles
  double* d_units2 = nullptr;    // the verify step's reversed-order unit terms
  size_t units2_cap = 0;
  int* d_ddlist = nullptr;       // the verify step's flagged units, [0] = count, list from [1]
  size_t ddlist_cap = 0;
  // ewh_refine_stats since the last query: 64-bit device counters [0] units
  // chol_dd_kernel refactored, [1] units that took the double-double route --
  // counted in stream order by the verify kernel (or, kernel mode 29, by
  // count_units_kernel), so graph replays count and captures do not
  unsigned long long* d_ddstat = nullptr;
  double* d_Glo = nullptr;       // varying white noise, bases past 16 blocks: the low part of G (contract_wide_kernel)
  int chunk = 0;
  int chunk_cap = 0;          // largest chunk the ~1.5 GB scratch budget allows
  int last_B = 0;
  // correlated common process (fixed white noise)
  bool corr = false;
  int nc = 0, keep = 0, Np = 0, cchunk = 0;
  double* d_orf = nullptr;
  DSpec* d_cspec = nullptr;
  int* d_cuniq = nullptr;     // distinct M_g: representative common column per slot
  int* d_crep = nullptr;      // common column -> slot
  int nuniq = 0;
  CommonPsr* d_cps = nullptr;
  double *d_keep = nullptr, *d_minv = nullptr, *d_mlog = nullptr, *d_dense = nullptr, *d_wbuf = nullptr;
  double *d_cldet = nullptr, *d_cq = nullptr;
  int* d_cfail = nullptr;
  size_t keep_cap = 0;
  int cchunk_cap = 0;         // samples the dense Sigma_c budget allows per chunk
  int n_param_desc = 0;
  bool osmode = false;        // EWH_COMMON_OPTSTAT handle (ewh_optstat only)
  // captured ewh_lnl_batch sequences (H2D, launches, D2H) per batch size:
  // a sampler's single-theta calls replay one graph instead of ~5 API calls
  struct Graph {
    int B, mode;
    const void *ht, *ho;
    hipGraphExec_t exec;
    long long last_use;
  };
  std::vector<Graph> graphs;
  long long graph_clock = 0;
  // latency path of small single-device batches (chol_lat.hip): every pulsar
  // has the same reduced block count lat_nb <= LAT_NB_MAX (0: not eligible)
  int lat_nb = 0;
  // correlated process: a second stream on which the M_g inverses of the
  // first sample chunk run beside the per-pulsar partial factorisations
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // multi-context batches: the theta entries this context's units read,
  // packed in pinned host memory (h_stage), copied to d_stage and scattered
  // into d_theta by expand_theta_kernel along the segment table d_seg
  double* h_stage = nullptr;
  size_t h_stage_cap = 0;
  int* h_seg = nullptr;
  size_t h_seg_cap = 0;
  double* d_stage = nullptr;
  size_t d_stage_cap = 0;
  int* d_seg = nullptr;
  size_t d_seg_cap = 0;
};

namespace {

// captured graphs hold device pointers: any (re)allocation invalidates them
void drop_graphs(DevCtx* h) {
  for (auto& g : h->graphs) (void)hipGraphExecDestroy(g.exec);
  h->graphs.clear();
}

template <typename T>
int dalloc(DevCtx* h, T** p, size_t count) {
  drop_graphs(h);
  *p = nullptr;
  if (count == 0) count = 1;
  hipError_t e = hipMalloc((void**)p, count * sizeof(T));
  if (e != hipSuccess) return set_err(EWH_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  h->allocs.push_back(*p);
  return 0;
}

template <typename T>
int dupload(DevCtx* h, T** p, const T* src, size_t count) {
  int rc = dalloc(h, p, count);
  if (rc) return rc;
  if (count) EWH_HIP(hipMemcpy(*p, src, count * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}

int nb_for(int cols_with_r) { return (cols_with_r + 15) / 16; }

size_t lds_bytes_chol(int mreal) {
  const size_t ma = (size_t)mreal + 1;
  return (ma * (ma + 1) / 2 + ma) * sizeof(double);
}

bool pref_uses_theta(const ewh_pref& r) { return r.idx >= 0; }

int validate(const ewh_pta_desc* d) {
  std::string msg;
  const int rc = ewh_desc::desc_check(d, msg);
  return rc ? set_err(rc, msg) : 0;
}

DSpec to_dspec(const ewh_spec_entry& e, int col) {
  DSpec d{};
  d.kind = e.kind;
  d.col = col;
  d.i0 = e.p0.idx; d.i1 = e.p1.idx; d.i2 = e.p2.idx;
  d.v0 = e.p0.cval; d.v1 = e.p1.cval; d.v2 = e.p2.cval;
  d.f = e.f;
  d.lnf = e.f > 0 ? std::log(e.f) : 0.0;
  d.lnfyr = e.fyr > 0 ? std::log(e.fyr) : 0.0;
  d.a = e.df > 0 ? std::log(e.df / (12.0 * M_PI * M_PI)) : 0.0;
  return d;
}

// CSR over columns [c0, c1) re-indexed to start at 0 (caller's entry order kept per column).
void build_csr(const ewh_pulsar_desc& s, int c0, int c1, std::vector<int>& ptr, std::vector<DSpec>& ent) {
  const int n = c1 - c0;
  ptr.assign(n + 1, 0);
  for (int e = 0; e < s.n_spec; ++e)
    if (s.spec[e].col >= c0 && s.spec[e].col < c1) ptr[s.spec[e].col - c0 + 1]++;
  for (int j = 0; j < n; ++j) ptr[j + 1] += ptr[j];
  ent.assign(ptr[n], DSpec{});
  std::vector<int> fill(ptr.begin(), ptr.end() - 1);
  for (int e = 0; e < s.n_spec; ++e) {
    const int cc = s.spec[e].col;
    if (cc >= c0 && cc < c1) ent[fill[cc - c0]++] = to_dspec(s.spec[e], cc - c0);
  }
}

// CSR over T_aug positions for the correlated varying-white-noise layout:
// basis column c at pos(c), and a CONST phi = 1 entry on each internal pad
// position [pad0, pad1) (an identity row / column: pivot 1, log phi 0)
void build_csr_mapped(const ewh_pulsar_desc& s, const std::vector<int>& pos, int ncols, int pad0, int pad1,
                      std::vector<int>& ptr, std::vector<DSpec>& ent) {
  ptr.assign(ncols + 1, 0);
  for (int e = 0; e < s.n_spec; ++e) ptr[pos[s.spec[e].col] + 1]++;
  for (int a = pad0; a < pad1; ++a) ptr[a + 1]++;
  for (int j = 0; j < ncols; ++j) ptr[j + 1] += ptr[j];
  ent.assign(ptr[ncols], DSpec{});
  std::vector<int> fill(ptr.begin(), ptr.end() - 1);
  for (int e = 0; e < s.n_spec; ++e) {
    const int a = pos[s.spec[e].col];
    ent[fill[a]++] = to_dspec(s.spec[e], a);
  }
  for (int a = pad0; a < pad1; ++a) {
    ewh_spec_entry one{};
    one.kind = EWH_SPEC_CONST;
    one.col = a;
    one.p0 = ewh_pref{-1, 0, 1.0};
    one.p1 = ewh_pref{-1, 0, 0.0};
    one.p2 = ewh_pref{-1, 0, 0.0};
    ent[fill[a]++] = to_dspec(one, a);
  }
}

// CSR over the fixed (reduced) layout's fx_ld positions: basis column c >=
// nlead lands at c - nlead (own) or gstart + (c - nlead - nloc) (common).
void build_csr_fixed(const ewh_pulsar_desc& s, int nlead, int nloc, int gstart, int fx_ld, std::vector<int>& ptr,
                     std::vector<DSpec>& ent) {
  auto pos = [&](int c) { return c - nlead < nloc ? c - nlead : gstart + (c - nlead - nloc); };
  ptr.assign(fx_ld + 1, 0);
  for (int e = 0; e < s.n_spec; ++e)
    if (s.spec[e].col >= nlead) ptr[pos(s.spec[e].col) + 1]++;
  for (int j = 0; j < fx_ld; ++j) ptr[j + 1] += ptr[j];
  ent.assign(ptr[fx_ld], DSpec{});
  std::vector<int> fill(ptr.begin(), ptr.end() - 1);
  for (int e = 0; e < s.n_spec; ++e) {
    const int cc = s.spec[e].col;
    if (cc >= nlead) ent[fill[pos(cc)]++] = to_dspec(s.spec[e], pos(cc));
  }
}

// columns of a CSR whose spectral entries equal (all fields but `col`, bit
// for bit, same order) those of an earlier column: rep[a] = that column (a
// itself when first or without entries); ulist = the first columns with
// entries.  The sin / cos columns of one frequency share a spectrum.
void build_spec_rep(const std::vector<int>& ptr, const std::vector<DSpec>& ent, std::vector<int>& rep,
                    std::vector<int>& ulist) {
  const int ncol = (int)ptr.size() - 1;
  rep.assign(ncol, 0);
  ulist.clear();
  std::map<std::string, int> first;
  for (int a = 0; a < ncol; ++a) {
    rep[a] = a;
    if (ptr[a] == ptr[a + 1]) continue;
    std::string key;
    for (int e = ptr[a]; e < ptr[a + 1]; ++e) {
      DSpec d = ent[e];
      const int f[5] = {d.kind, d.i0, d.i1, d.i2, 0};
      const double v[7] = {d.v0, d.v1, d.v2, d.a, d.lnf, d.lnfyr, d.f};
      key.append((const char*)f, sizeof f);
      key.append((const char*)v, sizeof v);
    }
    auto it = first.find(key);
    if (it == first.end()) {
      first.emplace(key, a);
      ulist.push_back(a);
    } else {
      rep[a] = it->second;
    }
  }
}

// kernel mode 27: every factorisation (full and partial) by chol_wide_kernel
// (routing only: the wide kernel is part of the product; tests compare it
// with the register kernels); 29: the double-double path for every unit it
// covers, without the verify step
constexpr int MODE_WIDE = 27, MODE_DD = 29;

// The double-double factorisation (chol_dd_kernel) takes the uncorrelated
// units the fp64 register kernels do not cover with fixed white noise
// (reduced width > 9 blocks: the cached S is double-double) and every basis
// wider than 16 blocks; kernel mode 27 routes them to the fp64 chol_wide
// instead, mode 1 to the LDS kernel (A/B)
// (MODE_DD: every unit in double-double; the default: verify-and-refine --
// the forward and the reversed-order fp64 chol_wide factorisations, and
// chol_dd_kernel only for the units on which they disagree by more than
// 1/16 of the strict bound (VERIFY_FRAC, chol_dd.hip; 1/4 until r05j let 5 of
// 4096 system-model prior draws through at up to 4.4x strict from double-
// double): near-truth draws stay on fp64 MFMA, the ill-conditioned prior
// draws get the double-double value)
// Round 6: MODE_DD also takes the fixed-white-noise pulsars at the register
// kernels' widths (nb <= 9: the headline C3 model), so the headline batch has a
// device-side double-double twin (tests/test_gpu_parity.py::
// test_headline_matches_dd_at_scale); their S_lo is kept from the mode's
// setting on (ewh_set_kernel_mode re-runs setup_fixed)
bool dd_path(const DevCtx* h, int nb, bool fixed) {
  if (h->corr || h->osmode || h->kernel_mode == MODE_WIDE || h->kernel_mode == 1) return false;
  if (h->kernel_mode == MODE_DD && fixed) return true;
  return nb > BIG_NB_MAX || (fixed && nb > MFMA_NB_MAX);
}

// Scratch budgets of the wide / double-double factorisations: one slot per
// resident workgroup.  Round 5 sized them to fill the chip -- 4 GB of the
// 288 GB HBM: chol_dd_kernel at 384 columns (2.4 MB per workgroup) had run on
// 56 workgroups (56 of 256 CUs) under the earlier 128 MB, chol_wide_kernel at
// 24 blocks (600 KB) on 218 waves per launch.  Dev mode 34 keeps the 128 MB
// budgets and the separate forward / reversed launches (A/B).
constexpr int MODE_WIDE_R05A = 34;
// (capped at an eighth of the device memory free when first sized, so several
// handles on one device -- multi-context tests, one handle per sampler
// thread -- cannot take it all; at least the round-5a 128 MB)
long long scratch_budget(DevCtx* h) {
  if (h->kernel_mode == MODE_WIDE_R05A) return 1LL << 27;
  if (h->scr_budget == 0) {
    size_t fr = 0, tot = 0;
    (void)hipSetDevice(h->device);
    h->scr_budget = hipMemGetInfo(&fr, &tot) == hipSuccess
                        ? std::max<long long>(1LL << 27, std::min<long long>(1LL << 32, (long long)(fr / 8)))
                        : (1LL << 27);
  }
  return h->scr_budget;
}

long long ensure_dd_scratch(DevCtx* h, int ld) {
  const long long per = dd_scratch_per_wg(ld);
  const long long want = std::min<long long>(1024, std::max<long long>(1, scratch_budget(h) / per)) * per;
  if (h->ddscr_len < want) {
    if (h->d_ddscr) {
      (void)hipFree(h->d_ddscr);
      h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), (void*)h->d_ddscr));
      h->d_ddscr = nullptr;
    }
    h->ddscr_len = 0;
    if (dalloc(h, &h->d_ddscr, (size_t)want)) return 0;
    h->ddscr_len = want;
  }
  return std::min<long long>(1024, std::min(h->ddscr_len, want) / per);
}

// scratch of chol_wide_kernel for (nb, keep): workgroups per launch it holds
// (0: allocation failed); at most 4096 workgroups, <= 4 GB
long long ensure_wide_scratch(DevCtx* h, int nb, int keep) {
  const long long per = wide_scratch_per_wg(nb, keep);
  const long long want = std::min<long long>(4096, std::max<long long>(1, scratch_budget(h) / per)) * per;
  if (h->widescr_len < want) {
    if (h->d_widescr) {
      (void)hipFree(h->d_widescr);
      h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), (void*)h->d_widescr));
      h->d_widescr = nullptr;
    }
    h->widescr_len = 0;
    if (dalloc(h, &h->d_widescr, (size_t)want)) return 0;
    h->widescr_len = want;
  }
  return std::min<long long>(4096, std::min(h->widescr_len, want) / per);
}

int launch_wide(DevCtx* h, int nb, int keep, const CholJob* jobs, int B, long long u0, long long n, int b_off,
                const double* theta, int ldth, double* units, double* keep_out, hipStream_t st, int rev = 0,
                double* units_rev = nullptr) {
  if (nb > WIDE_NB_MAX) return set_err(EWH_E_UNSUPPORTED, "basis wider than 1023 columns");
  const long long cap = ensure_wide_scratch(h, nb, keep);
  if (cap <= 0 || (units_rev && cap < 2)) return EWH_E_NOMEM;
  return launch_chol_wide(jobs, B, u0, n, b_off, theta, ldth, units, h->d_widescr, wide_scratch_per_wg(nb, keep), cap,
                          keep, keep_out, 0, B, st, rev, units_rev, h->kernel_mode != MODE_WIDE_R05A);
}

template <typename T>
int ensure_buf(DevCtx* h, T** p, size_t* cap, size_t need) {
  if (need <= *cap) return 0;
  if (*p) {
    (void)hipFree(*p);
    h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), (void*)*p));
    *p = nullptr;
  }
  *cap = 0;
  int rc = dalloc(h, p, need);
  if (rc) return rc;
  *cap = need;
  return 0;
}

// The double-double path of units [u0, u0 + n) (dd_path): verify-and-refine
// by default, every unit under MODE_DD
int launch_dd_path(DevCtx* h, int nb, const CholJob* jobs, int B, long long u0, long long n, int b_off,
                   const double* theta, int ldth, double* units, hipStream_t st) {
  const long long cap = ensure_dd_scratch(h, 16 * nb);
  if (cap <= 0) return EWH_E_NOMEM;
  const long long per = dd_scratch_per_wg(16 * nb);
  int rc;
  if (!h->d_ddstat) {
    if ((rc = dalloc(h, &h->d_ddstat, 2))) return rc;
    EWH_HIP(hipMemsetAsync(h->d_ddstat, 0, 2 * sizeof(unsigned long long), st));
  }
  if (h->kernel_mode == MODE_DD) {
    if ((rc = launch_count_units(h->d_ddstat, n, st))) return rc;
    return launch_chol_dd(jobs, B, u0, n, b_off, theta, ldth, units, h->d_ddscr, per, cap, 16 * nb, st,
                          h->kernel_mode == MODE_WIDE_R05A);
  }
  const size_t U = (size_t)(h->P + (h->corr ? 1 : 0)) * B;
  if ((rc = ensure_buf(h, &h->d_units2, &h->units2_cap, U)) || (rc = ensure_buf(h, &h->d_ddlist, &h->ddlist_cap, U + 1)))
    return rc;
  // the forward and reversed fp64 passes: one launch (both in one grid) when
  // one pass alone would leave SIMD slots empty (chol_wide_kernel: two waves
  // per SIMD), else two -- past that point the doubled set of resident
  // scratch slots only adds memory traffic (measured, profiles/r05h: w372
  // near 2.91 -> 2.40 ms fused at 1024 units; the system model at 4096 units
  // 1.46 -> 1.75 ms fused); dev mode 34: always two (the round-5a form)
  const bool fuse = h->kernel_mode != MODE_WIDE_R05A && 2 * n <= 8LL * h->n_cu;
  if (!fuse) {
    if ((rc = launch_wide(h, nb, 0, jobs, B, u0, n, b_off, theta, ldth, units, nullptr, st, 0)) ||
        (rc = launch_wide(h, nb, 0, jobs, B, u0, n, b_off, theta, ldth, h->d_units2, nullptr, st, 1)))
      return rc;
  } else if ((rc = launch_wide(h, nb, 0, jobs, B, u0, n, b_off, theta, ldth, units, nullptr, st, 0, h->d_units2))) {
    return rc;
  }
  EWH_HIP(hipMemsetAsync(h->d_ddlist, 0, sizeof(int), st));
  if ((rc = launch_verify_units(units, h->d_units2, u0, n, h->d_ddlist + 1, h->d_ddlist, h->d_ddstat, st))) return rc;
  return launch_chol_dd_list(jobs, B, b_off, theta, ldth, units, h->d_ddscr, per, std::min<long long>(cap, n),
                             h->d_ddlist + 1, h->d_ddlist, 16 * nb, st, h->kernel_mode == MODE_WIDE_R05A);
}

// Round 6: an -inf unit term from an fp64 factorisation is a rounding failure
// wherever the exact Sigma is positive definite (every full-rank basis: T^T
// N^-1 T + diag(phi^-1)), so the units [u0, u0 + n) whose term is not finite
// are listed (verify_units_kernel on the terms alone) and refactored by
// chol_dd_kernel on a double-double matrix: the cached S_hi + S_lo (fixed
// white noise), or G_hi + G_lo of those samples from gram_dd_units_kernel
// (varying white noise: psr != NULL, the chunk's weights in h->d_w / d_beta).
// The -inf that remains is the double-double factorisation's (or a failed
// timing-model block, CholJob::fail).  Four launches per run, empty lists exit
// at once.  Not in the cross-check modes 1 / 27 (fp64 kernels compared as such).
bool refine_on(const DevCtx* h) {
  return !h->corr && !h->osmode && h->kernel_mode != 1 && h->kernel_mode != MODE_WIDE;
}

int refine_failed(DevCtx* h, const CholJob* jobs, int nb, int B, long long u0, long long n, int b_off,
                  const double* theta, int ldth, double* units, hipStream_t st, const PsrHost* psr) {
  if (n <= 0) return 0;
  const long long cap = ensure_dd_scratch(h, 16 * nb);
  if (cap <= 0) return EWH_E_NOMEM;
  int rc;
  if (!h->d_ddstat) {
    if ((rc = dalloc(h, &h->d_ddstat, 2))) return rc;
    EWH_HIP(hipMemsetAsync(h->d_ddstat, 0, 2 * sizeof(unsigned long long), st));
  }
  const size_t U = (size_t)(h->P + (h->corr ? 1 : 0)) * B;
  if ((rc = ensure_buf(h, &h->d_ddlist, &h->ddlist_cap, U + 1))) return rc;
  EWH_HIP(hipMemsetAsync(h->d_ddlist, 0, sizeof(int), st));
  // (kernel mode 29: every unit listed -- the double-double twin of the fp64
  // routes; a basis on the double-double path was factored so already, and
  // only its -inf units are refined here)
  const bool all = h->kernel_mode == MODE_DD && !dd_path(h, nb, psr == nullptr);
  if ((rc = launch_verify_units(units, units, u0, n, h->d_ddlist + 1, h->d_ddlist, h->d_ddstat, st, all)))
    return rc;
  if (psr) {
    const int nbk = psr->nb * (psr->nb + 1) / 2;
    const unsigned slots = (unsigned)std::min<long long>(n, 64);
    hipLaunchKernelGGL(gram_dd_units_kernel, dim3(nbk, slots), dim3(256), 0, st, psr->dev, psr->d_Tlo, h->d_w, h->d_beta,
                       h->d_ddlist + 1, h->d_ddlist, B, b_off, h->d_G, h->d_Glo);
    EWH_HIP(hipGetLastError());
  }
  return launch_chol_dd_list(jobs, B, b_off, theta, ldth, units, h->d_ddscr, dd_scratch_per_wg(16 * nb),
                             std::min<long long>(cap, n), h->d_ddlist + 1, h->d_ddlist, 16 * nb, st, false);
}

// the partial factorisation (correlated common process) of units [u0, u0 + n)
// of one run of pulsars with nb blocks: the register kernel where it fits
// (chol_mfma_kernel<NB <= 9, KEEP>, phase split permitting), else chol_wide
int partial_units(DevCtx* h, const CholJob* jobs, int nb, int B, long long u0, long long n, int b_off,
                  const double* theta, double* units, double* keep_out, hipStream_t st) {
  const bool regs = nb <= MFMA_NB_MAX && nb - h->keep >= (nb == 8 ? 3 : nb / 2);
  if (regs && h->kernel_mode != MODE_WIDE)
    return launch_partial_nb(nb, h->keep, jobs, B, u0, n, b_off, theta, h->n_param, units, keep_out, B, st);
  return launch_wide(h, nb, h->keep, jobs, B, u0, n, b_off, theta, h->n_param, units, keep_out, st);
}

int dispatch_chol(DevCtx* h, int nb, int mreal, const CholJob* jobs, int B, long long u0, long long n, int b_off,
                  const double* theta, int ldth, double* units, hipStream_t st, bool fixed) {
  if (n <= 0) return 0;
  const int mode = h->kernel_mode;
  if (dd_path(h, nb, fixed)) return launch_dd_path(h, nb, jobs, B, u0, n, b_off, theta, ldth, units, st);
  if (mode == MODE_WIDE || nb > BIG_NB_MAX)
    return launch_wide(h, nb, 0, jobs, B, u0, n, b_off, theta, ldth, units, nullptr, st);
  double* bigscr = h->d_bigscr;
  const long long bigcap = h->bigscr_cap;
  if (mode != 1 && nb > MFMA_NB_MAX && nb <= BIG_NB_MAX && bigscr)
    return launch_chol_big_nb(nb, jobs, B, u0, n, b_off, theta, ldth, units, bigscr, bigcap, st);
  if (mode != 1 && nb <= MFMA_NB_MAX) {
    const int rc = launch_chol_small(mode, nb, jobs, B, u0, n, b_off, theta, ldth, units, st);
    if (rc <= 0) return rc;
  }
  const size_t lds = lds_bytes_chol(mreal);
  if (lds > LDS_MAX - 64) return set_err(EWH_E_UNSUPPORTED, "reduced matrix too large for the LDS Cholesky kernel");
  // (the dynamic-LDS attribute of chol_lds_kernel is set per device in create_ctx)
  hipLaunchKernelGGL(chol_lds_kernel, dim3((unsigned)n), dim3(256), lds, st, jobs, B, u0, b_off, theta, ldth, units);
  return 0;
}

// scratch of chol_big_kernel for NB: BIG_SLOTS workgroups x NB(NB+1)/2 blocks of 2 KiB
constexpr long long BIG_SLOTS = 2048;
int ensure_big_scratch(DevCtx* h, int nb) {
  if (nb <= MFMA_NB_MAX || nb > BIG_NB_MAX || nb <= h->bigscr_nb) return 0;
  if (h->d_bigscr) {
    (void)hipFree(h->d_bigscr);
    h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), (void*)h->d_bigscr));
    h->d_bigscr = nullptr;
  }
  int rc = dalloc(h, &h->d_bigscr, (size_t)BIG_SLOTS * (nb * (nb + 1) / 2) * 256);
  if (rc) return rc;
  h->bigscr_cap = BIG_SLOTS;
  h->bigscr_nb = nb;
  return 0;
}

int ensure_units(DevCtx* h, int B) {
  const size_t need = (size_t)(h->P + (h->corr ? 1 : 0)) * B;   // + the common term row
  if (need <= h->units_cap) return 0;
  if (h->d_units) {
    (void)hipFree(h->d_units);
    h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), (void*)h->d_units));
  }
  h->units_cap = 0;
  int rc = dalloc(h, &h->d_units, need);
  if (rc) return rc;
  h->units_cap = need;
  return 0;
}

int ensure_var_scratch(DevCtx* h, int B) {
  if (h->white_fixed) return 0;
  // reuse while the chunk covers the batch or already sits at its cap (the
  // memory-derived limit, at most 1024): no free / re-malloc per call
  if (h->chunk > 0 && (h->chunk >= B || h->chunk >= h->chunk_cap)) return 0;
  for (void* p : {(void*)h->d_w, (void*)h->d_beta, (void*)h->d_s, (void*)h->d_G, (void*)h->d_Kb, (void*)h->d_fac,
                  (void*)h->d_rho,
                  (void*)h->d_Glo}) {
    if (p) {
      (void)hipFree(p);
      h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), p));
    }
  }
  size_t maxn = 1, maxe = 1, maxld = 16, maxfac = 1;
  for (auto& ps : h->psr) {
    maxn = std::max(maxn, (size_t)ps.n_toa);
    maxe = std::max(maxe, (size_t)ps.n_epoch);
    maxld = std::max(maxld, (size_t)ps.ld);
    maxfac = std::max(maxfac, (size_t)ps.n_toa * ps.dev.n_bgroup);
  }
  // chunk: keep G (ld^2) and s (E*ld) scratch under ~1.5 GB (8 GB for wide bases)
  // epoch-sum rows per sample: whole CT_ROWS tiles (+1) so the pipelined
  // contraction's last epoch tile reads zero-initialised pad rows
  const size_t sstride = ((maxe + CT_ROWS - 1) / CT_ROWS + 1) * CT_ROWS * maxld;
  const bool wide = maxld > 16 * BIG_NB_MAX;
  // G_lo for the double-double factorisation: of every unit past 16 blocks,
  // and (round 6) of the units whose fp64 factorisation fails (refine_failed)
  const size_t per = (2 * maxld * maxld + sstride + maxn + maxe + maxfac + 1) * sizeof(double);
  // (bases past 16 blocks: 8 GB of the 288 GB HBM, so a batch of up to 1024
  // samples is one chunk -- one GEMM-form contraction over all of it and one
  // factorisation launch with 4 units per CU instead of 4 launches of 256
  // one-wave units)
  const size_t budget = (wide ? (size_t)8192 : (size_t)1536) * 1024 * 1024;
  size_t cap = std::min<size_t>(1024, std::max<size_t>(1, budget / per));
  // whole rounds of workgroups over the 256 CUs (a chunk of 853 samples of
  // C2 ran 2 rounds of 512 workgroups, the second two-thirds empty)
  if (cap > 256) cap -= cap % 256;
  h->chunk_cap = (int)cap;
  const size_t chunk = std::min<size_t>(cap, (size_t)std::max(B, 1));
  int rc;
  if ((rc = dalloc(h, &h->d_w, chunk * maxn))) return rc;
  if ((rc = dalloc(h, &h->d_beta, chunk * maxe))) return rc;
  if ((rc = dalloc(h, &h->d_s, chunk * sstride))) return rc;
  EWH_HIP(hipMemset(h->d_s, 0, chunk * sstride * sizeof(double)));
  h->s_stride = (long long)sstride;
  if ((rc = dalloc(h, &h->d_G, chunk * maxld * maxld))) return rc;
  if ((rc = dalloc(h, &h->d_Kb, chunk))) return rc;
  if ((rc = dalloc(h, &h->d_rho, chunk))) return rc;
  if ((rc = dalloc(h, &h->d_fac, chunk * maxfac))) return rc;
  h->d_Glo = nullptr;
  if ((rc = dalloc(h, &h->d_Glo, chunk * maxld * maxld))) return rc;
  h->chunk = (int)chunk;
  std::vector<CholJob> jobs(h->P);
  for (int p = 0; p < h->P; ++p) {
    const PsrHost& ps = h->psr[p];
    // (correlated: the columns before the common block take phi^-1; the
    // common block is assembled globally)
    const int mreal = h->corr ? ps.gstart_v : ps.m;
    jobs[p] = CholJob{h->d_G, (long long)ps.ld * ps.ld, ps.ld, mreal, ps.d_colptr, ps.d_spec, h->d_Kb, 1, 0};
    jobs[p].mats_lo = h->d_Glo;
  }
  EWH_HIP(hipMemcpy(h->d_jobs_var, jobs.data(), sizeof(CholJob) * h->P, hipMemcpyHostToDevice));
  return 0;
}

// white-noise terms of one pulsar for samples [b0, b0 + nb) into the chunk scratch
int run_white(DevCtx* h, int p, const double* theta, int ldth, int b0, int nb) {
  PsrHost& ps = h->psr[p];
  const bool c2 = ps.dev.n_bgroup == 0 && h->kernel_mode != 7 && ps.nb <= CONTRACT2_NB_MAX;
  // the r-separated contraction (contract2 RSEP): when the residual alone
  // fills the last 16-column block (m <= 16 (NB - 1): C4's 192 columns + r
  // = 13 blocks), the MFMAs form only the NB - 1 block Gram; d = T^T W r by
  // VALU from the staged tiles, r^T W r in wn_weights_kernel.  No ECORR
  // (the epoch pass would need the same split).  Dev mode 36: off (A/B)
  const bool rsep = c2 && ps.dev.n_epoch == 0 && ps.nb >= 2 && ps.dev.m <= 16 * (ps.nb - 1) &&
                    h->kernel_mode != 36 && h->kernel_mode != 30 &&
                    h->kernel_mode != 38 && h->kernel_mode != 39;
  hipLaunchKernelGGL(wn_weights_kernel, dim3(nb), dim3(256), 0, h->stream, ps.dev, theta, ldth, b0, h->d_w,
                     h->d_beta, h->d_Kb, h->d_fac, rsep ? h->d_rho : nullptr);
  if (c2) {
    // (dev library A/B: mode 15 = 4 waves per sample, mode 16 = 8)
    // (30: TwoSum accumulation up to 10 blocks)
    // (35: the run remainder on the first waves, as in round 4-5a)
    // (38 / 39: blocked accumulation up to 10 blocks, 4 / 8 waves)
    const int waves = h->kernel_mode == 15 ? 4 : h->kernel_mode == 16 ? 8 : h->kernel_mode == 30 ? 30
                    : h->kernel_mode == 35 ? 35 : h->kernel_mode == 38 ? 38 : h->kernel_mode == 39 ? 39 : 0;
    int rc = launch_contract2_nb(ps.nb, waves, ps.dev, h->d_w, h->d_beta, h->d_s, h->s_stride, h->d_G, nb, h->stream,
                                 rsep ? h->d_rho : nullptr);
    if (rc) return rc;
    EWH_HIP(hipGetLastError());
    return 0;
  }
  if (ps.n_epoch > 0) {
    // (dev mode 37: one sample per workgroup, as in round 5a)
    if (ps.dev.n_bgroup == 0 && ps.max_epoch <= ES_RMAX && h->kernel_mode != 37)
      hipLaunchKernelGGL(epoch_sums_multi_kernel, dim3(ps.n_epoch, (nb + ES_S - 1) / ES_S), dim3(256), 0, h->stream,
                         ps.dev, h->d_w, nb, h->d_s);
    else
      hipLaunchKernelGGL(epoch_sums_kernel, dim3(ps.n_epoch, nb), dim3(256), 0, h->stream, ps.dev, h->d_w, h->d_fac,
                         h->d_s);
  }
  int rc = launch_contract_nb(ps.nb, ps.dev, h->d_w, h->d_beta, h->d_s, h->d_fac, h->d_G, nb, h->stream,
                              ps.nb > BIG_NB_MAX ? h->d_Glo : nullptr);
  if (rc) return rc;
  EWH_HIP(hipGetLastError());
  return 0;
}

// Temporary device buffers of a one-off setup step (freed on scope exit).
struct TmpBufs {
  std::vector<void*> p;
  template <typename T>
  int get(T** out, size_t count) {
    *out = nullptr;
    hipError_t e = hipMalloc((void**)out, std::max<size_t>(1, count) * sizeof(T));
    if (e != hipSuccess) return set_err(EWH_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    p.push_back(*out);
    return 0;
  }
  ~TmpBufs() {
    for (void* q : p) (void)hipFree(q);
  }
};

// Fixed white noise: G = T_aug^T N^-1 T_aug of every pulsar at the constant
// white-noise values, then the timing-model elimination (schur_kernel) into
// the cached reduced matrix S_p and constant K_p.  Called by create and again
// by ewh_set_fixed_white (new constants, same layout: buffers are reused).
int setup_fixed(DevCtx* h) {
  int rc;
  size_t maxn = 1, maxe = 1, maxld = 16;
  for (auto& ps : h->psr) {
    maxn = std::max(maxn, (size_t)ps.n_toa);
    maxe = std::max(maxe, (size_t)ps.n_epoch);
    maxld = std::max(maxld, (size_t)ps.ld);
  }
  TmpBufs tmp;
  double *w, *beta, *s, *G, *Glo, *Kb, *dummy_theta;
  if ((rc = tmp.get(&w, maxn)) || (rc = tmp.get(&beta, maxe)) || (rc = tmp.get(&s, maxe * maxld)) ||
      (rc = tmp.get(&G, maxld * maxld)) || (rc = tmp.get(&Glo, maxld * maxld)) || (rc = tmp.get(&Kb, 1)) ||
      (rc = tmp.get(&dummy_theta, std::max(1, h->n_param))))
    return rc;
  // theta is never read (every white-noise slot is constant)
  EWH_HIP(hipMemsetAsync(dummy_theta, 0, sizeof(double) * std::max(1, h->n_param), h->stream));
  if (!h->d_fxK && (rc = dalloc(h, &h->d_fxK, h->P))) return rc;
  if (!h->d_fxfail && (rc = dalloc(h, &h->d_fxfail, h->P))) return rc;
  std::vector<CholJob> jobs(h->P);
  std::vector<int> fails(h->P, 0);
  for (int p = 0; p < h->P; ++p) {
    PsrHost& ps = h->psr[p];
    hipLaunchKernelGGL(wn_weights_kernel, dim3(1), dim3(256), 0, h->stream, ps.dev, dummy_theta, 0, 0, w, beta, Kb,
                       nullptr, nullptr);
    if (ps.n_epoch > 0)
      hipLaunchKernelGGL(epoch_sums_kernel, dim3(ps.n_epoch, 1), dim3(256), 0, h->stream, ps.dev, w, nullptr, s);
    if (ps.dev.n_bgroup == 0 && h->kernel_mode != 7) {
      // (the exactly projected basis: T_aug + its projection residual d_Tlo;
      // the epoch sums formed inside from both)
      hipLaunchKernelGGL(gram_dd_kernel, dim3(ps.nb * (ps.nb + 1) / 2), dim3(256), 0, h->stream, ps.dev, ps.d_Tlo, w,
                         beta, G, Glo);
      EWH_HIP(hipGetLastError());
    } else {
      EWH_HIP(hipMemsetAsync(Glo, 0, sizeof(double) * (size_t)ps.ld * ps.ld, h->stream));
      if ((rc = launch_contract_nb(ps.nb, ps.dev, w, beta, s, nullptr, G, 1, h->stream))) return rc;
    }
    double Kb_h = 0.0;
    EWH_HIP(hipMemcpyAsync(&Kb_h, Kb, sizeof(double), hipMemcpyDeviceToHost, h->stream));
    EWH_HIP(hipStreamSynchronize(h->stream));
    if (!ps.d_S && (rc = dalloc(h, &ps.d_S, (size_t)ps.fx_ld * ps.fx_ld))) return rc;
    // the low part of S for the double-double factorisation: bases past the
    // register kernels (dd_path), and (round 6) every unit whose fp64
    // factorisation fails (refine_failed)
    if (!ps.d_Slo && (rc = dalloc(h, &ps.d_Slo, (size_t)ps.fx_ld * ps.fx_ld))) return rc;
    if (ps.d_Slo && !ps.d_Srev && (rc = dalloc(h, &ps.d_Srev, (size_t)ps.fx_ld * ps.fx_ld))) return rc;
    hipLaunchKernelGGL(schur_kernel, dim3(1), dim3(256), 0, h->stream, G, Glo, ps.ld, ps.m, ps.nlead, ps.d_colptr,
                       ps.d_spec, Kb_h, ps.d_S, ps.fx_ld, ps.nloc, ps.gstart, ps.ncommon, h->d_fxK + p,
                       h->d_fxfail + p, ps.d_Slo);
    EWH_HIP(hipGetLastError());
    // mreal: columns that take phi^-1 in the factorisation -- the own columns
    // (correlated: the common block is assembled globally), or every column
    // with entries (optimal statistic: the CURN Sigma of each pulsar)
    const int mreal = h->osmode ? ps.fx_ld - 1 : ps.nloc;
    jobs[p] = CholJob{ps.d_S, 0, ps.fx_ld, mreal, ps.d_fx_colptr, ps.d_fx_spec, h->d_fxK + p, 0, 0,
                      ps.d_fx_rep, ps.d_fx_ulist, ps.fx_nu, h->stage_spectra ? ps.d_fx_urec : nullptr, ps.d_fx_urep};
    jobs[p].mats_lo = ps.d_Slo;
    if (ps.d_Slo) {          // the reversed verify pass's input, once (chol_wide.hip)
      const long long ne = (long long)ps.fx_ld * ps.fx_ld;
      hipLaunchKernelGGL(rev_input_kernel, dim3((unsigned)((ne + 255) / 256)), dim3(256), 0, h->stream, ps.d_S, ps.d_Slo,
                         ps.d_Srev, ne);
      EWH_HIP(hipGetLastError());
      jobs[p].mats_rev = ps.d_Srev;
    }
    if (jobs[p].urec != nullptr) {
      jobs[p].ntidx = (int)ps.fx_tidx.size();
      for (int i = 0; i < jobs[p].ntidx; ++i) jobs[p].tidx[i] = ps.fx_tidx[i];
    }
  }
  EWH_HIP(hipMemcpyAsync(fails.data(), h->d_fxfail, sizeof(int) * h->P, hipMemcpyDeviceToHost, h->stream));
  EWH_HIP(hipStreamSynchronize(h->stream));
  for (int p = 0; p < h->P; ++p) jobs[p].fail = fails[p];
  EWH_HIP(hipMemcpy(h->d_jobs_fixed, jobs.data(), sizeof(CholJob) * h->P, hipMemcpyHostToDevice));
  return 0;
}

int setup_common(DevCtx* h, const ewh_pta_desc* d) {
  const ewh_common_desc& c = *d->common;
  const int P = h->P;
  h->corr = true;
  h->nc = c.n_col;
  h->keep = (c.n_col + 1 + 15) / 16;
  for (auto& ps : h->psr) {
    const int nbk = h->white_fixed ? ps.fx_nb : ps.nb;
    const int gs = h->white_fixed ? ps.gstart : ps.gstart_v;
    if (nbk - gs / 16 != h->keep) return set_err(EWH_E_INVALID, "common: inconsistent reduced layout");
    if (nbk > WIDE_NB_MAX) return set_err(EWH_E_UNSUPPORTED, "common: basis wider than 1023 columns");
  }
  int rc;
  if ((rc = dupload(h, &h->d_orf, c.orf, (size_t)P * P))) return rc;
  // per pulsar: the CSR whose positions gstart.. hold the common columns'
  // own entries (fixed white noise: the reduced layout; varying: T_aug's)
  auto common_psr = [&](int p) {
    const PsrHost& ps = h->psr[p];
    return h->white_fixed ? CommonPsr{ps.d_fx_colptr, ps.d_fx_spec, ps.gstart, 0}
                          : CommonPsr{ps.d_colptr, ps.d_spec, ps.gstart_v, 0};
  };
  if (h->osmode) {               // optimal statistic: the CURN likelihood layout + the ORF only
    h->corr = false;
    std::vector<CommonPsr> cps(P);
    for (int p = 0; p < P; ++p) cps[p] = common_psr(p);
    return dupload(h, &h->d_cps, cps.data(), cps.size());
  }
  std::vector<DSpec> cs(c.n_col);
  for (int g = 0; g < c.n_col; ++g) cs[g] = to_dspec(c.spec[g], g);
  if ((rc = dupload(h, &h->d_cspec, cs.data(), cs.size()))) return rc;
  // columns whose M_g is identical (the sin / cos pair of a frequency: same
  // common spectrum, same own spectra in every pulsar) share one inverse
  auto same_ent = [](const ewh_spec_entry& x, const ewh_spec_entry& y) {
    auto pr = [](const ewh_pref& a, const ewh_pref& b) { return a.idx == b.idx && a.cval == b.cval; };
    return x.kind == y.kind && pr(x.p0, y.p0) && pr(x.p1, y.p1) && pr(x.p2, y.p2) && x.f == y.f && x.df == y.df &&
           x.fyr == y.fyr;
  };
  auto own_entries = [&](int p, int g) {
    const ewh_pulsar_desc& sd = d->pulsars[p];
    const int col = sd.n_col - sd.n_common + g;
    std::vector<ewh_spec_entry> v;
    for (int e = 0; e < sd.n_spec; ++e)
      if (sd.spec[e].col == col) v.push_back(sd.spec[e]);
    return v;
  };
  std::vector<int> uniq, rep(c.n_col);
  for (int g = 0; g < c.n_col; ++g) {
    int found = -1;
    for (size_t u = 0; u < uniq.size() && found < 0; ++u) {
      const int g2 = uniq[u];
      bool eq = same_ent(c.spec[g], c.spec[g2]);
      for (int p = 0; p < P && eq; ++p) {
        const auto a = own_entries(p, g), b = own_entries(p, g2);
        eq = a.size() == b.size();
        for (size_t k = 0; k < a.size() && eq; ++k) eq = same_ent(a[k], b[k]);
      }
      if (eq) found = (int)u;
    }
    if (found < 0) {
      found = (int)uniq.size();
      uniq.push_back(g);
    }
    rep[g] = found;
  }
  h->nuniq = (int)uniq.size();
  if ((rc = dupload(h, &h->d_cuniq, uniq.data(), uniq.size()))) return rc;
  if ((rc = dupload(h, &h->d_crep, rep.data(), rep.size()))) return rc;
  std::vector<CommonPsr> cps(P);
  for (int p = 0; p < P; ++p) cps[p] = common_psr(p);
  if ((rc = dupload(h, &h->d_cps, cps.data(), cps.size()))) return rc;
  h->Np = DCB * ((P * h->nc + 1 + DCB - 1) / DCB);
  // the dense kernels address a sample's Sigma_c by 32-bit byte offsets
  // (dchol_rowpair_kernel, dchol_rowupdate2_kernel): < 4 GB per sample
  if ((double)h->Np * h->Np * 8.0 >= 4294967296.0)
    return set_err(EWH_E_UNSUPPORTED, "correlated common process: Sigma_c of " + std::to_string(h->Np) +
                                          " columns exceeds 4 GB per sample (P x common columns <= 23168)");
  const double per = (double)h->Np * h->Np * 8.0;
  h->cchunk_cap = (int)std::max(1.0, std::min(1024.0, 40.0e9 / per));   // <= 40 GB of dense Sigma_c per chunk
  h->cchunk = 0;              // the chunk scratch is allocated on first use, sized to the batch
  const size_t lds = ((size_t)P * (P + 1) + 3 * P) * sizeof(double);
  EWH_HIP(hipFuncSetAttribute((const void*)common_minv_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  return 0;
}

// per-chunk scratch of the dense cross-pulsar factorisation, sized to
// min(B, cap) on first use and grown (up to the cap) when a larger batch comes
int ensure_common_scratch(DevCtx* h, int B) {
  const int want = std::min(std::max(B, 1), h->cchunk_cap);
  if (h->cchunk >= want) return 0;
  for (void* p : {(void*)h->d_minv, (void*)h->d_mlog, (void*)h->d_dense, (void*)h->d_wbuf, (void*)h->d_cldet,
                  (void*)h->d_cq, (void*)h->d_cfail}) {
    if (p) {
      (void)hipFree(p);
      h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), p));
    }
  }
  h->cchunk = 0;
  const size_t Bc = want, P = h->P;
  int rc;
  if ((rc = dalloc(h, &h->d_minv, Bc * h->nc * P * P)) || (rc = dalloc(h, &h->d_mlog, Bc * h->nc)) ||
      (rc = dalloc(h, &h->d_dense, Bc * h->Np * h->Np)) || (rc = dalloc(h, &h->d_wbuf, Bc * DCB * DCB)) ||
      (rc = dalloc(h, &h->d_cldet, Bc)) || (rc = dalloc(h, &h->d_cq, Bc)) || (rc = dalloc(h, &h->d_cfail, Bc)))
    return rc;
  h->cchunk = want;
  return 0;
}

int ensure_keep(DevCtx* h, int B) {
  const int KD = 16 * h->keep;
  int rc;
  const size_t need = (size_t)B * h->P * KD * KD;
  if (need > h->keep_cap) {
    if (h->d_keep) {
      (void)hipFree(h->d_keep);
      h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), (void*)h->d_keep));
      h->d_keep = nullptr;
    }
    h->keep_cap = 0;
    if ((rc = dalloc(h, &h->d_keep, need))) return rc;
    h->keep_cap = need;
  }
  return 0;
}

// Step 1 of a correlated batch for pulsars [p_begin, p_end): the partial
// factorisations (own columns eliminated), writing each unit's local term to
// units[p B + b] and its kept common block to keep (pulsar-major, B samples
// per pulsar).
int corr_partial(DevCtx* h, const double* theta_dev, int B, int p_begin, int p_end, double* units, double* keep,
                 hipStream_t st) {
  int rc;
  if (!h->white_fixed) {
    // white noise varying: per pulsar and sample chunk the contraction
    // (run_white: N^-1, ECORR, G = T_aug^T N^-1 T_aug on h->stream) and the
    // partial factorisation of G + diag(phi^-1) with the timing model in
    if ((rc = ensure_var_scratch(h, B))) return rc;
    hipStream_t saved = h->stream;
    h->stream = st;
    for (int p = p_begin; p < p_end && !rc; ++p)
      for (int c0 = 0; c0 < B && !rc; c0 += h->chunk) {
        const int nb = std::min(h->chunk, B - c0);
        rc = run_white(h, p, theta_dev, h->n_param, c0, nb);
        if (!rc)
          rc = partial_units(h, h->d_jobs_var, h->psr[p].nb, B, (long long)p * B + c0, nb, c0, theta_dev, units, keep,
                             st);
      }
    h->stream = saved;
    return rc;
  }
  for (long long u = (long long)p_begin * B; u < (long long)p_end * B;) {
    const int p0 = (int)(u / B);
    const int nb0 = h->psr[p0].fx_nb;
    int p1 = p0 + 1;
    while (p1 < p_end && h->psr[p1].fx_nb == nb0) ++p1;
    const long long seg_end = (long long)p1 * B;
    if ((rc = partial_units(h, h->d_jobs_fixed, nb0, B, u, seg_end - u, 0, theta_dev, units, keep, st))) return rc;
    u = seg_end;
  }
  return 0;
}

// Step 2, once every pulsar's kept block is in `keep`: per sample chunk the
// M_g inverses, the dense Sigma_c assembly and factorisation; the global term
// of sample b goes to units[P B + b].
// the M_g inverses and log-determinants of samples [c0, c0 + nb)
void launch_minv(DevCtx* h, const double* theta_dev, int c0, int nb, hipStream_t st) {
  const int P = h->P, ldth = h->n_param;
  const size_t lds = ((size_t)P * (P + 1) + 3 * P) * sizeof(double);
  if (P <= MINV_PMAX && h->kernel_mode != 7)
    hipLaunchKernelGGL(common_minv_reg_kernel, dim3(h->nuniq, nb), dim3(512), 0, st, h->d_cps, P, h->d_orf,
                       h->d_cspec, h->nc, h->d_cuniq, theta_dev, ldth, c0, h->d_minv, h->d_mlog);
  else
    hipLaunchKernelGGL(common_minv_kernel, dim3(h->nuniq, nb), dim3(256), lds, st, h->d_cps, P, h->d_orf,
                       h->d_cspec, h->nc, h->d_cuniq, theta_dev, ldth, c0, h->d_minv, h->d_mlog);
}

// first_minv_done: the M_g inverses of the first chunk are already in
// d_minv (lnl_correlated ran them beside the partial factorisations)
int corr_finish(DevCtx* h, const double* theta_dev, int B, const double* keep, double* units, hipStream_t st,
                bool first_minv_done = false) {
  const int P = h->P, KD = 16 * h->keep;
  int rc;
  if ((rc = ensure_common_scratch(h, B))) return rc;
  const int nbk = h->Np / DCB;
  for (int c0 = 0; c0 < B; c0 += h->cchunk) {
    const int nb = std::min(h->cchunk, B - c0);
    if (!(first_minv_done && c0 == 0)) launch_minv(h, theta_dev, c0, nb, st);
    hipLaunchKernelGGL(common_assemble_kernel, dim3((h->Np + 3) / 4, nb), dim3(256), 0, st, keep, KD, P, h->nc,
                       (long long)B, c0, h->d_minv, h->d_crep, h->Np, h->d_dense, h->d_cldet, h->d_cq, h->d_cfail);
    // one or a few proposals (PTMCMC): right-looking -- after each panel the
    // trailing tiles (i, j > k) are updated in parallel (m (m + 1) / 2 tiles
    // per launch, K = 64), instead of the left-looking row update whose
    // K = 64 k accumulation of one tile is a serial chain on one CU.  Tile
    // (i, j) takes the same K = 64 slabs in the same order into the same
    // accumulator (stored and reloaded in full between panels): bit-identical.
    const bool right = (h->kernel_mode == 0 || h->kernel_mode == 33) && nb <= CORR_RIGHT_LOOKING_MAX;
    for (int k = 0; k < nbk; ++k) {
      const int m = nbk - k - 1;
      if (right) {
        // the diagonal block k + 1 is factored inside the update launch of
        // step k (dchol_update_diag_kernel); dev mode 33 launches it apart
        const bool fuse_diag = h->kernel_mode != 33;
        if (k == 0 || !fuse_diag) {
          if (m == 0)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(dchol_diag_reg_kernel<true>), dim3(nb), dim3(64), 0, st, h->d_dense,
                               h->Np, k, h->d_wbuf, h->d_cldet, h->d_cq, h->d_cfail);
          else
            hipLaunchKernelGGL(HIP_KERNEL_NAME(dchol_diag_reg_kernel<false>), dim3(nb), dim3(64), 0, st, h->d_dense,
                               h->Np, k, h->d_wbuf, h->d_cldet, h->d_cq, h->d_cfail);
        }
        if (m == 0) continue;
        hipLaunchKernelGGL(dchol_panel_reg_kernel, dim3(4 * m, nb), dim3(64), 0, st, h->d_dense, h->Np, k, h->d_wbuf);
        if (!fuse_diag)
          hipLaunchKernelGGL(dchol_update_kernel, dim3(m * (m + 1) / 2, nb), dim3(256), 0, st, h->d_dense, h->Np, k);
        else if (m == 1)   // block k + 1 is the last one (its pivot q_c)
          hipLaunchKernelGGL(HIP_KERNEL_NAME(dchol_update_diag_kernel<true>), dim3(1, nb), dim3(256), 0, st,
                             h->d_dense, h->Np, k, h->d_wbuf, h->d_cldet, h->d_cq, h->d_cfail);
        else
          hipLaunchKernelGGL(HIP_KERNEL_NAME(dchol_update_diag_kernel<false>), dim3(m * (m + 1) / 2, nb), dim3(256),
                             0, st, h->d_dense, h->Np, k, h->d_wbuf, h->d_cldet, h->d_cq, h->d_cfail);
        continue;
      }
      // default for large sample chunks: row update + panel fused (the updated
      // tile never round-trips through HBM); small chunks keep the row update
      // of every tile in one launch, which shortens the dependent chain per
      // block row
      const bool fused = h->kernel_mode != 1 && h->kernel_mode != 7 && nb >= 64;
      // two block rows per update pass (dchol_rowpair_kernel) for the large
      // chunks: at an even k with a row k + 1 following, the rows p < k of
      // both rows' tiles j > k first; row k + 1 then takes only p = k
      const bool pairs = fused && h->kernel_mode != 28 && h->kernel_mode != 31;
      int p0 = 0;                                       // the first row p this block row still needs
      if (pairs && (k & 1)) p0 = k - 1;
      const bool pair_here = pairs && !(k & 1) && m > 0 && k > 0;
      if (h->kernel_mode == 1 && k > 0)     // round-1 row update (both operands staged through LDS)
        hipLaunchKernelGGL(dchol_rowupdate_kernel, dim3(m + 1, nb), dim3(256), 0, st, h->d_dense, h->Np, k);
      else if (k > 0 && h->kernel_mode != 7)   // the diagonal tile's row update only (fused), or the whole row
        hipLaunchKernelGGL(dchol_rowupdate2_kernel, dim3(fused ? 1 : m + 1, nb), dim3(256), 0, st, h->d_dense, h->Np,
                           k, p0);

      if (h->kernel_mode == 7 || h->kernel_mode == 1) {   // A/B: round-1 LDS diagonal block + LDS-staged panel
        hipLaunchKernelGGL(dchol_diag_kernel, dim3(nb), dim3(256), 0, st, h->d_dense, h->Np, k, h->d_wbuf,
                           h->d_cldet, h->d_cq, h->d_cfail);
        if (m > 0)
          hipLaunchKernelGGL(dchol_panel_kernel, dim3(m, nb), dim3(256), 0, st, h->d_dense, h->Np, k, h->d_wbuf);
      } else {
        if (m > 0)
          hipLaunchKernelGGL(HIP_KERNEL_NAME(dchol_diag_reg_kernel<false>), dim3(nb), dim3(64), 0, st, h->d_dense,
                             h->Np, k, h->d_wbuf, h->d_cldet, h->d_cq, h->d_cfail);
        else
          hipLaunchKernelGGL(HIP_KERNEL_NAME(dchol_diag_reg_kernel<true>), dim3(nb), dim3(64), 0, st, h->d_dense,
                             h->Np, k, h->d_wbuf, h->d_cldet, h->d_cq, h->d_cfail);
        if (m > 0 && fused)
        {
          if (h->kernel_mode == 28)   // (dev A/B: one tile per workgroup, one row per pass: the round-3 form)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(dchol_rowpanel_kernel<1>), dim3(m, nb), dim3(256), 0, st, h->d_dense,
                               h->Np, k, 0, h->d_wbuf);
          else if (pair_here && h->kernel_mode == 32)   // (dev A/B: U_pj loaded at the top of each step)
            hipLaunchKernelGGL(HIP_KERNEL_NAME(dchol_rowpair_kernel<false>), dim3(m, nb), dim3(512), 0, st,
                               h->d_dense, h->Np, k, h->d_wbuf);
          else if (pair_here)         // rows k and k + 1 over p < k, row k's panel
            hipLaunchKernelGGL(HIP_KERNEL_NAME(dchol_rowpair_kernel<true>), dim3(m, nb), dim3(512), 0, st,
                               h->d_dense, h->Np, k, h->d_wbuf);
          else
            hipLaunchKernelGGL(HIP_KERNEL_NAME(dchol_rowpanel_kernel<2>), dim3((m + 1) / 2, nb), dim3(512), 0, st,
                               h->d_dense, h->Np, k, p0, h->d_wbuf);
        }
        else if (m > 0)
          hipLaunchKernelGGL(dchol_panel_reg_kernel, dim3(4 * m, nb), dim3(64), 0, st, h->d_dense, h->Np, k,
                             h->d_wbuf);
      }
      if (m > 0 && h->kernel_mode == 7)   // A/B: right-looking trailing update
        hipLaunchKernelGGL(dchol_update_kernel, dim3(m * (m + 1) / 2, nb), dim3(256), 0, st, h->d_dense, h->Np, k);
    }
    hipLaunchKernelGGL(common_final_kernel, dim3((nb + 255) / 256), dim3(256), 0, st, h->d_cldet, h->d_cq,
                       h->d_cfail, h->d_mlog, h->d_crep, h->nc, nb, c0, P, B, units);
    EWH_HIP(hipGetLastError());
  }
  return 0;
}

// correlated batch on one device: step 1 for every pulsar, then step 2
int lnl_correlated(DevCtx* h, const double* theta_dev, int B, hipStream_t st) {
  int rc;
  if ((rc = ensure_keep(h, B)) || (rc = ensure_common_scratch(h, B))) return rc;
  // the first chunk's M_g inverses depend on theta only: they run on the
  // side stream while the partial factorisations run on st (forked after
  // whatever st produced theta with; joined before the assembly)
  // (large chunks only: for one proposal the fork / join costs more than the
  // overlap gains -- B = 1: 1.61 vs 1.49 ms)
  const bool overlap = h->P <= MINV_PMAX && h->kernel_mode != 7 && B >= 64;
  if (overlap) {
    if (!h->side) {
      EWH_HIP(hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking));
      EWH_HIP(hipEventCreateWithFlags(&h->ev_fork, hipEventDisableTiming));
      EWH_HIP(hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming));
    }
    EWH_HIP(hipEventRecord(h->ev_fork, st));
    EWH_HIP(hipStreamWaitEvent(h->side, h->ev_fork, 0));
    launch_minv(h, theta_dev, 0, std::min(h->cchunk, B), h->side);
    EWH_HIP(hipEventRecord(h->ev_join, h->side));
  }
  if ((rc = corr_partial(h, theta_dev, B, 0, h->P, h->d_units, h->d_keep, st))) return rc;
  if (overlap) EWH_HIP(hipStreamWaitEvent(st, h->ev_join, 0));
  return corr_finish(h, theta_dev, B, h->d_keep, h->d_units, st, overlap);
}

}  // namespace

namespace {

void destroy_ctx(DevCtx* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->stream) (void)hipStreamSynchronize(h->stream);
  drop_graphs(h);
  if (h->h_stage) (void)hipHostFree(h->h_stage);
  if (h->h_seg) (void)hipHostFree(h->h_seg);
  if (h->side) (void)hipStreamSynchronize(h->side);
  for (void* p : h->allocs) (void)hipFree(p);
  if (h->ev_fork) (void)hipEventDestroy(h->ev_fork);
  if (h->ev_join) (void)hipEventDestroy(h->ev_join);
  if (h->side) (void)hipStreamDestroy(h->side);
  if (h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

// Timing-model projection of one pulsar's basis.  Every
// basis column that does not depend on theta, and the residual, loses its
// least-squares component along the leading constant-phi (timing-model)
// columns M under the weights 1/sigma^2:
//   X' = X - M C,   C = (M^T W0 M)^-1 M^T W0 X.
// With phi_M = 1e40 this is an exact reparametrisation of the same
// likelihood: the timing-model coefficients absorb M C b (prior ~ flat), so
// lnL, log|Sigma| and the quadratic form change by O(|C|^2 / phi_M) ~ 1e-36
// relative, and log|phi| is untouched (the map is unit triangular).  What it
// removes is the cancellation: the low-frequency Fourier columns lie close
// to the span of the spin-down / astrometric columns, so in the original
// basis the timing-model elimination subtracts two nearly equal Gram blocks
// (~1e14 each) and fp64 rounding of the Gram -- or an asymmetric panel --
// was amplified into the prior-draw lnL (tests/golden, c2_small: 7e5x the
// strict bound).  C needs no special accuracy: any C is an exact
// reparametrisation; only X' = X - M C is rounded (once, by fma), a
// perturbation of X of O(eps |X|) -- the size of X's own representation.
// Computed once per handle (ProjCoef), applied when T_aug is built.
struct ProjCoef {
  int nl = 0;
  std::vector<int> cols;     // projected basis columns (the residual is cols.size()-th)
  std::vector<double> C;     // nl x (cols.size() + 1), row-major
};

ProjCoef projection_coef(const ewh_pulsar_desc& s) {
  ProjCoef pc;
  const int nl = s.n_lead_const, n = s.n_toa;
  if (nl <= 0 || nl >= s.n_col + 1) return pc;
  for (int j = nl; j < s.n_col; ++j)
    if (s.n_bgroup == 0 || s.col_bgroup[j] < 0) pc.cols.push_back(j);
  const int nc = (int)pc.cols.size() + 1;
  std::vector<double> G0((size_t)nl * nl, 0.0), Bm((size_t)nl * nc, 0.0), x(nc);
  for (int t = 0; t < n; ++t) {
    const double* row = s.basis + (size_t)t * s.n_col;
    const double w0 = 1.0 / (s.toaerr[t] * s.toaerr[t]);
    for (int k = 0; k < nc - 1; ++k) x[k] = row[pc.cols[k]];
    x[nc - 1] = s.resid[t];
    for (int a = 0; a < nl; ++a) {
      const double wa = w0 * row[a];
      if (wa == 0.0) continue;
      for (int b = 0; b < nl; ++b) G0[(size_t)a * nl + b] += wa * row[b];
      double* br = &Bm[(size_t)a * nc];
      for (int k = 0; k < nc; ++k) br[k] += wa * x[k];
    }
  }
  // Cholesky of G0; a column of M with (numerically) no weight of its own --
  // e.g. a zero-norm design-matrix column -- is left out of the projection
  double dmax = 0.0;
  for (int a = 0; a < nl; ++a) dmax = std::max(dmax, G0[(size_t)a * nl + a]);
  std::vector<double> L((size_t)nl * nl, 0.0);
  std::vector<char> use(nl, 0);
  for (int k = 0; k < nl; ++k) {
    double v = G0[(size_t)k * nl + k];
    for (int j = 0; j < k; ++j) v -= L[(size_t)k * nl + j] * L[(size_t)k * nl + j];
    if (!(v > 1e-12 * dmax)) continue;
    use[k] = 1;
    const double lkk = std::sqrt(v);
    L[(size_t)k * nl + k] = lkk;
    for (int i = k + 1; i < nl; ++i) {
      double u = G0[(size_t)i * nl + k];
      for (int j = 0; j < k; ++j) u -= L[(size_t)i * nl + j] * L[(size_t)k * nl + j];
      L[(size_t)i * nl + k] = u / lkk;
    }
  }
  // C = G0^-1 Bm over the used columns (forward, then back substitution)
  pc.nl = nl;
  pc.C.assign((size_t)nl * nc, 0.0);
  for (int k = 0; k < nc; ++k) {
    std::vector<double> y(nl, 0.0);
    for (int i = 0; i < nl; ++i) {
      if (!use[i]) continue;
      double v = Bm[(size_t)i * nc + k];
      for (int j = 0; j < i; ++j) v -= L[(size_t)i * nl + j] * y[j];
      y[i] = v / L[(size_t)i * nl + i];
    }
    for (int i = nl - 1; i >= 0; --i) {
      if (!use[i]) continue;
      double v = y[i];
      for (int j = i + 1; j < nl; ++j) v -= L[(size_t)j * nl + i] * pc.C[(size_t)j * nc + k];
      pc.C[(size_t)i * nc + k] = v / L[(size_t)i * nl + i];
    }
  }
  return pc;
}

// X' = X - M C on T_aug (row-major, leading dimension ld, residual at ld-1),
// formed in double-double (round 6): TwoProd of each M_ta C_ak (by fma) and
// TwoSum into (s, e), so s + e = X - M C to ~2^-106; T_aug takes the rounded
// value fl(s + e) and, when lo is given, lo takes the residual (s + e) -
// fl(s + e), the part of the exact projection that the fp64 T_aug drops
// (rounds 2-5: one fma chain, its rounding -- up to eps |M C|, cancellation
// included -- entered every Gram)
void apply_projection(const ProjCoef& pc, int n_toa, int ld, std::vector<double>& Ta, std::vector<double>* lo) {
#pragma clang fp contract(off)
  const int nl = pc.nl, nc = (int)pc.cols.size() + 1;
  if (nl == 0) return;
  for (int t = 0; t < n_toa; ++t) {
    double* row = &Ta[(size_t)t * ld];
    for (int k = 0; k < nc; ++k) {
      const int col = k < nc - 1 ? pc.cols[k] : ld - 1;
      double hs = row[col], es = 0.0;
      for (int a = 0; a < nl; ++a) {
        const double p = -row[a] * pc.C[(size_t)a * nc + k];
        const double pe = std::fma(-row[a], pc.C[(size_t)a * nc + k], -p);   // -M C = p + pe exactly
        const double sum = hs + p, bp = sum - hs;
        es += ((hs - (sum - bp)) + (p - bp)) + pe;                           // TwoSum error + product error
        hs = sum;
      }
      const double v = hs + es;
      row[col] = v;
      if (lo) (*lo)[(size_t)t * ld + col] = (hs - v) + es;                   // (hs - v exact: v ~ hs)
    }
  }
}

// One device's copy of the PTA (every table, the fixed-WN cache, scratch).
int create_ctx(const ewh_pta_desc* d, const std::vector<ProjCoef>& proj, int device, DevCtx** out) {
  *out = nullptr;
  int rc;
  EWH_HIP(hipSetDevice(device));
  DevCtx* h = new DevCtx();
  h->device = device;
  h->P = d->n_pulsar;
  h->n_param = d->n_param;
  h->psr.resize(h->P);
  auto bail = [&](int code) {
    destroy_ctx(h);
    return code;
  };
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess)
    return bail(set_err(EWH_E_HIP, "hipStreamCreate failed"));
  if (hipDeviceGetAttribute(&h->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || h->n_cu <= 0)
    h->n_cu = 256;
  // per device (the attribute is a property of the kernel on the current device)
  if (hipFuncSetAttribute((const void*)chol_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)(LDS_MAX - 64)) != hipSuccess)
    return bail(set_err(EWH_E_HIP, "hipFuncSetAttribute(chol_lds_kernel) failed"));
  if ((rc = set_contract_attributes()) || (rc = set_dd_attributes())) return bail(rc);
  bool any_theta_white = false;
  for (int p = 0; p < h->P; ++p) {
    const ewh_pulsar_desc& s = d->pulsars[p];
    for (int i = 0; i < s.n_slot; ++i) any_theta_white |= pref_uses_theta(s.slots[i]);
    any_theta_white |= s.n_bgroup > 0;
  }
  // a correlated common process with white noise varying (or a theta-dependent
  // basis): per sample, the contraction of a T_aug laid out with the common
  // columns in whole blocks, then the partial factorisation (corr_partial)
  const bool corr_var = d->common && d->common->kind == EWH_COMMON_CORRELATED &&
                        !((d->white_fixed != 0) && !any_theta_white);
  for (int p = 0; p < h->P; ++p) {
    const ewh_pulsar_desc& s = d->pulsars[p];
    PsrHost& ps = h->psr[p];
    ps.n_toa = s.n_toa;
    ps.m = s.n_col;
    ps.nlead = s.n_lead_const;
    // T_aug position of basis column j (identity, or the corr_var layout)
    std::vector<int> vpos(s.n_col);
    for (int j = 0; j < s.n_col; ++j) vpos[j] = j;
    int pad0 = 0, pad1 = 0;
    if (corr_var) {
      const int nlo = s.n_col - s.n_common;
      ps.gstart_v = 16 * ((nlo + 15) / 16);
      for (int j = nlo; j < s.n_col; ++j) vpos[j] = ps.gstart_v + (j - nlo);
      pad0 = nlo;
      pad1 = ps.gstart_v;
      ps.m = ps.gstart_v + s.n_common;
    }
    ps.nb = nb_for(ps.m + 1);
    ps.ld = 16 * ps.nb;
    ps.n_epoch = s.n_epoch;
    ps.max_epoch = 0;
    for (int e = 0; e < s.n_epoch; ++e) ps.max_epoch = std::max(ps.max_epoch, s.epoch_stop[e] - s.epoch_start[e]);
    ps.fx_m = s.n_col - s.n_lead_const;
    ps.ncommon = d->common ? s.n_common : 0;
    ps.nloc = ps.fx_m - ps.ncommon;
    if (ps.ncommon > 0) {          // [own | pad to 16 | common | pad | r]
      ps.gstart = 16 * ((ps.nloc + 15) / 16);
      ps.fx_nb = nb_for(ps.gstart + ps.ncommon + 1);
    } else {                       // [own | pad | r]
      ps.gstart = ps.nloc;
      ps.fx_nb = nb_for(ps.fx_m + 1);
    }
    ps.fx_ld = 16 * ps.fx_nb;
    for (int i = 0; i < s.n_slot; ++i) ps.has_theta_white |= pref_uses_theta(s.slots[i]);
    // T_aug: [basis | 0-pad | r], row-major n x ld
    // (+CT_ROWS zero rows: the pipelined contraction copies whole tiles)
    std::vector<double> Ta((size_t)(s.n_toa + CT_ROWS) * ps.ld, 0.0), sig2(s.n_toa);
    for (int t = 0; t < s.n_toa; ++t) {
      for (int j = 0; j < s.n_col; ++j) Ta[(size_t)t * ps.ld + j] = s.basis[(size_t)t * s.n_col + j];
      Ta[(size_t)t * ps.ld + ps.ld - 1] = s.resid[t];
      sig2[t] = s.toaerr[t] * s.toaerr[t];
    }
    // the projection residual for the double-double Grams (PsrHost::d_Tlo)
    const bool want_lo = !corr_var && s.n_bgroup == 0 && proj[p].nl > 0;
    std::vector<double> Tlo(want_lo ? Ta.size() : 0, 0.0);
    apply_projection(proj[p], s.n_toa, ps.ld, Ta, want_lo ? &Tlo : nullptr);
    if (want_lo && (rc = dupload(h, &ps.d_Tlo, Tlo.data(), Tlo.size()))) return bail(rc);
    if (corr_var) {       // common columns to their block-aligned positions (from the top: pos >= j)
      for (int t = 0; t < s.n_toa; ++t) {
        double* row = &Ta[(size_t)t * ps.ld];
        for (int j = s.n_col - 1; j >= pad0; --j) {
          const double v = row[j];
          row[j] = 0.0;
          row[vpos[j]] = v;
        }
      }
    }
    double* dT;
    double* dsig2;
    int *d_ef, *d_eq, *d_es, *d_ee, *d_eslot;
    ps.n_slot = s.n_slot;
    ps.slots.assign(s.slots, s.slots + s.n_slot);
    if ((rc = dupload(h, &dT, Ta.data(), Ta.size()))) return bail(rc);
    if ((rc = dupload(h, &dsig2, sig2.data(), sig2.size()))) return bail(rc);
    if ((rc = dupload(h, &d_ef, s.efac_slot, (size_t)s.n_toa))) return bail(rc);
    if ((rc = dupload(h, &d_eq, s.equad_slot, (size_t)s.n_toa))) return bail(rc);
    if ((rc = dupload(h, &ps.d_slots, s.slots, (size_t)s.n_slot))) return bail(rc);
    if ((rc = dupload(h, &d_es, s.epoch_start, (size_t)s.n_epoch))) return bail(rc);
    if ((rc = dupload(h, &d_ee, s.epoch_stop, (size_t)s.n_epoch))) return bail(rc);
    if ((rc = dupload(h, &d_eslot, s.epoch_slot, (size_t)s.n_epoch))) return bail(rc);
    std::vector<int> toa_ep((size_t)s.n_toa + CT_ROWS, -1);
    for (int e = 0; e < s.n_epoch; ++e)
      for (int t = s.epoch_start[e]; t < s.epoch_stop[e]; ++t) toa_ep[t] = 2 * e + (t == s.epoch_stop[e] - 1);
    int* d_tep;
    if ((rc = dupload(h, &d_tep, toa_ep.data(), toa_ep.size()))) return bail(rc);
    int* d_cbg = nullptr;
    double* d_lnc = nullptr;
    ewh_pref* d_bg = nullptr;
    if (s.n_bgroup > 0) {
      std::vector<int> cbg(ps.ld, -1);
      for (int j = 0; j < s.n_col; ++j) cbg[vpos[j]] = s.col_bgroup[j];
      if ((rc = dupload(h, &d_cbg, cbg.data(), cbg.size()))) return bail(rc);
      if ((rc = dupload(h, &d_lnc, s.ln_chrom, (size_t)s.n_toa))) return bail(rc);
      if ((rc = dupload(h, &d_bg, s.bgroup_idx, (size_t)s.n_bgroup))) return bail(rc);
    }
    ps.dev = PsrDev{s.n_toa, ps.m, ps.ld, ps.nb, s.n_epoch, dT, dsig2, d_ef, d_eq, ps.d_slots, d_es, d_ee, d_eslot,
                    s.n_bgroup, d_cbg, d_lnc, d_bg, d_tep};
    std::vector<int> ptr;
    std::vector<DSpec> ent;
    if (corr_var) build_csr_mapped(s, vpos, ps.m, pad0, pad1, ptr, ent);
    else build_csr(s, 0, s.n_col, ptr, ent);
    if ((rc = dupload(h, &ps.d_colptr, ptr.data(), ptr.size()))) return bail(rc);
    if ((rc = dupload(h, &ps.d_spec, ent.data(), ent.size()))) return bail(rc);
    build_csr_fixed(s, ps.nlead, ps.nloc, ps.gstart, ps.fx_ld, ptr, ent);
    if ((rc = dupload(h, &ps.d_fx_colptr, ptr.data(), ptr.size()))) return bail(rc);
    if ((rc = dupload(h, &ps.d_fx_spec, ent.data(), ent.size()))) return bail(rc);
    {
      std::vector<int> rep, ulist;
      build_spec_rep(ptr, ent, rep, ulist);
      ps.fx_nu = (int)ulist.size();
      // staged records: ulist order; urep[a] = record of column a's spectrum
      std::vector<int> urep(rep.size(), -1), uidx(rep.size(), -1);
      for (size_t u = 0; u < ulist.size(); ++u) uidx[ulist[u]] = (int)u;
      bool fits = true;
      std::vector<URec> urec(std::max<size_t>(1, ulist.size()));
      for (size_t u = 0; u < ulist.size(); ++u) {
        const int a = ulist[u];
        const int ne = ptr[a + 1] - ptr[a];
        if (ne > URec::NE) fits = false;
        urec[u] = URec{};
        urec[u].ne = std::min(ne, URec::NE);
        for (int e = 0; e < urec[u].ne; ++e) urec[u].e[e] = ent[ptr[a] + e];
      }
      // the theta entries the records read: staged alone when there are at
      // most TIDX_MAX of them (the records then index that list)
      std::vector<int> tl;
      for (size_t u = 0; u < ulist.size(); ++u)
        for (int e = 0; e < urec[u].ne; ++e)
          for (int idx : {urec[u].e[e].i0, urec[u].e[e].i1, urec[u].e[e].i2})
            if (idx >= 0 && std::find(tl.begin(), tl.end(), idx) == tl.end()) tl.push_back(idx);
      std::sort(tl.begin(), tl.end());
      ps.fx_tidx.clear();
      if (fits && (int)tl.size() <= TIDX_MAX) {
        ps.fx_tidx = tl;
        auto pos = [&](int idx) { return idx < 0 ? idx : (int)(std::lower_bound(tl.begin(), tl.end(), idx) - tl.begin()); };
        for (size_t u = 0; u < ulist.size(); ++u)
          for (int e = 0; e < urec[u].ne; ++e) {
            urec[u].e[e].i0 = pos(urec[u].e[e].i0);
            urec[u].e[e].i1 = pos(urec[u].e[e].i1);
            urec[u].e[e].i2 = pos(urec[u].e[e].i2);
          }
      }
      for (size_t a = 0; a < rep.size(); ++a)
        if (ptr[a] < ptr[a + 1]) urep[a] = uidx[rep[a]];
      if (fits) {
        if ((rc = dupload(h, &ps.d_fx_urec, urec.data(), urec.size()))) return bail(rc);
        if ((rc = dupload(h, &ps.d_fx_urep, urep.data(), urep.size()))) return bail(rc);
      }
      if (ulist.empty()) ulist.push_back(0);
      if ((rc = dupload(h, &ps.d_fx_rep, rep.data(), rep.size()))) return bail(rc);
      if ((rc = dupload(h, &ps.d_fx_ulist, ulist.data(), ulist.size()))) return bail(rc);
    }
  }
  h->white_fixed = (d->white_fixed != 0) && !any_theta_white;
  if ((rc = dalloc(h, &h->d_jobs_fixed, h->P))) return bail(rc);
  if ((rc = dalloc(h, &h->d_jobs_var, h->P))) return bail(rc);
  h->osmode = d->common && d->common->kind == EWH_COMMON_OPTSTAT;
  if (h->osmode && !h->white_fixed)
    return bail(set_err(EWH_E_UNSUPPORTED, "optimal statistic: white noise must be fixed (TNT cached)"));
  if (h->white_fixed && (rc = setup_fixed(h))) return bail(rc);
  if (d->common && (rc = setup_common(h, d))) return bail(rc);
  if (h->white_fixed && !h->corr && !h->osmode) {
    int nb = h->psr[0].fx_nb;
    for (const auto& ps : h->psr)
      if (ps.fx_nb != nb) nb = 0;
    if (nb >= 1 && nb <= LAT_NB_MAX) h->lat_nb = nb;
  }
  *out = h;
  return 0;
}

// lnL terms of units [u_begin, u_end) (u = pulsar * B + sample) into h->d_units
// (rows outside the range zeroed); reduce: also out_dev[b] = sum over the rows.
int ctx_units(DevCtx* h, const double* theta_dev, int B, int64_t u_begin, int64_t u_end, double* out_dev,
              hipStream_t st, bool reduce) {
  const long long U = (long long)h->P * B;
  u_begin = std::max<int64_t>(0, u_begin);
  u_end = std::min<int64_t>(U, u_end);
  EWH_HIP(hipSetDevice(h->device));
  int rc;
  if ((rc = ensure_units(h, B))) return rc;
  const int rows = h->P + (h->corr ? 1 : 0);
  EWH_HIP(hipMemsetAsync(h->d_units, 0, sizeof(double) * (size_t)rows * B, st));
  const int ldth = h->n_param;
  hipStream_t saved = h->stream;
  h->stream = st;
  struct Restore {
    DevCtx* h;
    hipStream_t s;
    ~Restore() { h->stream = s; }
  } restore{h, saved};
  if (h->corr) {
    if (u_begin != 0 || u_end != U)
      return set_err(EWH_E_UNSUPPORTED, "correlated common process: pass the whole batch (shard samples, not units)");
    if ((rc = lnl_correlated(h, theta_dev, B, st))) return rc;
  } else if (h->white_fixed) {
    // one launch per run of consecutive pulsars with the same kernel class
    long long u = u_begin;
    while (u < u_end) {
      const int p0 = (int)(u / B);
      const int nb0 = h->psr[p0].fx_nb;
      int p1 = p0 + 1;
      while (p1 < h->P && h->psr[p1].fx_nb == nb0 && (long long)p1 * B < u_end) ++p1;
      const long long seg_end = std::min<long long>(u_end, (long long)p1 * B);
      int maxm = 0;
      for (int p = p0; p < p1; ++p) maxm = std::max(maxm, h->psr[p].fx_m);
      if ((rc = ensure_big_scratch(h, nb0)) ||
          (rc = dispatch_chol(h, nb0, maxm, h->d_jobs_fixed, B, u, seg_end - u, 0, theta_dev, ldth, h->d_units, st,
                              true)))
        return rc;
      if (!dd_path(h, nb0, true) && refine_on(h) &&
          (rc = refine_failed(h, h->d_jobs_fixed, nb0, B, u, seg_end - u, 0, theta_dev, ldth, h->d_units, st,
                              nullptr)))
        return rc;
      u = seg_end;
    }
  } else {
    if ((rc = ensure_var_scratch(h, B))) return rc;
    for (long long u = u_begin; u < u_end;) {
      const int p = (int)(u / B);
      const long long pend = std::min<long long>(u_end, (long long)(p + 1) * B);
      const int bs = (int)(u - (long long)p * B), be = (int)(pend - (long long)p * B);
      for (int c0 = bs; c0 < be; c0 += h->chunk) {
        const int nb = std::min(h->chunk, be - c0);
        if ((rc = run_white(h, p, theta_dev, ldth, c0, nb))) return rc;
        if ((rc = ensure_big_scratch(h, h->psr[p].nb)) ||
            (rc = dispatch_chol(h, h->psr[p].nb, h->psr[p].m, h->d_jobs_var, B, (long long)p * B + c0, nb, c0,
                                theta_dev, ldth, h->d_units, st, false)))
          return rc;
        // (past 16 blocks too: the verify route's double-double factorisation
        // reads the compensated -- not error-free -- G_hi + G_lo of the wide
        // contraction, so a unit it still leaves at -inf gets the error-free
        // Gram here)
        const PsrHost& ps = h->psr[p];
        if (ps.dev.n_bgroup == 0 && refine_on(h) &&
            (rc = refine_failed(h, h->d_jobs_var, ps.nb, B, (long long)p * B + c0, nb, c0, theta_dev, ldth,
                                h->d_units, st, &ps)))
          return rc;
      }
      u = pend;
    }
  }
  if (reduce)
    hipLaunchKernelGGL(reduce_units_kernel, dim3((B + 255) / 256), dim3(256), 0, st, h->d_units, rows, B, out_dev);
  EWH_HIP(hipGetLastError());
  h->last_B = B;
  return 0;
}

// device theta / out buffers of one context, grown as needed
int ensure_io(DevCtx* h, int B) {
  const size_t need = (size_t)B * std::max(1, h->n_param) + B;
  if (need > h->io_cap) {
    if (h->d_theta) {
      (void)hipFree(h->d_theta);
      h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), (void*)h->d_theta));
      h->d_theta = nullptr;
    }
    h->io_cap = 0;
    int rc = dalloc(h, &h->d_theta, need);
    if (rc) return rc;
    h->io_cap = need;
  }
  h->d_out = h->d_theta + (size_t)B * std::max(1, h->n_param);
  return 0;
}

// Cost-balanced contiguous unit ranges (the same rule as
// enterprise_warp_amd.sharding.unit_ranges).
std::vector<std::pair<long long, long long>> unit_ranges(const std::vector<double>& cost, int B, int world) {
  const int P = (int)cost.size();
  std::vector<std::pair<long long, long long>> out;
  if (world <= 1) {
    out.push_back({0, (long long)P * B});
    return out;
  }
  std::vector<double> cum(P + 1, 0.0);
  for (int p = 0; p < P; ++p) cum[p + 1] = cum[p] + cost[p] * B;
  std::vector<long long> bounds{0};
  for (int r = 1; r < world; ++r) {
    const double target = cum[P] * r / world;
    int p = (int)(std::upper_bound(cum.begin(), cum.end(), target) - cum.begin()) - 1;
    p = std::min(std::max(p, 0), P - 1);
    const double within = cost[p] > 0 ? (target - cum[p]) / cost[p] : 0.0;
    long long u = (long long)p * B + (long long)std::llround(within);
    u = std::min<long long>(std::max<long long>(u, bounds.back()), (long long)P * B);
    bounds.push_back(u);
  }
  bounds.push_back((long long)P * B);
  for (int i = 0; i < world; ++i) out.push_back({bounds[i], bounds[i + 1]});
  return out;
}

int ctx_optstat(DevCtx* h, const double* theta_host, int32_t B, const double* phihat_host, double* rho_host,
                double* sig_host, double* os_host, double* os_sig_host) {
  if (!h || !theta_host || !phihat_host || !os_host || !os_sig_host || B <= 0)
    return set_err(EWH_E_INVALID, "bad arguments");
  if (!h->osmode) return set_err(EWH_E_INVALID, "handle was not created with common->kind = EWH_COMMON_OPTSTAT");
  EWH_HIP(hipSetDevice(h->device));
  const int P = h->P, nc = h->nc, KD = 16 * h->keep, np = std::max(1, h->n_param);
  hipStream_t st = h->stream;
  int rc;
  double *th, *ph, *xh, *wh, *rho, *sig, *os;
  std::vector<void*> tmp;
  auto alloc = [&](double** p, size_t n) {
    int r = dalloc(h, p, n);
    if (!r) tmp.push_back(*p);
    return r;
  };
  auto release = [&]() {
    for (void* p : tmp) {
      (void)hipFree(p);
      h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), p));
    }
  };
  if ((rc = alloc(&th, (size_t)B * np)) || (rc = alloc(&ph, (size_t)B * nc)) ||
      (rc = alloc(&xh, (size_t)B * P * nc)) || (rc = alloc(&wh, (size_t)B * P * nc * nc)) ||
      (rc = alloc(&rho, (size_t)B * P * P)) || (rc = alloc(&sig, (size_t)B * P * P)) || (rc = alloc(&os, 2 * (size_t)B))) {
    release();
    return rc;
  }
  if (h->n_param > 0)
    EWH_HIP(hipMemcpyAsync(th, theta_host, sizeof(double) * (size_t)B * h->n_param, hipMemcpyHostToDevice, st));
  EWH_HIP(hipMemcpyAsync(ph, phihat_host, sizeof(double) * (size_t)B * nc, hipMemcpyHostToDevice, st));
  EWH_HIP(hipMemsetAsync(rho, 0, sizeof(double) * (size_t)B * P * P, st));
  EWH_HIP(hipMemsetAsync(sig, 0, sizeof(double) * (size_t)B * P * P, st));
  if ((rc = ensure_units(h, B))) {
    release();
    return rc;
  }
  const size_t need = (size_t)B * P * KD * KD;
  if (need > h->keep_cap) {
    if (h->d_keep) {
      (void)hipFree(h->d_keep);
      h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), (void*)h->d_keep));
      h->d_keep = nullptr;
    }
    h->keep_cap = 0;
    if ((rc = dalloc(h, &h->d_keep, need))) {
      release();
      return rc;
    }
    h->keep_cap = need;
  }
  const long long U = (long long)P * B;
  for (long long u = 0; u < U;) {      // per-pulsar factorisations, common block kept
    const int p0 = (int)(u / B);
    const int nb0 = h->psr[p0].fx_nb;
    int p1 = p0 + 1;
    while (p1 < P && h->psr[p1].fx_nb == nb0) ++p1;
    const long long seg_end = (long long)p1 * B;
    if ((rc = partial_units(h, h->d_jobs_fixed, nb0, B, u, seg_end - u, 0, th, h->d_units, h->d_keep, st))) {
      release();
      return rc;
    }
    u = seg_end;
  }
  hipLaunchKernelGGL(os_xz_kernel, dim3(P, B), dim3(64), 0, st, h->d_keep, KD, P, nc, h->d_cps, th, h->n_param, ph,
                     xh, wh);
  hipLaunchKernelGGL(os_pairs_kernel, dim3(P, B), dim3(256), 0, st, xh, wh, P, nc, rho, sig);
  hipLaunchKernelGGL(os_final_kernel, dim3((B + 255) / 256), dim3(256), 0, st, rho, sig, h->d_orf, P, B, os, os + B);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && rho_host)
    e = hipMemcpyAsync(rho_host, rho, sizeof(double) * (size_t)B * P * P, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess && sig_host)
    e = hipMemcpyAsync(sig_host, sig, sizeof(double) * (size_t)B * P * P, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipMemcpyAsync(os_host, os, sizeof(double) * B, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipMemcpyAsync(os_sig_host, os + B, sizeof(double) * B, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  release();
  if (e != hipSuccess) return set_err(EWH_E_HIP, std::string("ewh_optstat: ") + hipGetErrorString(e));
  return 0;
}

double ctx_unit_cost(const DevCtx* h, int p) {
  const PsrHost& ps = h->psr[p];
  if (h->white_fixed) return (double)ps.fx_ld * ps.fx_ld * ps.fx_ld / 3.0;
  return (double)ps.n_toa * ps.ld * ps.ld + (double)ps.ld * ps.ld * ps.ld / 3.0;
}

}  // namespace

// The handle: one DevCtx per device of the node (a full replica of the PTA in
// each device's HBM -- C3 is 0.5 GB of bases against 288 GB), plus pinned
// host staging shared by all of them.
struct ewh_handle {
  std::vector<DevCtx*> ctx;
  int P = 0, n_param = 0;
  bool corr = false;
  // pinned (portable) host staging: theta rows, and the outputs / unit terms
  double* h_theta = nullptr;
  size_t h_theta_cap = 0;
  double* h_out = nullptr;
  size_t h_out_cap = 0;
  // last ewh_lnl_batch split: per context, unit range (uncorrelated) or
  // sample range (correlated)
  std::vector<std::pair<long long, long long>> last_split;
  int last_B = 0;
  // multi-context fold on the first context's device: per-context partial
  // B-vectors (peer-copied in), and one event per context
  double* d_part = nullptr;
  size_t part_cap = 0;
  std::vector<hipEvent_t> ev;
  // latency path: device addresses of h_theta / h_out (for the host pointers recorded)
  const double *lat_th_host = nullptr, *lat_out_host = nullptr;
  double *lat_th_dev = nullptr, *lat_out_dev = nullptr;
  // theta columns each pulsar's units read (white-noise slots, spectra,
  // chromatic index groups; a correlated process's common spectra)
  std::vector<std::vector<int>> psr_cols;
  // ewh_transfer_stats: theta bytes host -> device of the last batch, and the
  // contexts with peer access to the first one
  long long h2d_bytes = 0;
  long long peer_mask = 1;
  // peer-access directions (from, to) this handle holds a reference on
  // (peer_acquire); released in ewh_destroy
  std::vector<std::pair<int, int>> peer_held;
};

namespace {

// Peer access is process-global state.  Handles share it by reference count:
// a direction (from, to) a handle enabled, or found enabled by another
// handle, is counted; the last handle to release it disables it.  A direction
// that was already on when no handle held it (the caller's own) is never
// counted, so never turned off here.
std::mutex g_peer_mu;
std::map<std::pair<int, int>, int> g_peer_refs;

bool peer_acquire(ewh_handle* H, int from, int to) {
  std::lock_guard<std::mutex> lk(g_peer_mu);
  if (hipSetDevice(from) != hipSuccess) return false;
  const hipError_t e = hipDeviceEnablePeerAccess(to, 0);
  (void)hipGetLastError();
  const auto key = std::make_pair(from, to);
  auto it = g_peer_refs.find(key);
  if (e == hipSuccess || (e == hipErrorPeerAccessAlreadyEnabled && it != g_peer_refs.end())) {
    ++g_peer_refs[key];
    H->peer_held.push_back(key);
    return true;
  }
  return e == hipErrorPeerAccessAlreadyEnabled;   // on outside any handle: usable, not ours
}

void peer_release_all(ewh_handle* H) {
  std::lock_guard<std::mutex> lk(g_peer_mu);
  for (const auto& key : H->peer_held) {
    auto it = g_peer_refs.find(key);
    if (it == g_peer_refs.end()) continue;
    if (--it->second == 0) {
      g_peer_refs.erase(it);
      if (hipSetDevice(key.first) == hipSuccess) (void)hipDeviceDisablePeerAccess(key.second);
      (void)hipGetLastError();
    }
  }
  H->peer_held.clear();
}

// cached: the latency path's record of which host buffer its device address
// belongs to -- cleared on reallocation (a new buffer may reuse the address)
int ensure_pinned(double** p, size_t* cap, size_t need, const double** cached = nullptr) {
  if (need <= *cap) return 0;
  if (cached) *cached = nullptr;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *cap = 0;
  // coherent: the latency kernel's stores to it are visible to a spinning
  // host thread before the launch completes (and its theta reads bypass L2)
  hipError_t e = hipHostMalloc((void**)p, std::max<size_t>(need, 1) * sizeof(double),
                               hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return set_err(EWH_E_NOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
  *cap = need;
  return 0;
}

}  // namespace

namespace {

// enqueue one single-context batch on h->stream: H2D of theta from the pinned
// staging, the unit launches + reduction, D2H of lnL into the pinned staging
int enqueue_single(ewh_handle* H, DevCtx* h, int B) {
  const int np = H->n_param;
  int rc;
  if (np > 0)
    EWH_HIP(hipMemcpyAsync(h->d_theta, H->h_theta, sizeof(double) * (size_t)B * np, hipMemcpyHostToDevice,
                           h->stream));
  if ((rc = ctx_units(h, h->d_theta, B, 0, (long long)H->P * B, h->d_out, h->stream, true))) return rc;
  EWH_HIP(hipMemcpyAsync(H->h_out, h->d_out, sizeof(double) * B, hipMemcpyDeviceToHost, h->stream));
  return 0;
}

constexpr size_t GRAPH_CACHE = 8;

template <typename T>
int ensure_host_pinned(T** p, size_t* cap, size_t need) {
  if (need <= *cap) return 0;
  if (*p) (void)hipHostFree(*p);
  *p = nullptr;
  *cap = 0;
  hipError_t e = hipHostMalloc((void**)p, std::max<size_t>(need, 1) * sizeof(T), hipHostMallocPortable);
  if (e != hipSuccess) return set_err(EWH_E_NOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
  *cap = need;
  return 0;
}

template <typename T>
int ensure_dev(DevCtx* h, T** p, size_t* cap, size_t need) {
  if (need <= *cap) return 0;
  if (*p) {
    (void)hipFree(*p);
    h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), (void*)*p));
    *p = nullptr;
  }
  *cap = 0;
  int rc = dalloc(h, p, need);
  if (rc) return rc;
  *cap = need;
  return 0;
}

// Theta of one context's unit range [a, b) (u = pulsar * B + sample): per
// column, the sample rows its pulsars read (the union of their row ranges);
// columns with the same rows form one segment.  Packed into pinned memory,
// copied to the device and scattered into h->d_theta (full layout) on
// h->stream.  Returns the payload bytes (or a negative error code).
long long stage_theta_range(ewh_handle* H, DevCtx* h, const double* theta_host, int B, long long a, long long b) {
  const int np = H->n_param;
  if (b <= a || np <= 0) return 0;
  std::map<int, std::pair<int, int>> rows;                 // column -> [lo, hi)
  const int p0 = (int)(a / B), p1 = (int)((b - 1) / B);
  for (int p = p0; p <= p1; ++p) {
    const int lo = p == p0 ? (int)(a % B) : 0, hi = p == p1 ? (int)((b - 1) % B) + 1 : B;
    for (int c : H->psr_cols[p]) {
      auto it = rows.find(c);
      if (it == rows.end()) rows.emplace(c, std::make_pair(lo, hi));
      else it->second = {std::min(it->second.first, lo), std::max(it->second.second, hi)};
    }
  }
  std::map<std::pair<int, int>, std::vector<int>> segs;
  for (auto& kv : rows) segs[kv.second].push_back(kv.first);
  const int nseg = (int)segs.size();
  if (nseg == 0) return 0;
  size_t ncolsum = 0, payload = 0;
  for (auto& kv : segs) {
    ncolsum += kv.second.size();
    payload += (size_t)(kv.first.second - kv.first.first) * kv.second.size();
  }
  int rc;
  if ((rc = ensure_host_pinned(&h->h_stage, &h->h_stage_cap, payload)) ||
      (rc = ensure_host_pinned(&h->h_seg, &h->h_seg_cap, 5 * (size_t)nseg + ncolsum)) ||
      (rc = ensure_dev(h, &h->d_stage, &h->d_stage_cap, payload)) ||
      (rc = ensure_dev(h, &h->d_seg, &h->d_seg_cap, 5 * (size_t)nseg + ncolsum)))
    return rc;
  int si = 0, coloff = 0;
  size_t dataoff = 0;
  for (auto& kv : segs) {
    const int lo = kv.first.first, hi = kv.first.second, nc = (int)kv.second.size();
    int* rec = h->h_seg + 5 * si;
    rec[0] = lo; rec[1] = hi; rec[2] = nc; rec[3] = coloff; rec[4] = (int)dataoff;
    for (int j = 0; j < nc; ++j) h->h_seg[5 * nseg + coloff + j] = kv.second[j];
    for (int r = lo; r < hi; ++r) {
      const double* src = theta_host + (size_t)r * np;
      double* dst = h->h_stage + dataoff + (size_t)(r - lo) * nc;
      for (int j = 0; j < nc; ++j) dst[j] = src[kv.second[j]];
    }
    dataoff += (size_t)(hi - lo) * nc;
    coloff += nc;
    ++si;
  }
  EWH_HIP(hipMemcpyAsync(h->d_seg, h->h_seg, sizeof(int) * (5 * (size_t)nseg + ncolsum), hipMemcpyHostToDevice,
                         h->stream));
  EWH_HIP(hipMemcpyAsync(h->d_stage, h->h_stage, sizeof(double) * payload, hipMemcpyHostToDevice, h->stream));
  // every entry the segments do not cover reads as NaN (all bits set): a
  // column some kernel reads but psr_cols does not list gives a non-finite
  // phi -- a failed sample, not a stale value from an earlier batch
  EWH_HIP(hipMemsetAsync(h->d_theta, 0xFF, sizeof(double) * (size_t)B * np, h->stream));
  hipLaunchKernelGGL(expand_theta_kernel, dim3(nseg), dim3(256), 0, h->stream, h->d_stage, h->d_seg, nseg, np,
                     h->d_theta);
  EWH_HIP(hipGetLastError());
  return (long long)(payload * sizeof(double));
}

// Correlated common process, batch smaller than the device count (one
// PTMCMC proposal): the pulsars are split over the devices (the exchange step
// of SURVEY.md §8(e)) -- each device runs the partial factorisations of its
// pulsars, its kept common blocks and local terms are copied peer-to-peer into
// the first device's buffers (the all-gather), and the first device assembles
// and factors Sigma_c.  Per-pulsar results do not depend on the device, so the
// value equals the one-device result bit for bit.
int lnl_batch_corr_pulsars(ewh_handle* H, int B, double* out_host) {
  const int nd = (int)H->ctx.size(), P = H->P, np = H->n_param;
  DevCtx* h0 = H->ctx[0];
  const size_t kd2 = (size_t)(16 * h0->keep) * (16 * h0->keep);
  int rc;
  if ((rc = ensure_pinned(&H->h_out, &H->h_out_cap, (size_t)B, &H->lat_out_host))) return rc;
  for (int i = 0; i < nd; ++i) {
    DevCtx* h = H->ctx[i];
    EWH_HIP(hipSetDevice(h->device));
    if ((rc = ensure_io(h, B)) || (rc = ensure_units(h, B)) || (rc = ensure_keep(h, B))) return rc;
  }
  EWH_HIP(hipSetDevice(h0->device));
  EWH_HIP(hipMemsetAsync(h0->d_units, 0, sizeof(double) * (size_t)(P + 1) * B, h0->stream));
  // theta on the first device always: corr_finish reads it there even when
  // the first context gets no pulsars (P < number of contexts)
  if (np > 0)
    EWH_HIP(hipMemcpyAsync(h0->d_theta, H->h_theta, sizeof(double) * (size_t)B * np, hipMemcpyHostToDevice,
                           h0->stream));
  H->h2d_bytes += (long long)sizeof(double) * B * np;
  EWH_HIP(hipStreamSynchronize(h0->stream));
  for (int i = 0; i < nd; ++i) {
    DevCtx* h = H->ctx[i];
    const int p0 = (int)((long long)P * i / nd), p1 = (int)((long long)P * (i + 1) / nd);
    if (p1 <= p0) continue;
    EWH_HIP(hipSetDevice(h->device));
    if (np > 0 && i > 0) {
      EWH_HIP(hipMemcpyAsync(h->d_theta, H->h_theta, sizeof(double) * (size_t)B * np, hipMemcpyHostToDevice,
                             h->stream));
      H->h2d_bytes += (long long)sizeof(double) * B * np;
    }
    if ((rc = corr_partial(h, h->d_theta, B, p0, p1, h->d_units, h->d_keep, h->stream))) return rc;
    if (i > 0) {   // gather: this device's pulsar slices into the first device
      EWH_HIP(hipMemcpyPeerAsync(h0->d_keep + (size_t)p0 * B * kd2, h0->device, h->d_keep + (size_t)p0 * B * kd2,
                                 h->device, sizeof(double) * (size_t)(p1 - p0) * B * kd2, h->stream));
      EWH_HIP(hipMemcpyPeerAsync(h0->d_units + (size_t)p0 * B, h0->device, h->d_units + (size_t)p0 * B, h->device,
                                 sizeof(double) * (size_t)(p1 - p0) * B, h->stream));
    }
  }
  for (int i = 1; i < nd; ++i) {
    EWH_HIP(hipSetDevice(H->ctx[i]->device));
    EWH_HIP(hipStreamSynchronize(H->ctx[i]->stream));
  }
  EWH_HIP(hipSetDevice(h0->device));
  if ((rc = corr_finish(h0, h0->d_theta, B, h0->d_keep, h0->d_units, h0->stream))) return rc;
  hipLaunchKernelGGL(reduce_units_kernel, dim3((B + 255) / 256), dim3(256), 0, h0->stream, h0->d_units, P + 1, B,
                     h0->d_out);
  EWH_HIP(hipGetLastError());
  EWH_HIP(hipMemcpyAsync(H->h_out, h0->d_out, sizeof(double) * B, hipMemcpyDeviceToHost, h0->stream));
  EWH_HIP(hipStreamSynchronize(h0->stream));
  std::memcpy(out_host, H->h_out, sizeof(double) * B);
  H->last_split.assign(1, {0, (long long)P * B});     // unit terms live on the first device
  H->last_B = B;
  h0->last_B = B;
  return 0;
}

// One device: replay the captured graph of this batch size when there is one;
// otherwise run the batch eagerly (that also sizes every scratch buffer) and
// capture the same sequence for the next call.
constexpr uint64_t LAT_SENTINEL = 0x7ff4dead0ebeef01ull;   // a NaN no kernel writes
// batches up to this size take the latency kernel (round 4, interleaved on
// C3: B = 12 / 16 / 24 at 57.9 / 57.5 / 80.0 us vs 64.2 / 65.8 / 83.3 us
// batched; B = 32 even, larger batched -- profiles/r04d/latency_sweep_bmax.log)
constexpr int LAT_B_MAX = 24;

int lnl_batch_single(ewh_handle* H, DevCtx* h, int B, double* out_host) {
  int rc;
  EWH_HIP(hipSetDevice(h->device));
  if ((rc = ensure_pinned(&H->h_out, &H->h_out_cap, (size_t)B, &H->lat_out_host))) return rc;
  const int km = h->kernel_mode;
  if (h->lat_nb > 0 && B <= LAT_B_MAX && (km == 0 || km == 22 || km == 23 || km == 24 || km == 25)) {
    // latency path: one launch reads theta from the pinned staging and writes
    // the unit terms to pinned memory (chol_lat.hip); the host folds them
    if ((rc = ensure_units(h, B)) || (rc = ensure_pinned(&H->h_out, &H->h_out_cap, (size_t)h->P * B, &H->lat_out_host))) return rc;
    // device addresses of the pinned staging (looked up again only after a reallocation)
    if (H->lat_th_host != H->h_theta) {
      EWH_HIP(hipHostGetDevicePointer((void**)&H->lat_th_dev, H->h_theta, 0));
      H->lat_th_host = H->h_theta;
    }
    if (H->lat_out_host != H->h_out) {
      EWH_HIP(hipHostGetDevicePointer((void**)&H->lat_out_dev, H->h_out, 0));
      H->lat_out_host = H->h_out;
    }
    double *th_dev = H->lat_th_dev, *out_dev = H->lat_out_dev;
    // every unit term lands in pinned memory; the host waits for them by
    // spinning on a sentinel (a NaN payload the kernel never writes: its
    // terms are finite or -inf) instead of a stream synchronisation, whose
    // wake-up is a sizeable share of a ~30 us call.  Every workgroup reads
    // theta before it writes its term, so the staging is free once all terms
    // are in; a launch error or a stall falls back to the stream (2 s)
    const size_t nu = (size_t)h->P * B;
    volatile uint64_t* hu = reinterpret_cast<volatile uint64_t*>(H->h_out);
    for (size_t i = 0; i < nu; ++i) hu[i] = LAT_SENTINEL;
    if ((rc = launch_chol_lat(h->lat_nb, h->d_jobs_fixed, B, h->P, th_dev, h->n_param, h->d_units, out_dev,
                              h->stream, km == 22, km == 24 ? 1 : km == 25 ? 2 : km == 23 ? 3 : 0)) < 0)
      return rc;
    if (rc == 0) {
      const auto t0 = std::chrono::steady_clock::now();
      size_t seen = 0;
      for (long spins = 0;; ++spins) {
        while (seen < nu && hu[seen] != LAT_SENTINEL) ++seen;
        if (seen == nu) break;
        if ((spins & 4095) == 4095) {
          const hipError_t q = hipStreamQuery(h->stream);
          if (q != hipSuccess && q != hipErrorNotReady)
            return set_err(EWH_E_HIP, std::string("chol_lat_kernel: ") + hipGetErrorString(q));
          if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
            EWH_HIP(hipStreamSynchronize(h->stream));
            for (seen = 0; seen < nu && hu[seen] != LAT_SENTINEL; ++seen) {
            }
            if (seen != nu) return set_err(EWH_E_HIP, "chol_lat_kernel: unit terms missing after the launch");
            break;
          }
        }
      }
      std::atomic_thread_fence(std::memory_order_acquire);
      // a unit whose dataflow wait ran out carries LAT_STALL_BITS: an error,
      // never a NaN lnL (the ABI promises finite values or -inf)
      for (size_t i = 0; i < nu; ++i)
        if (hu[i] == LAT_STALL_BITS) {
          (void)hipStreamSynchronize(h->stream);
          return set_err(EWH_E_HIP, "chol_lat_kernel: a dataflow wait of unit " + std::to_string(i) +
                                        " ran out (LAT_SPIN_MAX); no lnL was produced");
        }
      // lnL_b = sum over pulsars in pulsar order (reduce_units_kernel's fold)
      bool failed = false;
      for (int b = 0; b < B; ++b) {
        double s = 0.0;
        for (int p = 0; p < h->P; ++p) s += H->h_out[(size_t)p * B + b];
        out_host[b] = s;
        failed = failed || !std::isfinite(s);
      }
      // an fp64 pivot failure (-inf term) is refactored in double-double by
      // the batched path (refine_failed): take it for this call instead
      if (!failed) {
        H->last_split.assign(1, {0, (long long)H->P * B});
        H->last_B = B;
        h->last_B = B;
        return 0;
      }
      EWH_HIP(hipStreamSynchronize(h->stream));
    }
  }
  if ((rc = ensure_io(h, B))) return rc;
  DevCtx::Graph* hit = nullptr;
  for (auto& g : h->graphs)
    if (g.B == B && g.mode == h->kernel_mode && g.ht == H->h_theta && g.ho == H->h_out) hit = &g;
  if (hit) {
    hit->last_use = ++h->graph_clock;
    EWH_HIP(hipGraphLaunch(hit->exec, h->stream));
  } else {
    if ((rc = enqueue_single(H, h, B))) return rc;
  }
  EWH_HIP(hipStreamSynchronize(h->stream));
  std::memcpy(out_host, H->h_out, sizeof(double) * B);
  H->last_split.assign(1, {0, (long long)H->P * B});
  H->last_B = B;
  if (hit || h->corr) return 0;     // (correlated batches are long: launch overhead is immaterial)
  // capture for the next call of this size (buffers are sized now, so the
  // sequence makes no allocation or synchronous call)
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  if (hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) return 0;
  rc = enqueue_single(H, h, B);
  const hipError_t e = hipStreamEndCapture(h->stream, &graph);
  if (rc || e != hipSuccess || !graph) {
    if (graph) (void)hipGraphDestroy(graph);
    (void)hipGetLastError();
    return 0;                       // no graph: the eager path stays correct
  }
  const hipError_t ei = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  (void)hipGraphDestroy(graph);
  if (ei != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  if (h->graphs.size() >= GRAPH_CACHE) {
    auto lru = std::min_element(h->graphs.begin(), h->graphs.end(),
                                [](const DevCtx::Graph& a, const DevCtx::Graph& b) { return a.last_use < b.last_use; });
    (void)hipGraphExecDestroy(lru->exec);
    h->graphs.erase(lru);
  }
  h->graphs.push_back({B, h->kernel_mode, H->h_theta, H->h_out, exec, ++h->graph_clock});
  return 0;
}

}  // namespace

extern "C" {

int ewh_version(void) { return EWH_ABI_VERSION; }
int ewh_lat_b_max(void) { return LAT_B_MAX; }

const char* ewh_last_error(void) { return g_err.c_str(); }

int ewh_create(const ewh_pta_desc* d, const int32_t* device_ids, int32_t ndev, ewh_handle** out) {
  if (!out) return set_err(EWH_E_INVALID, "out is NULL");
  *out = nullptr;
  if (ndev < 0 || (ndev > 0 && !device_ids) || ndev > 64) return set_err(EWH_E_INVALID, "bad device list");
  int rc = validate(d);
  if (rc) return rc;
  int count = 0;
  EWH_HIP(hipGetDeviceCount(&count));
  std::vector<int> ids = ndev ? std::vector<int>(device_ids, device_ids + ndev) : std::vector<int>{0};
  for (int id : ids)
    if (id < 0 || id >= count) return set_err(EWH_E_INVALID, "device id " + std::to_string(id) + " out of range");
  ewh_handle* H = new ewh_handle();
  H->P = d->n_pulsar;
  H->n_param = d->n_param;
  H->psr_cols.resize(d->n_pulsar);
  for (int p = 0; p < d->n_pulsar; ++p) {
    const ewh_pulsar_desc& sd = d->pulsars[p];
    std::vector<int>& cols = H->psr_cols[p];
    auto add = [&](const ewh_pref& r) {
      if (r.idx >= 0) cols.push_back(r.idx);
    };
    for (int i = 0; i < sd.n_slot; ++i) add(sd.slots[i]);
    for (int e = 0; e < sd.n_spec; ++e) {
      add(sd.spec[e].p0);
      add(sd.spec[e].p1);
      add(sd.spec[e].p2);
    }
    for (int g = 0; g < sd.n_bgroup; ++g) add(sd.bgroup_idx[g]);
    if (d->common && d->common->spec)
      for (int g = 0; g < d->common->n_col; ++g) {
        add(d->common->spec[g].p0);
        add(d->common->spec[g].p1);
        add(d->common->spec[g].p2);
      }
    std::sort(cols.begin(), cols.end());
    cols.erase(std::unique(cols.begin(), cols.end()), cols.end());
  }
  std::vector<ProjCoef> proj(d->n_pulsar);
  for (int p = 0; p < d->n_pulsar; ++p) proj[p] = projection_coef(d->pulsars[p]);
  for (int id : ids) {
    DevCtx* c = nullptr;
    if ((rc = create_ctx(d, proj, id, &c))) {
      ewh_destroy(H);
      return rc;
    }
    H->ctx.push_back(c);
  }
  H->corr = H->ctx[0]->corr;
  // peer access between every context's device and the first one (both
  // directions: partial B-vectors and gathered kept blocks move device to
  // device); bit i of peer_mask records context i
  H->peer_mask = 1;
  for (size_t i = 1; i < ids.size(); ++i) {
    bool ok = ids[i] == ids[0];
    if (!ok) {
      int a = 0, b = 0;
      if (hipDeviceCanAccessPeer(&a, ids[i], ids[0]) == hipSuccess && hipDeviceCanAccessPeer(&b, ids[0], ids[i]) ==
                                                                             hipSuccess && a && b) {
        const bool a1 = peer_acquire(H, ids[i], ids[0]);
        const bool a2 = peer_acquire(H, ids[0], ids[i]);
        ok = a1 && a2;
      }
    }
    if (ok) H->peer_mask |= 1LL << i;
  }
  *out = H;
  return 0;
}

int ewh_transfer_stats(const ewh_handle* H, int64_t* h2d_bytes, int64_t* peer) {
  if (!H) return set_err(EWH_E_INVALID, "bad handle");
  if (h2d_bytes) *h2d_bytes = H->h2d_bytes;
  if (peer) *peer = H->peer_mask;
  return 0;
}

int ewh_refine_stats(ewh_handle* H, int64_t* checked, int64_t* refined) {
  if (!H) return set_err(EWH_E_INVALID, "bad handle");
  long long c = 0, r = 0;
  for (DevCtx* h : H->ctx) {
    EWH_HIP(hipSetDevice(h->device));
    // (the whole device: ewh_lnl_units_device runs the route on the caller's
    // stream, whose work must be counted before the reset)
    EWH_HIP(hipDeviceSynchronize());
    unsigned long long v[2] = {0, 0};
    if (h->d_ddstat) {
      EWH_HIP(hipMemcpy(v, h->d_ddstat, sizeof v, hipMemcpyDeviceToHost));
      EWH_HIP(hipMemset(h->d_ddstat, 0, sizeof v));
    }
    c += (long long)v[1];
    r += (long long)v[0];
  }
  if (checked) *checked = c;
  if (refined) *refined = r;
  return 0;
}

int ewh_num_devices(const ewh_handle* H) { return H ? (int)H->ctx.size() : 0; }

int ewh_set_fixed_white(ewh_handle* H, const double* values) {
  if (!H || !values) return set_err(EWH_E_INVALID, "bad arguments");
  for (DevCtx* h : H->ctx) {
    EWH_HIP(hipSetDevice(h->device));
    size_t off = 0;
    for (auto& ps : h->psr) {
      for (int i = 0; i < ps.n_slot; ++i)
        if (ps.slots[i].idx < 0) ps.slots[i].cval = values[off + i];
      off += ps.n_slot;
      if (ps.n_slot)
        EWH_HIP(hipMemcpyAsync(ps.d_slots, ps.slots.data(), sizeof(ewh_pref) * ps.n_slot, hipMemcpyHostToDevice,
                               h->stream));
    }
    EWH_HIP(hipStreamSynchronize(h->stream));
    drop_graphs(h);
    if (h->white_fixed) {
      int rc = setup_fixed(h);
      if (rc) return rc;
    }
  }
  return 0;
}

int ewh_set_kernel_mode(ewh_handle* H, int32_t mode) {
  if (!H || mode < 0 || mode > 39) return set_err(EWH_E_INVALID, "bad handle / mode");
#ifdef EWH_DEV
  constexpr bool dev_lib = true;   // mode 33 (the one-proposal C5 schedule with the diagonal launched apart)
#else
  constexpr bool dev_lib = false;
#endif
  if (mode != 0 && mode != 1 && mode != 2 && mode != 7 && mode != MODE_WIDE && mode != MODE_DD && !variant_built(mode) &&
      !((mode == 33 || mode == MODE_WIDE_R05A || (mode >= 35 && mode <= 39)) && dev_lib))
    return set_err(EWH_E_UNSUPPORTED, "kernel mode " + std::to_string(mode) +
                                          " is not built into this library (A/B variants: the dev library, make dev)");
  for (DevCtx* h : H->ctx) {
    h->kernel_mode = mode;
    (void)hipSetDevice(h->device);
    drop_graphs(h);
    const bool stage = mode != 19;   // dev mode 19: the register kernels' CSR spectrum prologue
    // MODE_DD on a pulsar whose S_lo was not kept (register widths): set up again
    bool need_lo = false;
    if (h->white_fixed)
      for (const auto& ps : h->psr) need_lo = need_lo || (!ps.d_Slo && dd_path(h, ps.fx_nb, true));
    if (stage != h->stage_spectra || need_lo) {
      h->stage_spectra = stage;
      if (h->white_fixed) {
        const int rc = setup_fixed(h);
        if (rc) return rc;
      }
    }
  }
  return 0;
}

double ewh_unit_cost(const ewh_handle* H, int32_t p) {
  if (!H || p < 0 || p >= H->P) return 0.0;
  return ctx_unit_cost(H->ctx[0], p);
}

int ewh_lnl_units_device(ewh_handle* H, const double* theta_dev, int32_t B, int64_t u_begin, int64_t u_end,
                         double* out_dev, void* stream) {
  if (!H || !theta_dev || !out_dev || B <= 0) return set_err(EWH_E_INVALID, "bad arguments");
  DevCtx* h = H->ctx[0];
  if (h->osmode) return set_err(EWH_E_UNSUPPORTED, "an optimal-statistic handle evaluates ewh_optstat only");
  int rc = ctx_units(h, theta_dev, B, u_begin, u_end, out_dev, (hipStream_t)stream, true);
  if (rc) return rc;
  H->last_split.assign(1, {std::max<int64_t>(0, u_begin), std::min<int64_t>((long long)H->P * B, u_end)});
  H->last_B = B;
  return 0;
}

int ewh_lnl_batch(ewh_handle* H, const double* theta_host, int32_t B, double* out_host) {
  if (!H || !theta_host || !out_host || B <= 0) return set_err(EWH_E_INVALID, "bad arguments");
  if (H->ctx[0]->osmode) return set_err(EWH_E_UNSUPPORTED, "an optimal-statistic handle evaluates ewh_optstat only");
  const int nd = (int)H->ctx.size(), np = H->n_param;
  int rc;
  H->h2d_bytes = 0;
  if (nd == 1 || H->corr) {
    // (single context: the batch's theta rows, read by the latency kernel
    // straight from the pinned staging or copied once; correlated: each
    // context's sample slice, or every pulsar partition its copy)
    if ((rc = ensure_pinned(&H->h_theta, &H->h_theta_cap, (size_t)B * std::max(1, np), &H->lat_th_host))) return rc;
    if (np > 0) std::memcpy(H->h_theta, theta_host, sizeof(double) * (size_t)B * np);
  }
  if (nd == 1) {
    H->h2d_bytes = (long long)sizeof(double) * B * np;
    return lnl_batch_single(H, H->ctx[0], B, out_host);
  }
  if (H->corr && B < nd) return lnl_batch_corr_pulsars(H, B, out_host);
  std::vector<std::pair<long long, long long>> split;
  if (H->corr) {
    // samples: contiguous slices (the cross-pulsar factorisation needs every
    // pulsar of a sample on one device)
    for (int i = 0; i < nd; ++i) split.push_back({(long long)B * i / nd, (long long)B * (i + 1) / nd});
  } else {
    std::vector<double> cost(H->P);
    for (int p = 0; p < H->P; ++p) cost[p] = ctx_unit_cost(H->ctx[0], p);
    split = unit_ranges(cost, B, nd);
  }
  if ((rc = ensure_pinned(&H->h_out, &H->h_out_cap, (size_t)B, &H->lat_out_host))) return rc;
  DevCtx* h0 = H->ctx[0];
  if (!H->corr) {
    // per-context partial sums are folded on the first device: a partial
    // B-vector per context there, one event per context
    EWH_HIP(hipSetDevice(h0->device));
    const size_t need = (size_t)nd * B;
    if (need > H->part_cap) {
      if (H->d_part) (void)hipFree(H->d_part);
      H->d_part = nullptr;
      H->part_cap = 0;
      hipError_t e = hipMalloc((void**)&H->d_part, need * sizeof(double));
      if (e != hipSuccess) return set_err(EWH_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
      H->part_cap = need;
    }
    while ((int)H->ev.size() < nd) {
      const int i = (int)H->ev.size();
      EWH_HIP(hipSetDevice(H->ctx[i]->device));
      hipEvent_t e;
      EWH_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      H->ev.push_back(e);
    }
  }
  for (int i = 0; i < nd; ++i) {
    DevCtx* h = H->ctx[i];
    const long long a = split[i].first, b = split[i].second;
    EWH_HIP(hipSetDevice(h->device));
    if (H->corr) {
      if (b <= a) continue;
      const int Bd = (int)(b - a);
      if ((rc = ensure_io(h, Bd))) return rc;
      if (np > 0)
        EWH_HIP(hipMemcpyAsync(h->d_theta, H->h_theta + (size_t)a * np, sizeof(double) * (size_t)Bd * np,
                               hipMemcpyHostToDevice, h->stream));
      H->h2d_bytes += (long long)sizeof(double) * Bd * np;
      if ((rc = ctx_units(h, h->d_theta, Bd, 0, (long long)H->P * Bd, h->d_out, h->stream, true))) return rc;
      EWH_HIP(hipMemcpyAsync(H->h_out + a, h->d_out, sizeof(double) * Bd, hipMemcpyDeviceToHost, h->stream));
    } else {
      // every context evaluates its unit range and sums it over its pulsars
      // (rows outside the range are zero) into a B-vector, which goes to the
      // first device; only B doubles ever come back to the host
      if ((rc = ensure_io(h, B))) return rc;
      // only the theta entries this context's units read (the host packs
      // context i + 1's while context i's copy and launches run)
      const long long nbytes = stage_theta_range(H, h, theta_host, B, a, b);
      if (nbytes < 0) return (int)nbytes;
      H->h2d_bytes += nbytes;
      if ((rc = ctx_units(h, h->d_theta, B, a, b, h->d_out, h->stream, true))) return rc;
      EWH_HIP(hipMemcpyPeerAsync(H->d_part + (size_t)i * B, h0->device, h->d_out, h->device, sizeof(double) * B,
                                 h->stream));
      EWH_HIP(hipEventRecord(H->ev[i], h->stream));
    }
  }
  if (!H->corr) {
    EWH_HIP(hipSetDevice(h0->device));
    for (int i = 1; i < nd; ++i) EWH_HIP(hipStreamWaitEvent(h0->stream, H->ev[i], 0));
    hipLaunchKernelGGL(fold_partials_kernel, dim3((B + 255) / 256), dim3(256), 0, h0->stream, H->d_part, nd, B,
                       h0->d_out);
    EWH_HIP(hipGetLastError());
    EWH_HIP(hipMemcpyAsync(H->h_out, h0->d_out, sizeof(double) * B, hipMemcpyDeviceToHost, h0->stream));
    EWH_HIP(hipStreamSynchronize(h0->stream));
  } else {
    for (int i = 0; i < nd; ++i) {
      if (split[i].second <= split[i].first) continue;
      EWH_HIP(hipSetDevice(H->ctx[i]->device));
      EWH_HIP(hipStreamSynchronize(H->ctx[i]->stream));
    }
  }
  std::memcpy(out_host, H->h_out, sizeof(double) * B);
  H->last_split = split;
  H->last_B = B;
  return 0;
}

int ewh_contract_device(ewh_handle* H, const double* theta_dev, int32_t B, void* stream) {
  if (!H || !theta_dev || B <= 0) return set_err(EWH_E_INVALID, "bad arguments");
  DevCtx* h = H->ctx[0];
  if (h->white_fixed || h->corr || h->osmode)
    return set_err(EWH_E_UNSUPPORTED, "ewh_contract_device: white noise must vary (uncorrelated / CURN handle)");
  EWH_HIP(hipSetDevice(h->device));
  int rc;
  if ((rc = ensure_var_scratch(h, B))) return rc;
  hipStream_t saved = h->stream;
  h->stream = (hipStream_t)stream;
  for (int p = 0; p < h->P && !rc; ++p)
    for (int c0 = 0; c0 < B && !rc; c0 += h->chunk) rc = run_white(h, p, theta_dev, h->n_param, c0, std::min(h->chunk, B - c0));
  h->stream = saved;
  return rc;
}

int ewh_keep_dim(const ewh_handle* H) {
  if (!H || !H->corr) return 0;
  return 16 * H->ctx[0]->keep;
}

int ewh_corr_partial_device(ewh_handle* H, const double* theta_dev, int32_t B, int32_t p_begin, int32_t p_end,
                            double* keep_dev, double* local_dev, void* stream) {
  if (!H || !H->corr || !theta_dev || !keep_dev || !local_dev || B <= 0 || p_begin < 0 || p_end > H->P ||
      p_begin > p_end)
    return set_err(EWH_E_INVALID, "bad arguments (needs a correlated-common-process handle)");
  DevCtx* h = H->ctx[0];
  EWH_HIP(hipSetDevice(h->device));
  int rc = corr_partial(h, theta_dev, B, p_begin, p_end, local_dev, keep_dev, (hipStream_t)stream);
  if (rc) return rc;
  EWH_HIP(hipGetLastError());
  return 0;
}

int ewh_corr_finish_device(ewh_handle* H, const double* theta_dev, int32_t B, const double* keep_dev,
                           const double* local_dev, double* out_dev, void* stream) {
  if (!H || !H->corr || !theta_dev || !keep_dev || !local_dev || !out_dev || B <= 0)
    return set_err(EWH_E_INVALID, "bad arguments (needs a correlated-common-process handle)");
  DevCtx* h = H->ctx[0];
  hipStream_t st = (hipStream_t)stream;
  EWH_HIP(hipSetDevice(h->device));
  int rc;
  if ((rc = ensure_units(h, B))) return rc;
  EWH_HIP(hipMemcpyAsync(h->d_units, local_dev, sizeof(double) * (size_t)H->P * B, hipMemcpyDeviceToDevice, st));
  if ((rc = corr_finish(h, theta_dev, B, keep_dev, h->d_units, st))) return rc;
  hipLaunchKernelGGL(reduce_units_kernel, dim3((B + 255) / 256), dim3(256), 0, st, h->d_units, H->P + 1, B, out_dev);
  EWH_HIP(hipGetLastError());
  H->last_split.assign(1, {0, (long long)H->P * B});
  H->last_B = B;
  h->last_B = B;
  return 0;
}

int ewh_optstat(ewh_handle* H, const double* theta_host, int32_t B, const double* phihat_host, double* rho_host,
                double* sig_host, double* os_host, double* os_sig_host) {
  if (!H) return set_err(EWH_E_INVALID, "bad arguments");
  return ctx_optstat(H->ctx[0], theta_host, B, phihat_host, rho_host, sig_host, os_host, os_sig_host);
}

int ewh_last_unit_terms(ewh_handle* H, double* out_host, int32_t B) {
  if (!H || !out_host || B != H->last_B || H->last_split.empty()) return set_err(EWH_E_INVALID, "no matching previous call");
  const int P = H->P, nd = (int)H->last_split.size();
  const bool by_samples = nd == 1 ? false : H->corr;
  std::memset(out_host, 0, sizeof(double) * (size_t)P * B);
  std::vector<double> tmp;
  for (int i = 0; i < nd; ++i) {
    DevCtx* h = H->ctx[i];
    const long long a = H->last_split[i].first, b = H->last_split[i].second;
    if (b <= a || !h->d_units) continue;
    EWH_HIP(hipSetDevice(h->device));
    EWH_HIP(hipStreamSynchronize(h->stream));
    EWH_HIP(hipDeviceSynchronize());
    if (nd == 1 && !H->corr) {
      EWH_HIP(hipMemcpy(out_host, h->d_units, sizeof(double) * (size_t)P * B, hipMemcpyDeviceToHost));
    } else if (by_samples || nd == 1) {
      const int Bd = nd == 1 ? B : (int)(b - a);
      const long long s0 = nd == 1 ? 0 : a;
      tmp.resize((size_t)P * Bd);
      EWH_HIP(hipMemcpy(tmp.data(), h->d_units, sizeof(double) * (size_t)P * Bd, hipMemcpyDeviceToHost));
      for (int p = 0; p < P; ++p)
        for (int k = 0; k < Bd; ++k) out_host[(size_t)p * B + s0 + k] = tmp[(size_t)p * Bd + k];
    } else {
      EWH_HIP(hipMemcpy(out_host + a, h->d_units + a, sizeof(double) * (size_t)(b - a), hipMemcpyDeviceToHost));
    }
  }
  return 0;
}

void ewh_destroy(ewh_handle* H) {
  if (!H) return;
  for (size_t i = 0; i < H->ev.size(); ++i) {
    (void)hipSetDevice(H->ctx[i]->device);
    (void)hipEventDestroy(H->ev[i]);
  }
  if (H->d_part) {
    (void)hipSetDevice(H->ctx[0]->device);
    (void)hipFree(H->d_part);
  }
  for (DevCtx* c : H->ctx) destroy_ctx(c);
  peer_release_all(H);
  if (H->h_theta) (void)hipHostFree(H->h_theta);
  if (H->h_out) (void)hipHostFree(H->h_out);
  delete H;
}

#ifdef EWH_DEV
// ---- dev library only (make dev): intermediate quantities for diagnostics ----
// G = T_aug^T N^-1 T_aug of pulsar p for samples [0, B) (B <= the varying-WN
// chunk), row-major ld x ld per sample; returns ld (or a negative code).
int ewh_dev_gram(ewh_handle* H, int32_t p, const double* theta_host, int32_t B, double* G_out) {
  DevCtx* h = H->ctx[0];
  if (p < 0 || p >= h->P || B <= 0) return set_err(EWH_E_INVALID, "bad arguments");
  int rc;
  EWH_HIP(hipSetDevice(h->device));
  const bool wf = h->white_fixed;
  h->white_fixed = false;
  rc = ensure_var_scratch(h, B);
  h->white_fixed = wf;
  if (rc) return rc;
  if (B > h->chunk) return set_err(EWH_E_INVALID, "B exceeds the varying-WN chunk");
  if ((rc = ensure_io(h, B))) return rc;
  if (h->n_param > 0)
    EWH_HIP(hipMemcpy(h->d_theta, theta_host, sizeof(double) * (size_t)B * h->n_param, hipMemcpyHostToDevice));
  if ((rc = run_white(h, p, h->d_theta, h->n_param, 0, B))) return rc;
  EWH_HIP(hipStreamSynchronize(h->stream));
  const int ld = h->psr[p].ld;
  EWH_HIP(hipMemcpy(G_out, h->d_G, sizeof(double) * (size_t)B * ld * ld, hipMemcpyDeviceToHost));
  return ld;
}

// the double-double G_hi / G_lo of gram_dd_units_kernel (the fp64-failure
// refinement, varying white noise) of pulsar p for samples [0, B); returns ld
int ewh_dev_gram_dd(ewh_handle* H, int32_t p, const double* theta_host, int32_t B, double* G_out, double* Glo_out) {
  DevCtx* h = H->ctx[0];
  if (p < 0 || p >= h->P || B <= 0 || h->white_fixed) return set_err(EWH_E_INVALID, "bad arguments");
  int rc;
  EWH_HIP(hipSetDevice(h->device));
  if ((rc = ensure_var_scratch(h, B))) return rc;
  if (B > h->chunk) return set_err(EWH_E_INVALID, "B exceeds the varying-WN chunk");
  if ((rc = ensure_io(h, B)) || (rc = ensure_units(h, B))) return rc;
  EWH_HIP(hipMemcpy(h->d_theta, theta_host, sizeof(double) * (size_t)B * h->n_param, hipMemcpyHostToDevice));
  if ((rc = run_white(h, p, h->d_theta, h->n_param, 0, B))) return rc;
  std::vector<int> lst(B + 1);
  lst[0] = B;
  for (int b = 0; b < B; ++b) lst[b + 1] = p * B + b;
  const size_t U = (size_t)(h->P + 1) * B;
  if ((rc = ensure_buf(h, &h->d_ddlist, &h->ddlist_cap, U + 1))) return rc;
  EWH_HIP(hipMemcpy(h->d_ddlist, lst.data(), sizeof(int) * (B + 1), hipMemcpyHostToDevice));
  const PsrHost& ps = h->psr[p];
  hipLaunchKernelGGL(gram_dd_units_kernel, dim3(ps.nb * (ps.nb + 1) / 2, std::min(B, 64)), dim3(256), 0, h->stream,
                     ps.dev, ps.d_Tlo, h->d_w, h->d_beta, h->d_ddlist + 1, h->d_ddlist, B, 0, h->d_G, h->d_Glo);
  EWH_HIP(hipStreamSynchronize(h->stream));
  const int ld = ps.ld;
  EWH_HIP(hipMemcpy(G_out, h->d_G, sizeof(double) * (size_t)B * ld * ld, hipMemcpyDeviceToHost));
  EWH_HIP(hipMemcpy(Glo_out, h->d_Glo, sizeof(double) * (size_t)B * ld * ld, hipMemcpyDeviceToHost));
  return ld;
}

// the cached reduced matrix S_p (fx_ld x fx_ld) and K_p of a fixed-WN handle; returns fx_ld
int ewh_dev_reduced(ewh_handle* H, int32_t p, double* S_out, double* K_out) {
  DevCtx* h = H->ctx[0];
  if (!h->white_fixed || p < 0 || p >= h->P) return set_err(EWH_E_INVALID, "bad arguments");
  EWH_HIP(hipSetDevice(h->device));
  EWH_HIP(hipDeviceSynchronize());
  const int n = h->psr[p].fx_ld;
  EWH_HIP(hipMemcpy(S_out, h->psr[p].d_S, sizeof(double) * (size_t)n * n, hipMemcpyDeviceToHost));
  EWH_HIP(hipMemcpy(K_out, h->d_fxK + p, sizeof(double), hipMemcpyDeviceToHost));
  return n;
}
#endif

}  // extern "C"
