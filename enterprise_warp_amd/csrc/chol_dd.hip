// chol_dd.hip — the factorisation in double-double for the
// bases the fp64 register kernels do not cover: the reduced matrix of a
// fixed-white-noise pulsar wider than 9 blocks (the reference's own
// system_noise_example: enterprise_models.py:256-338, 208 reduced columns)
// and every basis wider than 16 blocks (X_<n>_nfreqs models,
// enterprise_models.py:148-167, :436-468).
//
// Why: on ill-conditioned prior draws the fp64 factorisation of such a
// matrix carries errors of tens to thousands of times the strict lnL bound
// whatever its order of operations (tests/golden c1_system sample 0: the
// blocked LDL^T 15-50x, unblocked Cholesky 25-40x, enterprise's own LAPACK
// order 17x; c1_wide sample 6: the two-level panel's explicit 16x16 inverse
// 300x); the input matrix itself is held to double-double (the fixed-WN
// cache S = S_hi + S_lo from schur_kernel, the wide contraction's G_hi +
// G_lo), so the factorisation in double-double leaves the lnL within ~1
// strict of the exact value.
//
// Blocked right-looking Cholesky, one 512-thread workgroup per (pulsar,
// sample); the trailing matrix lives in a per-workgroup scratch as hi / lo
// planes (upper triangle + the lower halves of the 4x4 diagonal tiles), r
// last.  Panels of PW rows (16; 8 past 512 columns, for the LDS):
//   A. panel solve: U_k = U_kk^-T A_k, the panel's rows right of its
//      diagonal block, by forward substitution, one thread per column -> LDS
//      (an explicit inverse E = U_kk^-T, which parallelises over rows too,
//      lost 1e3 x strict on an ill-conditioned diagonal block even in
//      double-double: golden c1_wide sample 6);
//   B. trailing update A_ij -= sum_p U_pi U_pj over 4x4 tiles (one thread
//      per tile, products exact by fma, sums carried in double-double), and
//      -- lookahead -- wave 0 first updates the next panel's diagonal block
//      (2x2 tiles) and factors it (readlane pivots), while the other seven
//      waves update the rest.
// Two barriers per panel (the round-4 kernel: one per pivot, and the whole
// trailing triangle read and written through scratch at every pivot, ~300 MB
// per 384-column unit: 77.7 us per unit at B = 1024; profiles/r05a).
// log d_p summed per pivot; the last pivot is q = r^T N^-1 r - d^T Sigma^-1 d.
#include "ewarp_dev.h"

#include <cstdlib>

// every function below: error-free transformations -- no contraction of a
// product into a later sum (ewarp_dev.h, the double-double helpers)
#pragma clang fp contract(off)

namespace ewh_dev {
namespace {

constexpr int DD_THREADS = 512;

__device__ __forceinline__ dd dd_sub_mul(dd a, dd x, dd y) {   // a - x y
  const double p = x.hi * y.hi;
  const double pe = fma(x.hi, y.hi, -p) + (x.hi * y.lo + x.lo * y.hi);
  const dd s = dd_two_sum(a.hi, -p);
  return dd_fast(s.hi, s.lo + a.lo - pe);
}
// t -= x y, t = (th, tl) carried unnormalised (tl collects the rounding of
// each step; dd_two_sum(th, tl) at the end)
__device__ __forceinline__ void dd_acc_sub(double& th, double& tl, dd x, dd y) {
  const double p = x.hi * y.hi;
  const double e = fma(x.hi, y.hi, -p) + fma(x.hi, y.lo, x.lo * y.hi);
  const double s = th - p, bp = s - th;
  tl += ((th - (s - bp)) + (-p - bp)) - e;
  th = s;
}
// one wave's LDS writes visible to its own later reads (other lanes): the
// writes complete, and the compiler moves no LDS access across
__device__ __forceinline__ void lds_wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ dd ld2(const double2& v) { return {v.x, v.y}; }
__device__ __forceinline__ double2 st2(dd v) { return make_double2(v.hi, v.lo); }
__device__ __forceinline__ dd readlane_dd(dd x, int lane) { return {readlane_d(x.hi, lane), readlane_d(x.lo, lane)}; }

// row-major upper triangle of T x T tiles: idx -> (ti, tj)
__device__ __forceinline__ void tri_decode(int T, int idx, int& ti, int& tj) {
  const double b = 2.0 * T + 1.0;
  int i = (int)((b - sqrt(b * b - 8.0 * idx)) * 0.5);
  auto start = [&](int r) { return r * T - r * (r - 1) / 2; };
  while (i > 0 && start(i) > idx) --i;
  while (start(i + 1) <= idx) ++i;
  ti = i;
  tj = i + (idx - start(i));
}

template <int PW>
struct DdLds {
  // dynamic LDS: U [PW][n] | DG [PW][PW] | SC [PW] | phinv [n] | red [8]
  double2 *U, *DG, *SC, *ph;
  double* red;
  int* ctr;                  // the trailing update's tile counter
  __device__ DdLds(double2* base, int n) {
    U = base;
    DG = U + PW * n;
    SC = DG + PW * PW;
    ph = SC + PW;
    red = (double*)(ph + n);
    ctr = (int*)(red + 8);
  }
};

template <int PW>
size_t dd_lds(int n) { return (size_t)(PW * n + PW * PW + PW + n) * sizeof(double2) + 8 * sizeof(double) + 16; }

// 1 / sqrt(d) in double-double: the fp64 reciprocal square root and one
// Newton step y + y (1 - d y^2) / 2 with d y^2 formed in double-double (the
// step's own error ~ (3/8) e^2 with e ~ 1e-16).  Round 5 (r05j): replaces
// dd_div(1, dd_sqrt(d)) -- one IEEE sqrt and three IEEE divisions in every
// pivot of wave 0's serial chain
__device__ __forceinline__ dd dd_rsqrt(dd d) {
  const double y = rsqrt_fast(d.hi);
  const double t = y * y, te = fma(y, y, -t);
  const dd u = dd_mul(d, {t, te});
  const double e = (1.0 - u.hi) - u.lo;
  return dd_fast(y, y * (0.5 * e));
}

// Wave 0, lanes c < PW: factor the diagonal block DG (upper part valid) of
// the panel starting at r0; pivots r0 + p < n - 1 add log d_p to ldet (lane
// p's own term: the logs are taken after the chain, one per lane, and
// summed over the wave at the end) and must be positive; the pivot n - 1 is
// q.  Leaves the strict upper part of U_kk in DG and the scales 1/sqrt(d_p)
// in SC for the panel solve.
template <int PW>
__device__ __forceinline__ void dd_factor_diag(const DdLds<PW>& S, int r0, int n, int lane, double& ldet, bool& ok, double& qv) {
  dd a[PW];
#pragma unroll
  for (int r = 0; r < PW; ++r) a[r] = (lane < PW && r <= lane) ? ld2(S.DG[r * PW + lane]) : dd{0.0, 0.0};
  double my_d = 1.0, my_c = 0.0;                     // lane p: d_p.hi and d_p.lo / d_p.hi
#pragma unroll
  for (int p = 0; p < PW; ++p) {
    const dd d = readlane_dd(a[p], p);
    if (r0 + p == n - 1) {
      qv = d.hi + d.lo;
      if (lane == 0) S.SC[p] = st2({1.0, 0.0});
      continue;
    }
    ok = ok && d.hi > 0.0;
    const dd s = dd_rsqrt(d);
    if (lane == p) {
      my_d = d.hi;
      my_c = d.lo * (s.hi * s.hi);
    }
    if (lane == 0) S.SC[p] = st2(s);
    if (lane > p) a[p] = dd_mul(a[p], s);           // U[p][c], c > p
#pragma unroll
    for (int r = p + 1; r < PW; ++r) {
      const dd ur = readlane_dd(a[p], r);
      if (lane >= r) a[r] = dd_sub_mul(a[r], ur, a[p]);
    }
  }
  // publish U_kk (strict upper part) for the panel solve
#pragma unroll
  for (int p = 0; p < PW; ++p)
    if (lane > p && lane < PW) S.DG[p * PW + lane] = st2(a[p]);
  if (lane < PW) ldet += log(my_d) + my_c;           // (1, 0 for q and the lanes past PW)
  lds_wave_sync();
}

// RSOLVE (round 5): the panel solve column-oriented -- as soon as U[p][j] is
// formed it is subtracted from every later row's running sum -- instead of
// each row summing the earlier ones: the same dd_acc_sub terms in the same
// order per row (bit-identical), but 15 - p independent updates after each
// step instead of one dependent chain of p (the solve is one thread per
// column, so this chain was the panel's critical path).  RSOLVE = false: the
// round-5a form (dev mode 34).
template <int PW, bool RSOLVE>
__device__ __forceinline__ void chol_ddb_unit(const CholJob* __restrict__ jobs, int B, long long u, int b_off,
                              const double* __restrict__ theta, double* __restrict__ out_units,
                              double* __restrict__ scratch, long long scr_per_wg, double2* lds, int dbg) {
  // (theta: the unit's own row; dbg: dev timing probe only -- bit 0 skips the
  // trailing update, bit 1 the panel solve, bit 2 wave 0's diagonal chain;
  // the results are then meaningless.  0 in the product)
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  constexpr bool RSOLVE_STATIC = !RSOLVE;          // (dev mode 34: the r05a tile dealing too)
  // (uniform: the job's fields load into scalar registers, not 50 VGPRs)
  const int p_ = __builtin_amdgcn_readfirstlane((int)(u / B)), b = __builtin_amdgcn_readfirstlane((int)(u % B));
  const CholJob& J = jobs[p_];
  const int n = J.ld;
  const DdLds<PW> S(lds, n);
  const long long moff = (long long)(b - b_off) * J.mstride;
  const double* Shi = J.mats + moff;
  const double* Slo = J.mats_lo ? J.mats_lo + moff : nullptr;
  double* H = scratch + (long long)blockIdx.x * scr_per_wg;
  double* L = H + (long long)n * n;
  EWH_DCHECK(2LL * n * n <= scr_per_wg && n % 16 == 0 && n >= PW, "chol_dd scratch slot holds the unit");
  // phi^-1 per column in double-double (pads and r carry no entry: 0)
  double lphi = 0.0;
  for (int a = tid; a < n; a += DD_THREADS) {
    dd pinv = {0.0, 0.0};
    if (a < J.mreal && J.col_ptr[a] < J.col_ptr[a + 1]) {
      double ph = 0.0;
      for (int e = J.col_ptr[a]; e < J.col_ptr[a + 1]; ++e) ph += spec_phi_body(J.spec[e], theta);
      pinv = dd_div({1.0, 0.0}, {ph, 0.0});
      lphi += log(ph);
    }
    S.ph[a] = st2(pinv);
  }
  lphi = wave_sum(lphi);
  if (lane == 0) S.red[wave] = lphi;
  __syncthreads();
  lphi = 0.0;
#pragma unroll
  for (int w = 0; w < DD_THREADS / 64; ++w) lphi += S.red[w];
  // element (i, j) of the matrix before panel k = 0: S + phi^-1 on the diagonal
  auto src0 = [&](int i, int j) -> dd {
    const long long o = (long long)i * n + j;
    dd v = {Shi[o], Slo ? Slo[o] : 0.0};
    if (i == j) v = dd_add(v, ld2(S.ph[i]));
    return v;
  };
  double ldet = 0.0, qv = 0.0;
  bool ok = true;
  // panel 0's diagonal block
  if (wave == 0) {
    for (int e = lane; e < PW * PW; e += 64) {
      const int r = e / PW, c = e % PW;
      if (c >= r) S.DG[e] = st2(src0(r, c));
    }
    lds_wave_sync();
    dd_factor_diag<PW>(S, 0, n, lane, ldet, ok, qv);
  }
  __syncthreads();
  for (int r0 = 0; r0 + PW < n; r0 += PW) {
    const bool first = r0 == 0;
    const int t0 = r0 + PW, m = n - t0;
    if (tid == 0 && !RSOLVE_STATIC) *S.ctr = 0;      // (phase B's tile counter; nothing reads it in A)
    // A. panel solve by forward substitution, one thread per column j:
    // U[p][j] = s_p (A[r0 + p][j] - sum_{r < p} U_kk[r][p] U[r][j])
    for (int jj = tid; jj < ((dbg & 2) ? 0 : m); jj += DD_THREADS) {
      const int j = t0 + jj;
      EWH_DCHECK(j < n && (long long)(r0 + PW - 1) * n + j < (long long)n * n, "chol_dd panel solve: column in range");
      dd a[PW];
#pragma unroll
      for (int r = 0; r < PW; ++r) {
        const long long o = (long long)(r0 + r) * n + j;
        a[r] = first ? dd{Shi[o], Slo ? Slo[o] : 0.0} : dd{H[o], L[o]};
      }
      if constexpr (RSOLVE) {
        double hh[PW], ll[PW];
#pragma unroll
        for (int r = 0; r < PW; ++r) {
          hh[r] = a[r].hi;
          ll[r] = a[r].lo;
        }
#pragma unroll
        for (int p = 0; p < PW; ++p) {
          const dd up = dd_mul(dd_two_sum(hh[p], ll[p]), ld2(S.SC[p]));
          S.U[p * n + j] = st2(up);
#pragma unroll
          for (int r = p + 1; r < PW; ++r) dd_acc_sub(hh[r], ll[r], ld2(S.DG[p * PW + r]), up);
        }
      } else {
#pragma unroll
        for (int p = 0; p < PW; ++p) {
          double hh = a[p].hi, ll = a[p].lo;
#pragma unroll
          for (int r = 0; r < p; ++r) dd_acc_sub(hh, ll, ld2(S.DG[r * PW + p]), a[r]);
          a[p] = dd_mul(dd_two_sum(hh, ll), ld2(S.SC[p]));
          S.U[p * n + j] = st2(a[p]);
        }
      }
    }
    __syncthreads();
    // B. trailing update of [t0, n)^2; wave 0: the next diagonal block first
    const int T = m / 4;
    if (wave == 0) {
      constexpr int Q = PW / 2;                  // 2x2 tiles of the PW x PW block
      for (int e = lane; e < Q * (Q + 1) / 2; e += 64) {
        int qi, qj;
        tri_decode(Q, e, qi, qj);
        const int i0 = t0 + 2 * qi, j0 = t0 + 2 * qj;
        double ah[2][2], al[2][2];
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int y = 0; y < 2; ++y) {
            const dd v = first ? src0(i0 + x, j0 + y) : dd{H[(long long)(i0 + x) * n + j0 + y], L[(long long)(i0 + x) * n + j0 + y]};
            ah[x][y] = v.hi;
            al[x][y] = v.lo;
          }
#pragma unroll 1
        for (int p = 0; p < PW; ++p) {
          const dd ui[2] = {ld2(S.U[p * n + i0]), ld2(S.U[p * n + i0 + 1])};
          const dd uj[2] = {ld2(S.U[p * n + j0]), ld2(S.U[p * n + j0 + 1])};
#pragma unroll
          for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) dd_acc_sub(ah[x][y], al[x][y], ui[x], uj[y]);
        }
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int y = 0; y < 2; ++y) {
            const int r = 2 * qi + x, c = 2 * qj + y;
            if (c >= r) S.DG[r * PW + c] = st2(dd_two_sum(ah[x][y], al[x][y]));
          }
      }
      lds_wave_sync();
      if (!(dbg & 4)) dd_factor_diag<PW>(S, t0, n, lane, ldet, ok, qv);
    }
    // the rest of the trailing update, 64 tiles per grab from an LDS counter
    // (r05j; wave 0 joins after its chain -- the tiles were dealt to waves
    // 1-7 by a fixed stride before): per tile the same operations
    if (RSOLVE_STATIC ? wave != 0 : true) {
      constexpr int QD = PW / 4;                 // 4x4 tiles inside the next diagonal block
      const int ntiles = (dbg & 1) ? 0 : T * (T + 1) / 2;
      for (int gi = 0;; ++gi) {
        int idx;
        if constexpr (RSOLVE_STATIC) {
          idx = tid - 64 + gi * (DD_THREADS - 64);
          if (idx >= ntiles) break;
        } else {
          // (every lane of the wave is active here: one grab per wave, the
          // base broadcast from the lane that made it)
          EWH_DCHECK(__builtin_amdgcn_read_exec() == ~0ull, "chol_dd tile grab: every lane active");
          EWH_DCHECK(gi <= ntiles / 64 + 1, "chol_dd tile grab: iteration bound");
          int base = 0;
          if (lane == 0) base = atomicAdd(S.ctr, 64);
          base = __shfl(base, 0);
          if (base >= ntiles) break;
          idx = base + lane;
        }
        int ti = 0, tj = 0;
        if (idx < ntiles) tri_decode(T, idx, ti, tj);
        if (idx < ntiles && tj >= QD) {          // (tj < QD: wave 0's)
        const int i0 = t0 + 4 * ti, j0 = t0 + 4 * tj;
        EWH_DCHECK(ti <= tj && j0 + 3 < n && i0 >= t0, "chol_dd trailing tile inside the trailing triangle");
        double ah[4][4], al[4][4];
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
          for (int y = 0; y < 4; ++y) {
            const long long o = (long long)(i0 + x) * n + j0 + y;
            if (first) {
              const dd v = src0(i0 + x, j0 + y);
              ah[x][y] = v.hi;
              al[x][y] = v.lo;
            } else {
              ah[x][y] = H[o];
              al[x][y] = L[o];
            }
          }
#pragma unroll 1
        for (int p = 0; p < PW; ++p) {
          dd ui[4], uj[4];
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            ui[x] = ld2(S.U[p * n + i0 + x]);
            uj[x] = ld2(S.U[p * n + j0 + x]);
          }
#pragma unroll
          for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y) dd_acc_sub(ah[x][y], al[x][y], ui[x], uj[y]);
        }
#pragma unroll
        for (int x = 0; x < 4; ++x)
#pragma unroll
          for (int y = 0; y < 4; ++y) {
            const long long o = (long long)(i0 + x) * n + j0 + y;
            const dd v = dd_two_sum(ah[x][y], al[x][y]);
            H[o] = v.hi;
            L[o] = v.lo;
          }
        }
      }
    }
    __threadfence_block();
    __syncthreads();
  }
  if (wave == 0) ldet = wave_sum(ldet);              // (each lane holds its own pivots' logs)
  if (tid == 0) {
    double lnl = J.K[(long long)(b - b_off) * J.kstride] - 0.5 * qv - 0.5 * ldet - 0.5 * lphi;
    if (!ok || J.fail) lnl = -INFINITY;
    out_units[(long long)p_ * B + b] = lnl;
  }
  __syncthreads();                         // (the workgroup's next unit reuses LDS and scratch)
}

// list != NULL: the units are list[0 .. *count) (absolute unit indices, the
// verify step's flags); the grid loops over them (a workgroup exits at once
// when there are none).  list == NULL: units u0 + blockIdx.x.
template <int PW, bool RSOLVE = true>
__global__ __launch_bounds__(DD_THREADS) void chol_dd_kernel(const CholJob* __restrict__ jobs, int B, long long u0,
                                                             int b_off, const double* __restrict__ theta, int ldth,
                                                             double* __restrict__ out_units,
                                                             double* __restrict__ scratch, long long scr_per_wg,
                                                             const int* __restrict__ list,
                                                             const int* __restrict__ count, int dbg) {
  extern __shared__ __attribute__((aligned(16))) double2 dd_smem[];
  // one call site (the unit body is inlined once)
  const int cnt = list ? *count : (int)gridDim.x;
  EWH_DCHECK(!list || cnt >= 0, "chol_dd list count");
  for (int i = blockIdx.x; i < cnt; i += gridDim.x) {
    const long long u = list ? (long long)list[i] : u0 + i;
    chol_ddb_unit<PW, RSOLVE>(jobs, B, u, b_off, theta + (long long)(u % B) * ldth, out_units, scratch, scr_per_wg,
                              dd_smem, dbg);
  }
}

// The verify step: the forward (a) and reversed (b) fp64 factorisations of
// units [u0, u0 + n) agree to VERIFY_FRAC of the strict bound of the unit's
// own term (and on -inf), or the unit goes to the list for chol_dd_kernel.
// 1/16: at 1/4 (to r05i) two fp64 orders that agreed while both were off let
// 5 of the system model's 4096 prior draws through at up to 4.4x strict from
// the all-double-double value; at 1/16 the largest difference is 0.72x strict
// on those draws and 0.24x on the 372-column pulsar's 1024, for 53 % / 26 %
// of units refined instead of 48 % / 23 % (scripts/verify_calibrate.sh,
// profiles/r05j/verify_calibrate).  Tighter fractions buy nothing measurable:
// the residual is the double-double kernel's own floor.
constexpr double VERIFY_FRAC = 0.0625;
__global__ __launch_bounds__(256) void verify_units_kernel(const double* __restrict__ a, const double* __restrict__ b,
                                                           long long u0, long long n, double frac,
                                                           int* __restrict__ list, int* __restrict__ count,
                                                           unsigned long long* __restrict__ total) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (total && i == 0) atomicAdd(total + 1, (unsigned long long)n);     // (ewh_refine_stats: units checked)
  if (i >= n) return;
  const long long u = u0 + i;
  const double x = a[u], y = b[u];
  const bool fx = x - x == 0.0, fy = y - y == 0.0;           // finite
  // (round 6: a non-finite term of either order is refactored too -- the two
  // agreeing on -inf is a rounding failure of both wherever the exact Sigma
  // is positive definite; with a == b this is the failure scan of
  // refine_failed)
  const bool bad = frac < 0.0 || !fx || !fy || fabs(x - y) > frac * (1e-6 + 1e-10 * fabs(x));
  if (bad) {
    const int slot = atomicAdd(count, 1);
    EWH_DCHECK(slot < n, "verify list slot within the units checked");
    list[slot] = (int)u;
    if (total) atomicAdd(total, 1ull);    // (ewh_refine_stats: units refined)
  }
}

__global__ void count_units_kernel(unsigned long long* __restrict__ total, long long n) {
  if (threadIdx.x == 0) {
    atomicAdd(total, (unsigned long long)n);
    atomicAdd(total + 1, (unsigned long long)n);
  }
}

constexpr int DD_PW_WIDE = 8;            // panel rows past DD_LD_PW16 columns (LDS)
constexpr int DD_LD_PW16 = 512;

template <int PW>
void launch_dd(const CholJob* jobs, int B, long long u0, int b_off, const double* theta, int ldth, double* units,
               double* scr, long long scr_per_wg, unsigned grid, const int* list, const int* count, int ld,
               hipStream_t st, bool r05a) {
  int dbg = 0;
#ifdef EWH_DEV
  if (const char* e = getenv("EWARP_DD_SKIP")) dbg = atoi(e);   // (dev timing probe, scripts only)
#endif
  if (r05a)
    hipLaunchKernelGGL(HIP_KERNEL_NAME(chol_dd_kernel<PW, false>), dim3(grid), dim3(DD_THREADS), dd_lds<PW>(ld), st,
                       jobs, B, u0, b_off, theta, ldth, units, scr, scr_per_wg, list, count, dbg);
  else
    hipLaunchKernelGGL(HIP_KERNEL_NAME(chol_dd_kernel<PW, true>), dim3(grid), dim3(DD_THREADS), dd_lds<PW>(ld), st,
                       jobs, B, u0, b_off, theta, ldth, units, scr, scr_per_wg, list, count, dbg);
}

int launch_dd_any(const CholJob* jobs, int B, long long u0, int b_off, const double* theta, int ldth, double* units,
                  double* scr, long long scr_per_wg, unsigned grid, const int* list, const int* count, int ld,
                  hipStream_t st, bool r05a) {
  if (ld <= DD_LD_PW16)
    launch_dd<16>(jobs, B, u0, b_off, theta, ldth, units, scr, scr_per_wg, grid, list, count, ld, st, r05a);
  else
    launch_dd<DD_PW_WIDE>(jobs, B, u0, b_off, theta, ldth, units, scr, scr_per_wg, grid, list, count, ld, st, r05a);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_err(EWH_E_HIP, std::string("chol_dd_kernel: ") + hipGetErrorString(e));
}

}  // namespace

int set_dd_attributes() {
  if (hipFuncSetAttribute((const void*)chol_dd_kernel<16, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)dd_lds<16>(DD_LD_PW16)) != hipSuccess ||
      hipFuncSetAttribute((const void*)chol_dd_kernel<DD_PW_WIDE, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)dd_lds<DD_PW_WIDE>(WIDE_LD_MAX)) != hipSuccess ||
      hipFuncSetAttribute((const void*)chol_dd_kernel<16, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)dd_lds<16>(DD_LD_PW16)) != hipSuccess ||
      hipFuncSetAttribute((const void*)chol_dd_kernel<DD_PW_WIDE, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)dd_lds<DD_PW_WIDE>(WIDE_LD_MAX)) != hipSuccess)
    return set_err(EWH_E_HIP, "hipFuncSetAttribute(chol_dd_kernel) failed");
  return 0;
}

int launch_count_units(unsigned long long* total, long long n, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(count_units_kernel, dim3(1), dim3(64), 0, st, total, n);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_err(EWH_E_HIP, std::string("count_units_kernel: ") + hipGetErrorString(e));
}

int launch_verify_units(const double* a, const double* b, long long u0, long long n, int* list, int* count,
                        unsigned long long* total, hipStream_t st, bool all) {
  if (n <= 0) return 0;
  double frac = all ? -1.0 : VERIFY_FRAC;
#ifdef EWH_DEV
  if (const char* e = getenv("EWARP_VERIFY_FRAC")) frac = atof(e);   // (dev calibration only)
#endif
  hipLaunchKernelGGL(verify_units_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, b, u0, n, frac,
                     list, count, total);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_err(EWH_E_HIP, std::string("verify_units_kernel: ") + hipGetErrorString(e));
}

long long dd_scratch_per_wg(int ld) { return 2LL * ld * ld; }

int launch_chol_dd(const CholJob* jobs, int B, long long u0, long long n, int b_off, const double* theta, int ldth,
                   double* units, double* scr, long long scr_per_wg, long long cap, int ld, hipStream_t st, bool r05a) {
  for (long long o = 0; o < n; o += cap) {   // one scratch slot per workgroup of a launch
    const int rc = launch_dd_any(jobs, B, u0 + o, b_off, theta, ldth, units, scr, scr_per_wg,
                                 (unsigned)std::min(cap, n - o), nullptr, nullptr, ld, st, r05a);
    if (rc) return rc;
  }
  return 0;
}

int launch_chol_dd_list(const CholJob* jobs, int B, int b_off, const double* theta, int ldth, double* units,
                        double* scr, long long scr_per_wg, long long cap, const int* list, const int* count, int ld,
                        hipStream_t st, bool r05a) {
  return launch_dd_any(jobs, B, 0LL, b_off, theta, ldth, units, scr, scr_per_wg, (unsigned)cap, list, count, ld, st,
                       r05a);
}

}  // namespace ewh_dev
