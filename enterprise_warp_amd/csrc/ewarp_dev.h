// ewarp_dev.h — device-side types, helpers and kernel templates shared by the
// translation units of libewarp_hip.so (split so hipcc builds them in parallel):
//   ewarp_hip.hip     host side (C ABI), non-template kernels
//   chol_small.hip    chol_mfma_kernel<NB <= 9> (register-resident factorisation)
//   chol_partial.hip  chol_mfma_kernel<..., KEEP> (correlated common process)
//   chol_big.hip      chol_big_kernel<NB 10..16>
//   contract.hip      contract_mfma_kernel / contract2_kernel
//   contract_wide.hip contract_xr_kernel / contract_wide_kernel (bases past 16 blocks)
// See ewarp_hip.hip for the formulation.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "ewarp_hip.h"

namespace ewh_dev {

// thread-local error message of the C ABI (defined in ewarp_hip.hip)
int set_err(int code, const std::string& msg);

#define EWH_HIP(expr)                                                          \
  do {                                                                         \
    hipError_t e_ = (expr);                                                    \
    if (e_ != hipSuccess)                                                      \
      return ::ewh_dev::set_err(EWH_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// Device-side invariant checks of the debug build (`make debug`: -DEWH_DEBUG,
// build/libewarp_hip_debug.so; SURVEY.md §5's sanitizer row for device code).
// A violated check prints its site, block and thread, then traps -- a bounded
// failure with a location instead of a hang or a silent out-of-bounds access.
// Sites: every work-grab / spin loop carries an iteration bound (and the
// grab a full exec mask), and LDS / scratch / operand indices are checked
// against their allocations in chol_dd, chol_wide and contract_xr.  The
// product and dev builds compile the checks away.
#ifdef EWH_DEBUG
#define EWH_DCHECK(cond, what)                                                                           \
  do {                                                                                                   \
    if (!(cond)) {                                                                                       \
      printf("EWH_DCHECK failed: %s (%s:%d) block %d,%d thread %d\n", what, __FILE__, __LINE__,          \
             (int)blockIdx.x, (int)blockIdx.y, (int)threadIdx.x);                                        \
      __builtin_trap();                                                                                  \
    }                                                                                                    \
  } while (0)
#else
#define EWH_DCHECK(cond, what) \
  do {                         \
  } while (0)
#endif

constexpr int MFMA_NB_MAX = 9;
constexpr int CONTRACT2_NB_MAX = 13;
constexpr int default_waves(int nb) { return nb <= 8 ? 2 : 1; }

typedef double v4d __attribute__((ext_vector_type(4)));

// ----------------------------------------------------------------------------
// device helpers
// ----------------------------------------------------------------------------
// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, typename F>
__host__ __device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

__device__ __forceinline__ double pref_val(const ewh_pref& r, const double* th) {
  return r.idx >= 0 ? th[r.idx] : r.cval;
}

// Device form of one spectral entry (built from ewh_spec_entry at create).
// phi is evaluated as one exp of a sum of logs:
//   POWERLAW  A^2/(12 pi^2) fyr^(g-3) f^-g df = exp(a + 2 ln10 lgA + (g-3) ln fyr - g ln f)
//   TURNOVER  A^2/(12 pi^2) fyr^-3 ((f+fc)/fyr)^-g df
//             = exp(a + 2 ln10 lgA - 3 ln fyr - g (ln(f+fc) - ln fyr)),  fc = 10^fc if fc < 0
//   FREESPEC  10^(2 rho) = exp(2 ln10 rho)
//   CONST     v0
// with a = ln(df / (12 pi^2)); the same quantities as [ent] utils.powerlaw,
// the reference's powerlaw_bpl (enterprise_models.py:553-563) and
// [ent] gp_priors.free_spectrum, re-associated (relative error ~1e-14).
struct DSpec {
  int kind, col;
  int i0, i1, i2, pad_;
  double v0, v1, v2;     // constant values of the three parameters
  double a, lnf, lnfyr, f;
};

__device__ __forceinline__ double dpar(int idx, double cval, const double* th) {
  return idx >= 0 ? th[idx] : cval;
}

constexpr double LN10 = 2.302585092994045684;

// spec_phi_body: the arithmetic; spec_phi: an out-of-line copy for the schur and
// LDS-Cholesky kernels (ROCm 7.2 clang crashes in the CGSCC inliner when one
// inlined copy serves both); the register-resident kernels inline the body
// (a call there reserves a scratch frame the unrolled factorisation then
// spills into).
template <int DUMMY = 0>
__device__ __forceinline__ double spec_phi_body(const DSpec& s, const double* th) {
  switch (s.kind) {
    case EWH_SPEC_POWERLAW: {
      const double lgA = dpar(s.i0, s.v0, th), gam = dpar(s.i1, s.v1, th);
      return exp(s.a + 2.0 * LN10 * lgA + (gam - 3.0) * s.lnfyr - gam * s.lnf);
    }
    case EWH_SPEC_TURNOVER: {
      const double lgA = dpar(s.i0, s.v0, th), gam = dpar(s.i1, s.v1, th);
      double fc = dpar(s.i2, s.v2, th);
      if (fc < 0) fc = exp(LN10 * fc);
      return exp(s.a + 2.0 * LN10 * lgA - 3.0 * s.lnfyr - gam * (log(s.f + fc) - s.lnfyr));
    }
    case EWH_SPEC_FREESPEC:
      return exp(2.0 * LN10 * dpar(s.i0, s.v0, th));
    case EWH_SPEC_CONST:
      return s.v0;
    default:
      return __builtin_nan("");
  }
}

static __device__ __noinline__ double spec_phi(const DSpec& s, const double* th) { return spec_phi_body(s, th); }

// running log-determinant without a log per term: product of frexp mantissas
// (each in [0.5, 1): >= 2^-1000 after 1000 terms, no underflow) + exponent sum.
struct LogAcc {
  double mant = 1.0;
  int ex = 0;
  __device__ __forceinline__ void add(double x) {
    mant *= __builtin_amdgcn_frexp_mant(x);   // <= 1000 terms: no renormalisation needed
    ex += __builtin_amdgcn_frexp_exp(x);
  }
  __device__ __forceinline__ double value() const { return log(mant) + ex * 0.69314718055994530942; }
};

__device__ __forceinline__ double readlane_d(double x, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), lane);
  return __hiloint2double(hi, lo);
}

// 1/sqrt(a): hardware estimate + two Newton steps (~1 ulp).
__device__ __forceinline__ double rsqrt_nr(double a) {
  double y = __builtin_amdgcn_rsq(a);
  const double h = 0.5 * a;
  double t = fma(-h * y, y, 0.5);
  y = fma(y, t, y);
  t = fma(-h * y, y, 0.5);
  return fma(y, t, y);
}

// XCD-aware unit order: the dispatcher deals workgroup b to XCD b % 8, so
// XCD x gets the contiguous unit range [x q, (x+1) q) (q = n / 8; the n % 8
// tail maps to itself).  Units are pulsar-major, so each pulsar's reduced
// matrix is fetched into ~one XCD's L2 instead of all eight.
__device__ __forceinline__ long long xcd_unit(unsigned b, unsigned n) {
  const unsigned q = n >> 3;
  return b < (q << 3) ? (long long)(b & 7) * q + (b >> 3) : (long long)b;
}

// 1/a: hardware estimate + two Newton steps (~1 ulp).
__device__ __forceinline__ double rcp_nr(double a) {
  double y = __builtin_amdgcn_rcp(a);
  double e = fma(-a, y, 1.0);
  y = fma(y, e, y);
  e = fma(-a, y, 1.0);
  return fma(y, e, y);
}

// x / a with one cubic correction: y = rcp(a) (|e| = |1 - a y| < 2^-24),
// x / a = x y (1 + e + e^2) + O(e^3).  t = x y forms beside e, so the chain
// after the estimate is e -> s -> result (3 ops; x * rcp_nr(a) is 5) and the
// whole quotient is 5 fp64 VALU ops instead of 6.  ~1 ulp.
__device__ __forceinline__ double div_fast(double x, double a) {
  const double y = __builtin_amdgcn_rcp(a);
  const double e = fma(-a, y, 1.0);
  const double t = x * y;
  const double s = fma(e, e, e);
  return fma(t, s, t);
}

// 1/sqrt(a) with one cubic correction: e = 1 - a y^2,
// a^-1/2 = y (1 + e/2 + 3e^2/8) + O(e^3).  6 fp64 VALU ops (rsqrt_nr is 8).
__device__ __forceinline__ double rsqrt_fast(double a) {
  const double y = __builtin_amdgcn_rsq(a);
  const double e = fma(-(a * y), y, 1.0);
  const double s = e * fma(0.375, e, 0.5);
  return fma(y, s, y);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// 256-thread block sum; `scratch` holds >= 4 doubles.
static __device__ double block_sum256(double v, double* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[w] = v;
  __syncthreads();
  double t = scratch[0] + scratch[1] + scratch[2] + scratch[3];
  __syncthreads();
  return t;
}

// ----------------------------------------------------------------------------
// double-double helpers (Knuth TwoSum, TwoProd by fma; Dekker / Bailey
// normalisation): value = hi + lo with |lo| <= ulp(hi) / 2.
// Every error-free transformation is compiled with floating-point
// contraction off (`#pragma clang fp contract(off)`, round 6): hipcc's device
// default (-ffp-contract=fast) fused `s = hi + x * y` into one fma while the
// TwoSum error term still used the separately rounded product, which left
// every "double-double" kernel (gram_dd, schur, chol_dd) only about fp64-
// accurate -- the ~15x strict floor of the device's double-double twin
// against the CPU double-double reference on C3 prior draws, and indefinite
// C4 refinements (ISA: v_fma_f64 in place of v_add_f64)
// ----------------------------------------------------------------------------
struct dd {
  double hi, lo;
};
__device__ __forceinline__ dd dd_two_sum(double a, double b) {
#pragma clang fp contract(off)
  const double s = a + b, bp = s - a;
  return {s, (a - (s - bp)) + (b - bp)};
}
__device__ __forceinline__ dd dd_fast(double a, double b) {   // |a| >= |b|
#pragma clang fp contract(off)
  const double s = a + b;
  return {s, b - (s - a)};
}
__device__ __forceinline__ dd dd_add(dd x, dd y) {
#pragma clang fp contract(off)
  const dd s = dd_two_sum(x.hi, y.hi);
  return dd_fast(s.hi, s.lo + x.lo + y.lo);
}
// x + y with both parts TwoSum-ed (the accurate double-double sum: a
// relative error of ~2^-106 of |x + y| even under cancellation, which the
// sloppy dd_add above does not bound)
__device__ __forceinline__ dd dd_add_ieee(dd x, dd y) {
#pragma clang fp contract(off)
  dd s = dd_two_sum(x.hi, y.hi);
  const dd t = dd_two_sum(x.lo, y.lo);
  s = dd_fast(s.hi, s.lo + t.hi);
  return dd_fast(s.hi, s.lo + t.lo);
}
__device__ __forceinline__ dd dd_mul(dd x, dd y) {
#pragma clang fp contract(off)
  const double p = x.hi * y.hi;
  return dd_fast(p, fma(x.hi, y.hi, -p) + (x.hi * y.lo + x.lo * y.hi));
}
__device__ __forceinline__ dd dd_div(dd x, dd y) {          // one Newton correction of x.hi / y.hi
#pragma clang fp contract(off)
  const double q = x.hi / y.hi;
  const dd r = dd_add(x, dd_mul({-q, 0.0}, y));
  return dd_fast(q, r.hi / y.hi);
}
__device__ __forceinline__ dd dd_sqrt(dd x) {
#pragma clang fp contract(off)
  const double r = sqrt(x.hi);
  const dd e = dd_add(x, dd_mul({-r, 0.0}, {r, 0.0}));
  return dd_fast(r, e.hi / (2.0 * r));
}

// ----------------------------------------------------------------------------
// per-pulsar device tables
// ----------------------------------------------------------------------------
constexpr int CT_ROWS = 32;   // TOA rows per contraction tile (8 MFMA k-steps); T_aug is padded by this many zero rows
constexpr int CT_GROUP = 2;   // contract2: tiles per accumulation group (a power of two)
constexpr int CT_SINGLE = 0, CT_BLOCKED = 1, CT_TWOSUM = 2;   // contract2 accumulation forms

struct PsrDev {
  int n_toa, m, ld, nb;      // varying layout: T_aug is n_toa x ld, r at ld-1
  int n_epoch;
  const double* T;           // n_toa x ld row-major
  const double* sig2;        // toaerr^2
  const int* efac_slot;
  const int* equad_slot;
  const ewh_pref* slots;
  const int* ep_start;
  const int* ep_stop;
  const int* ep_slot;
  int n_bgroup;              // theta-dependent chromatic basis groups (0: none)
  const int* col_bgroup;     // ld entries, -1 = fixed column
  const double* ln_chrom;    // n_toa: ln(1400 / nu)
  const ewh_pref* bgroup;    // n_bgroup: chromatic index per group
  const int* toa_ep;         // n_toa + CT_ROWS: 2 e + (last TOA of e), -1 = no epoch (pad rows -1)
};

// One factorisation job: (pulsar, sample) -> matrix + diagonal update.
struct CholJob {
  const double* mats;        // matrix of sample b at mats + (b - b_off) * mstride
  long long mstride;         // 0: one matrix shared by every sample
  int ld;                    // leading dimension (= 16 * NB)
  int mreal;                 // columns with a phi entry (0..mreal-1); r at ld-1
  const int* col_ptr;        // CSR of spectral entries over mreal columns
  const DSpec* spec;
  const double* K;           // additive constant, K[(b - b_off) * kstride]
  int kstride;
  int fail;                  // 1: lead block not positive definite -> -inf
  // fixed white noise: columns sharing one spectrum (the sin / cos pair of a
  // frequency) -- rep[a] = the first column with the same entries, ulist =
  // the nu representatives; the prologue then forms each spectrum once
  const int* rep = nullptr;
  const int* ulist = nullptr;
  int nu = 0;
  // the same, staged for the register kernels' prologue: one record per
  // distinct spectrum with its entries inline (URec), and per column the
  // record it takes (urep, -1 = no entry); theta is read from LDS.  One
  // global-load level instead of four (ulist -> col_ptr -> spec -> theta).
  // NULL: the CSR path (a spectrum with more than URec::NE entries)
  const struct URec* urec = nullptr;
  const int* urep = nullptr;
  // the theta entries the records reference, staged alone (their DSpec
  // indices are positions in this list); 0: the whole theta row is staged
  int ntidx = 0;
  int tidx[16] = {};
  // the low part of a double-double matrix (chol_dd_kernel; same stride as
  // mats), or NULL
  const double* mats_lo = nullptr;
  // the reversed verify pass's input fl(hi + 2 lo), formed once where the
  // matrix is shared by every sample (mstride 0: the fixed-WN cache), or NULL
  // (the pass then forms it from mats and mats_lo at every load)
  const double* mats_rev = nullptr;
};

// one distinct spectrum of a fixed-WN job: phi = sum of its ne entries
struct URec {
  static constexpr int NE = 3;
  DSpec e[NE];
  int ne, pad_[3];
};
constexpr int STAGE_THETA_MAX = 512;   // theta row staged in LDS up to this many parameters
constexpr int TIDX_MAX = 16;           // CholJob::tidx

// ----------------------------------------------------------------------------
// fp64 MFMA contraction G = T_aug^T W T_aug - sum_e beta_e s_e s_e^T
// One 256-thread workgroup (4 waves) per sample; the NB(NB+1)/2 upper 16x16
// output blocks are dealt round-robin to the waves; 32-row TOA tiles are
// staged in LDS and shared by the four waves.
// ----------------------------------------------------------------------------
template <int NB>
__global__ __launch_bounds__(256) void contract_mfma_kernel(PsrDev P, const double* __restrict__ w,
                                                            const double* __restrict__ beta,
                                                            const double* __restrict__ s,
                                                            const double* __restrict__ fac,
                                                            double* __restrict__ G) {
  constexpr int LD = 16 * NB;
  constexpr int NBLK = NB * (NB + 1) / 2;
  constexpr int SLOTS = (NBLK + 3) / 4;
  extern __shared__ __attribute__((aligned(16))) double smem[];
  double* tile = smem;                     // CT_ROWS x LD
  double* wt = smem + CT_ROWS * LD;        // CT_ROWS weights
  const int bl = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4, c = lane & 15;

  int bi[SLOTS], bj[SLOTS];
  bool valid[SLOTS];
#pragma unroll
  for (int sl = 0; sl < SLOTS; ++sl) {
    int blk = wave + 4 * sl;
    valid[sl] = blk < NBLK;
    int i = 0;
    while (blk >= NB - i && i < NB - 1) { blk -= NB - i; ++i; }
    bi[sl] = i;
    bj[sl] = i + blk;
  }
  v4d acc[SLOTS];
#pragma unroll
  for (int sl = 0; sl < SLOTS; ++sl) acc[sl] = v4d{0.0, 0.0, 0.0, 0.0};

  // pass 0: TOA rows (weights w), pass 1: epoch rows (weights -beta)
  for (int pass = 0; pass < 2; ++pass) {
    const int nrows = pass == 0 ? P.n_toa : P.n_epoch;
    const double* src = pass == 0 ? P.T : s + (long long)bl * P.n_epoch * LD;
    const double* wsrc = pass == 0 ? w + (long long)bl * P.n_toa : beta + (long long)bl * P.n_epoch;
    const double wsign = pass == 0 ? 1.0 : -1.0;
    for (int t0 = 0; t0 < nrows; t0 += CT_ROWS) {
      const int rows = min(CT_ROWS, nrows - t0);
      if (pass == 0 && P.n_bgroup) {   // theta-dependent chromatic columns: scale per TOA
        for (int idx = threadIdx.x; idx < CT_ROWS * LD; idx += 256) {
          const int r = idx / LD, cc = idx - r * LD;
          double v = idx < rows * LD ? src[(long long)t0 * LD + idx] : 0.0;
          const int g = P.col_bgroup[cc];
          if (g >= 0 && r < rows) v *= fac[((long long)bl * P.n_bgroup + g) * P.n_toa + t0 + r];
          tile[idx] = v;
        }
      } else {
        for (int idx = threadIdx.x; idx < CT_ROWS * LD; idx += 256)
          tile[idx] = idx < rows * LD ? src[(long long)t0 * LD + idx] : 0.0;
      }
      if (threadIdx.x < CT_ROWS) wt[threadIdx.x] = threadIdx.x < rows ? wsign * wsrc[t0 + threadIdx.x] : 0.0;
      __syncthreads();
#pragma unroll
      for (int kk = 0; kk < CT_ROWS / 4; ++kk) {
        const int row = 4 * kk + q;
        const double wr = wt[row];
        const double* trow = tile + row * LD + c;
#pragma unroll
        for (int sl = 0; sl < SLOTS; ++sl) {
          if (valid[sl]) {
            const double a = wr * trow[16 * bi[sl]];
            const double b = trow[16 * bj[sl]];
            acc[sl] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[sl], 0, 0, 0);
          }
        }
      }
      __syncthreads();
    }
  }
  // epilogue: C/D layout lane -> (row q + 4r, col c); mirror to the lower half,
  // unit diagonal on pad columns (m .. LD-2) so they factor as identity.
  double* out = G + (long long)bl * LD * LD;
#pragma unroll
  for (int sl = 0; sl < SLOTS; ++sl) {
    if (!valid[sl]) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * bi[sl] + q + 4 * r, col = 16 * bj[sl] + c;
      double v = acc[sl][r];
      if (row == col && row >= P.m && row < LD - 1) v = 1.0;
      out[(long long)row * LD + col] = v;
      out[(long long)col * LD + row] = v;
    }
  }
}

// ----------------------------------------------------------------------------
// fp64 MFMA contraction, pipelined (default for pulsars without theta-dependent
// basis columns).  One 256-thread workgroup (4 waves) per sample:
//   G = T_aug^T W T_aug - sum_e beta_e s_e s_e^T,  s_e = sum_{t in e} w_t T_aug[t].
//  * TOA tiles of CT_ROWS rows are copied global -> LDS by global_load_lds
//    (16 B per lane, 1 KiB per wave-instruction; T_aug is contiguous and padded
//    by CT_ROWS zero rows) into two buffers: tile i+1 streams in while the
//    MFMAs run on tile i.
//  * Wave WAVE owns the upper blocks blk = WAVE + 4 sl (compile-time, so the
//    operand set is known): per k-step it reads T[row][16 j + c] once per block
//    column j it touches and forms w_row * T[row][16 i + c] once per block row i.
//  * ECORR: the epoch sums s_e are accumulated from the same LDS tile (thread
//    = column; epochs are contiguous TOA runs that may straddle tiles) and
//    written to a per-sample scratch; a second pass runs them through the same
//    MFMA loop with weights -beta_e.  No second read of T from HBM.
// ----------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;
// global-address-space view of a device pointer: loads through it are
// global_load (vmcnt only), not flat_load, whose lgkmcnt share makes every
// ds_bpermute wait (s_waitcnt lgkmcnt(0)) for all matrix loads in flight
typedef const __attribute__((address_space(1))) double* gdptr;

// Contraction block ownership (contract2_body).  The upper blocks are put in
// a tiled order -- tiles of th x tw blocks, row-major over the tiles and
// within one -- and wave v of WS takes a contiguous run of that order (the
// first NBLK % WS waves one block more).  (th, tw) is picked at compile time
// to minimise the per-k-step work of the busiest wave: one LDS read per block
// column it touches and one multiply by the row weight per block row it
// owns.  Round 4 dealt the blocks round-robin (blk = v + WS sl): C4's 13
// blocks over 8 waves then read 13 columns and scaled 10 rows per k-step
// (23 instructions beside 12 MFMAs, and 52 operand registers, which spilled
// the blocked accumulator); tiled runs: 12 (C2's 9 blocks: 15 -> 8).
struct CtOrd {
  int ij[136];                        // i * 64 + j of the pos-th block (NB <= 16)
};
constexpr CtOrd ct_order(int nb, int th, int tw) {
  CtOrd o{};
  int n = 0;
  for (int I = 0; I < nb; I += th)
    for (int J = (I / tw) * tw; J < nb; J += tw)
      for (int i = I; i < I + th && i < nb; ++i)
        for (int j = J; j < J + tw && j < nb; ++j)
          if (j >= i) o.ij[n++] = i * 64 + j;
  return o;
}
// Runs: wave v of ws takes nblk / ws blocks, and the nblk % ws remainder goes
// one each to the LAST waves (LATE, round 5): waves 0 .. ceil(LD / 64) - 1
// also carry the ECORR epoch sums (threads tid < LD) and wave 0 the per-tile
// weight staging, so they take the shorter runs (round 4: the first waves
// took the extra blocks -- C2's 45 blocks put 6 MFMA blocks AND the epoch
// sums on waves 0-2; dev mode 35 keeps that order for the A/B).  Used where
// the accumulator is TwoSum-compensated, round 6; single until then (contract2_late: NB <= 9)
constexpr int ct_run_start(int nblk, int ws, int v, bool late = true) {
  const int b = nblk / ws, x = nblk % ws;
  return late ? v * b + (v > ws - x ? v - (ws - x) : 0) : v * b + (v < x ? v : x);
}
constexpr int ct_run_len(int nblk, int ws, int v, bool late = true) {
  const int b = nblk / ws, x = nblk % ws;
  return b + ((late ? v >= ws - x : v < x) ? 1 : 0);
}
constexpr int ct_cost(int nb, int ws, int th, int tw, bool late = true) {
  const CtOrd o = ct_order(nb, th, tw);
  const int nblk = nb * (nb + 1) / 2;
  int worst = 0;
  for (int v = 0; v < ws; ++v) {
    bool col[16] = {}, row[16] = {};
    const int s0 = ct_run_start(nblk, ws, v, late), n = ct_run_len(nblk, ws, v, late);
    for (int s = s0; s < s0 + n; ++s) {
      row[o.ij[s] >> 6] = col[o.ij[s] >> 6] = col[o.ij[s] & 63] = true;
    }
    int c = 0;
    for (int k = 0; k < nb; ++k) c += (col[k] ? 1 : 0) + (row[k] ? 1 : 0);
    worst = c > worst ? c : worst;
  }
  return worst;
}
constexpr int ct_shape(int nb, int ws, bool late = true) {   // th * 64 + tw
  int best = 1 << 30, shape = 64 + nb;
  for (int th = 1; th <= 6; ++th)
    for (int tw = 1; tw <= nb; ++tw) {
      const int c = ct_cost(nb, ws, th, tw, late);
      if (c < best) {
        best = c;
        shape = th * 64 + tw;
      }
    }
  return shape;
}
// the (i * 64 + j) of slot sl of wave v under shape SH
constexpr int ct_blk(int nb, int ws, int sh, int v, int sl, bool late = true) {
  return ct_order(nb, sh >> 6, sh & 63).ij[ct_run_start(nb * (nb + 1) / 2, ws, v, late) + sl];
}
// does wave v touch block index j as a block row (A operand) / at all?
constexpr bool ct_uses_row(int nb, int ws, int sh, int v, int j, bool late = true) {
  for (int sl = 0; sl < ct_run_len(nb * (nb + 1) / 2, ws, v, late); ++sl)
    if ((ct_blk(nb, ws, sh, v, sl, late) >> 6) == j) return true;
  return false;
}
constexpr bool ct_uses(int nb, int ws, int sh, int v, int j, bool late = true) {
  for (int sl = 0; sl < ct_run_len(nb * (nb + 1) / 2, ws, v, late); ++sl) {
    const int b = ct_blk(nb, ws, sh, v, sl, late);
    if ((b >> 6) == j || (b & 63) == j) return true;
  }
  return false;
}

// WAVE / W: the physical wave and waves per workgroup (tile copies, the
// per-tile weights); VW / WS: the virtual wave that picks the output blocks
// (blocks VW + WS sl) and the virtual waves per sample -- WS = W SPLIT when a
// sample's blocks are split over SPLIT workgroups (contract2_kernel).
// RSEP (round 5; the caller guarantees no ECORR and m <= 16 (NB - 1)): the
// last block column holds only r and pad columns, so the MFMAs form the Gram
// of the first NG = NB - 1 blocks only (C4: 78 instead of 91 blocks, -14 %),
// and d = T^T W r is summed by VALU from the staged tile -- one FMA per
// (row, column) on the last DW waves (column tid - 64 (W - DW)), blocked like
// the Gram; r^T W r comes from wn_weights_kernel (rho).  The epilogue writes
// block column NB - 1 itself: d, zeros, the pads' unit diagonal and rho.
template <int NB, int WAVE, int W, int VW = WAVE, int WS = W, int COMP = CT_BLOCKED, bool LATE = true,
          bool RSEP = false>
__device__ __forceinline__ void contract2_body(const PsrDev& P, const double* __restrict__ wrow,
                                               const double* __restrict__ brow, double* __restrict__ srow,
                                               double* __restrict__ Gout, const double* __restrict__ rho = nullptr) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int LD = 16 * NB;
  constexpr int NG = RSEP ? NB - 1 : NB;             // blocks the MFMAs form
  constexpr int NBLK = NG * (NG + 1) / 2;
  constexpr int SH = ct_shape(NG, WS, LATE);          // block ownership: tiled runs (ct_order)
  constexpr int SLOTS = ct_run_len(NBLK, WS, VW, LATE);
  constexpr int DW = RSEP ? (16 * NG + 63) / 64 : 0;  // the d waves (the last DW of W)
  constexpr bool DWAVE = RSEP && WAVE >= W - DW;
  static_assert(!RSEP || (DW <= W && WS == W), "r-separated contraction: one workgroup per sample");
  constexpr int TILE = CT_ROWS * LD;                 // doubles per tile
  constexpr int CHUNKS = TILE * 8 / 1024;            // 1-KiB glds pieces per tile (4 NB), dealt round-robin to the W waves
  static_assert(CHUNKS * 1024 == TILE * 8, "tile must split into pieces of 1 KiB");
  // LDS: [2][TILE] tiles | [2][CT_ROWS] weights | [2][CT_ROWS] epoch-sum
  // weights | [2][CT_ROWS] int flush epoch ids | [2] int flush masks
  const int tid = threadIdx.x, lane = tid & 63, q = lane >> 4, c = lane & 15;
  double* const wbase = smem + 2 * TILE;
  double* const ewbase = wbase + 2 * CT_ROWS;
  int* const ebase = (int*)(ewbase + 2 * CT_ROWS);
  int* const fmbase = ebase + 2 * CT_ROWS;

  // blocked accumulation: each group of CT_GROUP tiles
  // (CT_GROUP x 32 TOA rows) is summed by the MFMAs into a fresh accumulator
  // acc, which is then added into the running sum hi (CT_BLOCKED), or into hi
  // + lo by TwoSum (CT_TWOSUM, dev A/B); G = hi (+ lo) at the end.  A single
  // fp64 accumulator over all rows (CT_SINGLE) lost up to ~30x the strict
  // bound of lnL on ill-conditioned prior draws through the timing-model /
  // red-noise near-degeneracy (tests/golden c4_small sample 0: 4.0 vs
  // enterprise's 2.3 strict); per group the error grows only over CT_GROUP x
  // 32 rows, and the sum of the groups over n / 64 terms (restated on the
  // host, c4_small prior draws in strict units: single -2.1 / -27 / -8.6,
  // blocked -1.1 / -4.3 / -0.2, TwoSum -0.9 / 1.2 / 0.3 on samples 0 / 1 / 5,
  // against enterprise's -2.3 / -195 / -41).
  v4d acc[SLOTS > 0 ? SLOTS : 1], hi[SLOTS > 0 ? SLOTS : 1], lo[SLOTS > 0 ? SLOTS : 1];
#pragma unroll
  for (int sl = 0; sl < SLOTS; ++sl) {
    acc[sl] = v4d{0.0, 0.0, 0.0, 0.0};
    hi[sl] = v4d{0.0, 0.0, 0.0, 0.0};
    lo[sl] = v4d{0.0, 0.0, 0.0, 0.0};
  }
  // RSEP: d of column dc (the d waves), blocked like the Gram
  const int dc = DWAVE ? min(tid - 64 * (W - DW), 16 * NG - 1) : 0;
  double dacc = 0.0, dhi = 0.0, dlo = 0.0;
  auto flush = [&]() {
    if constexpr (COMP == CT_SINGLE) return;
    if constexpr (DWAVE) {
      if constexpr (COMP == CT_TWOSUM) {        // (d compensated like the Gram)
        const double sum = dhi + dacc, bp = sum - dhi;
        dlo += (dhi - (sum - bp)) + (dacc - bp);
        dhi = sum;
      } else {
        dhi += dacc;
      }
      dacc = 0.0;
    }
    static_for<0, SLOTS>([&](auto SL) {
      constexpr int sl = decltype(SL)::value;
      static_for<0, 4>([&](auto R) {
        constexpr int r = decltype(R)::value;
        if constexpr (COMP == CT_TWOSUM) {
          const double a = hi[sl][r], b = acc[sl][r];
          const double sum = a + b, bp = sum - a;
          lo[sl][r] += (a - (sum - bp)) + (b - bp);
          hi[sl][r] = sum;
        } else {
          hi[sl][r] += acc[sl][r];
        }
        acc[sl][r] = 0.0;
      });
    });
  };

  const bool ecorr = !RSEP && P.n_epoch > 0;       // (RSEP: none, by the caller's choice)
  double eacc = 0.0;                                 // running s_e of column `tid`
  // pass 0: TOA rows (weights w); pass 1: epoch rows (weights -beta)
  for (int pass = 0; pass < (ecorr ? 2 : 1); ++pass) {
    const bool epochs = pass == 0 && ecorr;
    const int nrows = pass == 0 ? P.n_toa : P.n_epoch;
    const double* src = pass == 0 ? P.T : srow;
    const double* wsrc = pass == 0 ? wrow : brow;
    const double wsign = pass == 0 ? 1.0 : -1.0;
    const int ntile = (nrows + CT_ROWS - 1) / CT_ROWS;
    auto issue = [&](int it) {
      const char* g = (const char*)(src + (long long)it * TILE) + lane * 16;
      char* l = (char*)(smem + (it & 1) * TILE);
#pragma unroll
      for (int k = WAVE; k < CHUNKS; k += W)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(g + k * 1024), (lds_void_t*)(l + k * 1024), 16, 0, 0);
    };
    // the tile's weights and epoch flags: wave 0 only (a compile-time branch,
    // no exec mask), loaded unconditionally from a clamped index and BEFORE
    // the tile's global_load_lds, so the wait for them is a counted vmcnt at
    // their use (the LDS store at the end of the iteration), never a
    // vmcnt(0) that would also wait for the next tile's DMA
    double wraw = 0.0, rraw = 0.0;
    int ev = -1;
    auto small = [&](int it) {
      if constexpr (WAVE == 0) {
        const int t = it * CT_ROWS + (lane & (CT_ROWS - 1));
        wraw = wsrc[min(t, nrows - 1)];
        ev = pass == 0 ? P.toa_ep[t] : -1;
        if constexpr (RSEP) rraw = P.T[(long long)min(t, nrows - 1) * LD + LD - 1];
      }
    };
    // staged per tile by wave 0: the Gram weights; the epoch-sum weights
    // (w on rows inside an epoch, 0 elsewhere); the mask of rows that close
    // an epoch and, in mask order, the epochs they close.  The epoch-sum loop
    // then runs on registers and one scalar mask: no per-row LDS round trip.
    auto stage = [&](int buf, int it) {
      if constexpr (WAVE == 0) {
        const int t = it * CT_ROWS + lane;
        const double w = (lane < CT_ROWS && t < nrows) ? wsign * wraw : 0.0;
        const bool fl = lane < CT_ROWS && ev >= 0 && (ev & 1);
        const unsigned long long fmask = __ballot(fl);
        if (lane < CT_ROWS) {
          wbase[buf * CT_ROWS + lane] = w;
          // (RSEP, no ECORR: the epoch-sum weights' slot carries w r, d's row weights)
          ewbase[buf * CT_ROWS + lane] = RSEP ? w * rraw : ev >= 0 ? w : 0.0;
        }
        if (fl) ebase[buf * CT_ROWS + __builtin_amdgcn_mbcnt_lo((unsigned)fmask, 0u)] = ev >> 1;
        if (lane == 0) fmbase[buf] = (int)(unsigned)fmask;
      }
    };
    small(0);
    issue(0);
    stage(0, 0);
    __syncthreads();
    for (int it = 0; it < ntile; ++it) {
      const int cur = it & 1;
      if (it + 1 < ntile) {
        small(it + 1);
        issue(it + 1);
      }
      const double* tile = smem + cur * TILE;
      const double* wt = wbase + cur * CT_ROWS;
#pragma unroll
      for (int kk = 0; kk < CT_ROWS / 4; ++kk) {
        const int row = 4 * kk + q;
        const double wr = wt[row];
        const double* trow = tile + row * LD + c;
        double tv[NG], av[NG];
        static_for<0, NG>([&](auto J) {
          constexpr int j = decltype(J)::value;
          if constexpr (ct_uses(NG, WS, SH, VW, j, LATE)) tv[j] = trow[16 * j];
          if constexpr (ct_uses_row(NG, WS, SH, VW, j, LATE)) av[j] = wr * tv[j];
        });
        static_for<0, SLOTS>([&](auto SL) {
          constexpr int blk = ct_blk(NG, WS, SH, VW, decltype(SL)::value, LATE);
          constexpr int bi = blk >> 6, bj = blk & 63;
          acc[decltype(SL)::value] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[bi], tv[bj], acc[decltype(SL)::value], 0, 0, 0);
        });
      }
      if (epochs && tid < LD) {                      // epoch sums of column tid
        // rows outside an epoch carry weight 0 (T is finite: fma(0, t, s) = s
        // exactly), so the running sum is a plain FMA chain over the tile,
        // its operands read 8 rows per LDS round trip; a row that closes an
        // epoch (bit of the wave-uniform mask) stores the sum and resets it.
        // (Interleaving the chain with the k-steps' MFMAs measured no faster
        // on C2 and 5 % slower on C4: more live registers.)
        const double* tcol = tile + tid;
        const double* ew = ewbase + cur * CT_ROWS;
        const int* fe = ebase + cur * CT_ROWS;
        const unsigned fm = (unsigned)__builtin_amdgcn_readfirstlane(fmbase[cur]);
        int nf = 0;
        // (4 rows per trip beside the blocked accumulator's second register
        // set, which leaves no room for 8)
        constexpr int ER = COMP != CT_SINGLE ? 4 : 8;
#pragma unroll
        for (int r0 = 0; r0 < CT_ROWS; r0 += ER) {
          double tc[ER], wc[ER];
#pragma unroll
          for (int i = 0; i < ER; ++i) {
            tc[i] = tcol[(r0 + i) * LD];
            wc[i] = ew[r0 + i];
          }
#pragma unroll
          for (int i = 0; i < ER; ++i) {
            eacc = fma(wc[i], tc[i], eacc);
            if ((fm >> (r0 + i)) & 1u) {
              const int e = __builtin_amdgcn_readfirstlane(fe[nf]);
              srow[(long long)e * LD + tid] = eacc;
              eacc = 0.0;
              ++nf;
            }
          }
        }
      }
      if constexpr (DWAVE) {                         // d of column dc: this tile's rows
        const double* ewr = ewbase + cur * CT_ROWS;
        constexpr int DR = COMP != CT_SINGLE ? 4 : 8;     // rows per LDS trip (registers, as the epoch sums)
#pragma unroll
        for (int r0 = 0; r0 < CT_ROWS; r0 += DR) {
          double tc[DR], wc[DR];
#pragma unroll
          for (int i = 0; i < DR; ++i) {
            tc[i] = tile[(r0 + i) * LD + dc];
            wc[i] = ewr[r0 + i];
          }
#pragma unroll
          for (int i = 0; i < DR; ++i) dacc = fma(wc[i], tc[i], dacc);
        }
      }
      if ((it & (CT_GROUP - 1)) == CT_GROUP - 1 || it + 1 == ntile) flush();
      if (it + 1 < ntile) stage(cur ^ 1, it + 1);
      __syncthreads();                               // drains the glds of tile it+1 (vmcnt(0))
    }
    if (pass == 0 && ecorr && tid < LD) {
      // pad rows [n_epoch, whole tiles) of the epoch pass: zero, so a value a
      // previous pulsar / sample left in the shared scratch never meets the
      // zero weight of the pad rows (0 * inf = NaN)
      const int epad = ((P.n_epoch + CT_ROWS - 1) / CT_ROWS) * CT_ROWS;
      for (int e = P.n_epoch; e < epad; ++e) srow[(long long)e * LD + tid] = 0.0;
    }
    if (pass == 0 && ecorr) __threadfence_block();   // s_e rows visible to the epoch pass
    __syncthreads();
  }
  // epilogue: C/D layout lane -> (row q + 4r, col c); mirror to the lower half,
  // unit diagonal on pad columns (m .. LD-2) so they factor as identity.
  if constexpr (DWAVE) {
    // block column NB - 1: d in column LD - 1, zeros in the pad columns
    // [16 NG, LD - 1) (their rows too); the d wave of column 0 also writes
    // the last diagonal block: unit diagonal on the pads, rho at the corner
    const int a = tid - 64 * (W - DW);
    if (a < 16 * NG) {
      const double d = COMP == CT_SINGLE ? dacc : COMP == CT_TWOSUM ? dhi + dlo : dhi;
      Gout[(long long)a * LD + LD - 1] = d;
      Gout[(long long)(LD - 1) * LD + a] = d;
#pragma unroll
      for (int pc = 16 * NG; pc < LD - 1; ++pc) {
        Gout[(long long)a * LD + pc] = 0.0;
        Gout[(long long)pc * LD + a] = 0.0;
      }
    }
    if (WAVE == W - DW) {
#pragma unroll
      for (int e = lane; e < 256; e += 64) {
        const int row = 16 * NG + (e >> 4), col = 16 * NG + (e & 15);
        Gout[(long long)row * LD + col] = row == LD - 1 && col == LD - 1 ? rho[blockIdx.x] : row == col ? 1.0 : 0.0;
      }
    }
  }
  static_for<0, SLOTS>([&](auto SL) {
    constexpr int blk = ct_blk(NG, WS, SH, VW, decltype(SL)::value, LATE);
    constexpr int bi = blk >> 6, bj = blk & 63;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * bi + q + 4 * r, col = 16 * bj + c;
      constexpr int sl = decltype(SL)::value;
      double v = COMP == CT_TWOSUM ? hi[sl][r] + lo[sl][r] : COMP == CT_BLOCKED ? hi[sl][r] : acc[sl][r];
      if (row == col && row >= P.m && row < LD - 1) v = 1.0;
      Gout[(long long)row * LD + col] = v;
      Gout[(long long)col * LD + row] = v;
    }
  });
}

// W = 4 or 8 waves per workgroup (8: half the accumulators per wave, so the
// narrow NB = 9 kernel fits 4 waves per SIMD and the wide NB = 13 one 2).
template <int NB, int W, int COMP = CT_BLOCKED, bool LATE = true, bool RSEP = false>
__global__ __launch_bounds__(64 * W) void contract2_kernel(PsrDev P, const double* __restrict__ w,
                                                           const double* __restrict__ beta, double* __restrict__ s,
                                                           long long s_stride, double* __restrict__ G,
                                                           const double* __restrict__ rho) {
  const int bl = blockIdx.x;
  const double* wrow = w + (long long)bl * P.n_toa;
  const double* brow = beta + (long long)bl * P.n_epoch;
  double* srow = s + (long long)bl * s_stride;
  double* Gout = G + (long long)bl * 16 * NB * 16 * NB;
  const int wv = threadIdx.x >> 6;
  static_for<0, W>([&](auto WV) {
    constexpr int wave = decltype(WV)::value;
    if (wv == wave) contract2_body<NB, wave, W, wave, W, COMP, LATE, RSEP>(P, wrow, brow, srow, Gout, rho);
  });
}
// the accumulation per width: blocked from 10 blocks on (C4's 13: the same
// registers as the single accumulator plus one set -- 2 waves per SIMD as
// before); below, the single accumulator meets the per-sample accuracy bound
// (c2_small, the C2 bench draws) and the extra set would halve C2's occupancy
// (4 -> 2 waves per SIMD).  (Round 4 first used TwoSum at 10+ blocks: three
// accumulator sets, so 11+ blocks had to split a sample over two workgroups;
// C4 5.44 k evals/s, vs 6.51 k with one accumulator.)  Dev kernel mode 30:
// TwoSum at every width up to 10 blocks (A/B).
// Round 6: TwoSum groups up to 10 blocks (C2's 9), blocked from 11 on.  The
// single accumulator C2 had kept since round 4 left 36 of its 4096 bench prior
// draws less accurate than enterprise's own fp64 order (at most 15x) against
// the double-double twin; TwoSum: none (worst 0.59), for 17.6 -> 20.8 ms per
// batch (scripts/c2_accum_ab.py, profiles/r06i).  Past 10 blocks the third
// accumulator set does not fit one workgroup per sample (round 4: C4 split
// over two workgroups, -16 %)
constexpr int contract2_comp(int nb) { return nb >= 11 ? CT_BLOCKED : CT_TWOSUM; }

// ----------------------------------------------------------------------------
// batched factorisation, MFMA register-blocked: one wave (64 lanes) per unit.
// The upper triangle of the LD x LD matrix (LD = 16 NB) is held as 16x16
// blocks in the v_mfma_f64_16x16x4_f64 C/D layout (lane l, reg r <-> row
// (l>>4) + 4r, col l&15).  A = U^T U (upper, as LAPACK dpotrf 'U' behind
// scipy cho_factor) by a blocked LDL^T: per block row bb the 16x16 diagonal
// block is eliminated (panel), the rest of the block row becomes
// V = L^-1 A_bj = E^T A_bj by four MFMAs per block (E = L^-T, built by the
// panel's column operations), the rows are scaled to U = D^-1/2 V, and the
// trailing blocks take A_ij -= U_bi^T U_bj by four MFMAs each with no data
// movement -- register s of a C/D-layout block IS the MFMA A / B operand of
// k-slice s.
//
// Three phases keep at most 26 blocks live for NB = 8 (36 in a plain
// right-looking order): (1) factor block rows 0..H-1 (H = NB/2) with the
// trailing update restricted to those rows; (2) load the trailing A22
// triangle and apply the H panel rows to it; (3) factor A22.  Same
// arithmetic, re-ordered (left-looking at the 2x2 block level).
// ----------------------------------------------------------------------------
template <int NB, bool FULL = false>
struct Split {
  // FULL (dev A/B, one wave per SIMD): the whole triangle resident, plain
  // right-looking order (phases 2 and 3 empty)
  static constexpr int H = FULL ? NB : NB == 8 ? 3 : NB / 2;
  static constexpr int M = NB - H;                    // A22 block order
  static constexpr int n1 = H * NB - H * (H - 1) / 2; // blocks (i < H, j >= i)
  static constexpr int n2 = M * (M + 1) / 2;          // blocks (H <= i <= j)
  static constexpr int i1(int i, int j) { return i * NB - (i * (i - 1)) / 2 + (j - i); }
  static constexpr int i2(int i, int j) { return (i - H) * M - ((i - H) * (i - H - 1)) / 2 + (j - i); }
};

// A -= U_i^T U_j : four f64 MFMAs.  For the f64 MFMAs of gfx940+ the last
// (blgp) field is the neg modifier (bit 0 negates A: `neg:[1,0,0]`), so no
// v_xor per negated operand.
__device__ __forceinline__ void syrk_update(v4d& C, const v4d& Ui, const v4d& Uj) {
#pragma unroll
  for (int sk = 0; sk < 4; ++sk) C = __builtin_amdgcn_mfma_f64_16x16x4f64(Ui[sk], Uj[sk], C, 0, 0, 1);
}

// lane (q, c) <- lane (q, K) of its 16-lane row (DPP row_newbcast, gfx90a+):
// one v_mov_b64_dpp (64-bit DPP takes row_newbcast; with bound_ctrl there is
// no `old` operand to materialise).
template <int K>
__device__ __forceinline__ double row_newbcast(double x) {
  const long v = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(long, x), 0x150 + K, 0xf, 0xf, true);
  return __builtin_bit_cast(double, v);
}

// One pivot k = 4 KR + KQ of the panel as fused DP-ALU DPP multiply-adds,
// each ONE v_fmac_f64_dpp whose src0 is read from lane k of its 16-lane row
// (row_newbcast: column k of the lane's row):
//  * row update A[q+4r][c] += A[q+4r][k] * nw of register KR in the 16-lane
//    rows q > KQ (row_mask) and, with FULLROWS (the one-level panel of round
//    2, dev A/B only), of every register r > KR;
//  * with DOE the column operation E[q+4r][c] += E[q+4r][k] * nwm on the
//    registers r <= KR (nwm is 0 in the lanes c <= k).
// Hazards the compiler cannot see inside the asm: (1) a DPP source must be
// written >= 2 wait states before it is read -- one statement per pivot, and
// the next pivot's statement needs nw, whose chain (readlane of this
// statement's output, rcp, 3 fma) lies in between; the first pivot of a
// sub-panel (NOP) follows the compiler's E initialisation or the sub-panel
// MFMA's copy-out, hence its s_nop; (2) E is an MFMA operand (V = E^T A)
// right after the last column operation (k = 14): a trailing s_nop covers
// VALU-write -> MFMA-read.  Only live registers (A, E) are written, so no
// in-flight MFMA reads them as a dead source.
template <int K, int KR, int KQ, bool DOE, bool NOP, bool FULLROWS>
__device__ __forceinline__ void pivot_fused(v4d& A, v4d& E, double nw, double nwm) {
  double a0 = A[0], a1 = A[1], a2 = A[2], a3 = A[3];
  double e0 = E[0], e1 = E[1], e2 = E[2], e3 = E[3];
  constexpr int RM = (0xf << (KQ + 1)) & 0xf;   // rows q > KQ of register KR
  asm(".if %[nop]\n s_nop 1\n .endif\n"
      ".if %[fr]\n"
      " .if %[kr] < 1\n v_fmac_f64_dpp %[a1], %[a1], %[nw] row_newbcast:%[k] row_mask:0xf bank_mask:0xf\n .endif\n"
      " .if %[kr] < 2\n v_fmac_f64_dpp %[a2], %[a2], %[nw] row_newbcast:%[k] row_mask:0xf bank_mask:0xf\n .endif\n"
      " .if %[kr] < 3\n v_fmac_f64_dpp %[a3], %[a3], %[nw] row_newbcast:%[k] row_mask:0xf bank_mask:0xf\n .endif\n"
      ".endif\n"
      ".if %[rm] != 0\n"
      " .if %[kr] == 0\n v_fmac_f64_dpp %[a0], %[a0], %[nw] row_newbcast:%[k] row_mask:%[rm] bank_mask:0xf\n .endif\n"
      " .if %[kr] == 1\n v_fmac_f64_dpp %[a1], %[a1], %[nw] row_newbcast:%[k] row_mask:%[rm] bank_mask:0xf\n .endif\n"
      " .if %[kr] == 2\n v_fmac_f64_dpp %[a2], %[a2], %[nw] row_newbcast:%[k] row_mask:%[rm] bank_mask:0xf\n .endif\n"
      " .if %[kr] == 3\n v_fmac_f64_dpp %[a3], %[a3], %[nw] row_newbcast:%[k] row_mask:%[rm] bank_mask:0xf\n .endif\n"
      ".endif\n"
      ".if %[doe]\n"
      " v_fmac_f64_dpp %[e0], %[e0], %[nwm] row_newbcast:%[k] row_mask:0xf bank_mask:0xf\n"
      " .if %[kr] >= 1\n v_fmac_f64_dpp %[e1], %[e1], %[nwm] row_newbcast:%[k] row_mask:0xf bank_mask:0xf\n .endif\n"
      " .if %[kr] >= 2\n v_fmac_f64_dpp %[e2], %[e2], %[nwm] row_newbcast:%[k] row_mask:0xf bank_mask:0xf\n .endif\n"
      " .if %[kr] >= 3\n v_fmac_f64_dpp %[e3], %[e3], %[nwm] row_newbcast:%[k] row_mask:0xf bank_mask:0xf\n .endif\n"
      " .if %[k] == 14\n s_nop 7\n s_nop 7\n .endif\n"
      ".endif\n"
      : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3), [e0] "+v"(e0), [e1] "+v"(e1), [e2] "+v"(e2),
        [e3] "+v"(e3)
      : [nw] "v"(nw), [nwm] "v"(nwm), [k] "i"(K), [kr] "i"(KR), [rm] "i"(RM), [doe] "i"(DOE ? 1 : 0),
        [nop] "i"(NOP ? 1 : 0), [fr] "i"(FULLROWS ? 1 : 0));
  A[0] = a0; A[1] = a1; A[2] = a2; A[3] = a3;
  E[0] = e0; E[1] = e1; E[2] = e2; E[3] = e3;
}

// upper-triangle blocks (i, j), r0 <= i < r1, i <= j < NB, enumerated row by
// row: count, and block t -> (i, j)
constexpr int tri_count(int nb, int r0, int r1) {
  int n = 0;
  for (int i = r0; i < r1; ++i) n += nb - i;
  return n;
}
constexpr int tri_row(int nb, int r0, int t) {
  int i = r0;
  while (t >= nb - i) { t -= nb - i; ++i; }
  return i;
}
constexpr int tri_col(int nb, int r0, int t) {
  int i = r0;
  while (t >= nb - i) { t -= nb - i; ++i; }
  return i + t;
}

// Hooks of the panel: the dense diagonal-tile kernel of the correlated
// factorisation exports E = L^-T of each 16-row sub-block (before V = E^T A)
// and each register's row scale D^-1/2.
struct NoHook {
  __device__ __forceinline__ void on_e(const v4d&) const {}
  __device__ __forceinline__ void on_scale(int, double) const {}
};


// PANEL_2L on the diagonal block D of block row BB (of NB): its 16 pivots in
// four sub-panels of 4 rows (register s of the C/D layout).  Inside a
// sub-panel the pivots update only register s (rows q > kq) and E; after it,
// the sub-panel's rows are scaled to U_s = D_s^-1/2 V_s and the rows below
// take D -= U_s^T U_s by ONE MFMA.  Leaves E = L^-T (column operations) and
// the row scales rsr[r] = D^-1/2 of register r; accumulates log d_k (lane
// c == 0 of each row) and d_k > 0.  RL: the last column of block row NB-1 is
// the residual (not pivoted); klim: pivots >= klim of that block row are pads
// (identity rows and columns: pivot 1, every multiplier 0) and are skipped.
// Rr[j] += Rr[j] (lane k of its row) * nw for the rows j in (KQ, 4): the
// replicated copies of the sub-panel's rows, updated exactly as pivot_fused
// updates their originals in register kr (bit-identical copies).  The
// leading s_nop covers a DPP read of a VGPR the previous pivot wrote.
template <int K, int KQ>
__device__ __forceinline__ void repl_rows_update(double (&Rr)[4], double nw) {
  double r1 = Rr[1], r2 = Rr[2], r3 = Rr[3];
  asm(" s_nop 1\n"
      ".if %[kq] < 1\n v_fmac_f64_dpp %[r1], %[r1], %[nw] row_newbcast:%[k] row_mask:0xf bank_mask:0xf\n .endif\n"
      ".if %[kq] < 2\n v_fmac_f64_dpp %[r2], %[r2], %[nw] row_newbcast:%[k] row_mask:0xf bank_mask:0xf\n .endif\n"
      ".if %[kq] < 3\n v_fmac_f64_dpp %[r3], %[r3], %[nw] row_newbcast:%[k] row_mask:0xf bank_mask:0xf\n .endif\n"
      : [r1] "+v"(r1), [r2] "+v"(r2), [r3] "+v"(r3)
      : [nw] "v"(nw), [k] "i"(K), [kq] "i"(KQ));
  Rr[1] = r1; Rr[2] = r2; Rr[3] = r3;
}

// REPL (the latency kernel): the four rows of each sub-panel are broadcast to
// every 16-lane row once, when the sub-panel starts (4 ds_bpermute pairs in
// flight together), and kept up to date by repl_rows_update, so no pivot
// waits on a ds_bpermute round trip: 6 more DPP multiply-adds per sub-panel
// for a shorter dependent chain.  Same values bit for bit.
// The pivot d = A[k][k] is read by two v_readlane_b32 from the register
// itself, in parallel with the ds_bpermute that broadcasts row k.  (Round 3
// A/B, profiles/r03e/chol_ab.log: taking d from the broadcast row by one
// v_mov_b64_dpp -- one instruction less per pivot -- put the bpermute's
// latency in front of the reciprocal: 3.70 vs 3.65 ms per launch; masking
// only the high dword of the E multiplier -- one v_cndmask_b32 less -- 3.70
// ms.  Neither is kept.)
// __shfl(x, 16 KQ + c) with the lane address formed at the use: an empty asm
// keeps the compiler from carrying the address of one KQ across the whole
// kernel (in the headline kernel's last block row it did, and spilled it:
// VERDICT r03 item 2)
template <int KQ>
__device__ __forceinline__ double shfl_row_fresh(double x, int c) {
  int a = c << 2;
  asm volatile("" : "+v"(a));
  const int lo = __builtin_amdgcn_ds_bpermute(a + 64 * KQ, __double2loint(x));
  const int hi = __builtin_amdgcn_ds_bpermute(a + 64 * KQ, __double2hiint(x));
  return __hiloint2double(hi, lo);
}

// The four rows of a sub-panel register x (row j = lanes 16 j .. 16 j + 15)
// broadcast to every 16-lane row by gfx950's lane-swap instructions:
// v_permlane32_swap of x with a copy gives rows (0, 1, 0, 1) and (2, 3, 2, 3),
// v_permlane16_swap of each with a copy the four broadcasts -- 6 swaps on the
// VALU instead of 8 ds_bpermute round trips through the LDS crossbar.  Same
// values bit for bit.  (In the batched kernel, issue-bound, the extra copies
// and replica updates cost more than the crossbar: 3.65 -> 3.76 ms, DESIGN.md
// §4a; the latency kernel waits on the round trip instead.)
__device__ __forceinline__ void bcast_rows4(double x, double (&R)[4]) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  const auto l32 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto h32 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  const auto l01 = __builtin_amdgcn_permlane16_swap(l32[0], l32[0], false, false);
  const auto h01 = __builtin_amdgcn_permlane16_swap(h32[0], h32[0], false, false);
  const auto l23 = __builtin_amdgcn_permlane16_swap(l32[1], l32[1], false, false);
  const auto h23 = __builtin_amdgcn_permlane16_swap(h32[1], h32[1], false, false);
  R[0] = __hiloint2double(h01[0], l01[0]);
  R[1] = __hiloint2double(h01[1], l01[1]);
  R[2] = __hiloint2double(h23[0], l23[0]);
  R[3] = __hiloint2double(h23[1], l23[1]);
}

// REPL: 0 = each pivot row broadcast by ds_bpermute when it is needed (the
// batched kernels); 1 = the sub-panel's four rows replicated up front by
// ds_bpermute; 2 = replicated by the lane swaps of bcast_rows4
template <int NB, int BB, bool RL, int REPL = 0>
__device__ __forceinline__ void diag_factor_2l(v4d& D, v4d& E, double (&rsr)[4], int q, int c, LogAcc& ldet,
                                               bool& ok, int klim) {
  constexpr bool LASTR = RL && BB == NB - 1;          // block row holding the residual
  static_for<0, 4>([&](auto R) {
    constexpr int r = decltype(R)::value;
    E[r] = (q + 4 * r == c) ? 1.0 : 0.0;
    rsr[r] = 1.0;
  });
  // (Folding the row scales into E's columns instead -- E D^-1/2, one gather,
  // four multiplies -- was tried in round 3: the wide chol_big_kernel and the
  // one-wave NB = 9 kernel then faulted with an illegal address on the GPU;
  // not kept.)
  static_for<0, 4>([&](auto KR) {
    constexpr int kr = decltype(KR)::value;
    constexpr int nk = (LASTR && kr == 3) ? 3 : 4;   // the r column is not pivoted
    double Rr[4];
    if constexpr (REPL == 1) {
      static_for<0, 4>([&](auto J) { Rr[decltype(J)::value] = __shfl(D[kr], 16 * decltype(J)::value + c); });
    } else if constexpr (REPL == 2) {
      bcast_rows4(D[kr], Rr);
    }
    static_for<0, nk>([&](auto KQc) {
      constexpr int kq = decltype(KQc)::value;
      constexpr int k = 4 * kr + kq;
      if constexpr (LASTR) {
        if (k >= klim) return;                         // wave-uniform: pad pivots
      }
      constexpr bool doe = !LASTR && k < 15;
      const double xk = REPL ? Rr[kq] : LASTR ? shfl_row_fresh<kq>(D[kr], c) : __shfl(D[kr], 16 * kq + c);  // A[k][c]
      const double d = REPL ? readlane_d(Rr[kq], k) : readlane_d(D[kr], 16 * kq + k);
      const double nw = div_fast(-xk, d);
      const double nwm = (doe && c > k) ? nw : 0.0;
      pivot_fused<k, kr, kq, doe, kq == 0, false>(D, E, nw, nwm);
      if constexpr (REPL && kq < 3) repl_rows_update<k, kq>(Rr, nw);
    });
    // sub-panel kr done: lane (q, c) takes the pivot of row 4 kr + q (lane
    // (q, 4 kr + q)): log-det, positivity, row scale; U_s = D_s^-1/2 V_s and
    // the rows below take D -= U_s^T U_s (one MFMA, in place: registers
    // <= kr are not read again)
    auto sub = [&]() {
      const double dg = __shfl(D[kr], 17 * q + 4 * kr);
      const double dv = (LASTR && kr == 3 && q == 3) ? 1.0 : dg;   // (the r row)
      ok = ok && (dv > 0.0);
      if (c == 0) ldet.add(dv);
      if constexpr (!(LASTR && kr == 3)) {
        const double rs = rsqrt_fast(dv);
        rsr[kr] = rs;
        if constexpr (kr < 3) {
          const double u = D[kr] * rs;
          D = __builtin_amdgcn_mfma_f64_16x16x4f64(u, u, D, 0, 0, 1);
        }
      }
    };
    if constexpr (LASTR) {
      if (4 * kr < klim) sub();                      // (a sub-panel of pads: pivots 1, no update)
    } else {
      sub();
    }
  });
}

// The rest of a block row after its diagonal block: V = E^T A (4 MFMAs)
// (row_v_2l), rows scaled to U = D^-1/2 V (row r of register r times rsr[r]).
__device__ __forceinline__ void row_v_2l(const v4d& E, v4d& A) {
  v4d acc = {0.0, 0.0, 0.0, 0.0};
  static_for<0, 4>([&](auto S) {
    constexpr int s = decltype(S)::value;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(E[s], A[s], acc, 0, 0, 0);
  });
  A = acc;
}

// The LDL^T panel of block row BB over the blocks blk(j), j = BB..NB-1 (C/D
// layout, upper triangle; the diagonal block is held in full): eliminates
// the diagonal block pivot by pivot (row k broadcast to every 16-lane row by
// ds_bpermute, pivot by readlane, quotient by div_fast), builds E = L^-T by
// column operations, turns the rest of the row into V = E^T A (4 MFMAs per
// block) and scales it to U = D^-1/2 V.  Accumulates log d_k (packed: one
// lane per row) and d_k > 0.
// RL: the last column of block row NB-1 is the residual (not pivoted), as in
// the per-pulsar factorisations; false for a plain SPD block (the dense
// cross-pulsar factorisation's diagonal tiles).
// PANEL_2L (the default): diag_factor_2l + row_v_2l + the row scales.  PANEL_1L (dev A/B
// only: the round-2 default): every pivot updates every register r >= kr by
// VALU.  The update A[i][c] -= A[i][k] (A[k][c] / d) rounds differently from
// its mirror A[c][i] -= A[c][k] (A[k][i] / d), so the lower triangle drifts
// from the upper one and, on ill-conditioned draws, the Schur complements
// drift with it (tests/golden: c1_turnover sample 0 at 4e3x the strict bound
// vs 22x for PANEL_2L and 79x for enterprise's LAPACK order).
// PACK (PANEL_1L): the row scales D^-1/2 of all 16 rows by one gather + one
// rsqrt per lane (lane (q, c) takes d of row q + 4 (c/4)); else one per
// register (the phase-1 form of chol_mfma_kernel<8>, where the packed
// temporaries spill).
// klim: pivots >= klim of the last block row are pads and are skipped.
constexpr int PANEL_1L = 11;
constexpr int PANEL_2L = 25;

template <int NB, int ALG, bool RL, bool PACK, typename BBt, typename Blk, typename Hook = NoHook>
__device__ __forceinline__ void panel_ldl_row(BBt BBc, Blk&& blk, int q, int c, LogAcc& ldet, bool& ok,
                                              const Hook& hook = Hook{}, int klim = 16) {
  constexpr int bb = decltype(BBc)::value;
  static_assert(ALG == PANEL_1L || ALG == PANEL_2L, "unknown panel form");
  constexpr bool LASTR = RL && bb == NB - 1;          // block row holding the residual
  if constexpr (ALG == PANEL_2L) {
    v4d E;
    double rsr[4];
    diag_factor_2l<NB, bb, RL>(blk(BBc), E, rsr, q, c, ldet, ok, klim);
    if constexpr (!LASTR) {
      hook.on_e(E);
      static_for<bb + 1, NB>([&](auto JJ) { row_v_2l(E, blk(JJ)); });
      static_for<0, 4>([&](auto R) {
        constexpr int r = decltype(R)::value;
        hook.on_scale(r, rsr[r]);
        static_for<bb + 1, NB>([&](auto JJ) { blk(JJ)[r] *= rsr[r]; });
      });
    }
    return;
  } else {
  v4d E;
  static_for<0, 4>([&](auto R) {
    constexpr int r = decltype(R)::value;
    E[r] = (q + 4 * r == c) ? 1.0 : 0.0;
  });
  static_for<0, 4>([&](auto KR) {
    constexpr int kr = decltype(KR)::value;
    constexpr int nk = (LASTR && kr == 3) ? 3 : 4;   // the r column is not pivoted
    static_for<0, nk>([&](auto KQc) {
      constexpr int kq = decltype(KQc)::value;
      constexpr int k = 4 * kr + kq;
      if constexpr (LASTR) {
        if (k >= klim) return;                         // wave-uniform: pad pivots
      }
      constexpr bool doe = !LASTR && k < 15;
      const double xk = __shfl(blk(BBc)[kr], 16 * kq + c);    // A[k][c]
      const double d = readlane_d(blk(BBc)[kr], 16 * kq + k);
      const double nw = div_fast(-xk, d);
      const double nwm = (doe && c > k) ? nw : 0.0;
      pivot_fused<k, kr, kq, doe, k == 0, true>(blk(BBc), E, nw, nwm);
    });
  });
  if constexpr (!LASTR) hook.on_e(E);
  static_for<bb + 1, NB>([&](auto JJ) {
    v4d acc = {0.0, 0.0, 0.0, 0.0};
    static_for<0, 4>([&](auto S) {
      constexpr int s = decltype(S)::value;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(E[s], blk(JJ)[s], acc, 0, 0, 0);
    });
    blk(JJ) = acc;
  });
  // rows of the block row -> U = d^-1/2 V (the diagonal block itself is not
  // needed after its panel; the last block row has nothing to scale)
  if constexpr (PACK) {
    // d of row q + 4r read from the diagonal (lane 17q + 4r); lane (q, c)
    // takes d of row q + 4 (c/4) -- held in register c/4 of lane
    // (q, q + 4 (c/4)), whose own c/4 is the same -- so one gather, one rsqrt
    // and one log-det term (lanes c % 4 == 0) cover all 16 rows; register r
    // then takes its rows' scale from lane (q, 4r) by DPP
    const int cr = c >> 2;
    const double own = cr == 0 ? blk(BBc)[0] : cr == 1 ? blk(BBc)[1] : cr == 2 ? blk(BBc)[2] : blk(BBc)[3];
    double dv = __shfl(own, 17 * q + 4 * cr);
    if constexpr (LASTR) dv = (q == 3 && cr == 3) ? 1.0 : dv;
    ok = ok && (dv > 0.0);
    if ((c & 3) == 0) ldet.add(dv);
    if constexpr (!LASTR) {
      const double rsp = rsqrt_nr(dv);
      static_for<0, 4>([&](auto R) {
        constexpr int r = decltype(R)::value;
        const double rs = row_newbcast<4 * r>(rsp);
        hook.on_scale(r, rs);
        static_for<bb + 1, NB>([&](auto JJ) { blk(JJ)[r] *= rs; });
      });
    }
  } else {
    static_for<0, 4>([&](auto R) {
      constexpr int r = decltype(R)::value;
      const bool rrow = LASTR && r == 3 && q == 3;
      const double dg = __shfl(blk(BBc)[r], 17 * q + 4 * r);
      const double dv = rrow ? 1.0 : dg;
      ok = ok && (dv > 0.0);
      if (c == 0) ldet.add(dv);
      if constexpr (!LASTR) {
        const double rs = rsqrt_nr(dv);
        hook.on_scale(r, rs);
        static_for<bb + 1, NB>([&](auto JJ) { blk(JJ)[r] *= rs; });
      }
    });
  }
  }
}

// KEEP > 0 (correlated common process): only block rows 0..NB-KEEP-1 (the
// pulsar's own columns) are factored; the trailing KEEP x KEEP blocks (the
// common columns + r: their Schur complement S^G, d', rho) are written to
// keep_out[(p * keep_bs + (b - keep_b0))] as a dense (16 KEEP)^2 square
// (pulsar-major: a device's pulsar range is one contiguous slice, the unit an
// all-gather moves), and
// the unit term is the local part K - 1/2 log|Sigma_LL| - 1/2 log|phi_L|.
#ifdef EWH_DEV
// STAMP (dev diagnostics): s_memtime stamps at the phase boundaries of the
// units with blockIdx < STAMP_UNITS (ewh_dev_stamps)
constexpr int STAMP_UNITS = 4096, STAMP_N = 24;
static __device__ long long g_stamps[STAMP_UNITS * STAMP_N];
#endif

// W: waves per SIMD the register budget is cut for (2 -> 256 VGPRs: the NB = 8
// three-phase kernel fits, so two units share each SIMD and one's MFMAs
// overlap the other's VALU / LDS latency).  Block row 0 is loaded before the
// spectra are formed (its latency overlaps the prologue); with fixed white
// noise each distinct spectrum is formed once (the sin / cos columns of a
// frequency share one: J.rep / J.ulist) and shared through LDS; the last
// panel's pad pivots are skipped.
template <int NB, int W, int ALG = PANEL_2L, bool STAMP = false, int KEEP = 0, bool FULL = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(W, W)))
void chol_mfma_kernel(const CholJob* __restrict__ jobs, int B, long long u0, int b_off,
                      const double* __restrict__ theta, int ldth, double* __restrict__ out_units,
                      double* __restrict__ keep_out, int keep_b0, int keep_bs) {
#ifdef EWH_DEV
  long long stp[STAMP_N];
#define EWH_STAMP(I)                                            \
  if constexpr (STAMP) {                                        \
    __builtin_amdgcn_sched_barrier(0);                          \
    stp[(I)] = (long long)__builtin_amdgcn_s_memtime();         \
    __builtin_amdgcn_sched_barrier(0);                          \
  }
#else
  static_assert(!STAMP, "phase stamps exist only in the dev library");
#define EWH_STAMP(I)
#endif
  EWH_STAMP(0)
  constexpr int LD = 16 * NB;
  using S = Split<NB, FULL>;
  constexpr int H = S::H;
  static_assert(!FULL || KEEP == 0, "the FULL form has no kept blocks");
  static_assert(FULL || NB - KEEP >= H, "kept blocks must lie in the phase-3 triangle");
  __shared__ double phinv[LD];
  __shared__ double phs[LD];
  const int lane = threadIdx.x;
  const int q = lane >> 4, c = lane & 15;
  const long long u = u0 + xcd_unit(blockIdx.x, gridDim.x);
  const int p = (int)(u / B), b = (int)(u % B);
  const CholJob J = jobs[p];
  const gdptr A = (gdptr)(J.mats + (long long)(b - b_off) * J.mstride);
  const double* th = theta + (long long)b * ldth;

  v4d pre[NB];
  static_for<0, NB>([&](auto BJ) {
    static_for<0, 4>([&](auto R) {
      constexpr int r = decltype(R)::value;
      pre[decltype(BJ)::value][r] = A[(long long)(q + 4 * r) * LD + 16 * decltype(BJ)::value + c];
    });
  });
  // log|phi| is summed into the per-lane log-det accumulator (one log() at
  // the end of the kernel)
  LogAcc ldet;
  if (J.urec != nullptr && (J.ntidx > 0 || ldth <= STAGE_THETA_MAX)) {
    // staged: the theta entries the spectra read (or the whole row) -> LDS,
    // each distinct spectrum's record by its lane, every column's record
    // index -- all loads issued together
    __shared__ double ths[STAGE_THETA_MAX];
    int ur[(LD + 63) / 64];
    static_for<0, (LD + 63) / 64>([&](auto I) {
      constexpr int i = decltype(I)::value;
      ur[i] = 64 * i + lane < J.mreal ? J.urep[64 * i + lane] : -1;
    });
    if (J.ntidx > 0) {
      if (lane < J.ntidx) ths[lane] = th[jobs[p].tidx[lane]];
    } else {
      for (int i = lane; i < ldth; i += 64) ths[i] = th[i];
    }
    __syncthreads();
    for (int u = lane; u < J.nu; u += 64) {
      const URec& R = J.urec[u];
      double ph = 0.0;
      for (int e = 0; e < R.ne; ++e) ph += spec_phi_body(R.e[e], ths);
      phs[u] = ph;
    }
    __syncthreads();
    static_for<0, (LD + 63) / 64>([&](auto I) {
      constexpr int i = decltype(I)::value;
      const int a = 64 * i + lane;
      if (a < LD) {
        double pi = 0.0;
        if (ur[i] >= 0) {
          const double ph = phs[ur[i]];
          pi = 1.0 / ph;
          ldet.add(ph);
        }
        phinv[a] = pi;
      }
    });
  } else {
    const bool dedup = J.rep != nullptr;
    if (dedup) {
      for (int i = lane; i < J.nu; i += 64) {
        const int a = J.ulist[i];
        double ph = 0.0;
        for (int e = J.col_ptr[a]; e < J.col_ptr[a + 1]; ++e) ph += spec_phi_body(J.spec[e], th);
        phs[a] = ph;
      }
      __syncthreads();
    }
    for (int a = lane; a < LD; a += 64) {
      double pi = 0.0;
      if (a < J.mreal && J.col_ptr[a] < J.col_ptr[a + 1]) {   // (pads carry no entry)
        double ph = 0.0;
        if (dedup) {
          ph = phs[J.rep[a]];
        } else {
          for (int e = J.col_ptr[a]; e < J.col_ptr[a + 1]; ++e) ph += spec_phi_body(J.spec[e], th);
        }
        pi = 1.0 / ph;
        ldet.add(ph);
      }
      phinv[a] = pi;
    }
  }
  __syncthreads();
  EWH_STAMP(1)

  auto load_block = [&](auto BI, auto BJ, v4d& v) {
    constexpr int bi = decltype(BI)::value, bj = decltype(BJ)::value;
    static_for<0, 4>([&](auto R) {
      constexpr int r = decltype(R)::value;
      v[r] = A[(long long)(16 * bi + q + 4 * r) * LD + 16 * bj + c];
    });
    if constexpr (bi == bj) {
      const double pd = phinv[16 * bi + c];
      static_for<0, 4>([&](auto R) {
        constexpr int r = decltype(R)::value;
        v[r] += (q + 4 * r == c) ? pd : 0.0;
      });
    }
  };

  bool ok = true;
  constexpr bool SKIPPAD = KEEP == 0;
  const int klast = SKIPPAD ? __builtin_amdgcn_readfirstlane(J.mreal - 16 * (NB - 1)) : 16;
  // phase 1 (NB = 8): per-register row scales (the packed form's temporaries spill there)
  constexpr bool PACK1 = NB != 8;

  // ---- phase 1: block rows 0..H-1 ----
  v4d U1[S::n1 > 0 ? S::n1 : 1];
  static_for<0, H>([&](auto BI) {
    constexpr int bi = decltype(BI)::value;
    static_for<bi, NB>([&](auto BJ) {
      constexpr int bj = decltype(BJ)::value;
      if constexpr (bi == 0) {
        U1[S::i1(0, bj)] = pre[bj];
        if constexpr (bj == 0) {
          const double pd = phinv[c];
          static_for<0, 4>([&](auto R) {
            constexpr int r = decltype(R)::value;
            U1[S::i1(0, 0)][r] += (q + 4 * r == c) ? pd : 0.0;
          });
        }
      } else {
        load_block(BI, BJ, U1[S::i1(bi, bj)]);
      }
    });
  });
  static_for<0, H>([&](auto BBc) {
    constexpr int bb = decltype(BBc)::value;
    panel_ldl_row<NB, ALG, KEEP == 0, PACK1>(BBc, [&](auto JJ) -> v4d& { return U1[S::i1(bb, decltype(JJ)::value)]; },
                                             q, c, ldet, ok, NoHook{}, klast);
    EWH_STAMP(2 + 2 * bb)
    static_for<bb + 1, H>([&](auto II) {
      constexpr int i = decltype(II)::value;
      static_for<i, NB>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        syrk_update(U1[S::i1(i, j)], U1[S::i1(bb, i)], U1[S::i1(bb, j)]);
      });
    });
    EWH_STAMP(3 + 2 * bb)
  });
  // ---- phase 2: A22 -= U12^T U12 ----
  // block by block in row order: U1 column i is dead once row i of A22 is done
  v4d U2[S::n2 > 0 ? S::n2 : 1];
  static_for<H, NB>([&](auto II) {
    constexpr int i = decltype(II)::value;
    static_for<i, NB>([&](auto JJ) {
      constexpr int j = decltype(JJ)::value;
      load_block(II, JJ, U2[S::i2(i, j)]);
      static_for<0, H>([&](auto BBc) {
        constexpr int bb = decltype(BBc)::value;
        syrk_update(U2[S::i2(i, j)], U1[S::i1(bb, i)], U1[S::i1(bb, j)]);
      });
    });
  });
  EWH_STAMP(2 + 2 * H)
  // ---- phase 3: factor A22 (up to the kept blocks) ----
  static_for<H, NB - KEEP>([&](auto BBc) {
    constexpr int bb = decltype(BBc)::value;
    panel_ldl_row<NB, ALG, KEEP == 0, true>(BBc, [&](auto JJ) -> v4d& { return U2[S::i2(bb, decltype(JJ)::value)]; },
                                            q, c, ldet, ok, NoHook{}, klast);
    EWH_STAMP(3 + 2 * bb)
    static_for<bb + 1, NB>([&](auto II) {
      constexpr int i = decltype(II)::value;
      static_for<i, NB>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        syrk_update(U2[S::i2(i, j)], U2[S::i2(bb, i)], U2[S::i2(bb, j)]);
      });
    });
    EWH_STAMP(4 + 2 * bb)
  });
  double qv = 0.0;
  if constexpr (FULL) {
    qv = readlane_d(U1[S::i1(NB - 1, NB - 1)][3], 63);
  } else if constexpr (KEEP == 0) {
    qv = readlane_d(U2[S::i2(NB - 1, NB - 1)][3], 63);
  } else {
    constexpr int KD = 16 * KEEP;
    double* ko = keep_out + ((long long)p * keep_bs + (b - keep_b0)) * (KD * KD);
    int qo = q, co = c;                     // (store addresses formed here, not hoisted: they spilled)
    asm volatile("" : "+v"(qo), "+v"(co));
    static_for<NB - KEEP, NB>([&](auto II) {
      constexpr int i = decltype(II)::value;
      static_for<i, NB>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        static_for<0, 4>([&](auto RR) {
          constexpr int r = decltype(RR)::value;
          const int row = 16 * (i - (NB - KEEP)) + qo + 4 * r, col = 16 * (j - (NB - KEEP)) + co;
          const double v = U2[S::i2(i, j)][r];
          if (i != j || row <= col) {
            ko[row * KD + col] = v;
            ko[col * KD + row] = v;
          }
        });
      });
    });
  }
  const double ldet_v = wave_sum(ldet.value());    // per-lane partial log-dets (pivots and phi)
  const bool ok_all = __all(ok);
  if (lane == 0) {
    double lnl = J.K[(long long)(b - b_off) * J.kstride] - 0.5 * qv - 0.5 * ldet_v;
    if (!ok_all || J.fail) lnl = -INFINITY;
    out_units[(long long)p * B + b] = lnl;
  }
#ifdef EWH_DEV
  if constexpr (STAMP) {
    EWH_STAMP(3 + 2 * NB)
    if (lane == 0 && blockIdx.x < STAMP_UNITS) {
      long long* o = g_stamps + (long long)blockIdx.x * STAMP_N;
      for (int i = 0; i < 4 + 2 * NB && i < STAMP_N - 2; ++i) o[i] = stp[i];
      o[STAMP_N - 2] = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_ID (wave, SIMD, CU, SE)
      o[STAMP_N - 1] = __builtin_amdgcn_s_getreg(20 | (31 << 11));   // XCC_ID
    }
  }
#endif
#undef EWH_STAMP
}
// ----------------------------------------------------------------------------
// batched factorisation for wide bases (NB > 9, e.g. C4's 193-wide Sigma):
// one wave per unit, LEFT-looking over block rows.  Block row i (<= NB
// blocks, C/D layout) is loaded into registers, takes the updates
// A_ij -= U_pi^T U_pj of every finished row p < i (4 MFMAs per block, the U
// blocks streamed back from a per-wave scratch in the same lane layout,
// double-buffered), is factored by the LDL^T panel and written to scratch.
// Same arithmetic as chol_mfma_kernel (right-looking), re-ordered.
// ----------------------------------------------------------------------------
constexpr int BIG_NB_MAX = 16;
// chol_wide_kernel (chol_wide.hip): any width up to WIDE_NB_MAX blocks
constexpr int WIDE_NB_MAX = 64;
constexpr int WIDE_LD_MAX = 16 * WIDE_NB_MAX;

template <int NB>
__device__ __forceinline__ long long big_blk(int p, int j) {   // packed upper block index
  return (long long)p * NB - (long long)p * (p - 1) / 2 + (j - p);
}

template <int NB>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
void chol_big_kernel(const CholJob* __restrict__ jobs, int B, long long u0, int b_off,
                     const double* __restrict__ theta, int ldth, double* __restrict__ out_units,
                     double* __restrict__ scratch) {
  constexpr int LD = 16 * NB;
  __shared__ double phinv[LD];
  const int lane = threadIdx.x;
  const int q = lane >> 4, c = lane & 15;
  const long long u = u0 + xcd_unit(blockIdx.x, gridDim.x);
  const int p = (int)(u / B), b = (int)(u % B);
  const CholJob J = jobs[p];
  const gdptr A = (gdptr)(J.mats + (long long)(b - b_off) * J.mstride);
  const double* th = theta + (long long)b * ldth;
  typedef __attribute__((address_space(1))) v4d gv4d;   // global_load / store (see gdptr)
  __attribute__((address_space(1))) double* scr =
      (__attribute__((address_space(1))) double*)(scratch + (long long)blockIdx.x * (NB * (NB + 1) / 2) * 256 + lane * 4);

  LogAcc lphi;
  for (int a = lane; a < LD; a += 64) {
    double pi = 0.0;
    if (a < J.mreal && J.col_ptr[a] < J.col_ptr[a + 1]) {   // (pads carry no entry)
      double ph = 0.0;
      for (int e = J.col_ptr[a]; e < J.col_ptr[a + 1]; ++e) ph += spec_phi_body(J.spec[e], th);
      pi = 1.0 / ph;
      lphi.add(ph);
    }
    phinv[a] = pi;
  }
  const double lphi_sum = wave_sum(lphi.value());
  __syncthreads();

  LogAcc ldet;
  bool ok = true;
  double qv = 0.0;
  const int klast = __builtin_amdgcn_readfirstlane(J.mreal - 16 * (NB - 1));   // the last row's pad pivots are skipped
  static_for<0, NB>([&](auto I) {
    constexpr int i = decltype(I)::value;
    constexpr int W = NB - i;                       // blocks in row i
    v4d R[W];
    static_for<0, W>([&](auto JJ) {
      constexpr int j = i + decltype(JJ)::value;
      static_for<0, 4>([&](auto RR) {
        constexpr int r = decltype(RR)::value;
        R[j - i][r] = A[(long long)(16 * i + q + 4 * r) * LD + 16 * j + c];
      });
      if constexpr (j == i) {
        const double pd = phinv[16 * i + c];
        static_for<0, 4>([&](auto RR) {
          constexpr int r = decltype(RR)::value;
          R[0][r] += (q + 4 * r == c) ? pd : 0.0;
        });
      }
    });
    if constexpr (i > 0) {
      // U blocks (p, i..NB-1) of earlier rows: Ui once, then each Uj in turn
      // (the compiler issues the row's loads ahead of its MFMAs)
#pragma unroll 1
      for (int pp = 0; pp < i; ++pp) {
        const v4d Ui = *(const gv4d*)(scr + big_blk<NB>(pp, i) * 256);
        static_for<0, W>([&](auto JJ) {
          constexpr int jj = decltype(JJ)::value;
          const v4d Uj = *(const gv4d*)(scr + big_blk<NB>(pp, i + jj) * 256);
          syrk_update(R[jj], Ui, Uj);
        });
      }
    }
    panel_ldl_row<NB, PANEL_2L, true, true>(I, [&](auto JJ) -> v4d& { return R[decltype(JJ)::value - i]; }, q, c,
                                            ldet, ok, NoHook{}, klast);
    if constexpr (i < NB - 1) {
      static_for<0, W>([&](auto JJ) {
        constexpr int j = i + decltype(JJ)::value;
        *(gv4d*)(scr + big_blk<NB>(i, j) * 256) = R[j - i];
      });
    } else {
      qv = readlane_d(R[0][3], 63);
    }
  });
  const double ldet_v = wave_sum(ldet.value());
  const bool ok_all = __all(ok);
  if (lane == 0) {
    double lnl = J.K[(long long)(b - b_off) * J.kstride] - 0.5 * qv - 0.5 * ldet_v - 0.5 * lphi_sum;
    if (!ok_all || J.fail) lnl = -INFINITY;
    out_units[(long long)p * B + b] = lnl;
  }
}

// ----------------------------------------------------------------------------
// correlated common process (HD / monopole / dipole ORF; [ent]
// FourierBasisCommonGP, enterprise_models.py:390-415), fixed white noise.
// Per sample b (after the per-pulsar partial factorisations):
//   M_g = Gamma phi_c(g) + diag_a(phi_own(a, g))          (P x P, per common column g)
//   Sigma_c = blockdiag_a(S^G_a) + [M_g^-1]_(a,g),(b,g)    (P n_c square, + r row)
//   lnL_b = sum_a local_a - 1/2 (log|Sigma_c| + q_c + sum_g log|M_g|)
// Sigma_c is factored densely (blocked right-looking, 64-wide panels: diagonal
// block by LDS Cholesky + explicit inverse, panel and trailing update by fp64
// MFMA); its last pivot is q_c = rho - d'^T Sigma_c^-1 d'.
// ----------------------------------------------------------------------------
struct CommonPsr {
  const int* colptr;     // reduced-layout CSR of the pulsar's own spectral entries
  const DSpec* spec;
  int gstart;            // reduced index of common column 0
  int pad_;
};

constexpr int DCB = 64;            // dense panel width


// ---- launchers defined in the other translation units ----------------------
// each returns 0 on success (negative EWH_E* on error)
// Glo: the low part of G (bases past 16 blocks only; may be NULL)
int launch_contract_nb(int nb, const PsrDev& P, const double* w, const double* beta, const double* s,
                       const double* fac, double* G, int nb_samples, hipStream_t st, double* Glo = nullptr);
// waves: 4 or 8 per sample (0 = the measured default for nb)
int launch_contract2_nb(int nb, int waves, const PsrDev& P, const double* w, const double* beta, double* s,
                        long long s_stride, double* G, int nb_samples, hipStream_t st, const double* rho = nullptr);
// mode: ewh_set_kernel_mode; returns 1 if no register kernel applies (caller falls back)
int launch_chol_small(int mode, int nb, const CholJob* jobs, int B, long long u0, long long n, int b_off,
                      const double* theta, int ldth, double* units, hipStream_t st);
int launch_chol_big_nb(int nb, const CholJob* jobs, int B, long long u0, long long n, int b_off,
                       const double* theta, int ldth, double* units, double* scr, long long cap, hipStream_t st);
// latency form for small batches (chol_lat.hip): one 4-wave workgroup per
// unit of units [0, P B); theta and host_units may be host-mapped pinned
// memory; every unit term goes to units[p B + b] and host_units[p B + b].
// Returns 1 if nb has no latency kernel (caller uses the batched path).
constexpr int LAT_NB_MAX = 8;
// unit term of a latency-kernel unit whose dataflow wait ran out (a NaN
// payload no other path writes; ewh_lnl_batch returns EWH_E_HIP on it)
constexpr unsigned long long LAT_STALL_BITS = 0x7ff4dead057a1100ull;
int launch_chol_lat(int nb, const CholJob* jobs, int B, int P, const double* theta, int ldth, double* units,
                    double* host_units, hipStream_t st, bool stamp = false, int var = 0);
// any width (chol_wide.hip): units [u0, u0 + n), slabs of at most cap
// workgroups, each with scr_per_wg doubles of scratch (wide_scratch_per_wg);
// keep > 0: the partial factorisation, kept blocks to keep_out as
// chol_mfma_kernel<KEEP> writes them
long long wide_scratch_per_wg(int nb, int keep);
// double-double factorisation (chol_dd.hip), one 512-thread workgroup per
// unit, 2 ld^2 doubles of scratch each (dd_scratch_per_wg); ld = the jobs'
// width (one width per launch)
long long dd_scratch_per_wg(int ld);
int launch_chol_dd(const CholJob* jobs, int B, long long u0, long long n, int b_off, const double* theta, int ldth,
                   double* units, double* scr, long long scr_per_wg, long long cap, int ld, hipStream_t st,
                   bool r05a = false);
// dynamic-LDS limits of chol_dd_kernel on the current device
int set_dd_attributes();
// the verify-and-refine form: units a (forward fp64) vs b (reversed fp64) of
// [u0, u0 + n) -> list / count of the disagreeing ones (count zeroed by the
// caller; total, if not NULL: total[0] += the count, total[1] += n; all:
// every unit listed -- kernel mode 29's refine_failed), then
// chol_dd_kernel over the list (cap workgroups looping) into units; r05a: the
// round-5a panel solve (row-oriented; dev mode 34)
int launch_verify_units(const double* a, const double* b, long long u0, long long n, int* list, int* count,
                        unsigned long long* total, hipStream_t st, bool all = false);
// kernel mode 29 (every unit in double-double): total[0] and total[1] += n on
// the device, in stream order (so graph replays count, captures do not)
int launch_count_units(unsigned long long* total, long long n, hipStream_t st);
int launch_chol_dd_list(const CholJob* jobs, int B, int b_off, const double* theta, int ldth, double* units,
                        double* scr, long long scr_per_wg, long long cap, const int* list, const int* count, int ld,
                        hipStream_t st, bool r05a = false);
// rev = 1 (keep == 0): the reversed column order (the verify step)
int launch_chol_wide(const CholJob* jobs, int B, long long u0, long long n, int b_off, const double* theta, int ldth,
                     double* units, double* scr, long long scr_per_wg, long long cap, int keep, double* keep_out,
                     int keep_b0, int keep_bs, hipStream_t st, int rev = 0, double* units_rev = nullptr,
                     bool pair = true);
// keep_out: pulsar-major kept blocks, keep_bs samples per pulsar (see chol_mfma_kernel KEEP)
int launch_partial_nb(int nb, int keep, const CholJob* jobs, int B, long long u0, long long n, int b_off,
                      const double* theta, int ldth, double* units, double* keep_out, int keep_bs, hipStream_t st);
// dynamic-LDS attributes of the contraction kernels on the current device
int set_contract_attributes();
// the contraction of a basis past 16 blocks (contract_wide.hip)
int launch_contract_wide(int nb, const PsrDev& P, const double* w, const double* beta, const double* s,
                         const double* fac, double* G, int nb_samples, hipStream_t st, double* Glo);
// true when kernel A/B mode `mode` (>= 3, not 7) is compiled into this library
// (dev library only: make dev, -DEWH_DEV)
bool variant_built(int mode);

}  // namespace ewh_dev
