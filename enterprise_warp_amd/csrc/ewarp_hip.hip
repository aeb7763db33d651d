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
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "ewarp_hip.h"

namespace {

thread_local std::string g_err;

int set_err(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define EWH_HIP(expr)                                                          \
  do {                                                                         \
    hipError_t e_ = (expr);                                                    \
    if (e_ != hipSuccess)                                                      \
      return set_err(EWH_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

typedef double v4d __attribute__((ext_vector_type(4)));

// ----------------------------------------------------------------------------
// device helpers
// ----------------------------------------------------------------------------
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

__device__ __noinline__ double spec_phi(const DSpec& s, const double* th) { return spec_phi_body(s, th); }

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

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// 256-thread block sum; `scratch` holds >= 4 doubles.
__device__ double block_sum256(double v, double* scratch) {
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
// per-pulsar device tables
// ----------------------------------------------------------------------------
constexpr int CT_ROWS = 32;   // TOA rows per contraction tile (8 MFMA k-steps); T_aug is padded by this many zero rows

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
};

// ----------------------------------------------------------------------------
// white noise: w_t = 1/N_t, ECORR beta_e, -1/2 log|N|     ([ent] ShermanMorrison)
// grid: one 256-thread block per sample of the chunk
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void wn_weights_kernel(PsrDev P, const double* __restrict__ theta,
                                                         int ldth, int b0, double* __restrict__ w,
                                                         double* __restrict__ beta,
                                                         double* __restrict__ Kb, double* __restrict__ fac) {
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

// block index blk of the upper triangle (row-major over i <= j) -> (i, j)
constexpr int tri_i(int nb, int blk) {
  int i = 0;
  while (blk >= nb - i) { blk -= nb - i; ++i; }
  return i;
}
constexpr int tri_j(int nb, int blk) {
  int i = 0;
  while (blk >= nb - i) { blk -= nb - i; ++i; }
  return i + blk;
}
// does wave `wave` (blocks wave + 4 sl) touch block column j as a row (A) / at all?
constexpr bool wave_uses_row(int nb, int wave, int j) {
  for (int blk = wave; blk < nb * (nb + 1) / 2; blk += 4)
    if (tri_i(nb, blk) == j) return true;
  return false;
}
constexpr bool wave_uses(int nb, int wave, int j) {
  for (int blk = wave; blk < nb * (nb + 1) / 2; blk += 4)
    if (tri_i(nb, blk) == j || tri_j(nb, blk) == j) return true;
  return false;
}

template <int NB, int WAVE>
__device__ __forceinline__ void contract2_body(const PsrDev& P, const double* __restrict__ wrow,
                                               const double* __restrict__ brow, double* __restrict__ srow,
                                               double* __restrict__ Gout) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int LD = 16 * NB;
  constexpr int NBLK = NB * (NB + 1) / 2;
  constexpr int SLOTS = (NBLK - WAVE + 3) / 4;
  constexpr int TILE = CT_ROWS * LD;                 // doubles per tile
  constexpr int CHUNKS = TILE * 8 / 1024 / 4;        // 1-KiB glds pieces per wave per tile (= NB)
  static_assert(CHUNKS * 4 * 1024 == TILE * 8, "tile must split into 4 x NB pieces of 1 KiB");
  // LDS: [2][TILE] tiles | [2][CT_ROWS] weights | [2][CT_ROWS] int epoch flags
  const int tid = threadIdx.x, lane = tid & 63, q = lane >> 4, c = lane & 15;
  double* const wbase = smem + 2 * TILE;
  int* const ebase = (int*)(smem + 2 * TILE + 2 * CT_ROWS);

  v4d acc[SLOTS > 0 ? SLOTS : 1];
#pragma unroll
  for (int sl = 0; sl < SLOTS; ++sl) acc[sl] = v4d{0.0, 0.0, 0.0, 0.0};

  const bool ecorr = P.n_epoch > 0;
  double eacc = 0.0;                                 // running s_e of column `tid`
  // pass 0: TOA rows (weights w); pass 1: epoch rows (weights -beta)
  for (int pass = 0; pass < (ecorr ? 2 : 1); ++pass) {
    const int nrows = pass == 0 ? P.n_toa : P.n_epoch;
    const double* src = pass == 0 ? P.T : srow;
    const double* wsrc = pass == 0 ? wrow : brow;
    const double wsign = pass == 0 ? 1.0 : -1.0;
    const int ntile = (nrows + CT_ROWS - 1) / CT_ROWS;
    auto issue = [&](int it) {
      const char* g = (const char*)(src + (long long)it * TILE) + (WAVE * CHUNKS) * 1024 + lane * 16;
      char* l = (char*)(smem + (it & 1) * TILE) + (WAVE * CHUNKS) * 1024;
#pragma unroll
      for (int k = 0; k < CHUNKS; ++k)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(g + k * 1024), (lds_void_t*)(l + k * 1024), 16, 0, 0);
    };
    double wv = 0.0;
    int ev = -1;
    auto small = [&](int it) {
      const int t = it * CT_ROWS + tid;
      wv = (tid < CT_ROWS && t < nrows) ? wsign * wsrc[t] : 0.0;
      ev = (pass == 0 && tid < CT_ROWS) ? P.toa_ep[t] : -1;
    };
    issue(0);
    small(0);
    if (tid < CT_ROWS) {
      wbase[tid] = wv;
      ebase[tid] = ev;
    }
    __syncthreads();
    for (int it = 0; it < ntile; ++it) {
      const int cur = it & 1;
      if (it + 1 < ntile) {
        issue(it + 1);
        small(it + 1);
      }
      const double* tile = smem + cur * TILE;
      const double* wt = wbase + cur * CT_ROWS;
#pragma unroll
      for (int kk = 0; kk < CT_ROWS / 4; ++kk) {
        const int row = 4 * kk + q;
        const double wr = wt[row];
        const double* trow = tile + row * LD + c;
        double tv[NB], av[NB];
        static_for<0, NB>([&](auto J) {
          constexpr int j = decltype(J)::value;
          if constexpr (wave_uses(NB, WAVE, j)) tv[j] = trow[16 * j];
          if constexpr (wave_uses_row(NB, WAVE, j)) av[j] = wr * tv[j];
        });
        static_for<0, SLOTS>([&](auto SL) {
          constexpr int blk = WAVE + 4 * decltype(SL)::value;
          constexpr int bi = tri_i(NB, blk), bj = tri_j(NB, blk);
          acc[decltype(SL)::value] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[bi], tv[bj], acc[decltype(SL)::value], 0, 0, 0);
        });
      }
      if (pass == 0 && ecorr && tid < LD) {          // epoch sums of column tid
        const double* tcol = tile + tid;
        const int* ecur = ebase + cur * CT_ROWS;
        for (int r = 0; r < CT_ROWS; ++r) {
          const int e = ecur[r];
          if (e >= 0) {
            eacc = fma(wt[r], tcol[r * LD], eacc);
            if (e & 1) {
              srow[(long long)(e >> 1) * LD + tid] = eacc;
              eacc = 0.0;
            }
          }
        }
      }
      if (it + 1 < ntile && tid < CT_ROWS) {
        wbase[(cur ^ 1) * CT_ROWS + tid] = wv;
        ebase[(cur ^ 1) * CT_ROWS + tid] = ev;
      }
      __syncthreads();                               // drains the glds of tile it+1 (vmcnt(0))
    }
    if (pass == 0 && ecorr) __threadfence_block();   // s_e rows visible to the epoch pass
    __syncthreads();
  }
  // epilogue: C/D layout lane -> (row q + 4r, col c); mirror to the lower half,
  // unit diagonal on pad columns (m .. LD-2) so they factor as identity.
  static_for<0, SLOTS>([&](auto SL) {
    constexpr int blk = WAVE + 4 * decltype(SL)::value;
    constexpr int bi = tri_i(NB, blk), bj = tri_j(NB, blk);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 16 * bi + q + 4 * r, col = 16 * bj + c;
      double v = acc[decltype(SL)::value][r];
      if (row == col && row >= P.m && row < LD - 1) v = 1.0;
      Gout[(long long)row * LD + col] = v;
      Gout[(long long)col * LD + row] = v;
    }
  });
}

template <int NB>
__global__ __launch_bounds__(256) void contract2_kernel(PsrDev P, const double* __restrict__ w,
                                                        const double* __restrict__ beta, double* __restrict__ s,
                                                        long long s_stride, double* __restrict__ G) {
  constexpr int LD = 16 * NB;
  const int bl = blockIdx.x;
  const double* wrow = w + (long long)bl * P.n_toa;
  const double* brow = beta + (long long)bl * P.n_epoch;
  double* srow = s + (long long)bl * s_stride;
  double* Gout = G + (long long)bl * LD * LD;
  switch (threadIdx.x >> 6) {
    case 0: contract2_body<NB, 0>(P, wrow, brow, srow, Gout); break;
    case 1: contract2_body<NB, 1>(P, wrow, brow, srow, Gout); break;
    case 2: contract2_body<NB, 2>(P, wrow, brow, srow, Gout); break;
    default: contract2_body<NB, 3>(P, wrow, brow, srow, Gout); break;
  }
}

// ----------------------------------------------------------------------------
// fixed white noise: eliminate the leading constant-phi (timing-model) block
// of G once; write the reduced matrix S (fx_ld x fx_ld, r last) and K.
// One 256-thread block per pulsar; G is modified in place.
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void schur_kernel(double* G, int ld, int m, int nlead,
                                                    const int* __restrict__ col_ptr,
                                                    const DSpec* __restrict__ spec,
                                                    double Kb, double* S, int fx_ld, int fx_m,
                                                    double* Kout, int* fail_out) {
  __shared__ double row[256 * 4];
  __shared__ double red[4];
  double lphi = 0.0;
  for (int a = threadIdx.x; a < nlead; a += 256) {
    double ph = 0.0;
    for (int e = col_ptr[a]; e < col_ptr[a + 1]; ++e) ph += spec_phi(spec[e], nullptr);
    G[(long long)a * ld + a] += 1.0 / ph;
    lphi += log(ph);
  }
  lphi = block_sum256(lphi, red);
  __syncthreads();
  double logdet = 0.0;
  int ok = 1;
  for (int k = 0; k < nlead; ++k) {
    const double piv = G[(long long)k * ld + k];
    ok &= piv > 0.0;
    const double d = sqrt(piv), rinv = 1.0 / d;
    logdet += log(d);
    __syncthreads();
    for (int j = k + 1 + threadIdx.x; j < ld; j += 256) row[j] = G[(long long)k * ld + j] * rinv;
    __syncthreads();
    for (int i = k + 1; i < ld; ++i) {
      const double ri = row[i];
      for (int j = k + 1 + threadIdx.x; j < ld; j += 256) G[(long long)i * ld + j] -= ri * row[j];
    }
    __syncthreads();
  }
  // reduced index a -> G column: a < fx_m -> nlead + a ; a == fx_ld-1 -> ld-1 ; else pad
  for (int idx = threadIdx.x; idx < fx_ld * fx_ld; idx += 256) {
    const int a = idx / fx_ld, bcol = idx % fx_ld;
    const int ga = a < fx_m ? nlead + a : (a == fx_ld - 1 ? ld - 1 : -1);
    const int gb = bcol < fx_m ? nlead + bcol : (bcol == fx_ld - 1 ? ld - 1 : -1);
    double v;
    if (ga < 0 || gb < 0) v = (a == bcol) ? 1.0 : 0.0;
    else v = G[(long long)ga * ld + gb];
    S[idx] = v;
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

// ----------------------------------------------------------------------------
// batched Cholesky, MFMA register-blocked: one wave (64 lanes) per unit.
// The upper triangle of the LD x LD matrix (LD = 16 NB) is held as 16x16
// blocks in the v_mfma_f64_16x16x4_f64 C/D layout (lane l, reg r <-> row
// (l>>4) + 4r, col l&15).  Factor A = U^T U (upper, as LAPACK dpotrf 'U'
// behind scipy cho_factor).  Per block row bb the 16 pivots of the panel are
// done by VALU (pivot by readlane, 1/sqrt by v_rsq_f64 + Newton, row k
// broadcast by ds_bpermute, only the rows that can still change are
// touched); trailing blocks get A_ij -= U_bi^T U_bj by four MFMAs each with
// no data movement — register s of a C/D-layout block IS the MFMA A / B
// operand of k-slice s.
//
// Three phases keep at most 26 blocks live for NB = 8 (36 in a plain
// right-looking order): (1) factor block rows 0..H-1 (H = NB/2) with the
// trailing update restricted to those rows; (2) load the trailing A22
// triangle and apply the H panel rows to it; (3) factor A22.  Same
// arithmetic, re-ordered (left-looking at the 2x2 block level).
// ----------------------------------------------------------------------------
template <int NB>
struct Split {
  // block rows of phase 1: NB/2, except 3 of 8 (phase 1's 21 blocks + panel
  // temporaries then fit 256 VGPRs without spills; phase 2 runs row by row)
  static constexpr int H = NB == 8 ? 3 : NB / 2;
  static constexpr int M = NB - H;                    // A22 block order
  static constexpr int n1 = H * NB - H * (H - 1) / 2; // blocks (i < H, j >= i)
  static constexpr int n2 = M * (M + 1) / 2;          // blocks (H <= i <= j)
  static constexpr int i1(int i, int j) { return i * NB - (i * (i - 1)) / 2 + (j - i); }
  static constexpr int i2(int i, int j) { return (i - H) * M - ((i - H) * (i - H - 1)) / 2 + (j - i); }
};

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// A -= U_i^T U_j : four f64 MFMAs (A operand = -U_i)
__device__ __forceinline__ void syrk_update(v4d& C, const v4d& Ui, const v4d& Uj) {
#pragma unroll
  for (int sk = 0; sk < 4; ++sk) C = __builtin_amdgcn_mfma_f64_16x16x4f64(-Ui[sk], Uj[sk], C, 0, 0, 0);
}

// FULL: 1 = every panel step unrolled (large code), 0 = runtime loop over the
// row's lane group (the default)
// W: waves per SIMD the register budget is cut for (2 -> 256 VGPRs: the NB = 8
// three-phase kernel fits with no spills, so two units share each SIMD and one's
// MFMAs overlap the other's VALU / LDS latency).
// ALG: panel form.  0 = Cholesky panel (row k scaled by 1/sqrt(pivot) before it
// is broadcast); 1 = square-root-free LDL^T panel: row k is broadcast raw while
// 1/d_k is formed, the lane's rows take the update with u_i = A_ki / d_k, and
// the 16 rows of the block row are scaled to U = D^-1/2 V together at the end
// (one vector rsqrt per register instead of one serial rsqrt per pivot).  The
// per-pivot dependency chain drops the scale -> ds_bpermute leg; log|Sigma| =
// sum log d_k is accumulated per block row from the lanes' own pivots.
// LDL^T panel of block row BB over the blocks blk(j), j = BB..NB-1 (C/D
// layout, upper triangle), used by the register-resident kernels: the 16
// pivots are factored by VALU (ALG 1: row k broadcast by ds_bpermute, ALG 2:
// through the per-wave LDS `rowbuf`), then the block row is scaled to
// U = D^-1/2 V.  Accumulates log d_k (one lane per row) and d_k > 0 per lane.
template <int NB, int FULL, int ALG, typename BBt, typename Blk>
__device__ __forceinline__ void panel_ldl_row(BBt BBc, Blk&& blk, int q, int c, LogAcc& ldet, bool& ok,
                                              double* rowbuf) {
  constexpr int LD = 16 * NB;
  (void)rowbuf;
  (void)LD;
  constexpr int bb = decltype(BBc)::value;
  static_for<0, 4>([&](auto KR) {
    constexpr int kr = decltype(KR)::value;
    auto step = [&](const int kq) {
      const int k = 4 * kr + kq;
      const double d = readlane_d(blk(BBc)[kr], 16 * kq + k);            // wave-uniform pivot
      // raw row k: A[k][q + 4r] for this lane's rows (masked to rows > k) and
      // A[k][col c] of every block of the row; both in flight while 1/d forms
      double ui[4];
      double rk[NB];
      if constexpr (ALG == 2) {
        // LDS broadcast: the 16 lanes of quad kq store row k of every block
        // (one ds_write_b64 per block), every lane reads it back with 16
        // distinct addresses per read (broadcast, bank-conflict free) --
        // several times cheaper on the CU's LDS than two ds_bpermute_b32
        // per double.  One wave per workgroup and LDS ops of a wave run in
        // order, so no barrier: the asm fences only stop the compiler from
        // moving the reads above the other lanes' writes.
        double* rb = rowbuf + (k & 1) * LD;
        if (q == kq) {
          static_for<bb, NB>([&](auto JJ) {
            constexpr int j = decltype(JJ)::value;
            rb[16 * j + c] = blk(JJ)[kr];
          });
        }
        asm volatile("" ::: "memory");
        static_for<kr, 4>([&](auto R) {
          constexpr int r = decltype(R)::value;
          const double v = rb[16 * bb + q + 4 * r];
          ui[r] = (r > kr || q > kq) ? v : 0.0;
        });
        static_for<bb, NB>([&](auto JJ) {
          constexpr int j = decltype(JJ)::value;
          rk[j] = rb[16 * j + c];
        });
        asm volatile("" ::: "memory");
      } else {
        static_for<kr, 4>([&](auto R) {
          constexpr int r = decltype(R)::value;
          const double v = __shfl(blk(BBc)[kr], 16 * kq + q + 4 * r);
          ui[r] = (r > kr || q > kq) ? v : 0.0;
        });
        static_for<bb, NB>([&](auto JJ) {
          constexpr int j = decltype(JJ)::value;
          rk[j] = __shfl(blk(JJ)[kr], 16 * kq + c);
        });
      }
      const double dinv = rcp_nr(d);
      static_for<kr, 4>([&](auto R) { ui[decltype(R)::value] *= dinv; });
      static_for<bb, NB>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        static_for<kr, 4>([&](auto R) {
          constexpr int r = decltype(R)::value;
          blk(JJ)[r] = fma(-ui[r], rk[j], blk(JJ)[r]);
        });
      });
    };
    constexpr int nk = (bb == NB - 1 && kr == 3) ? 3 : 4;   // the r column is not pivoted
    if constexpr (FULL) {
      static_for<0, nk>([&](auto KQ) {
        step(decltype(KQ)::value);
        // unrolled LDS-broadcast steps: keep the scheduler from hoisting the
        // next steps' LDS reads (it otherwise spills ~1 KB per lane)
        if constexpr (ALG == 2) __builtin_amdgcn_sched_barrier(0);
      });
    } else {
#pragma unroll 1
      for (int kq = 0; kq < nk; ++kq) step(kq);
    }
  });
  // rows of the block row -> U = d^-1/2 V, d of row q + 4r read from the
  // diagonal (lane 17q + 4r); log-det and positivity from one lane per row
  // (c == 0); the r row (last block, row 15) is left as it is
  static_for<0, 4>([&](auto R) {
    constexpr int r = decltype(R)::value;
    const bool rrow = (bb == NB - 1 && r == 3) && q == 3;
    const double dg = __shfl(blk(BBc)[r], 17 * q + 4 * r);
    const double dv = rrow ? 1.0 : dg;
    ok = ok && (dv > 0.0);
    if (c == 0) ldet.add(dv);
    const double rs = rrow ? 1.0 : rsqrt_nr(dv);
    static_for<bb, NB>([&](auto JJ) { blk(JJ)[r] *= rs; });
  });
}

template <int NB, int FULL, int W, int ALG = 0>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(W, W)))
void chol_mfma_kernel(const CholJob* __restrict__ jobs, int B, long long u0, int b_off,
                      const double* __restrict__ theta, int ldth, double* __restrict__ out_units) {
  constexpr int LD = 16 * NB;
  using S = Split<NB>;
  constexpr int H = S::H;
  __shared__ double phinv[LD];
  __shared__ double rowbuf[ALG == 2 ? 2 * LD : 1];   // ALG 2: double-buffered row-k broadcast
  const int lane = threadIdx.x;
  const int q = lane >> 4, c = lane & 15;
  const long long u = u0 + xcd_unit(blockIdx.x, gridDim.x);
  const int p = (int)(u / B), b = (int)(u % B);
  const CholJob J = jobs[p];
  const double* A = J.mats + (long long)(b - b_off) * J.mstride;
  const double* th = theta + (long long)b * ldth;

  LogAcc lphi;
  for (int a = lane; a < LD; a += 64) {
    double pi = 0.0;
    if (a < J.mreal) {
      double ph = 0.0;
      for (int e = J.col_ptr[a]; e < J.col_ptr[a + 1]; ++e) ph += spec_phi_body(J.spec[e], th);
      pi = 1.0 / ph;
      lphi.add(ph);
    }
    phinv[a] = pi;
  }
  const double lphi_sum = wave_sum(lphi.value());
  __syncthreads();

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

  LogAcc ldet;
  bool ok = true;
  // LDL^T panel row bb (ALG >= 1)
  auto panel_ldl = [&](auto BBc, auto&& blk) {
    panel_ldl_row<NB, FULL, ALG>(BBc, blk, q, c, ldet, ok, rowbuf);
  };
  // panel row bb over the blocks blk(j), j = bb..NB-1
  auto panel = [&](auto BBc, auto&& blk) {
    if constexpr (ALG >= 1) {
      panel_ldl(BBc, blk);
      return;
    }
    constexpr int bb = decltype(BBc)::value;
    static_for<0, 4>([&](auto KR) {
      constexpr int kr = decltype(KR)::value;
      auto step = [&](const int kq) {
        const int k = 4 * kr + kq;
        const double piv = readlane_d(blk(BBc)[kr], 16 * kq + k);           // wave-uniform
        ok = ok && (piv > 0.0);
        ldet.add(piv);
        const double rin = rsqrt_nr(piv);
        const double sc = (q == kq) ? rin : 1.0;                             // scales row k only
        const double xbb = blk(BBc)[kr] * sc;
        // U[k][q + 4r] for this lane's rows; rows <= k are final (r < kr never
        // changes, r == kr only for q > kq)
        double ui[4];
        static_for<kr, 4>([&](auto R) {
          constexpr int r = decltype(R)::value;
          const double v = __shfl(xbb, 16 * kq + q + 4 * r);
          ui[r] = (r > kr || q > kq) ? v : 0.0;
        });
        double rk[NB];
        static_for<bb, NB>([&](auto JJ) {
          constexpr int j = decltype(JJ)::value;
          const double x = (j == bb) ? xbb : blk(JJ)[kr] * sc;
          blk(JJ)[kr] = x;
          rk[j] = __shfl(x, 16 * kq + c);                                    // U[k][col c] of block (bb, j)
        });
        static_for<bb, NB>([&](auto JJ) {
          constexpr int j = decltype(JJ)::value;
          static_for<kr, 4>([&](auto R) {
            constexpr int r = decltype(R)::value;
            blk(JJ)[r] = fma(-ui[r], rk[j], blk(JJ)[r]);
          });
        });
      };
      constexpr int nk = (bb == NB - 1 && kr == 3) ? 3 : 4;   // the r column is not pivoted
      if constexpr (FULL) {
        static_for<0, nk>([&](auto KQ) { step(decltype(KQ)::value); });
      } else {
#pragma unroll 1
        for (int kq = 0; kq < nk; ++kq) step(kq);
      }
    });
  };

  // ---- phase 1: block rows 0..H-1 ----
  v4d U1[S::n1 > 0 ? S::n1 : 1];
  static_for<0, H>([&](auto BI) {
    constexpr int bi = decltype(BI)::value;
    static_for<bi, NB>([&](auto BJ) { load_block(BI, BJ, U1[S::i1(bi, decltype(BJ)::value)]); });
  });
  static_for<0, H>([&](auto BBc) {
    constexpr int bb = decltype(BBc)::value;
    panel(BBc, [&](auto JJ) -> v4d& { return U1[S::i1(bb, decltype(JJ)::value)]; });
    static_for<bb + 1, H>([&](auto II) {
      constexpr int i = decltype(II)::value;
      static_for<i, NB>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        syrk_update(U1[S::i1(i, j)], U1[S::i1(bb, i)], U1[S::i1(bb, j)]);
      });
    });
  });
  // ---- phase 2: A22 -= U12^T U12 ----
  // block by block in row order: U1 column i is dead once row i of A22 is done
  v4d U2[S::n2];
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
  // ---- phase 3: factor A22 ----
  static_for<H, NB>([&](auto BBc) {
    constexpr int bb = decltype(BBc)::value;
    panel(BBc, [&](auto JJ) -> v4d& { return U2[S::i2(bb, decltype(JJ)::value)]; });
    static_for<bb + 1, NB>([&](auto II) {
      constexpr int i = decltype(II)::value;
      static_for<i, NB>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        syrk_update(U2[S::i2(i, j)], U2[S::i2(bb, i)], U2[S::i2(bb, j)]);
      });
    });
  });
  const double qv = readlane_d(U2[S::i2(NB - 1, NB - 1)][3], 63);
  double ldet_v = ldet.value();
  bool ok_all = ok;
  if constexpr (ALG >= 1) {          // per-lane partial log-dets and checks
    ldet_v = wave_sum(ldet_v);
    ok_all = __all(ok);
  }
  if (lane == 0) {
    double lnl = J.K[(long long)(b - b_off) * J.kstride] - 0.5 * qv - 0.5 * ldet_v - 0.5 * lphi_sum;
    if (!ok_all || J.fail) lnl = -INFINITY;
    out_units[(long long)p * B + b] = lnl;
  }
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
  const double* A = J.mats + (long long)(b - b_off) * J.mstride;
  const double* th = theta + (long long)b * ldth;
  double* scr = scratch + (long long)blockIdx.x * (NB * (NB + 1) / 2) * 256 + lane * 4;

  LogAcc lphi;
  for (int a = lane; a < LD; a += 64) {
    double pi = 0.0;
    if (a < J.mreal) {
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
        const v4d Ui = *(const v4d*)(scr + big_blk<NB>(pp, i) * 256);
        static_for<0, W>([&](auto JJ) {
          constexpr int jj = decltype(JJ)::value;
          const v4d Uj = *(const v4d*)(scr + big_blk<NB>(pp, i + jj) * 256);
          syrk_update(R[jj], Ui, Uj);
        });
      }
    }
    panel_ldl_row<NB, 0, 1>(I, [&](auto JJ) -> v4d& { return R[decltype(JJ)::value - i]; }, q, c, ldet, ok,
                            nullptr);
    if constexpr (i < NB - 1) {
      static_for<0, W>([&](auto JJ) {
        constexpr int j = i + decltype(JJ)::value;
        *(v4d*)(scr + big_blk<NB>(i, j) * 256) = R[j - i];
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

// out[b] = sum_p units[p * B + b], pulsars in order.
__global__ void reduce_units_kernel(const double* __restrict__ units, int P, int B, double* __restrict__ out) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  double s = 0.0;
  for (int p = 0; p < P; ++p) s += units[(long long)p * B + b];
  out[b] = s;
}

// ----------------------------------------------------------------------------
// host side
// ----------------------------------------------------------------------------
constexpr int MFMA_NB_MAX = 9;
constexpr size_t LDS_MAX = 160 * 1024;

struct PsrHost {
  int n_toa = 0, m = 0, nlead = 0, ld = 0, nb = 0, n_epoch = 0;
  int fx_m = 0, fx_ld = 0, fx_nb = 0;
  PsrDev dev{};
  int* d_colptr = nullptr;        // varying CSR (m+1)
  DSpec* d_spec = nullptr;
  int* d_fx_colptr = nullptr;     // fixed CSR (fx_m+1), entries re-indexed
  DSpec* d_fx_spec = nullptr;
  double* d_S = nullptr;          // fx_ld^2
  bool has_theta_white = false;
};

}  // namespace

struct ewh_handle {
  int device = 0;
  int P = 0, n_param = 0;
  bool white_fixed = false;
  int kernel_mode = 0;
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
  long long s_stride = 0;     // doubles per sample in d_s (epoch rows padded to whole tiles)
  double* d_bigscr = nullptr; // chol_big_kernel: per-workgroup U blocks
  long long bigscr_cap = 0;   // workgroups per launch it holds
  int bigscr_nb = 0;
  int chunk = 0;
  int last_B = 0;
};

namespace {

template <typename T>
int dalloc(ewh_handle* h, T** p, size_t count) {
  *p = nullptr;
  if (count == 0) count = 1;
  hipError_t e = hipMalloc((void**)p, count * sizeof(T));
  if (e != hipSuccess) return set_err(EWH_E_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  h->allocs.push_back(*p);
  return 0;
}

template <typename T>
int dupload(ewh_handle* h, T** p, const T* src, size_t count) {
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
  if (!d || d->abi_version != EWH_ABI_VERSION) return set_err(EWH_E_INVALID, "bad descriptor / ABI version");
  if (d->n_pulsar <= 0 || !d->pulsars) return set_err(EWH_E_INVALID, "no pulsars");
  if (d->n_param < 0) return set_err(EWH_E_INVALID, "n_param < 0");
  for (int p = 0; p < d->n_pulsar; ++p) {
    const ewh_pulsar_desc& s = d->pulsars[p];
    const std::string tag = "pulsar " + std::to_string(p) + ": ";
    if (s.n_toa <= 0 || s.n_col < 0 || s.n_lead_const < 0 || s.n_lead_const > s.n_col)
      return set_err(EWH_E_INVALID, tag + "bad sizes");
    if ((s.n_col && !s.basis) || !s.resid || !s.toaerr || !s.efac_slot || !s.equad_slot ||
        (s.n_slot && !s.slots) || (s.n_spec && !s.spec))
      return set_err(EWH_E_INVALID, tag + "null pointer");
    if (s.n_epoch && (!s.epoch_start || !s.epoch_stop || !s.epoch_slot))
      return set_err(EWH_E_INVALID, tag + "null epoch pointer");
    for (int i = 0; i < s.n_slot; ++i)
      if (s.slots[i].idx >= d->n_param) return set_err(EWH_E_INVALID, tag + "slot theta index out of range");
    for (int t = 0; t < s.n_toa; ++t) {
      if (s.efac_slot[t] < 0 || s.efac_slot[t] >= s.n_slot) return set_err(EWH_E_INVALID, tag + "efac slot out of range");
      if (s.equad_slot[t] >= s.n_slot) return set_err(EWH_E_INVALID, tag + "equad slot out of range");
    }
    int prev = 0;
    for (int e = 0; e < s.n_epoch; ++e) {
      if (s.epoch_start[e] < prev || s.epoch_stop[e] <= s.epoch_start[e] + 1 || s.epoch_stop[e] > s.n_toa)
        return set_err(EWH_E_INVALID, tag + "epochs must be ordered, disjoint slices of >= 2 TOAs");
      if (s.epoch_slot[e] < 0 || s.epoch_slot[e] >= s.n_slot) return set_err(EWH_E_INVALID, tag + "epoch slot out of range");
      prev = s.epoch_stop[e];
    }
    if (s.n_bgroup < 0 || (s.n_bgroup > 0 && (!s.bgroup_idx || !s.col_bgroup || !s.ln_chrom)))
      return set_err(EWH_E_INVALID, tag + "bad basis-group tables");
    for (int g = 0; g < s.n_bgroup; ++g)
      if (s.bgroup_idx[g].idx >= d->n_param) return set_err(EWH_E_INVALID, tag + "basis-group theta index out of range");
    for (int j = 0; s.n_bgroup > 0 && j < s.n_col; ++j)
      if (s.col_bgroup[j] < -1 || s.col_bgroup[j] >= s.n_bgroup || (j < s.n_lead_const && s.col_bgroup[j] >= 0))
        return set_err(EWH_E_INVALID, tag + "bad column basis group");
    std::vector<int> cnt(s.n_col, 0);
    for (int e = 0; e < s.n_spec; ++e) {
      const ewh_spec_entry& sp = s.spec[e];
      if (sp.col < 0 || sp.col >= s.n_col) return set_err(EWH_E_INVALID, tag + "spectral column out of range");
      if (sp.kind < EWH_SPEC_POWERLAW || sp.kind > EWH_SPEC_CONST) return set_err(EWH_E_INVALID, tag + "bad spectral kind");
      if (sp.p0.idx >= d->n_param || sp.p1.idx >= d->n_param || sp.p2.idx >= d->n_param)
        return set_err(EWH_E_INVALID, tag + "spectral theta index out of range");
      if (sp.col < s.n_lead_const && sp.kind != EWH_SPEC_CONST)
        return set_err(EWH_E_INVALID, tag + "leading columns must have constant phi");
      cnt[sp.col]++;
    }
    for (int j = 0; j < s.n_col; ++j)
      if (!cnt[j]) return set_err(EWH_E_INVALID, tag + "column " + std::to_string(j) + " has no phi entry");
  }
  return 0;
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

template <int NB>
void launch_contract(const PsrDev& P, const double* w, const double* beta, const double* s, const double* fac,
                     double* G, int nb_samples, hipStream_t st) {
  const size_t lds = (size_t)(CT_ROWS * 16 * NB + CT_ROWS) * sizeof(double);
  hipLaunchKernelGGL(HIP_KERNEL_NAME(contract_mfma_kernel<NB>), dim3(nb_samples), dim3(256), lds, st, P, w, beta, s,
                     fac, G);
}

int dispatch_contract(int nb, const PsrDev& P, const double* w, const double* beta, const double* s,
                      const double* fac, double* G, int nb_samples, hipStream_t st) {
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
    default: return set_err(EWH_E_UNSUPPORTED, "basis too wide for the contraction kernel (> 207 columns)");
  }
  return 0;
}

constexpr int CONTRACT2_NB_MAX = 13;

template <int NB>
int launch_contract2(const PsrDev& P, const double* w, const double* beta, double* s, long long s_stride, double* G,
                     int nb_samples, hipStream_t st) {
  const size_t lds = (size_t)(2 * CT_ROWS * 16 * NB + 3 * CT_ROWS) * sizeof(double);
  static bool attr = false;
  if (!attr) {
    EWH_HIP(hipFuncSetAttribute((const void*)contract2_kernel<NB>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds));
    attr = true;
  }
  hipLaunchKernelGGL(HIP_KERNEL_NAME(contract2_kernel<NB>), dim3(nb_samples), dim3(256), lds, st, P, w, beta, s,
                     s_stride, G);
  return 0;
}

int dispatch_contract2(int nb, const PsrDev& P, const double* w, const double* beta, double* s, long long s_stride,
                       double* G, int nb_samples, hipStream_t st) {
  switch (nb) {
    case 1: return launch_contract2<1>(P, w, beta, s, s_stride, G, nb_samples, st);
    case 2: return launch_contract2<2>(P, w, beta, s, s_stride, G, nb_samples, st);
    case 3: return launch_contract2<3>(P, w, beta, s, s_stride, G, nb_samples, st);
    case 4: return launch_contract2<4>(P, w, beta, s, s_stride, G, nb_samples, st);
    case 5: return launch_contract2<5>(P, w, beta, s, s_stride, G, nb_samples, st);
    case 6: return launch_contract2<6>(P, w, beta, s, s_stride, G, nb_samples, st);
    case 7: return launch_contract2<7>(P, w, beta, s, s_stride, G, nb_samples, st);
    case 8: return launch_contract2<8>(P, w, beta, s, s_stride, G, nb_samples, st);
    case 9: return launch_contract2<9>(P, w, beta, s, s_stride, G, nb_samples, st);
    case 10: return launch_contract2<10>(P, w, beta, s, s_stride, G, nb_samples, st);
    case 11: return launch_contract2<11>(P, w, beta, s, s_stride, G, nb_samples, st);
    case 12: return launch_contract2<12>(P, w, beta, s, s_stride, G, nb_samples, st);
    case 13: return launch_contract2<13>(P, w, beta, s, s_stride, G, nb_samples, st);
    default: return set_err(EWH_E_UNSUPPORTED, "basis too wide for the contraction kernel (> 207 columns)");
  }
}

constexpr int default_waves(int nb) { return nb <= 8 ? 2 : 1; }

template <int NB, int FULL = 0, int W = default_waves(NB), int ALG = 0>
void launch_chol_mfma(const CholJob* jobs, int B, long long u0, long long n, int b_off, const double* theta, int ldth,
                      double* units, hipStream_t st) {
  hipLaunchKernelGGL(HIP_KERNEL_NAME(chol_mfma_kernel<NB, FULL, W, ALG>), dim3((unsigned)n), dim3(64), 0, st, jobs, B,
                     u0, b_off, theta, ldth, units);
}

template <int NB>
void launch_chol_big(const CholJob* jobs, int B, long long u0, long long n, int b_off, const double* theta, int ldth,
                     double* units, double* scr, long long cap, hipStream_t st) {
  for (long long o = 0; o < n; o += cap)   // one scratch slot per workgroup of a launch
    hipLaunchKernelGGL(HIP_KERNEL_NAME(chol_big_kernel<NB>), dim3((unsigned)std::min(cap, n - o)), dim3(64), 0, st,
                       jobs, B, u0 + o, b_off, theta, ldth, units, scr);
}

int dispatch_chol(int mode, int nb, int mreal, const CholJob* jobs, int B, long long u0, long long n, int b_off,
                  const double* theta, int ldth, double* units, hipStream_t st, double* bigscr = nullptr,
                  long long bigcap = 0) {
  if (n <= 0) return 0;
  if (mode != 1 && nb > MFMA_NB_MAX && nb <= BIG_NB_MAX && bigscr) {
    switch (nb) {
      case 10: launch_chol_big<10>(jobs, B, u0, n, b_off, theta, ldth, units, bigscr, bigcap, st); return 0;
      case 11: launch_chol_big<11>(jobs, B, u0, n, b_off, theta, ldth, units, bigscr, bigcap, st); return 0;
      case 12: launch_chol_big<12>(jobs, B, u0, n, b_off, theta, ldth, units, bigscr, bigcap, st); return 0;
      case 13: launch_chol_big<13>(jobs, B, u0, n, b_off, theta, ldth, units, bigscr, bigcap, st); return 0;
      case 14: launch_chol_big<14>(jobs, B, u0, n, b_off, theta, ldth, units, bigscr, bigcap, st); return 0;
      case 15: launch_chol_big<15>(jobs, B, u0, n, b_off, theta, ldth, units, bigscr, bigcap, st); return 0;
      case 16: launch_chol_big<16>(jobs, B, u0, n, b_off, theta, ldth, units, bigscr, bigcap, st); return 0;
      default: break;
    }
  }
  // A/B variants (NB = 8, the C3 reduced width); see ewh_set_kernel_mode
  if (nb == 8 && mode >= 3) {
    switch (mode) {
      case 3: launch_chol_mfma<8, 1, 1, 1>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // 1 wave/SIMD
      case 4: launch_chol_mfma<8, 0, 2, 1>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // LDL, looped
      case 5: launch_chol_mfma<8, 1, 2, 0>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // Cholesky, unrolled
      case 6: launch_chol_mfma<8, 0, 2, 2>(jobs, B, u0, n, b_off, theta, ldth, units, st); return 0;  // LDL, LDS bcast
      default: break;
    }
  }
  if (mode != 1 && nb <= MFMA_NB_MAX) {
    // default: LDL^T panel, panel steps unrolled up to NB = 8; mode 2: the
    // round-1 Cholesky panel (looped) as the A/B baseline
    const bool base = mode == 2;
#define EWH_CHOL_CASE(NBV)                                                                            \
  case NBV:                                                                                          \
    if (base) launch_chol_mfma<NBV, 0, default_waves(NBV), 0>(jobs, B, u0, n, b_off, theta, ldth, units, st); \
    else launch_chol_mfma<NBV, (NBV <= 8), default_waves(NBV), 1>(jobs, B, u0, n, b_off, theta, ldth, units, st); \
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
      default: break;
    }
#undef EWH_CHOL_CASE
  }
  const size_t lds = lds_bytes_chol(mreal);
  if (lds > LDS_MAX - 64) return set_err(EWH_E_UNSUPPORTED, "reduced matrix too large for the LDS Cholesky kernel");
  static bool attr_set = false;
  if (!attr_set) {
    EWH_HIP(hipFuncSetAttribute((const void*)chol_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)(LDS_MAX - 64)));
    attr_set = true;
  }
  hipLaunchKernelGGL(chol_lds_kernel, dim3((unsigned)n), dim3(256), lds, st, jobs, B, u0, b_off, theta, ldth, units);
  return 0;
}

// scratch of chol_big_kernel for NB: BIG_SLOTS workgroups x NB(NB+1)/2 blocks of 2 KiB
constexpr long long BIG_SLOTS = 2048;
int ensure_big_scratch(ewh_handle* h, int nb) {
  if (nb <= MFMA_NB_MAX || nb > BIG_NB_MAX || nb <= h->bigscr_nb) return 0;
  if (h->d_bigscr) {
    hipFree(h->d_bigscr);
    h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), (void*)h->d_bigscr));
    h->d_bigscr = nullptr;
  }
  int rc = dalloc(h, &h->d_bigscr, (size_t)BIG_SLOTS * (nb * (nb + 1) / 2) * 256);
  if (rc) return rc;
  h->bigscr_cap = BIG_SLOTS;
  h->bigscr_nb = nb;
  return 0;
}

int ensure_units(ewh_handle* h, int B) {
  const size_t need = (size_t)h->P * B;
  if (need <= h->units_cap) return 0;
  if (h->d_units) {
    hipFree(h->d_units);
    h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), (void*)h->d_units));
  }
  h->units_cap = 0;
  int rc = dalloc(h, &h->d_units, need);
  if (rc) return rc;
  h->units_cap = need;
  return 0;
}

int ensure_var_scratch(ewh_handle* h, int B) {
  if (h->white_fixed) return 0;
  if (h->chunk > 0 && (h->chunk >= B || h->chunk >= 1024)) return 0;
  for (void* p : {(void*)h->d_w, (void*)h->d_beta, (void*)h->d_s, (void*)h->d_G, (void*)h->d_Kb, (void*)h->d_fac}) {
    if (p) {
      hipFree(p);
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
  // chunk: keep G (ld^2) and s (E*ld) scratch under ~1.5 GB
  // epoch-sum rows per sample: whole CT_ROWS tiles (+1) so the pipelined
  // contraction's last epoch tile reads zero-initialised pad rows
  const size_t sstride = ((maxe + CT_ROWS - 1) / CT_ROWS + 1) * CT_ROWS * maxld;
  const size_t per = (maxld * maxld + sstride + maxn + maxe + maxfac + 1) * sizeof(double);
  size_t chunk = std::max<size_t>(1, (size_t)1536 * 1024 * 1024 / per);
  chunk = std::min<size_t>(chunk, std::min<size_t>(std::max(B, 1), 1024));
  int rc;
  if ((rc = dalloc(h, &h->d_w, chunk * maxn))) return rc;
  if ((rc = dalloc(h, &h->d_beta, chunk * maxe))) return rc;
  if ((rc = dalloc(h, &h->d_s, chunk * sstride))) return rc;
  EWH_HIP(hipMemset(h->d_s, 0, chunk * sstride * sizeof(double)));
  h->s_stride = (long long)sstride;
  if ((rc = dalloc(h, &h->d_G, chunk * maxld * maxld))) return rc;
  if ((rc = dalloc(h, &h->d_Kb, chunk))) return rc;
  if ((rc = dalloc(h, &h->d_fac, chunk * maxfac))) return rc;
  h->chunk = (int)chunk;
  std::vector<CholJob> jobs(h->P);
  for (int p = 0; p < h->P; ++p) {
    const PsrHost& ps = h->psr[p];
    jobs[p] = CholJob{h->d_G, (long long)ps.ld * ps.ld, ps.ld, ps.m, ps.d_colptr, ps.d_spec, h->d_Kb, 1, 0};
  }
  EWH_HIP(hipMemcpy(h->d_jobs_var, jobs.data(), sizeof(CholJob) * h->P, hipMemcpyHostToDevice));
  return 0;
}

// white-noise terms of one pulsar for samples [b0, b0 + nb) into the chunk scratch
int run_white(ewh_handle* h, int p, const double* theta, int ldth, int b0, int nb) {
  PsrHost& ps = h->psr[p];
  hipLaunchKernelGGL(wn_weights_kernel, dim3(nb), dim3(256), 0, h->stream, ps.dev, theta, ldth, b0, h->d_w,
                     h->d_beta, h->d_Kb, h->d_fac);
  if (ps.dev.n_bgroup == 0 && h->kernel_mode != 7 && ps.nb <= CONTRACT2_NB_MAX) {
    int rc = dispatch_contract2(ps.nb, ps.dev, h->d_w, h->d_beta, h->d_s, h->s_stride, h->d_G, nb, h->stream);
    if (rc) return rc;
    EWH_HIP(hipGetLastError());
    return 0;
  }
  if (ps.n_epoch > 0)
    hipLaunchKernelGGL(epoch_sums_kernel, dim3(ps.n_epoch, nb), dim3(256), 0, h->stream, ps.dev, h->d_w, h->d_fac,
                       h->d_s);
  int rc = dispatch_contract(ps.nb, ps.dev, h->d_w, h->d_beta, h->d_s, h->d_fac, h->d_G, nb, h->stream);
  if (rc) return rc;
  EWH_HIP(hipGetLastError());
  return 0;
}

int setup_fixed(ewh_handle* h, const ewh_pta_desc* d) {
  // one-sample scratch; theta is never read (all white-noise slots constant)
  int rc;
  size_t maxn = 1, maxe = 1, maxld = 16;
  for (auto& ps : h->psr) {
    maxn = std::max(maxn, (size_t)ps.n_toa);
    maxe = std::max(maxe, (size_t)ps.n_epoch);
    maxld = std::max(maxld, (size_t)ps.ld);
  }
  double *w, *beta, *s, *G, *Kb;
  if ((rc = dalloc(h, &w, maxn))) return rc;
  if ((rc = dalloc(h, &beta, maxe))) return rc;
  if ((rc = dalloc(h, &s, maxe * maxld))) return rc;
  if ((rc = dalloc(h, &G, maxld * maxld))) return rc;
  if ((rc = dalloc(h, &Kb, 1))) return rc;
  double* dummy_theta;
  if ((rc = dalloc(h, &dummy_theta, std::max(1, d->n_param)))) return rc;
  EWH_HIP(hipMemset(dummy_theta, 0, sizeof(double) * std::max(1, d->n_param)));
  if ((rc = dalloc(h, &h->d_fxK, h->P))) return rc;
  if ((rc = dalloc(h, &h->d_fxfail, h->P))) return rc;
  std::vector<CholJob> jobs(h->P);
  for (int p = 0; p < h->P; ++p) {
    PsrHost& ps = h->psr[p];
    hipLaunchKernelGGL(wn_weights_kernel, dim3(1), dim3(256), 0, h->stream, ps.dev, dummy_theta, 0, 0, w, beta, Kb,
                       nullptr);
    if (ps.n_epoch > 0)
      hipLaunchKernelGGL(epoch_sums_kernel, dim3(ps.n_epoch, 1), dim3(256), 0, h->stream, ps.dev, w, nullptr, s);
    if ((rc = dispatch_contract(ps.nb, ps.dev, w, beta, s, nullptr, G, 1, h->stream))) return rc;
    double Kb_h = 0.0;
    EWH_HIP(hipMemcpyAsync(&Kb_h, Kb, sizeof(double), hipMemcpyDeviceToHost, h->stream));
    EWH_HIP(hipStreamSynchronize(h->stream));
    if ((rc = dalloc(h, &ps.d_S, (size_t)ps.fx_ld * ps.fx_ld))) return rc;
    hipLaunchKernelGGL(schur_kernel, dim3(1), dim3(256), 0, h->stream, G, ps.ld, ps.m, ps.nlead, ps.d_colptr,
                       ps.d_spec, Kb_h, ps.d_S, ps.fx_ld, ps.fx_m, h->d_fxK + p, h->d_fxfail + p);
    EWH_HIP(hipGetLastError());
    EWH_HIP(hipStreamSynchronize(h->stream));
    int fail = 0;
    EWH_HIP(hipMemcpy(&fail, h->d_fxfail + p, sizeof(int), hipMemcpyDeviceToHost));
    jobs[p] = CholJob{ps.d_S, 0, ps.fx_ld, ps.fx_m, ps.d_fx_colptr, ps.d_fx_spec, h->d_fxK + p, 0, fail};
  }
  EWH_HIP(hipMemcpy(h->d_jobs_fixed, jobs.data(), sizeof(CholJob) * h->P, hipMemcpyHostToDevice));
  return 0;
}

}  // namespace

extern "C" {

int ewh_version(void) { return EWH_ABI_VERSION; }

const char* ewh_last_error(void) { return g_err.c_str(); }

int ewh_create(const ewh_pta_desc* d, int device, ewh_handle** out) {
  if (!out) return set_err(EWH_E_INVALID, "out is NULL");
  *out = nullptr;
  int rc = validate(d);
  if (rc) return rc;
  EWH_HIP(hipSetDevice(device));
  ewh_handle* h = new ewh_handle();
  h->device = device;
  h->P = d->n_pulsar;
  h->n_param = d->n_param;
  h->psr.resize(h->P);
  auto bail = [&](int code) {
    ewh_destroy(h);
    return code;
  };
  if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess)
    return bail(set_err(EWH_E_HIP, "hipStreamCreate failed"));
  bool any_theta_white = false;
  for (int p = 0; p < h->P; ++p) {
    const ewh_pulsar_desc& s = d->pulsars[p];
    PsrHost& ps = h->psr[p];
    ps.n_toa = s.n_toa;
    ps.m = s.n_col;
    ps.nlead = s.n_lead_const;
    ps.nb = nb_for(s.n_col + 1);
    ps.ld = 16 * ps.nb;
    ps.n_epoch = s.n_epoch;
    ps.fx_m = s.n_col - s.n_lead_const;
    ps.fx_nb = nb_for(ps.fx_m + 1);
    ps.fx_ld = 16 * ps.fx_nb;
    for (int i = 0; i < s.n_slot; ++i) ps.has_theta_white |= pref_uses_theta(s.slots[i]);
    any_theta_white |= ps.has_theta_white || s.n_bgroup > 0;
    // T_aug: [basis | 0-pad | r], row-major n x ld
    // (+CT_ROWS zero rows: the pipelined contraction copies whole tiles)
    std::vector<double> Ta((size_t)(s.n_toa + CT_ROWS) * ps.ld, 0.0), sig2(s.n_toa);
    for (int t = 0; t < s.n_toa; ++t) {
      for (int j = 0; j < s.n_col; ++j) Ta[(size_t)t * ps.ld + j] = s.basis[(size_t)t * s.n_col + j];
      Ta[(size_t)t * ps.ld + ps.ld - 1] = s.resid[t];
      sig2[t] = s.toaerr[t] * s.toaerr[t];
    }
    double* dT;
    double* dsig2;
    int *d_ef, *d_eq, *d_es, *d_ee, *d_eslot;
    ewh_pref* d_slots;
    if ((rc = dupload(h, &dT, Ta.data(), Ta.size()))) return bail(rc);
    if ((rc = dupload(h, &dsig2, sig2.data(), sig2.size()))) return bail(rc);
    if ((rc = dupload(h, &d_ef, s.efac_slot, (size_t)s.n_toa))) return bail(rc);
    if ((rc = dupload(h, &d_eq, s.equad_slot, (size_t)s.n_toa))) return bail(rc);
    if ((rc = dupload(h, &d_slots, s.slots, (size_t)s.n_slot))) return bail(rc);
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
      for (int j = 0; j < s.n_col; ++j) cbg[j] = s.col_bgroup[j];
      if ((rc = dupload(h, &d_cbg, cbg.data(), cbg.size()))) return bail(rc);
      if ((rc = dupload(h, &d_lnc, s.ln_chrom, (size_t)s.n_toa))) return bail(rc);
      if ((rc = dupload(h, &d_bg, s.bgroup_idx, (size_t)s.n_bgroup))) return bail(rc);
    }
    ps.dev = PsrDev{s.n_toa, s.n_col, ps.ld, ps.nb, s.n_epoch, dT, dsig2, d_ef, d_eq, d_slots, d_es, d_ee, d_eslot,
                    s.n_bgroup, d_cbg, d_lnc, d_bg, d_tep};
    std::vector<int> ptr;
    std::vector<DSpec> ent;
    build_csr(s, 0, s.n_col, ptr, ent);
    if ((rc = dupload(h, &ps.d_colptr, ptr.data(), ptr.size()))) return bail(rc);
    if ((rc = dupload(h, &ps.d_spec, ent.data(), ent.size()))) return bail(rc);
    build_csr(s, s.n_lead_const, s.n_col, ptr, ent);
    if ((rc = dupload(h, &ps.d_fx_colptr, ptr.data(), ptr.size()))) return bail(rc);
    if ((rc = dupload(h, &ps.d_fx_spec, ent.data(), ent.size()))) return bail(rc);
  }
  h->white_fixed = (d->white_fixed != 0) && !any_theta_white;
  if ((rc = dalloc(h, &h->d_jobs_fixed, h->P))) return bail(rc);
  if ((rc = dalloc(h, &h->d_jobs_var, h->P))) return bail(rc);
  if (h->white_fixed) {
    if ((rc = setup_fixed(h, d))) return bail(rc);
  }
  *out = h;
  return 0;
}

int ewh_set_kernel_mode(ewh_handle* h, int32_t mode) {
  if (!h || mode < 0 || mode > 7) return set_err(EWH_E_INVALID, "bad handle / mode");
  h->kernel_mode = mode;
  return 0;
}

double ewh_unit_cost(const ewh_handle* h, int32_t p) {
  if (!h || p < 0 || p >= h->P) return 0.0;
  const PsrHost& ps = h->psr[p];
  if (h->white_fixed) return (double)ps.fx_ld * ps.fx_ld * ps.fx_ld / 3.0;
  return (double)ps.n_toa * ps.ld * ps.ld + (double)ps.ld * ps.ld * ps.ld / 3.0;
}

int ewh_lnl_units_device(ewh_handle* h, const double* theta_dev, int32_t B, int64_t u_begin, int64_t u_end,
                         double* out_dev, void* stream) {
  if (!h || !theta_dev || !out_dev || B <= 0) return set_err(EWH_E_INVALID, "bad arguments");
  const long long U = (long long)h->P * B;
  u_begin = std::max<int64_t>(0, u_begin);
  u_end = std::min<int64_t>(U, u_end);
  EWH_HIP(hipSetDevice(h->device));
  hipStream_t st = (hipStream_t)stream;   // NULL = the default stream, as documented
  int rc;
  if ((rc = ensure_units(h, B))) return rc;
  EWH_HIP(hipMemsetAsync(h->d_units, 0, sizeof(double) * (size_t)h->P * B, st));
  const int ldth = h->n_param;
  hipStream_t saved = h->stream;
  h->stream = st;
  if (h->white_fixed) {
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
          (rc = dispatch_chol(h->kernel_mode, nb0, maxm, h->d_jobs_fixed, B, u, seg_end - u, 0, theta_dev, ldth,
                              h->d_units, st, h->d_bigscr, h->bigscr_cap))) {
        h->stream = saved;
        return rc;
      }
      u = seg_end;
    }
  } else {
    if ((rc = ensure_var_scratch(h, B))) {
      h->stream = saved;
      return rc;
    }
    for (long long u = u_begin; u < u_end;) {
      const int p = (int)(u / B);
      const long long pend = std::min<long long>(u_end, (long long)(p + 1) * B);
      const int bs = (int)(u - (long long)p * B), be = (int)(pend - (long long)p * B);
      for (int c0 = bs; c0 < be; c0 += h->chunk) {
        const int nb = std::min(h->chunk, be - c0);
        if ((rc = run_white(h, p, theta_dev, ldth, c0, nb))) {
          h->stream = saved;
          return rc;
        }
        if ((rc = ensure_big_scratch(h, h->psr[p].nb)) ||
            (rc = dispatch_chol(h->kernel_mode, h->psr[p].nb, h->psr[p].m, h->d_jobs_var, B,
                                (long long)p * B + c0, nb, c0, theta_dev, ldth, h->d_units, st, h->d_bigscr,
                                h->bigscr_cap))) {
          h->stream = saved;
          return rc;
        }
      }
      u = pend;
    }
  }
  h->stream = saved;
  hipLaunchKernelGGL(reduce_units_kernel, dim3((B + 255) / 256), dim3(256), 0, st, h->d_units, h->P, B, out_dev);
  EWH_HIP(hipGetLastError());
  h->last_B = B;
  return 0;
}

int ewh_lnl_batch(ewh_handle* h, const double* theta_host, int32_t B, double* out_host) {
  if (!h || !theta_host || !out_host || B <= 0) return set_err(EWH_E_INVALID, "bad arguments");
  EWH_HIP(hipSetDevice(h->device));
  const size_t need = (size_t)B * std::max(1, h->n_param) + B;
  if (need > h->io_cap) {
    for (void* p : {(void*)h->d_theta}) {
      if (p) {
        hipFree(p);
        h->allocs.erase(std::find(h->allocs.begin(), h->allocs.end(), p));
      }
    }
    h->io_cap = 0;
    int rc = dalloc(h, &h->d_theta, need);
    if (rc) return rc;
    h->io_cap = need;
  }
  h->d_out = h->d_theta + (size_t)B * std::max(1, h->n_param);
  if (h->n_param > 0)
    EWH_HIP(hipMemcpyAsync(h->d_theta, theta_host, sizeof(double) * (size_t)B * h->n_param, hipMemcpyHostToDevice,
                           h->stream));
  int rc = ewh_lnl_units_device(h, h->d_theta, B, 0, (long long)h->P * B, h->d_out, h->stream);
  if (rc) return rc;
  EWH_HIP(hipMemcpyAsync(out_host, h->d_out, sizeof(double) * B, hipMemcpyDeviceToHost, h->stream));
  EWH_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

int ewh_last_unit_terms(ewh_handle* h, double* out_host, int32_t B) {
  if (!h || !out_host || B != h->last_B || !h->d_units) return set_err(EWH_E_INVALID, "no matching previous call");
  EWH_HIP(hipSetDevice(h->device));
  EWH_HIP(hipStreamSynchronize(h->stream));
  EWH_HIP(hipDeviceSynchronize());
  EWH_HIP(hipMemcpy(out_host, h->d_units, sizeof(double) * (size_t)h->P * B, hipMemcpyDeviceToHost));
  return 0;
}

void ewh_destroy(ewh_handle* h) {
  if (!h) return;
  hipSetDevice(h->device);
  if (h->stream) hipStreamSynchronize(h->stream);
  for (void* p : h->allocs) hipFree(p);
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
}

}  // extern "C"
