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
// One 256-thread workgroup per (pulsar, sample): the n x n matrix (upper
// triangle used, r last) as hi / lo planes in a per-workgroup scratch, phi^-1
// added to the diagonal in double-double, then a right-looking LDL^T: per
// pivot k the row k and the multipliers w_j = A_kj / d_k staged in LDS, the
// trailing upper triangle A_ij -= A_ki w_j (wave w: rows i = k+1+w, +4, ...;
// lanes: columns) in double-double; log d_k summed per pivot; the last pivot
// is q = r^T N^-1 r - d^T Sigma^-1 d.
#include "ewarp_dev.h"

namespace ewh_dev {
namespace {

__device__ __forceinline__ dd dd_sub_mul(dd a, dd x, dd y) {   // a - x y
  const double p = x.hi * y.hi;
  const double pe = fma(x.hi, y.hi, -p) + (x.hi * y.lo + x.lo * y.hi);
  const dd s = dd_two_sum(a.hi, -p);
  return dd_fast(s.hi, s.lo + a.lo - pe);
}

// list != NULL: the units are list[0 .. *count) (absolute unit indices, the
// verify step's flags); the grid loops over them (a workgroup exits at once
// when there are none).  list == NULL: units u0 + blockIdx.x.
__device__ void chol_dd_unit(const CholJob* __restrict__ jobs, int B, long long u, int b_off,
                             const double* __restrict__ theta, int ldth, double* __restrict__ out_units,
                             double* __restrict__ scratch, long long scr_per_wg) {
  __shared__ double rh[WIDE_LD_MAX], rl[WIDE_LD_MAX], wh[WIDE_LD_MAX], wl[WIDE_LD_MAX];
  __shared__ double red[4];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int p = (int)(u / B), b = (int)(u % B);
  const CholJob J = jobs[p];
  const int n = J.ld;
  const double* Ahi = J.mats + (long long)(b - b_off) * J.mstride;
  const double* Alo = J.mats_lo ? J.mats_lo + (long long)(b - b_off) * J.mstride : nullptr;
  double* H = scratch + (long long)blockIdx.x * scr_per_wg;
  double* L = H + (long long)n * n;
  const double* th = theta + (long long)b * ldth;
  for (int i = wave; i < n; i += 4)
    for (int j = i + lane; j < n; j += 64) {
      const long long o = (long long)i * n + j;
      H[o] = Ahi[o];
      L[o] = Alo ? Alo[o] : 0.0;
    }
  __syncthreads();
  double lphi = 0.0;
  for (int a = tid; a < J.mreal; a += 256) {
    if (J.col_ptr[a] == J.col_ptr[a + 1]) continue;          // (pads carry no entry)
    double ph = 0.0;
    for (int e = J.col_ptr[a]; e < J.col_ptr[a + 1]; ++e) ph += spec_phi_body(J.spec[e], th);
    const dd pinv = dd_div({1.0, 0.0}, {ph, 0.0});
    const long long o = (long long)a * n + a;
    const dd v = dd_add({H[o], L[o]}, pinv);
    H[o] = v.hi;
    L[o] = v.lo;
    lphi += log(ph);
  }
  lphi = block_sum256(lphi, red);          // (its barriers also publish the diagonal)
  double ldet = 0.0;
  bool ok = true;
  for (int k = 0; k < n - 1; ++k) {
    const long long ok_ = (long long)k * n + k;
    const dd d = {H[ok_], L[ok_]};
    ok = ok && (d.hi > 0.0);
    ldet += log(d.hi) + d.lo / d.hi;
    for (int j = k + 1 + tid; j < n; j += 256) {
      const dd r = {H[(long long)k * n + j], L[(long long)k * n + j]};
      const dd wv = dd_div(r, d);
      rh[j] = r.hi;
      rl[j] = r.lo;
      wh[j] = wv.hi;
      wl[j] = wv.lo;
    }
    __syncthreads();
    for (int i = k + 1 + wave; i < n; i += 4) {
      const dd ri = {rh[i], rl[i]};
      for (int j = i + lane; j < n; j += 64) {
        const long long o = (long long)i * n + j;
        const dd v = dd_sub_mul({H[o], L[o]}, ri, {wh[j], wl[j]});
        H[o] = v.hi;
        L[o] = v.lo;
      }
    }
    __threadfence_block();
    __syncthreads();
  }
  if (tid == 0) {
    const long long o = (long long)(n - 1) * n + (n - 1);
    const double qv = H[o] + L[o];
    double lnl = J.K[(long long)(b - b_off) * J.kstride] - 0.5 * qv - 0.5 * ldet - 0.5 * lphi;
    if (!ok || J.fail) lnl = -INFINITY;
    out_units[(long long)p * B + b] = lnl;
  }
  __syncthreads();                         // (the workgroup's next unit reuses LDS and scratch)
}

__global__ __launch_bounds__(256) void chol_dd_kernel(const CholJob* __restrict__ jobs, int B, long long u0, int b_off,
                                                      const double* __restrict__ theta, int ldth,
                                                      double* __restrict__ out_units, double* __restrict__ scratch,
                                                      long long scr_per_wg, const int* __restrict__ list,
                                                      const int* __restrict__ count) {
  if (!list) {
    chol_dd_unit(jobs, B, u0 + blockIdx.x, b_off, theta, ldth, out_units, scratch, scr_per_wg);
    return;
  }
  const int n = *count;
  for (int i = blockIdx.x; i < n; i += gridDim.x)
    chol_dd_unit(jobs, B, list[i], b_off, theta, ldth, out_units, scratch, scr_per_wg);
}

// The verify step: the forward (a) and reversed (b) fp64 factorisations of
// units [u0, u0 + n) agree to a quarter of the strict bound of the unit's own
// term (and on -inf), or the unit goes to the list for chol_dd_kernel.
__global__ __launch_bounds__(256) void verify_units_kernel(const double* __restrict__ a, const double* __restrict__ b,
                                                           long long u0, long long n, int* __restrict__ list,
                                                           int* __restrict__ count, int* __restrict__ total) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (total && i == 0) atomicAdd(total + 1, (int)n);     // (ewh_refine_stats: units checked)
  if (i >= n) return;
  const long long u = u0 + i;
  const double x = a[u], y = b[u];
  const bool fx = x - x == 0.0, fy = y - y == 0.0;           // finite
  const bool bad = (fx != fy) || (fx && fabs(x - y) > 0.25 * (1e-6 + 1e-10 * fabs(x)));
  if (bad) {
    list[atomicAdd(count, 1)] = (int)u;
    if (total) atomicAdd(total, 1);       // (ewh_refine_stats: units refined)
  }
}

}  // namespace

int launch_verify_units(const double* a, const double* b, long long u0, long long n, int* list, int* count,
                        int* total, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(verify_units_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, b, u0, n, list,
                     count, total);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_err(EWH_E_HIP, std::string("verify_units_kernel: ") + hipGetErrorString(e));
}

long long dd_scratch_per_wg(int ld) { return 2LL * ld * ld; }

int launch_chol_dd(const CholJob* jobs, int B, long long u0, long long n, int b_off, const double* theta, int ldth,
                   double* units, double* scr, long long scr_per_wg, long long cap, hipStream_t st) {
  for (long long o = 0; o < n; o += cap)   // one scratch slot per workgroup of a launch
    hipLaunchKernelGGL(chol_dd_kernel, dim3((unsigned)std::min(cap, n - o)), dim3(256), 0, st, jobs, B, u0 + o, b_off,
                       theta, ldth, units, scr, scr_per_wg, nullptr, nullptr);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_err(EWH_E_HIP, std::string("chol_dd_kernel: ") + hipGetErrorString(e));
}


int launch_chol_dd_list(const CholJob* jobs, int B, int b_off, const double* theta, int ldth, double* units,
                        double* scr, long long scr_per_wg, long long cap, const int* list, const int* count,
                        hipStream_t st) {
  hipLaunchKernelGGL(chol_dd_kernel, dim3((unsigned)cap), dim3(256), 0, st, jobs, B, 0LL, b_off, theta, ldth, units,
                     scr, scr_per_wg, list, count);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : set_err(EWH_E_HIP, std::string("chol_dd_kernel: ") + hipGetErrorString(e));
}

}  // namespace ewh_dev
