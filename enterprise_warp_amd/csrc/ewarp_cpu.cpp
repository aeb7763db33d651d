// ewarp_cpu.cpp — host (C++) twin of the C ABI in include/ewarp_hip.h
// ("a C++ CPU twin has the same ABI").
//
// Same descriptor (validated by the same ewarp_desc.h), same entry points,
// same -inf semantics ([ent] LinAlgError -> -np.inf), evaluated on the host
// cores: OpenMP over samples in ewh_lnl_batch, over pulsars in the white-noise
// cache.  It is NOT a fallback of the GPU library: enterprise_warp_amd loads
// it only when EWARP_BACKEND=cpu (or EWARP_HIP_LIB names it), and it is a
// separate .so.  Scope: uncorrelated / CURN models with fixed or varying
// white noise (chromatic 'vary' bases included).  A correlated common
// process, the optimal statistic and the device-pointer entries return
// EWH_E_UNSUPPORTED (device-only in this ABI version).
//
// Per pulsar (enterprise's likelihood; the reference
// reaches it at bilby_warp.py:35):
//   N   = diag(efac^2 sigma^2 + 10^(2 log10_tnequad)) + ECORR epoch blocks,
//         applied by Sherman-Morrison ([ent] ShermanMorrison._solve_2D2 /
//         _solve_1D1: beta_e = 1 / (sum_e 1/N + 1/J_e), log|N| += log J_e -
//         log beta_e)
//   G   = [T r]^T N^-1 [T r], summed in long double (x87, 64-bit mantissa)
//   the timing-model block (leading columns, constant phi = 1e40) is
//   eliminated once in long double:  A = G_TT + diag(1/phi_T),
//   S = G_RR - G_RT A^-1 G_TR  (r last: S also carries d' and r^T N^-1 r')
//   per sample: Sigma_R = S + diag(1/phi_R), LDL^T in double, bordered by r,
//   whose last pivot is q = r^T N^-1 r - d^T Sigma^-1 d;
//   lnL_a = -1/2 (q + log|N| + log|A| + log|Sigma_R| + log|phi|).
// Fixed white noise caches S, log|N|, log|A| per pulsar (recomputed by
// ewh_set_fixed_white); varying white noise recomputes them per sample.
//   g++ -O3 -fopenmp -shared -fPIC -Iinclude ewarp_cpu.cpp -o libewarp_cpu.so
#include <cmath>
#include <cstring>
#include <limits>
#include <string>
#include <vector>

#include "ewarp_desc.h"
#include "ewarp_hip.h"

namespace {

thread_local std::string g_err;

int set_err(int code, const std::string& m) {
  g_err = m;
  return code;
}

typedef long double ld_t;
constexpr double LN10 = 2.302585092994045684;

double pref_val(const ewh_pref& r, const double* th) { return r.idx >= 0 ? th[r.idx] : r.cval; }

// phi of one spectral entry: the quantities of [ent] utils.powerlaw, the
// reference's powerlaw_bpl (enterprise_models.py:553-563) and [ent]
// gp_priors.free_spectrum
double spec_phi(const ewh_spec_entry& e, const double* th) {
  switch (e.kind) {
    case EWH_SPEC_POWERLAW: {
      const double lgA = pref_val(e.p0, th), gam = pref_val(e.p1, th);
      return std::pow(10.0, 2.0 * lgA) / (12.0 * M_PI * M_PI) * std::pow(e.fyr, gam - 3.0) * std::pow(e.f, -gam) *
             e.df;
    }
    case EWH_SPEC_TURNOVER: {
      const double lgA = pref_val(e.p0, th), gam = pref_val(e.p1, th);
      double fc = pref_val(e.p2, th);
      if (fc < 0) fc = std::pow(10.0, fc);
      return std::pow(10.0, 2.0 * lgA) / (12.0 * M_PI * M_PI) * std::pow(e.fyr, -3.0) *
             std::pow((e.f + fc) / e.fyr, -gam) * e.df;
    }
    case EWH_SPEC_FREESPEC:
      return std::exp(2.0 * LN10 * pref_val(e.p0, th));
    case EWH_SPEC_CONST:
      return e.p0.cval;
    default:
      return std::numeric_limits<double>::quiet_NaN();
  }
}

struct Psr {
  int n = 0, m = 0, nl = 0;             // TOAs, columns, leading constant-phi (timing model) columns
  std::vector<double> T, r, sig2;
  std::vector<ewh_pref> slots;
  std::vector<int> efac_slot, equad_slot, ep_start, ep_stop, ep_slot;
  std::vector<int> col_ptr;              // CSR of spectral entries per column
  std::vector<ewh_spec_entry> spec;
  std::vector<ewh_pref> bgroup;
  std::vector<int> col_bgroup;
  std::vector<double> ln_chrom;
  bool theta_white = false;              // a white-noise slot or a basis group reads theta
  // white-noise cache (fixed white noise): S (mR + 1)^2, log|N| + log|A|
  std::vector<double> S;
  double Kc = 0.0;
  bool fail = false;                     // timing-model block not positive definite
};

// G = [T r]^T N^-1 [T r] (upper triangle, (m+1)^2, long double) and log|N|
void gram(const Psr& P, const double* th, std::vector<ld_t>& G, ld_t& logN) {
  const int m = P.m, M = m + 1;
  G.assign((size_t)M * M, 0.0L);
  std::vector<double> w(P.n);
  logN = 0.0L;
  for (int t = 0; t < P.n; ++t) {
    const double ef = pref_val(P.slots[P.efac_slot[t]], th);
    double Nt = ef * ef * P.sig2[t];
    if (P.equad_slot[t] >= 0) Nt += std::pow(10.0, 2.0 * pref_val(P.slots[P.equad_slot[t]], th));
    w[t] = 1.0 / Nt;
    logN += std::log((ld_t)Nt);
  }
  std::vector<double> gfac(P.bgroup.size());
  for (size_t g = 0; g < P.bgroup.size(); ++g) gfac[g] = pref_val(P.bgroup[g], th);
  std::vector<ld_t> x(M);
  auto row = [&](int t) {
    for (int j = 0; j < m; ++j) {
      double v = P.T[(size_t)t * m + j];
      if (!P.col_bgroup.empty() && P.col_bgroup[j] >= 0) v *= std::exp(gfac[P.col_bgroup[j]] * P.ln_chrom[t]);
      x[j] = v;
    }
    x[m] = P.r[t];
  };
  for (int t = 0; t < P.n; ++t) {
    row(t);
    const ld_t wt = w[t];
    for (int i = 0; i < M; ++i) {
      const ld_t a = wt * x[i];
      ld_t* gi = &G[(size_t)i * M];
      for (int j = i; j < M; ++j) gi[j] += a * x[j];
    }
  }
  std::vector<ld_t> se(M);
  for (size_t e = 0; e < P.ep_start.size(); ++e) {
    const ld_t J = std::pow(10.0L, 2.0L * (ld_t)pref_val(P.slots[P.ep_slot[e]], th));
    ld_t sw = 0.0L;
    std::fill(se.begin(), se.end(), 0.0L);
    for (int t = P.ep_start[e]; t < P.ep_stop[e]; ++t) {
      row(t);
      sw += w[t];
      for (int i = 0; i < M; ++i) se[i] += (ld_t)w[t] * x[i];
    }
    const ld_t beta = 1.0L / (sw + 1.0L / J);
    logN += std::log(J) - std::log(beta);
    for (int i = 0; i < M; ++i) {
      const ld_t a = beta * se[i];
      ld_t* gi = &G[(size_t)i * M];
      for (int j = i; j < M; ++j) gi[j] -= a * se[j];
    }
  }
}

// the timing-model elimination: S (double, (m - nl + 1)^2, full) and
// Kc = log|N| + log|A| + log|phi_T|; fail when A is not positive definite
void reduce(const Psr& P, const double* th, std::vector<double>& S, double& Kc, bool& fail) {
  std::vector<ld_t> G;
  ld_t logN;
  gram(P, th, G, logN);
  const int M = P.m + 1, nl = P.nl, mR = M - nl;
  auto g = [&](int i, int j) -> ld_t& { return i <= j ? G[(size_t)i * M + j] : G[(size_t)j * M + i]; };
  ld_t ldA = 0.0L, ldphiT = 0.0L;
  fail = false;
  // A = G_TT + diag(1/phi_T): Cholesky in place (upper: A = U^T U)
  std::vector<ld_t> U((size_t)nl * nl, 0.0L);
  for (int i = 0; i < nl; ++i) {
    double ph = 0.0;
    for (int e = P.col_ptr[i]; e < P.col_ptr[i + 1]; ++e) ph += spec_phi(P.spec[e], th);
    ldphiT += std::log((ld_t)ph);
    for (int j = i; j < nl; ++j) U[(size_t)i * nl + j] = g(i, j) + (i == j ? 1.0L / ph : 0.0L);
  }
  for (int k = 0; k < nl; ++k) {
    ld_t d = U[(size_t)k * nl + k];
    for (int p = 0; p < k; ++p) d -= U[(size_t)p * nl + k] * U[(size_t)p * nl + k];
    if (!(d > 0.0L)) {
      fail = true;
      d = 1.0L;
    }
    const ld_t s = std::sqrt(d);
    ldA += std::log(d);
    U[(size_t)k * nl + k] = s;
    for (int j = k + 1; j < nl; ++j) {
      ld_t v = U[(size_t)k * nl + j];
      for (int p = 0; p < k; ++p) v -= U[(size_t)p * nl + k] * U[(size_t)p * nl + j];
      U[(size_t)k * nl + j] = v / s;
    }
  }
  // Y = U^-T G_TR (nl x mR), S = G_RR - Y^T Y
  std::vector<ld_t> Y((size_t)nl * mR);
  for (int c = 0; c < mR; ++c)
    for (int k = 0; k < nl; ++k) {
      ld_t v = g(k, nl + c);
      for (int p = 0; p < k; ++p) v -= U[(size_t)p * nl + k] * Y[(size_t)p * mR + c];
      Y[(size_t)k * mR + c] = v / U[(size_t)k * nl + k];
    }
  S.assign((size_t)mR * mR, 0.0);
  for (int i = 0; i < mR; ++i)
    for (int j = i; j < mR; ++j) {
      ld_t v = g(nl + i, nl + j);
      for (int k = 0; k < nl; ++k) v -= Y[(size_t)k * mR + i] * Y[(size_t)k * mR + j];
      S[(size_t)i * mR + j] = S[(size_t)j * mR + i] = (double)v;
    }
  Kc = (double)(logN + ldA + ldphiT);
}

// lnL term of one pulsar for one sample; work: (mR)^2 doubles
double unit_lnl(const Psr& P, const double* th, const std::vector<double>& S, double Kc, bool fail,
                std::vector<double>& A) {
  if (fail) return -INFINITY;
  const int nl = P.nl, mR = P.m + 1 - nl, nr = mR - 1;   // nr reduced columns, r last
  A = S;
  double ldphi = 0.0;
  for (int j = 0; j < nr; ++j) {
    double ph = 0.0;
    for (int e = P.col_ptr[nl + j]; e < P.col_ptr[nl + j + 1]; ++e) ph += spec_phi(P.spec[e], th);
    if (!std::isfinite(ph)) return -INFINITY;
    ldphi += std::log(ph);
    A[(size_t)j * mR + j] += 1.0 / ph;
  }
  // LDL^T (right-looking, upper triangle), the last pivot left as q
  double ldS = 0.0;
  for (int k = 0; k < nr; ++k) {
    const double d = A[(size_t)k * mR + k];
    if (!(d > 0.0)) return -INFINITY;
    ldS += std::log(d);
    const double* rk = &A[(size_t)k * mR];
    for (int i = k + 1; i < mR; ++i) {
      const double l = rk[i] / d;
      double* ri = &A[(size_t)i * mR];
      for (int j = i; j < mR; ++j) ri[j] -= l * rk[j];
    }
  }
  const double q = A[(size_t)nr * mR + nr];
  const double v = -0.5 * (q + Kc + ldS + ldphi);
  return std::isnan(v) ? -INFINITY : v;
}

}  // namespace

struct ewh_handle {
  int n_param = 0;
  bool white_fixed = false;
  std::vector<Psr> psr;
  std::vector<double> units;   // last call: P x B
  int last_B = 0;
};

namespace {

void refresh_fixed(ewh_handle* H) {
  std::vector<double> dummy(std::max(1, H->n_param), 0.0);   // constant slots never read theta
  const int P = (int)H->psr.size();
#pragma omp parallel for schedule(dynamic, 1)
  for (int p = 0; p < P; ++p) {
    Psr& ps = H->psr[p];
    if (!ps.theta_white) reduce(ps, dummy.data(), ps.S, ps.Kc, ps.fail);
  }
}

}  // namespace

extern "C" {

int ewh_version(void) { return EWH_ABI_VERSION; }
int ewh_lat_b_max(void) { return 0; }   // no latency kernel on the host

const char* ewh_last_error(void) { return g_err.c_str(); }

int ewh_create(const ewh_pta_desc* d, const int32_t* device_ids, int32_t ndev, ewh_handle** out) {
  (void)device_ids;
  (void)ndev;
  if (!out) return set_err(EWH_E_INVALID, "null output handle");
  *out = nullptr;
  std::string msg;
  if (const int rc = ewh_desc::desc_check(d, msg)) return set_err(rc, msg);
  if (d->common)
    return set_err(EWH_E_UNSUPPORTED, "host twin: a correlated common process / optimal statistic is device-only");
  ewh_handle* H = new ewh_handle;
  H->n_param = d->n_param;
  H->white_fixed = d->white_fixed != 0;
  H->psr.resize(d->n_pulsar);
  for (int p = 0; p < d->n_pulsar; ++p) {
    const ewh_pulsar_desc& s = d->pulsars[p];
    Psr& P = H->psr[p];
    P.n = s.n_toa;
    P.m = s.n_col;
    P.nl = s.n_lead_const;
    P.T.assign(s.basis, s.basis + (size_t)s.n_toa * s.n_col);
    P.r.assign(s.resid, s.resid + s.n_toa);
    P.sig2.resize(s.n_toa);
    for (int t = 0; t < s.n_toa; ++t) P.sig2[t] = s.toaerr[t] * s.toaerr[t];
    P.slots.assign(s.slots, s.slots + s.n_slot);
    P.efac_slot.assign(s.efac_slot, s.efac_slot + s.n_toa);
    P.equad_slot.assign(s.equad_slot, s.equad_slot + s.n_toa);
    P.ep_start.assign(s.epoch_start, s.epoch_start + s.n_epoch);
    P.ep_stop.assign(s.epoch_stop, s.epoch_stop + s.n_epoch);
    P.ep_slot.assign(s.epoch_slot, s.epoch_slot + s.n_epoch);
    P.col_ptr.assign(s.n_col + 1, 0);
    for (int e = 0; e < s.n_spec; ++e) P.col_ptr[s.spec[e].col + 1]++;
    for (int j = 0; j < s.n_col; ++j) P.col_ptr[j + 1] += P.col_ptr[j];
    P.spec.resize(s.n_spec);
    std::vector<int> fill(P.col_ptr.begin(), P.col_ptr.end() - 1);
    for (int e = 0; e < s.n_spec; ++e) P.spec[fill[s.spec[e].col]++] = s.spec[e];
    if (s.n_bgroup > 0) {
      P.bgroup.assign(s.bgroup_idx, s.bgroup_idx + s.n_bgroup);
      P.col_bgroup.assign(s.col_bgroup, s.col_bgroup + s.n_col);
      P.ln_chrom.assign(s.ln_chrom, s.ln_chrom + s.n_toa);
    }
    P.theta_white = !H->white_fixed || s.n_bgroup > 0;
    for (const auto& sl : P.slots)
      if (sl.idx >= 0) P.theta_white = true;
  }
  refresh_fixed(H);
  *out = H;
  return 0;
}

int ewh_num_devices(const ewh_handle* H) { return H ? 1 : 0; }

int ewh_set_fixed_white(ewh_handle* H, const double* values) {
  if (!H || !values) return set_err(EWH_E_INVALID, "bad arguments");
  size_t k = 0;
  for (auto& P : H->psr)
    for (auto& sl : P.slots) {
      if (sl.idx < 0) sl.cval = values[k];
      ++k;
    }
  refresh_fixed(H);
  return 0;
}

int ewh_lnl_batch(ewh_handle* H, const double* theta, int32_t B, double* out) {
  if (!H || !theta || !out || B <= 0) return set_err(EWH_E_INVALID, "bad arguments");
  const int P = (int)H->psr.size(), np = H->n_param;
  H->units.assign((size_t)P * B, 0.0);
#pragma omp parallel
  {
    std::vector<double> A, S;
#pragma omp for schedule(dynamic, 1)
    for (int b = 0; b < B; ++b) {
      const double* th = theta + (size_t)b * np;
      double s = 0.0;
      for (int p = 0; p < P; ++p) {
        const Psr& ps = H->psr[p];
        double v;
        if (ps.theta_white) {
          double Kc;
          bool fail;
          reduce(ps, th, S, Kc, fail);
          v = unit_lnl(ps, th, S, Kc, fail, A);
        } else {
          v = unit_lnl(ps, th, ps.S, ps.Kc, ps.fail, A);
        }
        H->units[(size_t)p * B + b] = v;
        s += v;                                      // pulsar order
      }
      out[b] = s;
    }
  }
  H->last_B = B;
  return 0;
}

int ewh_last_unit_terms(ewh_handle* H, double* out, int32_t B) {
  if (!H || !out || B != H->last_B) return set_err(EWH_E_INVALID, "bad arguments / B differs from the last call");
  std::memcpy(out, H->units.data(), sizeof(double) * H->units.size());
  return 0;
}

int ewh_refine_stats(ewh_handle* H, int64_t* checked, int64_t* refined) {
  if (!H) return set_err(EWH_E_INVALID, "bad handle");
  if (checked) *checked = 0;     // (no double-double route on the host: the twin factors in double)
  if (refined) *refined = 0;
  return 0;
}

int ewh_transfer_stats(const ewh_handle* H, int64_t* h2d_bytes, int64_t* peer) {
  if (!H) return set_err(EWH_E_INVALID, "bad handle");
  if (h2d_bytes) *h2d_bytes = 0;     // host twin: nothing crosses a bus
  if (peer) *peer = 1;
  return 0;
}

double ewh_unit_cost(const ewh_handle* H, int32_t p) {
  if (!H || p < 0 || p >= (int)H->psr.size()) return 0.0;
  const Psr& P = H->psr[p];
  const double mR = P.m + 1 - P.nl;
  return P.theta_white ? (double)P.n * (P.m + 1) * (P.m + 1) + mR * mR * mR / 3.0 : mR * mR * mR / 3.0;
}

int ewh_set_kernel_mode(ewh_handle* H, int32_t mode) {
  if (!H) return set_err(EWH_E_INVALID, "bad handle");
  return mode == 0 || mode == 2 ? 0 : set_err(EWH_E_UNSUPPORTED, "host twin: kernel modes are device-only");
}

int ewh_lnl_units_device(ewh_handle*, const double*, int32_t, int64_t, int64_t, double*, void*) {
  return set_err(EWH_E_UNSUPPORTED, "host twin: no device entries");
}
int ewh_contract_device(ewh_handle*, const double*, int32_t, void*) {
  return set_err(EWH_E_UNSUPPORTED, "host twin: no device entries");
}
int ewh_keep_dim(const ewh_handle*) { return 0; }
int ewh_corr_partial_device(ewh_handle*, const double*, int32_t, int32_t, int32_t, double*, double*, void*) {
  return set_err(EWH_E_UNSUPPORTED, "host twin: no device entries");
}
int ewh_corr_finish_device(ewh_handle*, const double*, int32_t, const double*, const double*, double*, void*) {
  return set_err(EWH_E_UNSUPPORTED, "host twin: no device entries");
}
int ewh_optstat(ewh_handle*, const double*, int32_t, const double*, double*, double*, double*, double*) {
  return set_err(EWH_E_UNSUPPORTED, "host twin: the optimal statistic is device-only");
}

void ewh_destroy(ewh_handle* H) { delete H; }

}  // extern "C"
