// Host-side AddressSanitizer driver for the C ABI (include/ewarp_hip.h).
// Built by `make -C enterprise_warp_amd/csrc asan` (every translation unit
// with -Xarch_host -fsanitize=address; device code unchanged) and run by
// tests/test_asan_abi.py.  It walks the descriptor validation, the CSR / table
// builders and the error paths with well-formed and malformed descriptors; on
// a host with a GPU it also runs create -> lnl_batch -> set_fixed_white ->
// multi-context create -> destroy.  Exit status 0 = every expectation held
// (ASan aborts the process on any host memory error).
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "ewarp_hip.h"

namespace {

struct Psr {
  int n = 96, ncol = 24, nlead = 4;
  std::vector<double> basis, resid, err;
  std::vector<ewh_pref> slots;
  std::vector<int32_t> efac, equad, es, ee, eslot;
  std::vector<ewh_spec_entry> spec;
  ewh_pulsar_desc d{};

  explicit Psr(bool fixed_white) {
    basis.resize((size_t)n * ncol);
    resid.resize(n);
    err.resize(n);
    for (int t = 0; t < n; ++t) {
      const double x = (t + 0.5) / n;
      for (int j = 0; j < ncol; ++j) {
        double v;
        if (j < nlead) v = std::pow(x - 0.5, j);
        else {
          const int f = (j - nlead) / 2 + 1;
          v = ((j - nlead) % 2 == 0) ? std::sin(2 * M_PI * f * x) : std::cos(2 * M_PI * f * x);
        }
        basis[(size_t)t * ncol + j] = v;
      }
      resid[t] = 1e-6 * std::sin(17.0 * t);
      err[t] = 1e-6 * (1.0 + 0.5 * (t % 3));
    }
    // slots: efac (theta 0 / const), equad (theta 1 / const), ecorr (const)
    slots = {ewh_pref{fixed_white ? -1 : 0, 0, 1.1}, ewh_pref{fixed_white ? -1 : 1, 0, -6.5}, ewh_pref{-1, 0, -6.8}};
    efac.assign(n, 0);
    equad.assign(n, 1);
    for (int e = 0; e + 3 <= n; e += 4) {
      es.push_back(e);
      ee.push_back(e + 3);
      eslot.push_back(2);
    }
    const double Tspan = 4.6e8, fyr = 1.0 / (365.25 * 86400.0);
    for (int j = 0; j < nlead; ++j) spec.push_back(ewh_spec_entry{EWH_SPEC_CONST, j, {-1, 0, 1e40}, {-1, 0, 0}, {-1, 0, 0}, 0, 0, fyr});
    for (int j = nlead; j < ncol; ++j) {
      const double f = ((j - nlead) / 2 + 1) / Tspan;
      spec.push_back(ewh_spec_entry{EWH_SPEC_POWERLAW, j, {2, 0, 0}, {3, 0, 0}, {-1, 0, 0}, f, 1.0 / Tspan, fyr});
    }
    refresh();
  }
  void refresh() {
    d = ewh_pulsar_desc{};
    d.n_toa = n;
    d.n_col = ncol;
    d.n_lead_const = nlead;
    d.n_spec = (int32_t)spec.size();
    d.basis = basis.data();
    d.resid = resid.data();
    d.toaerr = err.data();
    d.n_slot = (int32_t)slots.size();
    d.slots = slots.data();
    d.efac_slot = efac.data();
    d.equad_slot = equad.data();
    d.n_epoch = (int32_t)es.size();
    d.epoch_start = es.data();
    d.epoch_stop = ee.data();
    d.epoch_slot = eslot.data();
    d.spec = spec.data();
  }
};

int failures = 0;

void expect(bool ok, const char* what) {
  if (!ok) {
    std::printf("FAIL: %s (%s)\n", what, ewh_last_error());
    ++failures;
  } else {
    std::printf("ok: %s\n", what);
  }
}

int create(const ewh_pulsar_desc* p, int np, int n_param, int white_fixed, const int32_t* devs, int ndev,
           ewh_handle** h) {
  ewh_pta_desc d{EWH_ABI_VERSION, np, n_param, white_fixed, p, nullptr};
  return ewh_create(&d, devs, ndev, h);
}

}  // namespace

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && std::strcmp(argv[1], "--gpu") == 0;
  expect(ewh_version() == EWH_ABI_VERSION, "ABI version");
  ewh_handle* h = nullptr;
  // malformed descriptors: rejected before any device call
  {
    Psr p(false);
    p.efac[7] = 9;
    p.refresh();
    expect(create(&p.d, 1, 4, 0, nullptr, 0, &h) == EWH_E_INVALID && !h, "efac slot out of range");
  }
  {
    Psr p(false);
    p.ee[3] = p.es[3] + 1;      // a one-TOA epoch
    p.refresh();
    expect(create(&p.d, 1, 4, 0, nullptr, 0, &h) == EWH_E_INVALID, "one-TOA epoch");
  }
  {
    Psr p(false);
    p.es[5] = p.es[4];          // overlapping epochs
    p.refresh();
    expect(create(&p.d, 1, 4, 0, nullptr, 0, &h) == EWH_E_INVALID, "overlapping epochs");
  }
  {
    Psr p(false);
    p.spec[10].col = p.ncol;    // column out of range
    p.refresh();
    expect(create(&p.d, 1, 4, 0, nullptr, 0, &h) == EWH_E_INVALID, "spectral column out of range");
  }
  {
    Psr p(false);
    p.spec[12].p1.idx = 4;      // theta index == n_param
    p.refresh();
    expect(create(&p.d, 1, 4, 0, nullptr, 0, &h) == EWH_E_INVALID, "theta index out of range");
  }
  {
    Psr p(false);
    p.spec.pop_back();          // last column without a phi entry
    p.refresh();
    expect(create(&p.d, 1, 4, 0, nullptr, 0, &h) == EWH_E_INVALID, "column without phi");
  }
  {
    Psr p(false);
    p.d.basis = nullptr;
    expect(create(&p.d, 1, 4, 0, nullptr, 0, &h) == EWH_E_INVALID, "NULL basis");
  }
  {
    Psr p(false);
    p.d.n_common = 3;           // without a common descriptor
    expect(create(&p.d, 1, 4, 0, nullptr, 0, &h) == EWH_E_INVALID, "n_common without common");
  }
  {
    Psr p(false);
    const int32_t bad[2] = {0, -1};
    expect(create(&p.d, 1, 4, 0, bad, 2, &h) == EWH_E_INVALID || !gpu, "negative device id");
  }
  expect(ewh_create(nullptr, nullptr, 0, &h) == EWH_E_INVALID, "NULL descriptor");
  // well-formed descriptor
  Psr pv(false), pf(true);
  ewh_pulsar_desc two[2] = {pv.d, pf.d};
  const int rc = create(two, 2, 4, 0, nullptr, 0, &h);
  if (!gpu) {
    expect(rc == EWH_E_HIP && !h, "valid descriptor without a GPU: HIP error, no handle");
  } else {
    expect(rc == EWH_OK && h, "create (varying white noise)");
    std::vector<double> th = {1.05, -6.6, -13.5, 3.5, 0.95, -6.9, -14.0, 4.0}, out(2);
    expect(ewh_lnl_batch(h, th.data(), 2, out.data()) == EWH_OK && std::isfinite(out[0]), "lnl_batch");
    std::vector<double> wn = {1.0, -6.4, -6.9, 1.2, -6.3, -7.0};
    expect(ewh_set_fixed_white(h, wn.data()) == EWH_OK, "set_fixed_white");
    std::vector<double> terms(4);
    expect(ewh_last_unit_terms(h, terms.data(), 2) == EWH_OK, "last_unit_terms");
    ewh_destroy(h);
    ewh_handle* h2 = nullptr;
    ewh_pulsar_desc fx[1] = {pf.d};
    const int32_t devs[2] = {0, 0};
    expect(create(fx, 1, 4, 1, devs, 2, &h2) == EWH_OK, "create fixed white noise, two contexts");
    std::vector<double> out3(3);
    std::vector<double> th3 = {0, 0, -13.5, 3.5, 0, 0, -14.0, 4.0, 0, 0, -13.0, 2.5};
    expect(ewh_lnl_batch(h2, th3.data(), 3, out3.data()) == EWH_OK && std::isfinite(out3[2]), "two-context batch");
    ewh_destroy(h2);
  }
  std::printf("%d failure(s)\n", failures);
  return failures ? 1 : 0;
}
