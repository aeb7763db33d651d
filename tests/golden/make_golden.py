"""Generate the committed golden vectors (run in the dev container; CPU only).

    python tests/golden/make_golden.py

Each fixture `<name>.npz` holds the pulsar arrays, a JSON model recipe
(terms, common terms, Tspan, fixed-white flag, noise dict), a theta batch in
param_names order and the oracle's lnL for it.  The oracle is
oracle/enterprise_ref.py (the numpy/scipy restatement of enterprise's
likelihood; "parity unpinned" against enterprise itself, see
oracle/__init__.py).  Inputs are seeded synthetic data, except c1, whose
TOAs / errors / frequencies / flags come from the reference's example pulsar
(ref_examples/data/J1832-0836.tim) and whose residuals are drawn at the
reference's example noise file values.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from enterprise_warp_amd import synth  # noqa: E402
from oracle.device_order_ref import DeviceOrderPTA  # noqa: E402
from oracle.enterprise_ref import OraclePTA  # noqa: E402


ORDERINGS = ("enterprise", "device", "device_blas", "reverse_chol", "extended")


def oracle_lnl(pta, X):
    """Per sample, the lnL of five orderings of the same likelihood:
      enterprise    oracle/enterprise_ref.py (the full Sigma by cho_factor)
      device        the device's order (oracle/device_order_ref.py: projected
                    basis, the contraction kernels' FMA accumulation order for
                    a varying-white-noise Gram, double-double cache and
                    timing-model elimination for fixed white noise, two-level
                    blocked LDL^T)
      device_blas   the same with a BLAS Gram
      reverse_chol  original basis, the Gram summed over the TOAs in reverse,
                    unblocked Cholesky
      extended      near-exact: oracle/ddref.py (double-double) for
                    uncorrelated / CURN models, the extended-precision
                    restatement with an error-free Gram for correlated ones
    and the spread = max - min of the five (informational; 0 where all are
    -inf, inf where they disagree on -inf).  The GPU tests hold near-truth
    draws to strict and prior draws to |gpu - extended| <= max(|enterprise -
    extended|, strict) (tests/conftest.py check_accuracy).  Also returns the
    conditioning of what the device factors (informational)."""
    from oracle.ddref import DDReferencePTA
    const = pta.constant_values()
    fixed = const if pta.white_fixed() else None
    psrs = [c.psr for c in pta.signal_collections]
    terms = pta.oracle_terms()
    ent = OraclePTA(psrs, terms, fixed_params=fixed)
    exact = (DeviceOrderPTA(psrs, terms, fixed, np.longdouble) if ent.correlated()
             else DDReferencePTA(psrs, terms))
    models = [ent,
              DeviceOrderPTA(psrs, terms, fixed, np.float64, gram_mode="device"),
              DeviceOrderPTA(psrs, terms, fixed, np.float64, gram_mode="blas"),
              DeviceOrderPTA(psrs, terms, fixed, np.float64, gram_mode="reverse", factor="chol"),
              exact]
    vals = np.zeros((len(models), len(X)))
    cond = []
    for j, x in enumerate(X):
        d = dict(const)
        d.update(pta.map_params(x))
        for i, mdl in enumerate(models):
            vals[i, j] = mdl.lnlikelihood(d)
        cond.append(models[3].min_eig(d))
    fin = np.isfinite(vals).all(axis=0)
    spread = np.zeros(len(X))
    spread[fin] = vals[:, fin].max(axis=0) - vals[:, fin].min(axis=0)
    spread[~fin & np.isfinite(vals).any(axis=0)] = np.inf     # orderings disagree on -inf
    return vals, spread, np.array(cond)


def dump(name, pta, recipe, X, n_prior=8):
    psrs = [c.psr for c in pta.signal_collections]
    arrays = {}
    for i, p in enumerate(psrs):
        arrays[f"p{i}_toas"] = p.toas
        arrays[f"p{i}_residuals"] = p.residuals
        arrays[f"p{i}_toaerrs"] = p.toaerrs
        arrays[f"p{i}_freqs"] = p.freqs
        arrays[f"p{i}_Mmat"] = p.Mmat
        arrays[f"p{i}_pos"] = p.pos
        for k, v in p.flags.items():
            arrays[f"p{i}_flag_{k}"] = v.astype(str)
    recipe = dict(recipe, names=[p.name for p in psrs], flag_names=[sorted(p.flags) for p in psrs],
                  param_names=pta.param_names)
    vals, spread, cond = oracle_lnl(pta, X)
    lnl, dev, ex = vals[0], vals[1], vals[-1]
    near = np.arange(len(X)) >= n_prior          # rows [n_prior:) are near-truth draws
    np.savez_compressed(os.path.join(HERE, name + ".npz"), recipe=np.array(json.dumps(recipe)), theta=X, lnl=lnl,
                        lnl_dev=dev, lnl_exact=ex, lnl_orderings=vals, orderings=np.array(ORDERINGS),
                        spread=spread, near=near, min_eig=cond, **arrays)
    strict = 1e-6 + 1e-10 * np.abs(ex)
    with np.errstate(invalid="ignore", divide="ignore"):
        print(name, "n_psr", len(psrs), "nparam", X.shape[1], "n_inf", int(np.sum(~np.isfinite(lnl))),
              "spread/strict", np.array2string(spread / strict, precision=1, max_line_width=200),
              "log10 min_eig", np.round(np.log10(np.abs(cond)), 1))


def recipe_of(cfg, per_psr, common, fixed_white):
    pta = cfg.pta
    Tspan = None
    for c in pta.signal_collections:
        for b in c.bound:
            if hasattr(b, "basis_spec") and b.basis_spec.Tspan is not None:
                Tspan = float(b.basis_spec.Tspan)
                break
    return {"per_psr_terms": per_psr, "common_terms": common, "Tspan": Tspan, "fixed_white": fixed_white,
            "noisedict": {k: v for k, v in pta.constant_values().items() if v is not None}}


def main():
    only = sys.argv[1:]                    # optional fixture-name prefixes
    global dump
    _dump = dump

    def dump(name, *a, **k):               # noqa: F811 - filter by name
        if not only or any(name.startswith(o) for o in only):
            _dump(name, *a, **k)
    terms_ecorr = {"efac": "by_backend", "equad": "by_backend", "ecorr": "by_backend",
                   "spin_noise": "powerlaw_30_nfreqs", "dm_noise": "powerlaw_30_nfreqs"}
    # c1: the reference's example pulsar and model (default_noise_example_1.json)
    c1 = synth.config_c1(os.path.join(HERE, "ref_examples"))
    X = np.vstack([synth.prior_draws(c1.pta, 8, 11), synth.near_draws(c1.pta, c1.truth, 8, 12)])
    dump("c1_j1832", c1.pta, recipe_of(c1, {"efac": "by_backend", "equad": "by_backend", "spin_noise": "powerlaw",
                                            "dm_noise": "powerlaw"}, {}, False), X)
    # c2 small: varying white noise with ECORR
    c2 = synth.config_c2(n_toa=1500, epoch_size=4)
    X = np.vstack([synth.prior_draws(c2.pta, 8, 21), synth.near_draws(c2.pta, c2.truth, 8, 22)])
    dump("c2_small", c2.pta, recipe_of(c2, terms_ecorr, {}, False), X)
    # c3 small: fixed white noise, CURN merged with red noise
    c3 = synth.config_c3(n_psr=4, n_min=600, n_max=1500, epoch_size=4)
    X = np.vstack([synth.prior_draws(c3.pta, 8, 31), synth.near_draws(c3.pta, c3.truth, 8, 32)])
    dump("c3_small", c3.pta, recipe_of(c3, terms_ecorr, {"gwb": "vary_gamma_14_nfreqs"}, True), X)
    # c1 turnover: the reference's default_noise_example_2.json model for
    # J1832-0836 (efac by backend, spin_noise turnover, dm_noise powerlaw)
    c1t = synth.config_c1(os.path.join(HERE, "ref_examples"))
    psr = c1t.pta.signal_collections[0].psr
    ns = synth.params_namespace(np.ptp(psr.toas), False)
    terms_t = {"efac": "by_backend", "spin_noise": "turnover", "dm_noise": "powerlaw"}
    pta_t = synth.build_pta([psr], terms_t, {}, ns, None)
    truth_t = synth.truth_values(pta_t, 5)
    X = np.vstack([synth.prior_draws(pta_t, 8, 13), synth.near_draws(pta_t, truth_t, 8, 14)])
    dump("c1_turnover", pta_t, {"per_psr_terms": terms_t, "common_terms": {}, "Tspan": float(np.ptp(psr.toas)),
                                "fixed_white": False, "noisedict": {}}, X)
    # c3 free spectrum: fixed white noise, CURN as a 10-bin free spectrum
    c3f = synth.config_c3(n_psr=3, n_min=700, n_max=1400, epoch_size=4)
    psrs = [c.psr for c in c3f.pta.signal_collections]
    Tspan = max(p.toas.max() for p in psrs) - min(p.toas.min() for p in psrs)
    ns = synth.params_namespace(Tspan, True)
    wn = {k: v for k, v in c3f.pta.constant_values().items() if v is not None}
    common_f = {"gwb": "freesp_10_nfreqs"}
    pta_f = synth.build_pta(psrs, terms_ecorr, common_f, ns, wn)
    truth_f = synth.truth_values(pta_f, 6, white=wn)
    X = np.vstack([synth.prior_draws(pta_f, 8, 15), synth.near_draws(pta_f, truth_f, 8, 16)])
    dump("c3_freesp", pta_f, {"per_psr_terms": terms_ecorr, "common_terms": common_f, "Tspan": float(Tspan),
                              "fixed_white": True, "noisedict": wn}, X)
    # c4 small: varying white noise, band noise, wide basis (LDS kernel)
    c4 = synth.config_c4(n_psr=3, n_min=700, n_max=1200, epoch_size=4)
    X = np.vstack([synth.prior_draws(c4.pta, 8, 41), synth.near_draws(c4.pta, c4.truth, 8, 42)])
    dump("c4_small", c4.pta, recipe_of(c4, {"efac": "by_backend", "equad": "by_backend",
                                            "spin_noise": "powerlaw_30_nfreqs", "dm_noise": "powerlaw_30_nfreqs",
                                            "ppta_band_noise": ["20CM_30_nfreqs"]},
                                       {"gwb": "vary_gamma_14_nfreqs"}, False), X)
    # c2 chromatic: varying white noise, DM noise and a chromatic GP whose
    # spectral index is sampled (chromred "vary": the basis depends on theta)
    c2c = synth.config_c2(n_toa=1200, epoch_size=4)
    psr = c2c.pta.signal_collections[0].psr
    ns = synth.params_namespace(np.ptp(psr.toas), False)
    terms_c = {"efac": "by_backend", "equad": "by_backend", "ecorr": "by_backend",
               "spin_noise": "powerlaw_20_nfreqs", "dm_noise": "powerlaw_20_nfreqs", "chromred": "vary_15_nfreqs"}
    pta_c = synth.build_pta([psr], terms_c, {}, ns, None)
    truth_c = synth.truth_values(pta_c, 7)
    X = np.vstack([synth.prior_draws(pta_c, 8, 17), synth.near_draws(pta_c, truth_c, 8, 18)])
    dump("c2_chromvary", pta_c, {"per_psr_terms": terms_c, "common_terms": {}, "Tspan": float(np.ptp(psr.toas)),
                                 "fixed_white": False, "noisedict": {}}, X)
    # c5 small: fixed white noise + ECORR, Hellings-Downs correlated common
    # process (cross-pulsar Sigma), and the same model with a monopole ORF
    for name, gwb in (("c5_small", "hd_vary_gamma_5_nfreqs"), ("c5_mono", "mono_vary_gamma_4_nfreqs"),
                      ("c5_noauto", "hd_noauto_vary_gamma_5_nfreqs"), ("c5_dipo", "dipo_vary_gamma_4_nfreqs")):
        c5 = synth.config_c5(n_psr=4, n_toa=500, seed=50, epoch_size=4, gwb=gwb, nfreqs=10)
        truth = dict(c5.truth)
        if "noauto" in gwb:
            # Gamma without auto terms: M_g = diag(phi_red) + Gamma_off phi_gw is
            # positive definite only while the pulsars' own red noise dominates
            truth["gw_log10_A"] = -15.5
        X = np.vstack([synth.prior_draws(c5.pta, 8, 51), synth.near_draws(c5.pta, truth, 8, 52)])
        dump(name, c5.pta, recipe_of(c5, c5.terms, c5.common, True), X)
    # c1 system noise: the reference's system_noise_example.dat /
    # system_noise_example.json for J1832-0836 (efac / equad fixed from the
    # example noise file; spin + DM noise; system noise on the PDFB_40CM and
    # CASPSR_40CM groups; band noise on 10CM: enterprise_models.py:256-338)
    c1s = synth.config_c1(os.path.join(HERE, "ref_examples"))
    psr = c1s.pta.signal_collections[0].psr
    ns = synth.params_namespace(np.ptp(psr.toas), True)
    terms_s = {"efac": "by_backend", "equad": "by_backend", "spin_noise": "powerlaw", "dm_noise": "powerlaw",
               "system_noise": ["PDFB_40CM", "CASPSR_40CM"], "ppta_band_noise": ["10CM"]}
    wn = {k: v for k, v in c1s.truth.items() if k.endswith("_efac") or k.endswith("_log10_tnequad")}
    pta_s = synth.build_pta([psr], terms_s, {}, ns, wn)
    truth_s = synth.truth_values(pta_s, 8, white=wn)
    synth.simulate_residuals(pta_s, truth_s, 9)
    X = np.vstack([synth.prior_draws(pta_s, 8, 19), synth.near_draws(pta_s, truth_s, 8, 20)])
    dump("c1_system", pta_s, {"per_psr_terms": terms_s, "common_terms": {}, "Tspan": float(np.ptp(psr.toas)),
                              "fixed_white": True, "noisedict": wn}, X)
    # c5 varying white noise: the HD process stacked on sampled efac / equad /
    # ecorr (enterprise_models.py:108-146 under :390-403): per-sample
    # contraction, partial factorisation with the timing model in
    c5v = synth.config_c5(n_psr=4, n_toa=500, seed=57, epoch_size=4, gwb="hd_vary_gamma_5_nfreqs", nfreqs=10,
                          fixed_white=False)
    X = np.vstack([synth.prior_draws(c5v.pta, 8, 58), synth.near_draws(c5v.pta, c5v.truth, 8, 59)])
    dump("c5_varwn", c5v.pta, recipe_of(c5v, c5v.terms, c5v.common, False), X)
    # c1 wide: the reference's example pulsar with 60 frequencies per term
    # (X_60_nfreqs, enterprise_models.py:148-167; fake_psr_0's own rule gives
    # 60) for red, DM and chromatic noise: 376 basis columns, past the register
    # kernels (chol_wide_kernel / contract_wide_kernel); white noise sampled
    # (c1_wide) and fixed at the example noise file (c1_widefix)
    c1w = synth.config_c1(os.path.join(HERE, "ref_examples"))
    psr = c1w.pta.signal_collections[0].psr
    terms_w = {"efac": "by_backend", "equad": "by_backend", "spin_noise": "powerlaw_60_nfreqs",
               "dm_noise": "powerlaw_60_nfreqs", "chromred": "4_60_nfreqs"}
    for name, fixed in (("c1_wide", False), ("c1_widefix", True)):
        ns = synth.params_namespace(np.ptp(psr.toas), fixed)
        wn = {k: v for k, v in c1w.truth.items() if k.endswith("_efac") or k.endswith("_log10_tnequad")}
        pta_w = synth.build_pta([psr], terms_w, {}, ns, wn if fixed else None)
        truth_w = synth.truth_values(pta_w, 21, white=wn)
        synth.simulate_residuals(pta_w, truth_w, 22)
        X = np.vstack([synth.prior_draws(pta_w, 8, 23), synth.near_draws(pta_w, truth_w, 8, 24)])
        dump(name, pta_w, {"per_psr_terms": terms_w, "common_terms": {}, "Tspan": float(np.ptp(psr.toas)),
                           "fixed_white": fixed, "noisedict": wn if fixed else {}}, X)


if __name__ == "__main__":
    main()
