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
from oracle.enterprise_ref import OraclePTA  # noqa: E402


def oracle_lnl(pta, X):
    """lnL per sample and the sample's conditioning: min over pulsars of the
    smallest eigenvalue of the unit-diagonal-scaled Sigma (near 0 = the
    Cholesky-failure boundary, where -inf parity is inherently fragile)."""
    const = pta.constant_values()
    fixed = const if pta.white_fixed() else None
    o = OraclePTA([c.psr for c in pta.signal_collections], pta.oracle_terms(), fixed_params=fixed)
    out, cond = [], []
    for x in X:
        d = dict(const)
        d.update(pta.map_params(x))
        out.append(o.lnlikelihood(d))
        if o.correlated():
            cond.append(correlated_min_eig(o, d))
            continue
        mins = []
        for i, pp in enumerate(o.pulsars):
            TNT = o.fixed[i][0] if fixed is not None else pp.white_terms(d)[0]
            S = TNT + np.diag(1.0 / pp.phi(d))
            sc = 1.0 / np.sqrt(np.diag(S))
            mins.append(np.linalg.eigvalsh(S * sc[:, None] * sc[None, :])[0])
        cond.append(min(mins))
    return np.array(out), np.array(cond)


def correlated_min_eig(o, d):
    """lambda_min of the unit-diagonal-scaled global Sigma = blockdiag(TNT) +
    Phi^-1 of a correlated PTA (the conditioning of its one factorisation)."""
    terms = [o.fixed[i] if o.fixed is not None else pp.white_terms(d) for i, pp in enumerate(o.pulsars)]
    Phi, off = o.phi_global(d)
    S, _ = o.phiinv_cliques(Phi)
    for a, t in enumerate(terms):
        S[off[a]:off[a + 1], off[a]:off[a + 1]] += t[0]
    sc = 1.0 / np.sqrt(np.abs(np.diag(S)))
    return np.linalg.eigvalsh(S * sc[:, None] * sc[None, :])[0]


def dump(name, pta, recipe, X):
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
    lnl, cond = oracle_lnl(pta, X)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), recipe=np.array(json.dumps(recipe)), theta=X, lnl=lnl,
                        min_eig=cond, **arrays)
    print(name, "n_psr", len(psrs), "nparam", X.shape[1], "n_inf", int(np.sum(~np.isfinite(lnl))),
          "min_eig", np.round(np.log10(np.abs(cond)), 1))


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
    for name, gwb in (("c5_small", "hd_vary_gamma_5_nfreqs"), ("c5_mono", "mono_vary_gamma_4_nfreqs")):
        c5 = synth.config_c5(n_psr=4, n_toa=500, seed=50, epoch_size=4, gwb=gwb, nfreqs=10)
        X = np.vstack([synth.prior_draws(c5.pta, 8, 51), synth.near_draws(c5.pta, c5.truth, 8, 52)])
        dump(name, c5.pta, recipe_of(c5, c5.terms, c5.common, True), X)


if __name__ == "__main__":
    main()
