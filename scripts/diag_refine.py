"""Diagnostic: the fp64-failure refinement (refine_failed) on C4's first 64
prior draws -- refine counters and the per-pulsar terms of the -inf draws."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    from enterprise_warp_amd import synth
    cfg = synth.config_c4()
    pta = cfg.pta
    X = synth.prior_draws(pta, cfg.B, cfg.theta_seed)[:64]
    eng = pta.engine()
    print("stats before", eng.refine_stats())
    got = pta.get_lnlikelihood_batch(X)
    print("stats after first", eng.refine_stats())
    u = eng.unit_terms(64)
    bad = np.flatnonzero(~np.isfinite(got))
    print("-inf draws", bad.tolist())
    for b in bad:
        print(" draw", b, "pulsars -inf", np.flatnonzero(~np.isfinite(u[:, b])).tolist())
    got2 = pta.get_lnlikelihood_batch(X)
    print("stats after second (graph)", eng.refine_stats(), "same", np.array_equal(got, got2, equal_nan=True))
    eng.set_kernel_mode(2)
    got3 = pta.get_lnlikelihood_batch(X)
    print("mode 2 stats", eng.refine_stats(), np.flatnonzero(~np.isfinite(got3)).tolist())
    # kernel mode 29: every varying unit through gram_dd_units + chol_dd
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import oracle_lnl
    eng.set_kernel_mode(29)
    Xn = synth.near_draws(pta, cfg.truth, 4, 31)
    a = pta.get_lnlikelihood_batch(Xn)
    eng.set_kernel_mode(0)
    b = pta.get_lnlikelihood_batch(Xn)
    o = oracle_lnl(pta, Xn)
    print("near: mode29 - oracle", a - o, "default - oracle", b - o, "strict", 1e-6 + 1e-10 * np.abs(o))
    eng.set_kernel_mode(29)
    g29 = pta.get_lnlikelihood_batch(X)
    print("prior mode 29 stats", eng.refine_stats(), "-inf", np.flatnonzero(~np.isfinite(g29)).tolist())
    print("prior mode29 - default (finite)", np.nanmax(np.abs(np.where(np.isfinite(got) & np.isfinite(g29), g29 - got, np.nan))))
