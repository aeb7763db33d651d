"""Diagnostic: the headline batch (4096 C3 prior draws)
on the default route and under kernel mode 29 (every unit in double-double),
per-pulsar unit terms of both -> gpurun_out/hdd/hdd.npz for the host-side
analysis against oracle/ddref.py (scripts/analyse_headline_dd.py)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from enterprise_warp_amd import synth
    out = os.path.join(ROOT, "gpurun_out", "hdd")
    os.makedirs(out, exist_ok=True)
    cfg = synth.config_c3()
    pta = cfg.pta
    X = synth.prior_draws(pta, cfg.B, cfg.theta_seed)
    eng = pta.engine()
    got = pta.get_lnlikelihood_batch(X)
    u_got = eng.unit_terms(cfg.B)
    eng.set_kernel_mode(29)
    dd = pta.get_lnlikelihood_batch(X)
    u_dd = eng.unit_terms(cfg.B)
    eng.set_kernel_mode(0)
    np.savez(os.path.join(out, "hdd.npz"), got=got, dd=dd, u_got=u_got, u_dd=u_dd)
    s = 1e-6 + 1e-10 * np.abs(dd)
    print("outside strict:", int(np.sum(np.abs(got - dd) > s)), "max", float(np.max(np.abs(got - dd) / s)))


if __name__ == "__main__":
    main()
