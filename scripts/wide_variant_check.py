"""Bit-identity of the wide-route schedule against its round-5a form (dev
kernel mode 34: one block row per pass in chol_wide_kernel, separate forward
and reversed launches, 128 MB scratch budgets): the same lnL bit for bit
(-inf included) on the wide goldens, on 64 prior draws of the 372-column
10k-TOA pulsar (white noise fixed and sampled), on 512 prior draws of the
system_noise model (208 columns) and on the
correlated wide partial factorisation (chol_wide_kernel's KEEP form, 12
blocks).  Exit 1 on any difference.  Loads the dev library unless
EWARP_HIP_LIB names another.

    python scripts/wide_variant_check.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("EWARP_HIP_LIB", os.path.join(ROOT, "enterprise_warp_amd", "libewarp_hip_dev.so"))


MODES = (34,)


def both(pta, X):
    eng = pta.engine()
    out = {}
    for m in (0,) + MODES:
        eng.set_kernel_mode(m)
        out[m] = pta.get_lnlikelihood_batch(X)
    eng.set_kernel_mode(0)
    pta._drop_engine()
    return out


def main():
    from conftest import load_golden
    from enterprise_warp_amd import synth
    cases = []
    for name in ("c1_wide", "c1_widefix", "c1_system"):
        pta, z = load_golden(name, full=True)
        cases.append((name, pta, z["theta"]))
    for fixed in (True, False):
        cfg = synth.config_wide(fixed)
        cases.append((f"w372 fixed_white={fixed} prior", cfg.pta, synth.prior_draws(cfg.pta, 64, 65)))
    cfg = synth.config_system(os.path.join(ROOT, "tests", "golden", "ref_examples"))
    cases.append(("system_noise prior", cfg.pta, synth.prior_draws(cfg.pta, 512, 66)))
    base = synth.config_c5(n_psr=4, n_toa=600, seed=71, epoch_size=8, gwb="hd_vary_gamma_14_nfreqs", nfreqs=30)
    psrs = [c.psr for c in base.pta.signal_collections]
    Tspan = max(p.toas.max() for p in psrs) - min(p.toas.min() for p in psrs)
    for fixed in (True, False):
        wn = synth.white_noisedict(psrs, 73)
        pta = synth.build_pta(psrs, dict(base.terms, chromred="4_30_nfreqs"), base.common,
                              synth.params_namespace(Tspan, fixed), wn if fixed else None)
        truth = synth.truth_values(pta, 74, white=wn)
        synth.simulate_residuals(pta, truth, 75)
        cases.append((f"HD wide partial fixed_white={fixed}", pta, synth.prior_draws(pta, 16, 76)))
    bad = 0
    for name, pta, X in cases:
        out = both(pta, X)
        for m in MODES:
            same = np.array_equal(out[0], out[m], equal_nan=True)
            print(f"{name:40s} n={len(X):3d} finite={np.mean(np.isfinite(out[0])):.2f} mode {m}: bit-identical={same}",
                  flush=True)
            bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
