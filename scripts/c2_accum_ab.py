"""A/B (dev library): C2's contraction accumulation on the
whole 4096-draw bench batch: batch time, and per draw the error against the
device's double-double twin (kernel mode 29) beside enterprise's order
(host oracle, tests/_oracle_pool.py): how many draws exceed max(|ent - dd|,
strict), and the worst ratio.  Modes (argv, default "0,30"): 0 the product
(round 6: TwoSum groups up to 10 blocks; before: the single fp64
accumulator), 30 TwoSum groups, 38 / 39 blocked groups on 4 / 8 waves.

    EWARP_HIP_LIB=enterprise_warp_amd/libewarp_hip_dev.so python scripts/c2_accum_ab.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

if __name__ == "__main__":
    from _oracle_pool import map_reference
    cfg_ent = map_reference("c2", 4096, 4096, range(4096), "ent")[:, 0]   # (before the GPU is touched)
    from enterprise_warp_amd import synth
    cfg = synth.config_c2()
    assert cfg.theta_seed == 4096 and cfg.B == 4096
    pta = cfg.pta
    X = synth.prior_draws(pta, cfg.B, cfg.theta_seed)
    eng = pta.engine()
    eng.set_kernel_mode(29)
    dd = pta.get_lnlikelihood_batch(X)
    st = 1e-6 + 1e-10 * np.abs(dd)
    fe = np.isfinite(cfg_ent)
    modes = [int(m) for m in (sys.argv[1] if len(sys.argv) > 1 else "0,30").split(",")]
    for mode in modes + modes:
        eng.set_kernel_mode(mode)
        got = pta.get_lnlikelihood_batch(X)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            pta.get_lnlikelihood_batch(X)
            ts.append(time.perf_counter() - t0)
        r = np.abs(got[fe] - dd[fe]) / np.maximum(np.abs(cfg_ent[fe] - dd[fe]), st[fe])
        print(f"mode {mode}: {1e3 * np.median(ts):.2f} ms per 4096; |gpu - dd|/strict max "
              f"{np.max(np.abs(got - dd) / st):.3e}; draws past max(|ent - dd|, strict): {int(np.sum(r > 1))} of "
              f"{int(fe.sum())}, worst {r.max():.2f}", flush=True)
