"""Diagnostic: C4's whole 1024-draw bench batch on the
GPU (default route, per-pulsar unit terms) against the host enterprise-order
oracle's finiteness per pulsar (tests/_oracle_pool.py, spawned workers).
Writes gpurun_out/c4inf/c4inf.npz for the host-side analysis."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from _oracle_pool import map_reference
    out = os.path.join(ROOT, "gpurun_out", "c4inf")
    os.makedirs(out, exist_ok=True)
    t0 = time.time()
    # host oracle first (spawned workers, before this process touches the GPU)
    ent_psr = map_reference("c4", 30, 1024, range(1024), "ent_psr")
    print(f"ent_psr done {time.time() - t0:.1f} s; ent -inf draws {(ent_psr.min(1) == 0).sum()}", flush=True)
    from enterprise_warp_amd import synth
    cfg = synth.config_c4()
    assert cfg.theta_seed == 30 and cfg.B == 1024
    pta = cfg.pta
    X = synth.prior_draws(pta, cfg.B, cfg.theta_seed)
    got = pta.get_lnlikelihood_batch(X)
    units = pta.engine().unit_terms(cfg.B)
    print(f"gpu done {time.time() - t0:.1f} s; gpu -inf draws {(~np.isfinite(got)).sum()}", flush=True)
    np.savez(os.path.join(out, "c4inf.npz"), got=got, units=units, ent_psr=ent_psr)
    gi, ei = ~np.isfinite(got), ent_psr.min(1) == 0
    print(f"gpu -inf {gi.sum()}, ent -inf {ei.sum()}, both {(gi & ei).sum()}, gpu only {(gi & ~ei).sum()}, "
          f"ent only {(ei & ~gi).sum()}", flush=True)


if __name__ == "__main__":
    main()
