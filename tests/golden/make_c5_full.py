"""Oracle lnL for BASELINE config 5 at its stated size (100 pulsars x 20,000
TOAs, ECORR, red + DM noise 30 frequencies, Hellings-Downs GWB 14
frequencies, fixed white noise): the enterprise-order oracle factors the
dense 13,200 x 13,200 global Sigma = blockdiag(TNT_a) + Phi^-1 (cliques
Phi^-1), as enterprise's dense fallback does.  Run in the dev container
(CPU only, ~1 min):

    python tests/golden/make_c5_full.py

Writes tests/golden/c5_full.json: near-truth theta rows (param_names order),
the oracle's lnL, the device-order fp64 lnL, and a SHA-256 of the seeded
synthetic arrays so the GPU test can confirm it rebuilt the same PTA."""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from enterprise_warp_amd import synth  # noqa: E402


def synth_hash(pta):
    """SHA-256 of the seeded arrays that do not pass through transcendental
    functions (TOAs, TOA errors, radio frequencies, sky positions): identical
    on every host."""
    h = hashlib.sha256()
    for c in pta.signal_collections:
        p = c.psr
        for a in (p.toas, p.toaerrs, p.freqs, p.pos):
            h.update(np.ascontiguousarray(a, dtype=float).tobytes())
    return h.hexdigest()


def synth_sums(pta):
    """Per-pulsar sums of the residuals and timing-model columns: these pass
    through numpy's vectorised sin / cos / exp, whose last bits depend on the
    host's SIMD dispatch (the dev container's Xeon vs the GPU box's EPYC), so
    they are compared to a relative 1e-9 rather than hashed."""
    return [[float(np.sum(c.psr.residuals)), float(np.sum(np.abs(c.psr.residuals))), float(np.sum(c.psr.Mmat))]
            for c in pta.signal_collections]


def main(n_samples=3, seed=101):
    from oracle.device_order_ref import DeviceOrderPTA
    from oracle.enterprise_ref import OraclePTA
    t0 = time.time()
    c5 = synth.config_c5()
    pta = c5.pta
    X = synth.near_draws(pta, c5.truth, n_samples, seed)
    const = pta.constant_values()
    psrs = [c.psr for c in pta.signal_collections]
    o = OraclePTA(psrs, pta.oracle_terms(), fixed_params=const)
    dev = DeviceOrderPTA(psrs, pta.oracle_terms(), const, np.float64)
    print(f"setup {time.time() - t0:.1f}s", flush=True)
    ent, dv = [], []
    for x in X:
        d = dict(const)
        d.update(pta.map_params(x))
        t1 = time.time()
        ent.append(o.lnlikelihood(d))
        dv.append(dev.lnlikelihood(d))
        print(f"sample: enterprise-order {ent[-1]!r} device-order {dv[-1]!r} ({time.time() - t1:.1f}s)", flush=True)
    rec = {"config": "synth.config_c5() (100 psr x 20k TOAs, hd_vary_gamma_14_nfreqs)",
           "near_draws_seed": seed, "synth_sha256": synth_hash(pta), "synth_sums": synth_sums(pta),
           "param_names": pta.param_names,
           "theta": X.tolist(), "lnl": ent, "lnl_dev": dv}
    with open(os.path.join(HERE, "c5_full.json"), "w") as fh:
        json.dump(rec, fh)
    print(f"done {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
