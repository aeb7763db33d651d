"""Oracle lnL for the C5 bench's own workload: the first N of the prior draws
bench.py evaluates for BASELINE config 5 (synth.prior_draws(pta, 512,
cfg.theta_seed); 100 pulsars x 20,000 TOAs, Hellings-Downs GWB 14
frequencies, fixed white noise).  Per draw:

  * "lnl"     -- enterprise's order (oracle/enterprise_ref.py): the dense
                 13,200 x 13,200 global Sigma factored by cho_factor, -inf on
                 LinAlgError (/root/reference/enterprise_warp/bilby_warp.py:35
                 -> enterprise's PTA.get_lnlikelihood);
  * "lnl_dev" -- the device's order in fp64 (oracle/device_order_ref.py);
  * "lnl_ext" -- the near-exact value: the same Woodbury form in x86 extended
                 precision on the error-free Gram (device_order_ref with
                 np.longdouble).

Run in the dev container (CPU only, ~30 min for 24 draws; the extended-precision
dense 2,801 x 2,801 factorisation dominates):

    python tests/golden/make_c5_prior.py [N]

Writes tests/golden/c5_prior.json with the synthetic arrays' hash
(make_c5_full.synth_hash) so the GPU test confirms it rebuilt the same PTA."""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from enterprise_warp_amd import synth  # noqa: E402
from golden.make_c5_full import synth_hash, synth_sums  # noqa: E402


def main(n_samples=24):
    from oracle.device_order_ref import DeviceOrderPTA
    from oracle.enterprise_ref import OraclePTA
    t0 = time.time()
    c5 = synth.config_c5()
    pta = c5.pta
    assert c5.B == 512
    X = synth.prior_draws(pta, c5.B, c5.theta_seed)[:n_samples]
    const = pta.constant_values()
    psrs = [c.psr for c in pta.signal_collections]
    o = OraclePTA(psrs, pta.oracle_terms(), fixed_params=const)
    dev = DeviceOrderPTA(psrs, pta.oracle_terms(), const, np.float64)
    ext = DeviceOrderPTA(psrs, pta.oracle_terms(), const, np.longdouble)
    print(f"setup {time.time() - t0:.1f}s", flush=True)
    ent, dv, ex = [], [], []
    for i, x in enumerate(X):
        d = dict(const)
        d.update(pta.map_params(x))
        t1 = time.time()
        ent.append(float(o.lnlikelihood(d)))
        dv.append(float(dev.lnlikelihood(d)))
        ex.append(float(ext.lnlikelihood(d)))
        print(f"draw {i}: enterprise-order {ent[-1]!r} device-order {dv[-1]!r} extended {ex[-1]!r} "
              f"({time.time() - t1:.1f}s)", flush=True)
    rec = {"config": "synth.config_c5() (100 psr x 20k TOAs, hd_vary_gamma_14_nfreqs)",
           "draws": f"synth.prior_draws(pta, {c5.B}, {c5.theta_seed})[:{n_samples}] (the C5 bench's first draws)",
           "synth_sha256": synth_hash(pta), "synth_sums": synth_sums(pta),
           "param_names": pta.param_names,
           "theta": X.tolist(), "lnl": ent, "lnl_dev": dv, "lnl_ext": ex}
    with open(os.path.join(HERE, "c5_prior.json"), "w") as fh:
        json.dump(rec, fh)
    print(f"done {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 24)
