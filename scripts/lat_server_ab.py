"""The persistent latency server (dev kernel mode 33) against the
launch-per-call latency kernel (mode 0): interleaved rounds of single-theta
calls on full-size C3 (median us per call), the same lnL bit for bit, and
the server's life cycle -- a call after an idle gap longer than the host's
replacement bound, batch sizes changing (1 -> 4 -> 1), a batched call in
between (the server stops), the handle closed while it runs.  Dev library.

    python scripts/lat_server_ab.py [--rounds 5] [--calls 200]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("EWARP_HIP_LIB", os.path.join(ROOT, "enterprise_warp_amd", "libewarp_hip_dev.so"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--calls", type=int, default=200)
    args = ap.parse_args()
    from enterprise_warp_amd import synth
    cfg = synth.config_c3()
    pta = cfg.pta
    eng = pta.engine()
    X = synth.prior_draws(pta, args.calls, 5)
    res = {"mode0": [], "mode33": []}
    vals = {}
    for r in range(args.rounds):
        for md in (0, 33):
            eng.set_kernel_mode(md)
            pta.get_lnlikelihood_batch(X[:1])
            ts, v = [], []
            for i in range(args.calls):
                t0 = time.perf_counter()
                out = pta.get_lnlikelihood_batch(X[i:i + 1])
                ts.append(time.perf_counter() - t0)
                v.append(out[0])
            res[f"mode{md}"].append(1e6 * float(np.median(ts)))
            vals[md] = np.array(v)
        print(f"round {r}: mode0 {res['mode0'][-1]:.2f} us, mode33 {res['mode33'][-1]:.2f} us", flush=True)
    same = bool(np.array_equal(vals[0], vals[33]))
    # life cycle (mode 33)
    eng.set_kernel_mode(0)
    ref = pta.get_lnlikelihood_batch(X[:8])
    eng.set_kernel_mode(33)
    life = {}
    a = pta.get_lnlikelihood_batch(X[:1])
    time.sleep(0.05)                                   # > the host's 10 ms bound and the server's 20 ms
    b = pta.get_lnlikelihood_batch(X[:1])
    life["after_idle"] = bool(a[0] == ref[0] and b[0] == ref[0])
    c = pta.get_lnlikelihood_batch(X[:4])
    d = pta.get_lnlikelihood_batch(X[:1])
    life["batch_change"] = bool(np.array_equal(c, ref[:4]) and d[0] == ref[0])
    big = synth.prior_draws(pta, 64, 9)
    e1 = pta.get_lnlikelihood_batch(big)
    f = pta.get_lnlikelihood_batch(X[:1])
    eng.set_kernel_mode(0)
    e0 = pta.get_lnlikelihood_batch(big)
    life["batched_between"] = bool(np.array_equal(e1, e0) and f[0] == ref[0])
    eng.set_kernel_mode(33)
    pta.get_lnlikelihood_batch(X[:1])
    pta._drop_engine()                                 # (ewh_destroy stops the running server first)
    life["closed"] = True
    out = {"median_us_per_round": res, "mode0_us": float(np.median(res["mode0"])),
           "mode33_us": float(np.median(res["mode33"])), "bit_identical": same, "life": life}
    print(json.dumps(out, indent=1))
    return 0 if same and all(life.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
