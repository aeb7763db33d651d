"""Sampler-call latency on C3 (host theta in, host lnL out through
ewh_lnl_batch): per batch size, the median over `reps` calls with the
default kernels (mode 0: the latency kernel for B <= LAT_B_MAX) and with the
batched kernels only (mode 2).  Run under rocprofv3 --kernel-trace --stats to
see the kernel share.  Prints one JSON object.

    python scripts/latency_sweep.py [--reps 200] [--batches 1,2,4,8,16,32]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--batches", default="1,2,4,8,16,32")
    ap.add_argument("--modes", default="0,2")
    ap.add_argument("--rounds", type=int, default=1, help="interleave the modes over this many rounds")
    args = ap.parse_args()
    from enterprise_warp_amd import synth
    cfg = synth.config_c3()
    pta = cfg.pta
    eng = pta.engine()
    out = {}
    modes = [int(m) for m in args.modes.split(",")]
    for B in [int(b) for b in args.batches.split(",")]:
        X = synth.prior_draws(pta, B, 11 + B)
        ts = {m: [] for m in modes}
        vals = {}
        for _ in range(args.rounds):
            for mode in modes:
                eng.set_kernel_mode(mode)
                vals[mode] = pta.get_lnlikelihood_batch(X)
                for _ in range(args.reps // args.rounds):
                    t0 = time.perf_counter()
                    pta.get_lnlikelihood_batch(X)
                    ts[mode].append(time.perf_counter() - t0)
        for mode in modes:
            t = ts[mode]
            d = np.abs(np.asarray(vals[mode]) - np.asarray(vals[modes[0]]))
            out[f"B{B}/mode{mode}"] = {"us_median": 1e6 * float(np.median(t)), "us_p10": 1e6 * float(np.percentile(t, 10)),
                                       "evals_per_s": B / float(np.median(t)),
                                       "max_abs_diff_vs_first_mode": float(np.max(d))}
    eng.set_kernel_mode(0)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
