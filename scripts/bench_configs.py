"""Per-configuration throughput on one GPU (BASELINE.json configs 2-4) with a
parity spot check against the oracle on a few samples of each.

    python scripts/bench_configs.py [--configs c2,c3,c4] [--reps 3]

Prints one JSON object per config: evals/s, ms per batch, batch size, kernel
path, and the max |GPU - oracle| / tolerance over the spot-checked samples.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def oracle_vals(pta, X):
    from oracle.enterprise_ref import OraclePTA
    const = pta.constant_values()
    o = OraclePTA([c.psr for c in pta.signal_collections], pta.oracle_terms(),
                  fixed_params=const if pta.white_fixed() else None)
    out = []
    for x in X:
        d = dict(const)
        d.update(pta.map_params(x))
        out.append(o.lnlikelihood(d))
    return np.array(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c2,c3,c4")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--check", type=int, default=3)
    ap.add_argument("--mode", type=int, default=0, help="ewh_set_kernel_mode (7: round-1 contraction)")
    args = ap.parse_args()
    import torch
    from enterprise_warp_amd import synth
    for name in args.configs.split(","):
        t0 = time.time()
        cfg = getattr(synth, f"config_{name}")()
        build_s = time.time() - t0
        pta = cfg.pta
        B = cfg.B
        X = synth.near_draws(pta, cfg.truth, B, 11)
        t0 = time.time()
        eng = pta.engine(0)
        eng.set_kernel_mode(args.mode)
        create_s = time.time() - t0
        th = torch.from_numpy(X).cuda()
        out = torch.zeros(B, dtype=torch.float64, device="cuda")
        U = len(pta.signal_collections) * B
        eng.lnl_units_device(th.data_ptr(), B, 0, U, out.data_ptr(), 0)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            eng.lnl_units_device(th.data_ptr(), B, 0, U, out.data_ptr(), 0)
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e))
        got = out.cpu().numpy()
        idx = np.arange(min(args.check, B))
        want = oracle_vals(pta, X[idx]) if len(idx) else np.zeros(0)
        tol = 1e-6 + 1e-10 * np.abs(want)
        rec = {"config": name, "mode": args.mode, "n_pulsars": len(pta.signal_collections), "B": B,
               "basis": sorted({c.T.shape[1] for c in pta.signal_collections}),
               "white_fixed": pta.white_fixed(), "ms_per_batch": float(np.median(ts)),
               "evals_per_s": B / (np.median(ts) * 1e-3), "host_build_s": build_s, "engine_create_s": create_s,
               "finite": float(np.mean(np.isfinite(got))),
               "max_err_over_tol": float(np.max(np.abs(got[idx] - want) / tol)) if len(idx) else None}
        print(json.dumps(rec), flush=True)
        pta._drop_engine()


if __name__ == "__main__":
    main()
