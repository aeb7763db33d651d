"""Interleaved A/B timing of kernel modes -- written for the wide / double-double route (bases past the
register kernels: the 372-column 10k-TOA pulsar with white noise fixed and
sampled, and the reference's system_noise_example model) between kernel
modes, on prior and near-truth draws; per mode the median ms per batch, the
refined share (ewh_refine_stats) and the largest difference from the first
mode in strict units (modes that only change launch shapes must be 0).

    python scripts/wide_ab.py [--cases w372_fixed,system] [--modes 0,34,27,29] [--rounds 5]
    python scripts/wide_ab.py --cases c2,c4 --modes 0,35 --kinds prior --contract

Loads the dev library (mode 34 and the other A/B modes live there only)
unless EWARP_HIP_LIB names another build.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("EWARP_HIP_LIB", os.path.join(ROOT, "enterprise_warp_amd", "libewarp_hip_dev.so"))


def make_case(name):
    from enterprise_warp_amd import synth
    if name == "w372_fixed":
        return synth.config_wide(True)
    if name == "w372_varwn":
        return synth.config_wide(False)
    if name == "system":
        return synth.config_system(os.path.join(ROOT, "tests", "golden", "ref_examples"))
    if name in ("c2", "c3", "c4"):
        return getattr(synth, f"config_{name}")()
    raise SystemExit(f"unknown case {name}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="w372_fixed,system")
    ap.add_argument("--modes", default="0,34")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--kinds", default="prior,near")
    ap.add_argument("--seed-offset", type=int, default=0,
                    help="added to the case's theta seed (fresh draws beyond the bench's own batch)")
    ap.add_argument("--contract", action="store_true",
                    help="time the contraction stage alone (ewh_contract_device) instead of the lnL batch")
    args = ap.parse_args()
    import torch
    from enterprise_warp_amd import synth
    modes = [int(m) for m in args.modes.split(",")]
    res = {}
    for case in args.cases.split(","):
        cfg = make_case(case)
        pta, B = cfg.pta, cfg.B
        eng = pta.engine(0)
        U = len(pta.signal_collections) * B
        out = torch.zeros(B, dtype=torch.float64, device="cuda")
        sd = cfg.theta_seed + args.seed_offset
        draws = {"prior": lambda: synth.prior_draws(pta, B, sd),
                 "near": lambda: synth.near_draws(pta, cfg.truth, B, sd + 1)}
        for kind in args.kinds.split(","):
            th = torch.from_numpy(draws[kind]()).cuda()
            times = {m: [] for m in modes}
            vals, share = {}, {}
            for r in range(args.rounds + 1):
                for m in modes:
                    eng.set_kernel_mode(m)
                    eng.refine_stats()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    s.record()
                    if args.contract:
                        eng.contract_device(th.data_ptr(), B, 0)
                    else:
                        eng.lnl_units_device(th.data_ptr(), B, 0, U, out.data_ptr(), 0)
                    e.record()
                    torch.cuda.synchronize()
                    if args.contract:     # (the values: one lnL batch after the timed contraction)
                        eng.lnl_units_device(th.data_ptr(), B, 0, U, out.data_ptr(), 0)
                        torch.cuda.synchronize()
                    if r > 0:   # round 0 warms up (scratch allocation, first launches)
                        times[m].append(s.elapsed_time(e))
                    c, f = eng.refine_stats()
                    share[m] = f / c if c else None
                    vals[m] = out.cpu().numpy().copy()
            ref = vals[modes[0]]
            for m in modes:
                v = vals[m]
                same_fin = bool(np.array_equal(np.isfinite(ref), np.isfinite(v)))
                fin = np.isfinite(ref) & np.isfinite(v)
                d = float(np.max(np.abs(v[fin] - ref[fin]) / (1e-6 + 1e-10 * np.abs(ref[fin])))) if fin.any() else 0.0
                res[f"{case}/{kind}/mode{m}"] = {
                    "median_ms": float(np.median(times[m])), "min_ms": float(np.min(times[m])),
                    "evals_per_s": B / (np.median(times[m]) * 1e-3), "refined_share": share[m],
                    "finite": float(np.mean(np.isfinite(v))), "same_finiteness": same_fin,
                    "max_diff_over_strict_vs_first": d}
            del th
        eng.set_kernel_mode(0)
        pta._drop_engine()
        print(json.dumps({k: v for k, v in res.items() if k.startswith(case + "/")}, indent=1), flush=True)


if __name__ == "__main__":
    main()
