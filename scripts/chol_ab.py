"""Interleaved A/B timing of the Cholesky kernel variants on config C3
(one process, R rounds, median and min per variant; guide §5.4 rule 24).

    python scripts/chol_ab.py [--rounds 7] [--modes 0,2,1]

Modes 3-6 and 8-13 live in the dev library only (make -C
enterprise_warp_amd/csrc dev); this script loads it unless EWARP_HIP_LIB
names another build.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("EWARP_HIP_LIB", os.path.join(ROOT, "enterprise_warp_amd", "libewarp_hip_dev.so"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--modes", default="0,2,1")
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--npsr", type=int, default=45)
    args = ap.parse_args()
    import torch
    from enterprise_warp_amd import synth
    cfg = synth.config_c3(n_psr=args.npsr)
    pta = cfg.pta
    X = synth.prior_draws(pta, args.B, cfg.theta_seed)
    Xn = synth.near_draws(pta, cfg.truth, args.B, 5)
    eng = pta.engine(0)
    B = args.B
    U = len(pta.signal_collections) * B
    out = torch.zeros(B, dtype=torch.float64, device="cuda")
    modes = [int(m) for m in args.modes.split(",")]
    res = {}
    for name, XX in (("prior", X), ("near", Xn)):
        th = torch.from_numpy(XX).cuda()
        times = {m: [] for m in modes}
        vals = {}
        for r in range(args.rounds):
            for m in modes:
                eng.set_kernel_mode(m)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                s.record()
                eng.lnl_units_device(th.data_ptr(), B, 0, U, out.data_ptr(), 0)
                e.record()
                torch.cuda.synchronize()
                times[m].append(s.elapsed_time(e))
                vals[m] = out.cpu().numpy().copy()
        ref = vals[modes[0]]
        for m in modes:
            fin = np.isfinite(ref) & np.isfinite(vals[m])
            d = float(np.max(np.abs(vals[m][fin] - ref[fin]) / (1e-6 + 1e-10 * np.abs(ref[fin])))) if fin.any() else 0
            res[f"{name}/mode{m}"] = {"median_ms": float(np.median(times[m][1:])), "min_ms": float(np.min(times[m])),
                                      "units_per_s": U / (np.median(times[m][1:]) * 1e-3),
                                      "finite": float(np.mean(np.isfinite(vals[m]))), "max_err_over_tol_vs_mode0": d}
    eng.set_kernel_mode(0)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
