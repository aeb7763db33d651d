"""Interleaved A/B of the C5 (100 psr x 20k TOAs, HD) batched factorisation
between kernel modes (dev library): ms per 512-proposal batch (HIP events
around ewh_lnl_units_device), fp64 MFMA fraction, and bit identity against
the first mode.  python scripts/c5_ab.py [--modes 0,28] [--rounds 5]"""
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
    ap.add_argument("--modes", default="0,28")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--B", type=int, default=512)
    ap.add_argument("--n-psr", type=int, default=100)
    ap.add_argument("--n-toa", type=int, default=20000)
    args = ap.parse_args()
    import torch
    from bench import FP64_MFMA_PEAK_TFLOPS
    from enterprise_warp_amd import synth
    cfg = synth.config_c5(n_psr=args.n_psr, n_toa=args.n_toa)
    pta = cfg.pta
    eng = pta.engine(0)
    P, B = len(pta.signal_collections), args.B
    X = synth.prior_draws(pta, B, cfg.theta_seed)
    th = torch.from_numpy(X).cuda()
    out = torch.zeros(B, dtype=torch.float64, device="cuda")
    st = torch.cuda.current_stream()
    nc = pta.common_layout()["n_col"]
    m = np.array([c.T.shape[1] for c in pta.signal_collections])
    flops = (float(np.sum(m ** 3 / 3.0)) + (P * nc + 1) ** 3 / 3.0) * B
    modes = [int(v) for v in args.modes.split(",")]
    times = {md: [] for md in modes}
    vals = {}
    for r in range(args.rounds):
        for md in modes:
            eng.set_kernel_mode(md)
            eng.lnl_units_device(th.data_ptr(), B, 0, P * B, out.data_ptr(), st.cuda_stream)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(st)
            eng.lnl_units_device(th.data_ptr(), B, 0, P * B, out.data_ptr(), st.cuda_stream)
            b.record(st)
            torch.cuda.synchronize()
            times[md].append(a.elapsed_time(b))
            vals[md] = out.cpu().numpy().copy()
    eng.set_kernel_mode(0)
    res = {}
    for md in modes:
        ms = float(np.median(times[md]))
        res[f"mode{md}"] = {"ms_median": ms, "ms_all": times[md], "evals_per_s": B / (ms * 1e-3),
                            "fp64_mfma_frac": flops / (ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS,
                            "bit_identical_to_first": bool(np.array_equal(vals[md], vals[modes[0]]))}
    print(json.dumps(res, indent=1))
    return 0 if all(r["bit_identical_to_first"] for r in res.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
