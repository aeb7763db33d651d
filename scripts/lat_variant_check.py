"""Latency-kernel variant check (dev library): unit terms and lnL of kernel
mode --mode against the batched path (mode 2) on the goldens the latency
parity test uses (tests/test_gpu_properties.py
test_latency_kernel_matches_batched), B = 1, 5, 8.  Prints one JSON object.

    EWARP_HIP_LIB=.../libewarp_hip_dev.so python scripts/lat_variant_check.py --mode 26
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", type=int, required=True)
    args = ap.parse_args()
    from enterprise_warp_amd import synth
    from conftest import load_golden
    out = {}
    ok = True
    for name in ("c3_small", "c3_freesp", "c1_j1832", "c1_system", "full_c3"):
        if name == "full_c3":
            cfg = synth.config_c3()
            pta = cfg.pta
            X = np.vstack([synth.prior_draws(pta, 8, 45), synth.near_draws(pta, cfg.truth, 8, 3)])
        else:
            pta, X, _, _ = load_golden(name)
        eng = pta.engine()
        worst = 0.0
        for B in (1, 5, 8):
            XX = X[:B]
            eng.set_kernel_mode(2)
            ref = pta.get_lnlikelihood_batch(XX)
            rt = eng.unit_terms(B)
            eng.set_kernel_mode(args.mode)
            got = pta.get_lnlikelihood_batch(XX)
            gt = eng.unit_terms(B)
            again = pta.get_lnlikelihood_batch(XX)
            same_pattern = bool(np.array_equal(np.isfinite(got), np.isfinite(ref))) and not np.any(np.isnan(got))
            fin = np.isfinite(rt) & np.isfinite(gt)
            d = float(np.max(np.abs(gt[fin] - rt[fin]) / (1e-9 + 1e-12 * np.abs(rt[fin])))) if fin.any() else 0.0
            worst = max(worst, d)
            det = bool(np.array_equal(again, got))
            ok = ok and same_pattern and det and d <= 1.0
        out[name] = {"unit_terms_err_over_rtol1e-12": worst}
        eng.set_kernel_mode(0)
    out["ok"] = ok
    print(json.dumps(out, indent=1))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
