"""Every register-blocked Cholesky variant of the dev library (kernel modes
0, 2-6, 8-13: Cholesky / LDL^T panels, looped / unrolled, DPP / LDS
broadcasts, blocked panel, quotient and row-scale forms) against the oracle
on full-size C3: near-truth draws at the strict bound.  Exit status 0 when
all pass.  Run by tests/test_gpu_ab.py (marker gpu_ab) in its own process:

    python scripts/check_variants.py [--modes 0,2,3,...]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("EWARP_HIP_LIB", os.path.join(ROOT, "enterprise_warp_amd", "libewarp_hip_dev.so"))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="0,2,17,19,21,22,24,25,26")
    args = ap.parse_args()
    from conftest import check_parity, oracle_lnl
    from enterprise_warp_amd import synth
    c3 = synth.config_c3()
    pta = c3.pta
    X = synth.near_draws(pta, c3.truth, 16, 7)
    want = oracle_lnl(pta, X)
    bad = []
    for mode in [int(m) for m in args.modes.split(",")]:
        pta.engine().set_kernel_mode(mode)
        got = pta.get_lnlikelihood_batch(X)
        try:
            check_parity(got, want, f"C3 variant mode {mode}")
        except AssertionError as e:
            print(e)
            bad.append(mode)
    pta.engine().set_kernel_mode(0)
    print("failed modes:", bad)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
