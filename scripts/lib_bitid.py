"""Bit-identity of a kernel change across two builds: the lnL of one batch
under the library EWARP_HIP_LIB names, saved to (or compared with) an .npy.

    EWARP_HIP_LIB=.../libewarp_hip_prev.so python scripts/lib_bitid.py save gpurun_out/a.npy [case]
    python scripts/lib_bitid.py compare gpurun_out/a.npy [case]

case: w372_varwn (default), w372_fixed, system, c2, c4 -- 256 prior draws.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    from wide_ab import make_case
    from enterprise_warp_amd import synth
    what, path = sys.argv[1], sys.argv[2]
    case = sys.argv[3] if len(sys.argv) > 3 else "w372_varwn"
    cfg = make_case(case)
    X = synth.prior_draws(cfg.pta, 256, cfg.theta_seed + 7)
    got = cfg.pta.get_lnlikelihood_batch(X)
    if what == "save":
        np.save(path, got)
        print(f"{case}: saved {len(got)} values")
        return
    ref = np.load(path)
    same = np.array_equal(ref, got, equal_nan=True)
    print(f"{case}: bit-identical={same} max|diff|={np.nanmax(np.abs(ref - got)):.3e}")
    sys.exit(0 if same else 1)


if __name__ == "__main__":
    main()
