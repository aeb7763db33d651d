"""lnL of the headline workload's 4096 C3 prior draws and 64 near-truth draws
under the library EWARP_HIP_LIB names, saved to / compared with an .npy
(bit identity of a kernel change across builds).

    python scripts/c3_values.py save|compare <path.npy>
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if __name__ == "__main__":
    from enterprise_warp_amd import synth
    what, path = sys.argv[1], sys.argv[2]
    cfg = synth.config_c3()
    X = np.vstack([synth.prior_draws(cfg.pta, 4096, cfg.theta_seed), synth.near_draws(cfg.pta, cfg.truth, 64, 5)])
    got = cfg.pta.get_lnlikelihood_batch(X)
    if what == "save":
        np.save(path, got)
        print(f"saved {len(got)} values ({os.environ.get('EWARP_HIP_LIB')})")
    else:
        ref = np.load(path)
        same = np.array_equal(got, ref)
        d = np.abs(got - ref) / (1e-6 + 1e-10 * np.abs(ref))
        print(f"bit-identical: {same}; max |diff| / strict {np.nanmax(d):.3e}; "
              f"differing values {int(np.sum(got != ref))} of {len(got)} ({os.environ.get('EWARP_HIP_LIB')})")
