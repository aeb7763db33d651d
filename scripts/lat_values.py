"""lnL of C3 draws one theta per call (the latency kernel, B = 1) and in
batches of 8 and 24 under the library EWARP_HIP_LIB names, saved to /
compared with an .npy (bit identity of a latency-kernel change across builds).

    python scripts/lat_values.py save|compare <path.npy>
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
    X = np.vstack([synth.prior_draws(cfg.pta, 24, 11), synth.near_draws(cfg.pta, cfg.truth, 24, 12)])
    one = np.array([cfg.pta.get_lnlikelihood(x) for x in X[:16]])
    b8 = cfg.pta.get_lnlikelihood_batch(X[16:24])
    b24 = cfg.pta.get_lnlikelihood_batch(X[24:48])
    got = np.concatenate([one, b8, b24])
    if what == "save":
        np.save(path, got)
        print(f"saved {len(got)} values ({os.environ.get('EWARP_HIP_LIB')})")
    else:
        ref = np.load(path)
        print(f"bit-identical: {np.array_equal(got, ref)}; differing {int(np.sum(got != ref))} of {len(got)} "
              f"({os.environ.get('EWARP_HIP_LIB')})")
