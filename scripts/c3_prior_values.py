"""Print the GPU lnL of chosen prior draws of the C3 bench workload (the
first 4096 draws bench.py evaluates) with full precision, for accuracy
studies against the CPU orderings (oracle/)."""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from enterprise_warp_amd import synth

idx = [int(a) for a in (sys.argv[1] if len(sys.argv) > 1 else "3,10,0").split(",")]
cfg = synth.config_c3()
pta = cfg.pta
X = synth.prior_draws(pta, 4096, cfg.theta_seed)[idx]
got = pta.get_lnlikelihood_batch(X)
for i, g in zip(idx, got):
    print(i, repr(float(g)))
