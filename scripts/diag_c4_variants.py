"""Diagnostic: enterprise's algorithm in two further
fp64 orders (tests/_oracle_pool.py "entv_psr") on C4's 1024 bench draws, per
pulsar finiteness -> gpurun_out/c4inf/c4var.npz (host only)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

if __name__ == "__main__":
    from _oracle_pool import map_reference
    t0 = time.time()
    v = map_reference("c4", 30, 1024, range(1024), "entv_psr")
    os.makedirs(os.path.join(ROOT, "gpurun_out", "c4inf"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", "c4inf", "c4var.npz"), v=v)
    P = v.shape[1] // 2
    print(f"done {time.time() - t0:.1f} s; -inf draws: reversed+lower {(v[:, :P].min(1) == 0).sum()}, "
          f"lower {(v[:, P:].min(1) == 0).sum()}")
