"""GPU accuracy on every golden fixture: per sample |lnL_gpu - lnL_ext| and
|lnL_enterprise - lnL_ext| in units of the strict bound (1e-6 + 1e-10 |lnL|),
lnL_ext = the extended-precision value stored in the fixture.  Prints one
line per fixture and the samples where the GPU is less accurate than
enterprise's own fp64 order (the criterion of tests/test_gpu_parity.py::
test_golden_vectors).  Usage: python scripts/accuracy_goldens.py [mode]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import GOLDEN_NAMES, load_golden, strict_tolerance  # noqa: E402


def main():
    mode = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    worst = 0.0
    for name in GOLDEN_NAMES:
        pta, z = load_golden(name, full=True)
        if mode:
            pta.engine().set_kernel_mode(mode)
        got = pta.get_lnlikelihood_batch(z["theta"])
        ext, ent = z["lnl_exact"], z["lnl"]
        fin = np.isfinite(ext)
        st = strict_tolerance(ext[fin])
        eg = np.abs(got[fin] - ext[fin]) / st
        ee = np.abs(ent[fin] - ext[fin]) / st
        worse = np.flatnonzero(eg > np.maximum(ee, 1.0))
        worst = max(worst, float(np.max(eg / np.maximum(ee, 1.0))))
        print(f"{name:13s} gpu/ext max {eg.max():10.3g}  ent/ext max {ee.max():10.3g}  "
              f"-inf gpu {int(np.sum(~np.isfinite(got)))} ref {int(np.sum(~fin))}  worse-than-enterprise "
              + (", ".join(f"#{i}: {eg[i]:.3g} vs {ee[i]:.3g}" for i in worse) or "none"), flush=True)
    print(f"max over samples of gpu_err / max(ent_err, strict) = {worst:.3g}")


if __name__ == "__main__":
    main()
