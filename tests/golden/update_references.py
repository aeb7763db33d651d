"""Recompute the reference values of the committed golden fixtures in place
(run in the dev container; CPU only):

    python tests/golden/update_references.py [name ...]

Inputs (pulsar arrays, recipe, theta) are left exactly as committed; only
lnl_dev, lnl_exact, spread and min_eig are recomputed with
make_golden.oracle_lnl (the current device-order restatement and the
near-exact reference).  The enterprise-order value is recomputed too and must
equal the stored `lnl` (a check that the oracle is unchanged)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import GOLDEN_NAMES, load_golden  # noqa: E402
from golden.make_golden import oracle_lnl  # noqa: E402


def main(names):
    for name in names:
        path = os.path.join(HERE, name + ".npz")
        pta, z = load_golden(name, full=True)
        vals, spread, cond = oracle_lnl(pta, z["theta"])
        ent = vals[0]
        fin = np.isfinite(z["lnl"])
        assert np.array_equal(np.isfinite(ent), fin)
        dent = np.max(np.abs(ent[fin] - z["lnl"][fin]) / (1e-6 + 1e-10 * np.abs(z["lnl"][fin]))) if fin.any() else 0.0
        assert dent < 1e-3, f"{name}: enterprise-order value moved by {dent} x strict"
        arrays = dict(np.load(path, allow_pickle=False))
        arrays.update(lnl_dev=vals[1], lnl_exact=vals[4], spread=spread, min_eig=cond)
        np.savez_compressed(path, **arrays)
        st = 1e-6 + 1e-10 * np.abs(vals[4][fin])
        print(f"{name}: |ent - exact|/strict max {np.max(np.abs(ent[fin] - vals[4][fin]) / st) if fin.any() else 0:.3g}, "
              f"|device - exact|/strict max {np.max(np.abs(vals[1][fin] - vals[4][fin]) / st) if fin.any() else 0:.3g}",
              flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or GOLDEN_NAMES)
