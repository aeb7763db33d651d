"""Per-sample errors of the wide / double-double routes on a golden fixture:
the default route (verify-and-refine), kernel mode 29 (every unit in
double-double) and mode 27 (one fp64 chol_wide pass), against the fixture's
near-exact lnL, in units of the strict bound; and the verify step's counts.

    python scripts/diag_wide_route.py [c1_wide]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from conftest import load_golden, strict_tolerance
    name = sys.argv[1] if len(sys.argv) > 1 else "c1_wide"
    pta, z = load_golden(name, full=True)
    X, ext, ent = z["theta"], z["lnl_exact"], z["lnl"]
    eng = pta.engine()
    st = strict_tolerance(ext)
    np.set_printoptions(linewidth=200, precision=3)
    print("enterprise", np.abs(ent - ext) / st)
    for mode in (0, 29, 27):
        eng.set_kernel_mode(mode)
        eng.refine_stats()
        got = pta.get_lnlikelihood_batch(X)
        c, r = eng.refine_stats()
        print(f"mode {mode:2d} checked {c} refined {r}", np.abs(got - ext) / st)
    eng.set_kernel_mode(0)


if __name__ == "__main__":
    main()
