"""VERDICT r05 item 7 (the route): the verify-and-refine route's tail on
fresh prior-draw batches of the reference's system_noise_example model --
per batch, the samples where the default route and every unit in double-
double (kernel mode 29) differ by more than strict, their distance from the
CPU double-double value (oracle/ddref.py) against enterprise's order and the
all-double-double value, the refined share and the route's time.  Run with
the dev library to set the verify threshold (EWARP_VERIFY_FRAC, a fraction
of strict; product: 1/16):

    EWARP_HIP_LIB=enterprise_warp_amd/libewarp_hip_dev.so EWARP_VERIFY_FRAC=0.015625 \\
        python scripts/verify_tail.py --offsets 0,1000,2000,3000
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from conftest import reference_lnl, strict_tolerance
    from enterprise_warp_amd import synth
    offs = [int(v) for v in (sys.argv[sys.argv.index("--offsets") + 1] if "--offsets" in sys.argv
                             else "0,1000,2000,3000").split(",")]
    cfg = synth.config_system(os.path.join(ROOT, "tests", "golden", "ref_examples"))
    pta = cfg.pta
    eng = pta.engine()
    print(f"verify fraction {os.environ.get('EWARP_VERIFY_FRAC', '1/16 (product)')}", flush=True)
    for off in offs:
        X = synth.prior_draws(pta, cfg.B, cfg.theta_seed + off)
        route = pta.get_lnlikelihood_batch(X)
        eng.refine_stats()
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            route = pta.get_lnlikelihood_batch(X)
            ts.append(time.perf_counter() - t0)
        c, r = eng.refine_stats()
        eng.set_kernel_mode(29)
        dd = pta.get_lnlikelihood_batch(X)
        eng.set_kernel_mode(0)
        st = strict_tolerance(dd)
        ratio = np.abs(route - dd) / st
        bad = np.flatnonzero(ratio > 1.0)
        line = (f"offset {off}: refined {r / max(c, 1):.3f} of units, route {1e3 * np.median(ts):.2f} ms per "
                f"{len(X)}; |route - dd| / strict max {ratio.max():.3g}; past strict: {len(bad)}")
        if len(bad):
            ent, ext = reference_lnl(pta, X[bad], exact="dd")
            s = strict_tolerance(ext)
            line += (f"; vs CPU dd: route {np.round(np.abs(route[bad] - ext) / s, 3).tolist()}, all-dd "
                     f"{np.round(np.abs(dd[bad] - ext) / s, 4).tolist()}, enterprise "
                     f"{np.round(np.abs(ent - ext) / s, 1).tolist()}")
        print(line, flush=True)


if __name__ == "__main__":
    main()
