"""The verify-and-refine route's blind spot at scale: on a model's whole
prior-draw batch, the samples where the default route (two fp64 orders
verify each other; disagreeing units refactored in double-double) and
kernel mode 29 (every unit in double-double) differ by more than the strict
bound, each against the CPU double-double reference (oracle/ddref.py) and
enterprise's own fp64 order; plus the forward / reversed fp64 pass values
(mode 27 and the verify's own agreement) for those samples.

    python scripts/diag_verify_blindspot.py [system|w372_fixed] [--max 12] [--seed-offset 0]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from conftest import reference_lnl, strict_tolerance
    from enterprise_warp_amd import synth
    case = sys.argv[1] if len(sys.argv) > 1 else "system"
    nmax = int(sys.argv[sys.argv.index("--max") + 1]) if "--max" in sys.argv else 12
    off = int(sys.argv[sys.argv.index("--seed-offset") + 1]) if "--seed-offset" in sys.argv else 0
    cfg = (synth.config_system(os.path.join(ROOT, "tests", "golden", "ref_examples")) if case == "system"
           else synth.config_wide(True))
    pta = cfg.pta
    X = synth.prior_draws(pta, cfg.B, cfg.theta_seed + off)
    eng = pta.engine()
    route = pta.get_lnlikelihood_batch(X)
    out = {}
    for m in (29, 27):
        eng.set_kernel_mode(m)
        out[m] = pta.get_lnlikelihood_batch(X)
    eng.set_kernel_mode(0)
    st = strict_tolerance(out[29])
    bad = np.flatnonzero(np.abs(route - out[29]) > st)
    print(f"{case}: {len(bad)} of {len(X)} samples with |route - dd| > strict", flush=True)
    sel = bad[np.argsort(-np.abs(route - out[29])[bad])][:nmax]
    if len(sel) == 0:
        return
    ent, ext = reference_lnl(pta, X[sel], exact="dd")
    s = strict_tolerance(ext)
    np.set_printoptions(linewidth=220, precision=3)
    print("sample          ", sel)
    print("route - ref     ", (route[sel] - ext) / s)
    print("dd    - ref     ", (out[29][sel] - ext) / s)
    print("fp64 fwd - ref  ", (out[27][sel] - ext) / s)
    print("enterprise - ref", (ent - ext) / s)
    worse = np.abs(route[sel] - ext) > np.maximum(np.maximum(np.abs(ent - ext), np.abs(out[29][sel] - ext)), s)
    print(f"route worse than both enterprise's order and all-double-double (and strict): {int(worse.sum())} "
          f"of {len(sel)}", flush=True)


if __name__ == "__main__":
    main()
