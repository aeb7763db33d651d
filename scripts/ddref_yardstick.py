"""VERDICT r05 item 7 (the yardstick): oracle/ddref.py's own error on the
uncorrelated golden fixtures -- the double-double reference with 4 slices
per Gram operand (rounds 4-5: 72 bits below each column maximum) and with 6
(round 6: 108 bits), against each other and against the extended-precision
error-free-Gram restatement (oracle/device_order_ref.py, np.longdouble), in
units of strict per sample.  CPU only; prints one line per fixture.

    python scripts/ddref_yardstick.py [name ...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

UNCORR = ["c1_j1832", "c1_turnover", "c1_system", "c2_small", "c2_chromvary", "c3_small", "c3_freesp", "c4_small",
          "c1_wide", "c1_widefix"]


def main(names):
    from conftest import load_golden
    from oracle import ddref
    from oracle.device_order_ref import DeviceOrderPTA
    for name in names:
        pta, z = load_golden(name, full=True)
        psrs, terms = [c.psr for c in pta.signal_collections], pta.oracle_terms()
        const = pta.constant_values()
        fixed = const if pta.white_fixed() else None
        vals = {}
        for k in (4, 6):
            ddref.DD_SLICES = k
            r = ddref.DDReferencePTA(psrs, terms)
            v = []
            for x in z["theta"]:
                d = dict(const)
                d.update(pta.map_params(x))
                v.append(r.lnlikelihood(d))
            vals[k] = np.array(v)
        ext = DeviceOrderPTA(psrs, terms, fixed, np.longdouble)
        v = []
        for x in z["theta"]:
            d = dict(const)
            d.update(pta.map_params(x))
            v.append(ext.lnlikelihood(d))
        vals["ld"] = np.array(v)
        ddref.DD_SLICES = 6
        fin = np.isfinite(vals[6])
        s = 1e-6 + 1e-10 * np.abs(vals[6][fin])
        r46 = np.abs(vals[4][fin] - vals[6][fin]) / s
        rld = np.abs(vals["ld"][fin] - vals[6][fin]) / s
        rst = np.abs(z["lnl_exact"][fin] - vals[6][fin]) / s
        rent = np.abs(z["lnl"][fin] - vals[6][fin]) / s
        print(f"{name}: |dd(k=4) - dd(k=6)|/strict max {r46.max():.3e} (sample {np.argmax(r46)}); "
              f"|longdouble - dd(k=6)|/strict max {rld.max():.3e}; |stored lnl_exact - dd(k=6)|/strict max "
              f"{rst.max():.3e}; |enterprise - dd(k=6)|/strict max {rent.max():.3e}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or UNCORR)
