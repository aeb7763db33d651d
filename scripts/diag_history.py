"""Does a golden's GPU lnL depend on what ran before it in the process?"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
from conftest import GOLDEN_NAMES, load_golden  # noqa: E402

order = sys.argv[1].split(",") if len(sys.argv) > 1 else GOLDEN_NAMES
watch = ["c3_small", "c2_small"]
first = {}
for nm in watch:
    pta, z = load_golden(nm, full=True)
    first[nm] = pta.get_lnlikelihood_batch(z["theta"])
    print(nm, "fresh   err vs exact:", np.array2string(first[nm] - z["lnl_exact"], precision=3, max_line_width=300))
    again = pta.get_lnlikelihood_batch(z["theta"])
    print(nm, "same handle again identical:", np.array_equal(again, first[nm]))
for nm in order:
    try:
        pta, z = load_golden(nm, full=True)
        pta.get_lnlikelihood_batch(z["theta"])
        print("ran", nm)
    except Exception as e:  # noqa: BLE001
        print("ran", nm, "->", type(e).__name__, str(e)[:120])
    for w in watch:
        p2, z2 = load_golden(w, full=True)
        g = p2.get_lnlikelihood_batch(z2["theta"])
        if not np.array_equal(g, first[w]):
            print("   ", w, "CHANGED: err vs exact", np.array2string(g - z2["lnl_exact"], precision=3, max_line_width=300))
