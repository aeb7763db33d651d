"""Dump device intermediates (dev library) for offline comparison with the
numpy restatements: per-sample Gram matrices (varying white noise) and the
cached reduced matrices S_p / K_p (fixed white noise)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("EWARP_HIP_LIB", os.path.join(ROOT, "enterprise_warp_amd", "libewarp_hip_dev.so"))
import numpy as np  # noqa: E402
from conftest import load_golden  # noqa: E402

out = {}
for nm in ("c2_small", "c4_small"):
    pta, z = load_golden(nm, full=True)
    eng = pta.engine()
    out[f"{nm}_lnl"] = pta.get_lnlikelihood_batch(z["theta"])
    for p in range(len(pta.signal_collections)):
        out[f"{nm}_G{p}"] = eng.dev_gram(p, z["theta"])
for nm in ("c3_small", "c3_freesp", "c1_j1832"):
    pta, z = load_golden(nm, full=True)
    eng = pta.engine()
    out[f"{nm}_lnl"] = pta.get_lnlikelihood_batch(z["theta"])
    if pta.white_fixed():
        for p, c in enumerate(pta.signal_collections):
            n = 16 * ((c.T.shape[1] - c.n_lead_const + 1 + 15) // 16)
            S, K = eng.dev_reduced(p, n)
            out[f"{nm}_S{p}"] = S
            out[f"{nm}_K{p}"] = np.array([K])
    else:
        out[f"{nm}_G0"] = eng.dev_gram(0, z["theta"])
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "intermediates.npz"), **out)
print("saved", sorted(out))
