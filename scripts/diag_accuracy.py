"""Per-sample accuracy diagnostics (dev library): GPU lnL of every golden
sample (kernel mode 0 and the LDS kernel, mode 1), the per-pulsar unit
terms, and the device intermediates of the wide-basis fixtures -- the cached
reduced matrix S_p / K_p (fixed white noise) and the per-sample Gram
(varying white noise) -- for offline comparison with the restatements in
oracle/ (which stage carries the error).  Writes gpurun_out/diag_accuracy.npz.

    python scripts/diag_accuracy.py [fixture ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("EWARP_HIP_LIB", os.path.join(ROOT, "enterprise_warp_amd", "libewarp_hip_dev.so"))
import numpy as np  # noqa: E402

from conftest import GOLDEN_NAMES, load_golden, strict_tolerance  # noqa: E402

DUMP = ("c1_system", "c4_small", "c1_j1832", "c3_small")


def main():
    names = sys.argv[1:] or GOLDEN_NAMES
    out = {}
    for nm in names:
        pta, z = load_golden(nm, full=True)
        eng = pta.engine()
        X = z["theta"]
        got = pta.get_lnlikelihood_batch(X)
        out[f"{nm}_gpu"] = got
        out[f"{nm}_units"] = eng.unit_terms(len(X))
        from enterprise_warp_amd._lib import EngineError
        eng.set_kernel_mode(1)
        try:
            out[f"{nm}_gpu_lds"] = pta.get_lnlikelihood_batch(X)
        except EngineError:          # (wider than the LDS kernel takes)
            pass
        eng.set_kernel_mode(0)
        ext, ent = z["lnl_exact"], z["lnl"]
        fin = np.isfinite(ext)
        st = strict_tolerance(ext[fin])
        eg = (got[fin] - ext[fin]) / st
        ee = (ent[fin] - ext[fin]) / st
        print(f"{nm:13s} gpu " + " ".join(f"{v:8.2f}" for v in eg[:8]), flush=True)
        print(f"{'':13s} ent " + " ".join(f"{v:8.2f}" for v in ee[:8]), flush=True)
        if nm in DUMP:
            for p, c in enumerate(pta.signal_collections):
                if pta.white_fixed():
                    n = 16 * ((c.T.shape[1] - c.n_lead_const + 1 + 15) // 16)
                    S, K = eng.dev_reduced(p, n)
                    out[f"{nm}_S{p}"] = S
                    out[f"{nm}_K{p}"] = np.array([K])
                else:
                    out[f"{nm}_G{p}"] = eng.dev_gram(p, X[:8])
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "diag_accuracy.npz"), **out)
    print("saved", len(out), "arrays")


if __name__ == "__main__":
    main()
