"""Dev library: the latency kernel's stall path (kernel mode 23 forces every
LDS-counter wait of chol_lat_kernel to run out at once).  ewh_lnl_batch must
return an error -- never a NaN lnL -- and the handle must stay usable: the
next call in the default mode gives the batched path's value.  Exit 0 on
success (tests/test_gpu_ab.py::test_latency_stall_is_an_error)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ.setdefault("EWARP_HIP_LIB", os.path.join(ROOT, "enterprise_warp_amd", "libewarp_hip_dev.so"))
import numpy as np  # noqa: E402

from conftest import load_golden  # noqa: E402
from enterprise_warp_amd._lib import EngineError  # noqa: E402


def main():
    pta, X, _, _ = load_golden("c3_small")
    eng = pta.engine()
    eng.set_kernel_mode(2)
    ref = pta.get_lnlikelihood_batch(X[:4])
    eng.set_kernel_mode(23)
    for B in (1, 4):
        try:
            v = pta.get_lnlikelihood_batch(X[:B])
        except EngineError as e:
            assert "ran out" in str(e), str(e)
            print(f"B={B}: stall reported: {e}")
        else:
            print(f"B={B}: no error, got {v}")
            return 1
    eng.set_kernel_mode(0)
    got = pta.get_lnlikelihood_batch(X[:4])
    err = np.abs(got - ref) / (1e-6 + 1e-10 * np.abs(ref))
    print("after the stall, default mode vs batched: max err/strict", err.max())
    return 0 if err.max() <= 1e-3 else 1


if __name__ == "__main__":
    sys.exit(main())
