"""The device-side debug build (`make -C enterprise_warp_amd/csrc debug`:
build/libewarp_hip_debug.so, -DEWH_DEBUG; SURVEY.md §5's sanitizer row for
device code): the EWH_DCHECK invariants (ewarp_dev.h -- iteration bounds on
every grab / spin loop, a full exec mask at chol_dd's tile grab, LDS /
scratch / operand bounds in chol_dd, chol_wide and contract_xr) hold on the
15 goldens, the wide (372-column) and system_noise routes and the C4 fp64-
failure refinement.  The parity tests run in a child process on the debug
library (EWARP_HIP_LIB); a failed check prints "EWH_DCHECK failed" and traps.
Marker gpu_debug: outside the driver's -m gpu suite (run on purpose:
`pytest -m gpu_debug`)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEBUG_LIB = os.path.join(ROOT, "build", "libewarp_hip_debug.so")
CASES = "golden_vectors or wide_prior or system_noise or c4_bench_workload"

pytestmark = pytest.mark.gpu_debug


def test_debug_build_invariants(require_gpu):
    if not os.path.exists(DEBUG_LIB):
        pytest.fail(f"{DEBUG_LIB} not built: make -C enterprise_warp_amd/csrc debug")
    env = dict(os.environ, EWARP_HIP_LIB=DEBUG_LIB)
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_gpu_parity.py"), "-m", "gpu", "-k", CASES],
                       env=env, capture_output=True, text=True, timeout=1100)
    out = r.stdout + r.stderr
    print(out[-4000:])
    assert "EWH_DCHECK failed" not in out, "a device invariant failed in the debug build"
    assert r.returncode == 0, f"parity suite on the debug library: rc {r.returncode}"
