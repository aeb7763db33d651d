"""The host C++ twin of the C ABI (csrc/ewarp_cpu.cpp, libewarp_cpu.so;
SURVEY.md §8(b): "a C++ CPU twin has the same ABI"), on the CPU: every
uncorrelated / CURN golden fixture under the GPU's own accuracy criterion
(near-truth draws strict against the enterprise-order oracle and the
near-exact value; prior draws no less accurate than enterprise's order),
correlated fixtures refused with EWH_E_UNSUPPORTED, in-place white noise,
unit terms, refused device entries, and the exported symbol set."""
import ctypes
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(ROOT, "enterprise_warp_amd", "libewarp_cpu.so")


@pytest.fixture(scope="module")
def twin_lib():
    if not os.path.exists(LIB):
        subprocess.run(["make", "-C", os.path.join(ROOT, "enterprise_warp_amd", "csrc"), "cpu"], check=True,
                       capture_output=True)
    return LIB


def test_twin_exports_the_abi(twin_lib):
    from enterprise_warp_amd import _lib
    lib = ctypes.CDLL(twin_lib)
    for sym in _lib.EXPORTS:
        assert hasattr(lib, sym), sym
    lib.ewh_version.restype = ctypes.c_int
    assert lib.ewh_version() == _lib.EWH_ABI_VERSION


def test_twin_goldens_and_surface(twin_lib):
    env = dict(os.environ, EWARP_BACKEND="cpu", OMP_NUM_THREADS="4")
    env.pop("EWARP_HIP_LIB", None)
    p = subprocess.run([sys.executable, os.path.join(HERE, "_twin_worker.py")], env=env, capture_output=True,
                       text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    line = next(ln for ln in p.stdout.splitlines() if ln.startswith("TWIN_JSON "))
    res = json.loads(line[len("TWIN_JSON "):])
    print(p.stdout)
    assert res["lib"] == "libewarp_cpu.so"
    assert set(res["goldens"]) == {"c1_j1832", "c1_turnover", "c1_system", "c2_small", "c2_chromvary", "c3_small",
                                   "c3_freesp", "c4_small", "c1_wide", "c1_widefix"}
    assert set(res["refused"]) == {"c5_small", "c5_mono", "c5_noauto", "c5_dipo", "c5_varwn"}
    assert all("device-only" in v for v in res["refused"].values())
    assert res["set_fixed_white_equal"] and res["set_fixed_white_changed"]
    assert res["unit_terms_sum_ok"]
    assert res["device_entry_refused"]
