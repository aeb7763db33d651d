"""Host-side AddressSanitizer run of the C ABI (sanitizer build
of the host shim).  `make -C enterprise_warp_amd/csrc asan` compiles the host
translation unit with -Xarch_host -fsanitize=address (device code unchanged;
GPU sanitizers are not available on this pool) and links
tests/hip/abi_asan_driver.cpp against it.  The driver feeds well-formed and
malformed descriptors through ewh_create's validation, CSR and table builders
(CPU: every malformed descriptor is rejected with EWH_E_INVALID before any
device call), and on a GPU host runs create -> lnl_batch -> set_fixed_white
-> two-context create -> destroy.  ASan aborts on any host memory error."""
import os
import subprocess

import pytest

from conftest import ROOT, gpu_available

DRIVER = os.path.join(ROOT, "build", "abi_asan_driver")


def _build():
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "enterprise_warp_amd", "csrc"), "asan"],
                   check=True, capture_output=True, text=True, timeout=900)


def _run(*args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    r = subprocess.run([DRIVER, *args], capture_output=True, text=True, timeout=300, env=env)
    print(r.stdout[-3000:], r.stderr[-3000:])
    return r


def test_abi_validation_under_asan():
    _build()
    r = _run()
    assert r.returncode == 0 and "0 failure(s)" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr


@pytest.mark.gpu
def test_abi_device_path_under_asan(require_gpu):
    if not os.path.exists(DRIVER):      # prebuilt in-tree (build/ travels with the snapshot)
        _build()
    r = _run("--gpu")
    assert r.returncode == 0 and "0 failure(s)" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr
