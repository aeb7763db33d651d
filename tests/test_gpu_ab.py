"""Kernel A/B variants (dev library libewarp_hip_dev.so; marker gpu_ab, not
part of the driver's -m gpu suite): each variant against the oracle on
full-size C3 at the strict bound, in a separate process (the dev library is
a different build of the same ABI)."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu_ab


def test_chol_variants_vs_oracle():
    lib = os.path.join(ROOT, "enterprise_warp_amd", "libewarp_hip_dev.so")
    if not os.path.exists(lib):
        pytest.skip("dev library not built (make -C enterprise_warp_amd/csrc dev)")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "check_variants.py")], capture_output=True,
                       text=True, timeout=600)
    print(r.stdout[-4000:], r.stderr[-2000:])
    assert r.returncode == 0


@pytest.mark.parametrize("mode", [0, 24, 25])
def test_latency_variants_vs_batched(mode):
    """chol_lat_kernel variants (0: the dataflow default, 24: the same with
    block barriers, 25: the round-3 kernel) against the batched path on the
    latency-test goldens (scripts/lat_variant_check.py)."""
    lib = os.path.join(ROOT, "enterprise_warp_amd", "libewarp_hip_dev.so")
    if not os.path.exists(lib):
        pytest.skip("dev library not built (make -C enterprise_warp_amd/csrc dev)")
    env = dict(os.environ, EWARP_HIP_LIB=lib)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "lat_variant_check.py"), "--mode", str(mode)],
                       capture_output=True, text=True, timeout=600, env=env)
    print(r.stdout[-4000:], r.stderr[-2000:])
    assert r.returncode == 0


def test_latency_stall_is_an_error():
    """A chol_lat_kernel unit whose LDS-counter wait runs out is an error of
    ewh_lnl_batch (EWH_E_HIP), not a NaN lnL; forced by dev kernel mode 23
    (scripts/lat_stall_check.py)."""
    lib = os.path.join(ROOT, "enterprise_warp_amd", "libewarp_hip_dev.so")
    if not os.path.exists(lib):
        pytest.skip("dev library not built (make -C enterprise_warp_amd/csrc dev)")
    env = dict(os.environ, EWARP_HIP_LIB=lib)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "lat_stall_check.py")],
                       capture_output=True, text=True, timeout=600, env=env)
    print(r.stdout[-4000:], r.stderr[-2000:])
    assert r.returncode == 0


def test_c5_row_update_variants_bit_identical():
    """The C5 row-update schedules of the dev library (28: one block row per
    pass, one tile per workgroup -- round 3; 31: one row per pass, two tiles;
    32: the two-row pass with each streamed slab loaded at the top of its
    step) against the default (two rows per pass, pipelined slabs): the same
    lnL bit for bit (scripts/c5_ab.py on a 20-pulsar HD model, 9 block rows)."""
    lib = os.path.join(ROOT, "enterprise_warp_amd", "libewarp_hip_dev.so")
    if not os.path.exists(lib):
        pytest.skip("dev library not built (make -C enterprise_warp_amd/csrc dev)")
    env = dict(os.environ, EWARP_HIP_LIB=lib)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "c5_ab.py"), "--modes", "0,28,31,32",
                        "--rounds", "1", "--n-psr", "20", "--n-toa", "1200", "--B", "64"],
                       capture_output=True, text=True, timeout=600, env=env)
    print(r.stdout[-4000:], r.stderr[-2000:])
    assert r.returncode == 0


@pytest.mark.parametrize("B", [1, 3])
def test_c5_one_proposal_diag_fusion_bit_identical(B):
    """The one-proposal (right-looking) C5 schedule factors diagonal block
    k + 1 inside the step-k trailing update; dev mode 33 launches it apart:
    the same lnL bit for bit (against the left-looking schedule:
    test_gpu_properties.py::test_correlated_right_looking_small_chunks)."""
    lib = os.path.join(ROOT, "enterprise_warp_amd", "libewarp_hip_dev.so")
    if not os.path.exists(lib):
        pytest.skip("dev library not built (make -C enterprise_warp_amd/csrc dev)")
    env = dict(os.environ, EWARP_HIP_LIB=lib)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "c5_ab.py"), "--modes", "0,33",
                        "--rounds", "1", "--n-psr", "20", "--n-toa", "1200", "--B", str(B)],
                       capture_output=True, text=True, timeout=600, env=env)
    print(r.stdout[-4000:], r.stderr[-2000:])
    assert r.returncode == 0


def test_wide_route_schedule_bit_identical():
    """chol_wide_kernel's paired block rows, the fused forward / reversed
    verify launch and the chip-filling scratch budgets against the round-5a
    schedule (dev mode 34): the same lnL bit for bit on the wide goldens, 64
    prior draws of the 372-column pulsar (white noise fixed and sampled) and
    the correlated wide partial factorisation (scripts/wide_variant_check.py)."""
    lib = os.path.join(ROOT, "enterprise_warp_amd", "libewarp_hip_dev.so")
    if not os.path.exists(lib):
        pytest.skip("dev library not built (make -C enterprise_warp_amd/csrc dev)")
    env = dict(os.environ, EWARP_HIP_LIB=lib)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "wide_variant_check.py")],
                       capture_output=True, text=True, timeout=600, env=env)
    print(r.stdout[-4000:], r.stderr[-2000:])
    assert r.returncode == 0
