"""CPU tests of the C ABI: the library loads without a GPU, exports every
entry point include/ewarp_hip.h declares, and the ctypes structs match the C
layout (checked by compiling the header with gcc)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT
from enterprise_warp_amd import _lib

HEADER = os.path.join(ROOT, "include", "ewarp_hip.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"\b(ewh_[a-z_]+)\s*\(", src)))


def test_header_declares_bound_functions():
    assert declared_functions() == sorted(_lib.EXPORTS)


def test_library_loads_and_exports():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libewarp_hip.so not built (run __graft_entry__.build())")
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert lib.ewh_version() == _lib.EWH_ABI_VERSION
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for name in declared_functions():
        assert re.search(rf"\bT {name}\b", out), f"{name} not exported"


def test_struct_layout_matches_header(tmp_path):
    structs = {"ewh_pref": _lib.Pref, "ewh_spec_entry": _lib.SpecEntry, "ewh_pulsar_desc": _lib.PulsarDesc,
               "ewh_pta_desc": _lib.PtaDesc}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "ewarp_hip.h"', "int main(void){"]
    for cname, cls in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in cls._fields_:
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True)
    got = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True,
                                                               text=True).stdout.strip().splitlines())
    for cname, cls in structs.items():
        assert int(got[cname]) == C.sizeof(cls), cname
        for fname, _ in cls._fields_:
            assert int(got[f"{cname}.{fname}"]) == getattr(cls, fname).offset, f"{cname}.{fname}"


def test_engine_fails_loudly_without_gpu():
    """No CPU fallback: creating the engine on a host without a HIP device
    raises an EngineError instead of silently computing elsewhere."""
    import numpy as np
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except Exception:  # noqa: BLE001
        pass
    from conftest import load_golden
    pta, X, _, _ = load_golden("c1_j1832")
    with pytest.raises(_lib.EngineError):
        pta.get_lnlikelihood_batch(X[:2])
    assert np.isfinite(X).all()


def test_dev_exports_only_in_dev_library():
    """The kernel A/B variants and diagnostic exports are not in the product
    library (enterprise_warp_amd/csrc/Makefile `dev`)."""
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for name in _lib.DEV_EXPORTS:
        assert name not in out
    if os.path.exists(_lib.DEV_LIB_PATH):
        out = subprocess.run(["nm", "-D", "--defined-only", _lib.DEV_LIB_PATH], capture_output=True, text=True).stdout
        for name in _lib.DEV_EXPORTS + _lib.EXPORTS:
            assert re.search(rf"\bT {name}\b", out), name
