"""ctypes binding of libewarp_hip.so (include/ewarp_hip.h).

The library is built in-tree (`enterprise_warp_amd/libewarp_hip.so`, see
csrc/Makefile / __graft_entry__.build).  There is no CPU fallback: if the
library or a GPU is missing, the likelihood raises.  EWARP_HIP_LIB selects
another build of the same ABI (the dev library libewarp_hip_dev.so with the
kernel A/B variants and diagnostic exports: scripts/chol_ab.py, gpu_ab tests).
EWARP_BACKEND=cpu selects the host C++ twin of the same ABI,
libewarp_cpu.so (csrc/ewarp_cpu.cpp, `make -C enterprise_warp_amd/csrc cpu`):
an explicit choice for hosts without a GPU, never taken automatically.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
CPU_LIB_PATH = os.path.join(_HERE, "libewarp_cpu.so")
BACKEND = os.environ.get("EWARP_BACKEND", "hip").lower()
if BACKEND not in ("hip", "cpu"):
    raise ValueError(f"EWARP_BACKEND={BACKEND!r}: expected 'hip' (default) or 'cpu'")
LIB_PATH = os.environ.get("EWARP_HIP_LIB") or (CPU_LIB_PATH if BACKEND == "cpu" else
                                               os.path.join(_HERE, "libewarp_hip.so"))
DEV_LIB_PATH = os.path.join(_HERE, "libewarp_hip_dev.so")

EWH_ABI_VERSION = 7
COMMON_CORRELATED, COMMON_OPTSTAT = 0, 1
SPEC_POWERLAW, SPEC_TURNOVER, SPEC_FREESPEC, SPEC_CONST = 1, 2, 3, 4


class Pref(C.Structure):
    _fields_ = [("idx", C.c_int32), ("pad_", C.c_int32), ("cval", C.c_double)]


class SpecEntry(C.Structure):
    _fields_ = [("kind", C.c_int32), ("col", C.c_int32), ("p0", Pref), ("p1", Pref), ("p2", Pref),
                ("f", C.c_double), ("df", C.c_double), ("fyr", C.c_double)]


_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int32)


class PulsarDesc(C.Structure):
    _fields_ = [("n_toa", C.c_int32), ("n_col", C.c_int32), ("n_lead_const", C.c_int32), ("n_spec", C.c_int32),
                ("basis", _dp), ("resid", _dp), ("toaerr", _dp),
                ("n_slot", C.c_int32), ("slots", C.POINTER(Pref)),
                ("efac_slot", _ip), ("equad_slot", _ip),
                ("n_epoch", C.c_int32), ("epoch_start", _ip), ("epoch_stop", _ip), ("epoch_slot", _ip),
                ("spec", C.POINTER(SpecEntry)),
                ("n_bgroup", C.c_int32), ("bgroup_idx", C.POINTER(Pref)), ("col_bgroup", _ip), ("ln_chrom", _dp),
                ("n_common", C.c_int32)]


class CommonDesc(C.Structure):
    _fields_ = [("n_col", C.c_int32), ("orf", _dp), ("spec", C.POINTER(SpecEntry)), ("kind", C.c_int32)]


class PtaDesc(C.Structure):
    _fields_ = [("abi_version", C.c_int32), ("n_pulsar", C.c_int32), ("n_param", C.c_int32),
                ("white_fixed", C.c_int32), ("pulsars", C.POINTER(PulsarDesc)), ("common", C.POINTER(CommonDesc))]


EXPORTS = ["ewh_create", "ewh_num_devices", "ewh_set_fixed_white", "ewh_lnl_batch", "ewh_lnl_units_device",
           "ewh_keep_dim", "ewh_corr_partial_device", "ewh_corr_finish_device",
           "ewh_last_unit_terms", "ewh_unit_cost", "ewh_set_kernel_mode", "ewh_optstat", "ewh_contract_device",
           "ewh_transfer_stats", "ewh_lat_b_max", "ewh_refine_stats",
           "ewh_destroy", "ewh_last_error", "ewh_version"]
DEV_EXPORTS = ["ewh_dev_gram", "ewh_dev_reduced"]

_lib = None


class EngineError(RuntimeError):
    pass


def load():
    """Load and type the shared library (does not touch the GPU)."""
    global _lib
    if _lib is not None:
        return _lib
    # The HIP runtime must be loaded once per process.  torch ships its own
    # libamdhip64 (same SONAME as /opt/rocm's); if our library is loaded
    # first, torch later maps a second runtime and device queries fail.  Load
    # torch's runtime first so libewarp_hip.so binds to it.
    if BACKEND != "cpu":
        try:
            import torch  # noqa: F401
        except Exception:  # noqa: BLE001 - torch is optional for the ABI itself
            pass
    if not os.path.exists(LIB_PATH):
        raise EngineError(f"{LIB_PATH} not built: run `make -C enterprise_warp_amd/csrc` or "
                          "__graft_entry__.build(); there is no CPU fallback")
    lib = C.CDLL(LIB_PATH)
    # a library of an older ABI lacks entry points: say so before typing them
    missing = [n for n in EXPORTS if not hasattr(lib, n)]
    if missing or lib.ewh_version() != EWH_ABI_VERSION:
        raise EngineError(f"{LIB_PATH}: library out of date (ABI version mismatch"
                          f"{'; missing ' + ', '.join(missing) if missing else ''}); rebuild it "
                          "(make -C enterprise_warp_amd/csrc)")
    lib.ewh_create.argtypes = [C.POINTER(PtaDesc), _ip, C.c_int32, C.POINTER(C.c_void_p)]
    lib.ewh_create.restype = C.c_int
    lib.ewh_num_devices.argtypes = [C.c_void_p]
    lib.ewh_num_devices.restype = C.c_int
    lib.ewh_set_fixed_white.argtypes = [C.c_void_p, _dp]
    lib.ewh_set_fixed_white.restype = C.c_int
    lib.ewh_lnl_batch.argtypes = [C.c_void_p, _dp, C.c_int32, _dp]
    lib.ewh_lnl_batch.restype = C.c_int
    lib.ewh_lnl_units_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int64, C.c_int64, C.c_void_p,
                                         C.c_void_p]
    lib.ewh_lnl_units_device.restype = C.c_int
    lib.ewh_keep_dim.argtypes = [C.c_void_p]
    lib.ewh_keep_dim.restype = C.c_int
    lib.ewh_corr_partial_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p,
                                            C.c_void_p, C.c_void_p]
    lib.ewh_corr_partial_device.restype = C.c_int
    lib.ewh_corr_finish_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p,
                                           C.c_void_p]
    lib.ewh_corr_finish_device.restype = C.c_int
    lib.ewh_last_unit_terms.argtypes = [C.c_void_p, _dp, C.c_int32]
    lib.ewh_last_unit_terms.restype = C.c_int
    lib.ewh_unit_cost.argtypes = [C.c_void_p, C.c_int32]
    lib.ewh_unit_cost.restype = C.c_double
    lib.ewh_set_kernel_mode.argtypes = [C.c_void_p, C.c_int32]
    lib.ewh_set_kernel_mode.restype = C.c_int
    lib.ewh_optstat.argtypes = [C.c_void_p, _dp, C.c_int32, _dp, _dp, _dp, _dp, _dp]
    lib.ewh_optstat.restype = C.c_int
    lib.ewh_contract_device.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p]
    lib.ewh_contract_device.restype = C.c_int
    lib.ewh_transfer_stats.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    lib.ewh_transfer_stats.restype = C.c_int
    lib.ewh_refine_stats.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
    lib.ewh_refine_stats.restype = C.c_int
    lib.ewh_lat_b_max.argtypes = []
    lib.ewh_lat_b_max.restype = C.c_int
    lib.ewh_destroy.argtypes = [C.c_void_p]
    lib.ewh_destroy.restype = None
    lib.ewh_last_error.argtypes = []
    lib.ewh_last_error.restype = C.c_char_p
    lib.ewh_version.argtypes = []
    lib.ewh_version.restype = C.c_int
    if hasattr(lib, "ewh_dev_gram"):
        lib.ewh_dev_gram.argtypes = [C.c_void_p, C.c_int32, _dp, C.c_int32, _dp]
        lib.ewh_dev_gram.restype = C.c_int
        lib.ewh_dev_reduced.argtypes = [C.c_void_p, C.c_int32, _dp, _dp]
        lib.ewh_dev_reduced.restype = C.c_int
    _lib = lib
    return lib


def check(rc):
    if rc != 0:
        raise EngineError(f"libewarp_hip error {rc}: {_lib.ewh_last_error().decode(errors='replace')}")
