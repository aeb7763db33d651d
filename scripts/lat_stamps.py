"""Phase timing of the latency kernel (chol_lat_kernel, dev mode 22) at a
sampler's batch size: s_memtime stamps per wave of the first 64 workgroups
(chol_lat.hip LAT_STAMP).  Prints, per stamp, the mean cycles since the
workgroup's start (max over its four waves), and the spread of workgroup
start times (launch / dispatch skew).

    python scripts/lat_stamps.py [--B 1]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("EWARP_HIP_LIB", os.path.join(ROOT, "enterprise_warp_amd", "libewarp_hip_dev.so"))
WG, NS = 64, 16
NAMES = {0: "start", 1: "theta staged", 2: "phi^-1 ready", 10: "factorised", 11: "unit term",}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1)
    args = ap.parse_args()
    from enterprise_warp_amd import _lib, synth
    cfg = synth.config_c3()
    pta = cfg.pta
    X = synth.prior_draws(pta, args.B, 3)
    eng = pta.engine()
    ref = pta.get_lnlikelihood_batch(X)
    eng.set_kernel_mode(22)
    for _ in range(5):
        got = pta.get_lnlikelihood_batch(X)
    eng.set_kernel_mode(0)
    lib = C.CDLL(_lib.LIB_PATH)
    lib.ewh_dev_lat_stamps.argtypes = [C.POINTER(C.c_longlong), C.c_longlong]
    buf = (C.c_longlong * (WG * 4 * NS))()
    assert lib.ewh_dev_lat_stamps(buf, WG * 4 * NS) == 0
    st = np.frombuffer(buf, dtype=np.int64).reshape(WG, 4, NS).astype(np.float64)
    nwg = min(WG, len(pta.signal_collections) * args.B)
    st = st[:nwg]
    t0 = st[:, :, 0].min(axis=1)                       # workgroup start
    res = {"B": args.B, "workgroups": nwg, "same_as_mode0": bool(np.array_equal(got, ref))}
    rel = {}
    for i in range(NS):
        v = st[:, :, i]
        if np.all(v == 0):
            continue
        m = np.where(v > 0, v - t0[:, None], np.nan)
        rel[NAMES.get(i, f"panel {i - 3} E published")] = float(np.nanmean(np.nanmax(m, axis=1)))
    res["cycles_since_wg_start"] = rel
    res["wg_start_spread_cycles"] = float(t0.max() - t0.min())
    ends = st[:, :, 11].max(axis=1)
    res["kernel_span_to_last_unit_cycles"] = float(ends.max() - t0.min())
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
