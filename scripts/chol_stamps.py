"""Phase timing of the C3 Cholesky kernel from in-kernel s_memtime stamps
(dev library, kernel mode 21 = the default two-level panel with stamps at
every panel / trailing-update boundary of the first 4096 units; phase split
H = 3 block rows for NB = 8).

    python scripts/chol_stamps.py [--B 4096]

Prints the mean cycles per phase and, for units that shared a SIMD (same
XCC / SE / CU / SIMD in HW_ID) and overlapped in time, how much of one
unit's panel time overlapped the other's panels.
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

UNITS, NST = 4096, 24


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--mode", type=int, default=21)
    ap.add_argument("--H", type=int, default=3)
    args = ap.parse_args()
    import torch
    from enterprise_warp_amd import _lib, synth
    cfg = synth.config_c3()
    pta = cfg.pta
    X = synth.prior_draws(pta, args.B, cfg.theta_seed)
    eng = pta.engine(0)
    U = len(pta.signal_collections) * args.B
    out = torch.zeros(args.B, dtype=torch.float64, device="cuda")
    th = torch.from_numpy(X).cuda()
    lib = C.CDLL(_lib.LIB_PATH)
    lib.ewh_dev_stamps.argtypes = [C.POINTER(C.c_longlong), C.c_longlong]
    res = {}
    for mode in (0, args.mode):
        eng.set_kernel_mode(mode)
        for _ in range(3):
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            eng.lnl_units_device(th.data_ptr(), args.B, 0, U, out.data_ptr(), 0)
            e.record()
            torch.cuda.synchronize()
        res[f"mode{mode}_ms"] = s.elapsed_time(e)
    eng.set_kernel_mode(0)
    buf = (C.c_longlong * (UNITS * NST))()
    assert lib.ewh_dev_stamps(buf, UNITS * NST) == 0
    st = np.frombuffer(buf, dtype=np.int64).reshape(UNITS, NST)
    nb = 8
    nstamp = 4 + 2 * nb
    t = st[:, :nstamp].astype(np.float64)
    d = np.diff(t, axis=1)
    names = ["phi prologue"]
    for bb in range(args.H):
        names += [f"panel {bb}", f"trailing {bb}"]
    names += ["phase-2 A22 update"]
    for bb in range(args.H, nb):
        names += [f"panel {bb}", f"trailing {bb}"]
    names += ["epilogue"]
    names = names[: d.shape[1]]
    valid = t[:, 0] > 0
    dm = d[valid].mean(axis=0)
    res["phase_cycles_mean"] = {n: float(v) for n, v in zip(names, dm)}
    res["unit_cycles_mean"] = float((t[valid, -1] - t[valid, 0]).mean())
    panel_idx = [i for i, n in enumerate(names) if n.startswith("panel")]
    res["panel_cycles_total"] = float(dm[panel_idx].sum())
    res["trailing_cycles_total"] = float(dm[[i for i, n in enumerate(names) if not n.startswith("panel")]].sum())
    # SIMD sharing: HW_ID fields (gfx9): wave [3:0], simd [5:4], cu [11:8], sh [12], se [15:13]
    hw = st[:, NST - 2]
    xcc = st[:, NST - 1] & 0xf
    simd_key = (xcc << 16) | (hw & 0xFF30) | ((hw >> 13) & 7) << 20
    keys, counts = np.unique(simd_key[valid], return_counts=True)
    res["units_per_simd_key_hist"] = {int(k): int(v) for k, v in zip(*np.unique(counts, return_counts=True))}
    # overlap of panel intervals between the units of one SIMD that ran concurrently
    ov, tot = 0.0, 0.0
    for k in keys[:512]:
        idx = np.flatnonzero(valid & (simd_key == k))
        ivs = []
        for u in idx:
            for i in panel_idx:
                ivs.append((u, t[u, i], t[u, i + 1]))
        for u in idx:
            for i in panel_idx:
                a, b = t[u, i], t[u, i + 1]
                tot += b - a
                for (v, c0, c1) in ivs:
                    if v != u:
                        ov += max(0.0, min(b, c1) - max(a, c0))
    res["panel_time_overlapping_partner_panels_frac"] = ov / tot if tot else None
    starts = t[valid, 0]
    res["start_spread_cycles"] = float(np.percentile(starts - starts.min(), 90))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
