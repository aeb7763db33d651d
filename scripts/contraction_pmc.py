"""Contraction PMC summary of a round profile (scripts/gpu_profile_round.sh TAG):
fp64 MFMA-busy fraction and HBM read rate of contract2_kernel on C2 / C4 from
gpurun_out/cpmc_<TAG>_{busy,fetch,write}, written to
profiles/<TAG>/contraction_pmc.json.

    python scripts/contraction_pmc.py <tag>
"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def dispatches(tag, name):
    rows = defaultdict(lambda: {"c": defaultdict(float)})
    for r in csv.DictReader(open(os.path.join(OUT, f"cpmc_{tag}_{name}", "run_counter_collection.csv"))):
        d = rows[r["Dispatch_Id"]]
        d["kernel"] = r["Kernel_Name"]
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d["c"][r["Counter_Name"]] += float(r["Counter_Value"])
    return rows


def short(k):
    i = k.find("contract2_kernel<")
    return k[i:k.index(">", i) + 1] if i >= 0 else k


def main():
    tag = sys.argv[1]
    busy, fetch, write = (dispatches(tag, n) for n in ("busy", "fetch", "write"))
    out = {}
    for kname in sorted({short(d["kernel"]) for d in busy.values()}):
        b = [d for d in busy.values() if short(d["kernel"]) == kname]
        f = [d for d in fetch.values() if short(d["kernel"]) == kname]
        w = [d for d in write.values() if short(d["kernel"]) == kname]
        frac = [d["c"]["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (d["c"]["GRBM_GUI_ACTIVE"] / 8) for d in b]
        rb = [2 * d["c"]["FETCH_SIZE"] * 1024 for d in f]
        out[kname] = {
            "mfma_busy_fraction": sum(frac) / len(frac),
            "dispatches": len(b),
            "rule_mfma": "SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs), mean over dispatches",
            "hbm_read_bytes_per_dispatch_mean": sum(rb) / len(rb),
            "hbm_read_GBps_mean": sum(x / (d["ns"] * 1e-9) / 1e9 for x, d in zip(rb, f)) / len(f),
            "hbm_write_bytes_per_dispatch_mean": sum(d["c"]["WRITE_SIZE"] * 1024 for d in w) / max(len(w), 1),
            "rule_hbm": "2 * FETCH_SIZE KiB per dispatch (gfx950 correction) / the profiled dispatch's duration",
            "mfma_insts_per_wave": sum(d["c"]["SQ_INSTS_MFMA"] / d["c"]["SQ_WAVES"] for d in b) / len(b),
        }
    os.makedirs(os.path.join(ROOT, "profiles", tag), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", tag, "contraction_pmc.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
