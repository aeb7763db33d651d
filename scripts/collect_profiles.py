"""Copy a round's GPU profile outputs into profiles/<tag>/ and derive the
contraction figures the north star asks for (fp64 MFMA utilisation and
achieved HBM GB/s of contract2_kernel on C2 / C4).

    python scripts/collect_profiles.py <tag>
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def per_dispatch(tag, name, counter):
    f = os.path.join(OUT, f"pmc_{tag}_{name}", "run_counter_collection.csv")
    rows = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        key = r["Dispatch_Id"]
        d = rows.setdefault(key, {"kernel": r["Kernel_Name"], "v": 0.0, "grid": int(r["Grid_Size"]),
                                  "ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
        d["v"] += float(r["Counter_Value"])
    return rows


def main():
    tag = sys.argv[1]
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    for src, name in ((f"prof_{tag}/run_kernel_stats.csv", "kernel_stats_bench.csv"),
                      (f"prof_{tag}/run_domain_stats.csv", "domain_stats_bench.csv"),
                      (f"profcfg_{tag}/run_kernel_stats.csv", "kernel_stats_configs.csv"),
                      (f"bench_{tag}.log", "bench.log"), (f"configs_{tag}.log", "configs.log"),
                      (f"profc5_{tag}/run_kernel_stats.csv", "kernel_stats_c5_b512.csv"),
                      (f"c5prof_{tag}.log", "c5_ab.log"), (f"kernel_sources_sha_{tag}.txt", "kernel_sources_sha.txt")):
        p = os.path.join(OUT, src)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, name))
    # contraction: MFMA busy fraction and HBM bytes per dispatch
    res = {}
    busy = per_dispatch(tag, "csq", "SQ_VALU_MFMA_BUSY_CYCLES")
    gui = per_dispatch(tag, "csq", "GRBM_GUI_ACTIVE")
    fetch = per_dispatch(tag, "cfetch", "FETCH_SIZE")
    write = per_dispatch(tag, "cwrite", "WRITE_SIZE")
    for src, agg in ((busy, "busy"), (gui, "gui")):
        for k, d in src.items():
            if "contract2" not in d["kernel"]:
                continue
            kn = d["kernel"].split("contract2_kernel")[1].split("(")[0]
            e = res.setdefault(kn, {"busy": [], "gui": [], "bytes": [], "ns": []})
            e[agg].append(d["v"])
    for src in (fetch, write):
        pass
    for k, d in fetch.items():
        if "contract2" in d["kernel"]:
            kn = d["kernel"].split("contract2_kernel")[1].split("(")[0]
            w = next((x["v"] for kk, x in write.items() if x["kernel"] == d["kernel"]), 0.0)
            res[kn]["bytes"].append((2 * d["v"] + w) * 1024)
            res[kn]["ns"].append(d["ns"])
    summary = {}
    for kn, e in res.items():
        n = min(len(e["busy"]), len(e["gui"]))
        util = sum(e["busy"][i] / 1024.0 / (e["gui"][i] / 8.0) for i in range(n)) / max(n, 1)
        gbs = [b / ns for b, ns in zip(e["bytes"], e["ns"])] if e["ns"] else []
        summary[f"contract2_kernel{kn}"] = {
            "mfma_busy_fraction": util,
            "rule_mfma": "SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs), mean over dispatches",
            "hbm_bytes_per_dispatch_mean": sum(e["bytes"]) / max(len(e["bytes"]), 1),
            "hbm_GBps_mean": sum(gbs) / max(len(gbs), 1),
            "rule_hbm": "(2*FETCH_SIZE + WRITE_SIZE) KiB per dispatch / the profiled dispatch's duration",
            "dispatches": n}
    with open(os.path.join(dst, "contraction_pmc.json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
