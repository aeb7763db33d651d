"""Reduce rocprofv3 --pmc passes to per-kernel means and the HBM traffic of
the dominant kernel (CPU only; reads gpurun_out/pmc_<tag>_*).

    python scripts/pmc_summary.py <tag> [--kernel chol_mfma_kernel] [--units N]

Writes profiles/<tag>/pmc_summary.json (every kernel, every counter: mean per
dispatch, dispatch count) and profiles/pmc_chol.json, which bench.py reads for
`roofline.traffic` (with the kernel-source sha the profiling run recorded in
gpurun_out/pmc_<tag>_sha.txt).  HBM bytes per launch follow MI355X_MICROARCH.md § HBM:
FETCH_SIZE and WRITE_SIZE are in KiB, and on gfx950 FETCH_SIZE reports half
the bytes of wide coalesced reads, so bytes = (2 * FETCH_SIZE + WRITE_SIZE)
* 1024.  The SQ counters are per dispatch totals over all waves.
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    """'void (anonymous namespace)::k<8, 0>(args)' -> 'k<8, 0>'."""
    n = name.replace("(anonymous namespace)::", "").replace("void ", "", 1)
    return n.split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="chol_mfma_kernel<8, 2, 25, false, 0,")   # (the headline; not the C5 KEEP form)
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    args = ap.parse_args()
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    order = []
    grid = {}
    for d in sorted(glob.glob(os.path.join(args.src, f"pmc_{args.tag}_*"))):
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if k not in per:
                order.append(k)
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            grid[k] = {"grid": int(r["Grid_Size"]), "block": int(r["Workgroup_Size"]),
                       "vgpr": int(r["VGPR_Count"]), "agpr": int(r["Accum_VGPR_Count"]),
                       "lds": int(r["LDS_Block_Size"]), "scratch": int(r["Scratch_Size"])}
    if not per:
        raise SystemExit(f"no pmc_{args.tag}_* counter files under {args.src}")
    summary = {}
    for k in order:
        c = {n: {"mean": sum(v) / len(v), "dispatches": len(v)} for n, v in per[k].items()}
        summary[short(k)] = {"name": k, "launch": grid[k], "counters": c}
    out_dir = os.path.join(ROOT, "profiles", args.tag)
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "pmc_summary.json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    hits = [k for k in order if args.kernel in k and "FETCH_SIZE" in per[k] and "WRITE_SIZE" in per[k]]
    if not hits:
        raise SystemExit(f"no kernel matching {args.kernel!r} with FETCH_SIZE and WRITE_SIZE")
    k = hits[0]
    fetch = summary[short(k)]["counters"]["FETCH_SIZE"]["mean"]
    write = summary[short(k)]["counters"]["WRITE_SIZE"]["mean"]
    rec = {"tag": args.tag, "kernel": k, "fetch_kib": fetch, "write_kib": write,
           "hbm_bytes_per_launch": (2.0 * fetch + write) * 1024.0,
           "rule": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md, HBM section)"}
    sq = summary[short(k)]["counters"]
    if "SQ_WAVES" in sq:
        waves = sq["SQ_WAVES"]["mean"]
        rec["per_wave"] = {n: sq[n]["mean"] / waves for n in sq if n.startswith("SQ_") and n != "SQ_WAVES"}
    # the sha of the PROFILED kernel sources, recorded on the GPU box by the
    # profiling script (gpurun_out/pmc_<tag>_sha.txt); bench.py uses the
    # traffic only while its own tree has the same sha
    shaf = os.path.join(args.src, f"pmc_{args.tag}_sha.txt")
    if not os.path.exists(shaf):
        raise SystemExit(f"{shaf} missing: the profiling run must record bench.kernel_sources_sha()")
    with open(shaf) as fh:
        rec["kernel_sources_sha"] = fh.read().split()[-1]
    with open(os.path.join(ROOT, "profiles", "pmc_chol.json"), "w") as fh:
        json.dump(rec, fh, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
