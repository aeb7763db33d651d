"""Per-kernel, per-wave PMC table from rocprofv3 counter_collection.csv files.
    python scripts/pmc_table.py <dir-or-csv>... [--match chol]"""
import collections
import csv
import glob
import os
import sys


def load(paths, match):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    waves = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for p in paths:
        files = glob.glob(os.path.join(p, "*counter_collection.csv")) if os.path.isdir(p) else [p]
        for f in files:
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                if match and match not in k:
                    continue
                k = k.replace("(anonymous namespace)::", "").split("(")[0]
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                key = (f, r["Dispatch_Id"])
                if key not in disp[k]:
                    disp[k].add(key)
                    waves[(k, f)] += int(r["Grid_Size"]) / int(r["Workgroup_Size"]) * (int(r["Workgroup_Size"]) + 63) // 64
    return agg, waves


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    match = None
    if "--match" in sys.argv:
        match = sys.argv[sys.argv.index("--match") + 1]
        args = [a for a in args if a != match]
    agg, waves = load(args, match)
    for k, v in agg.items():
        print(k)
        for c, x in sorted(v.items()):
            # counters were summed over files; divide by waves of the file they came from
            nw = sum(w for (kk, f), w in waves.items() if kk == k and any(True for _ in [0]))
            print(f"   {c:28s} total {x:12.4g}")


if __name__ == "__main__":
    main()
