"""Table of a scripts/wide_ab.py log: case/kind/mode, median ms, refined share,
largest difference from the first mode (strict units).

    python scripts/ab_table.py gpurun_out/<tag>_ab.log
"""
import json
import re
import sys

t = open(sys.argv[1]).read()
for blk in re.findall(r"^\{.*?^\}", t, re.S | re.M):
    for k, v in json.loads(blk).items():
        sh = v["refined_share"]
        print(f"{k:28s} {v['median_ms']:9.3f} ms  share {'-' if sh is None else f'{sh:.3f}':>6s}  "
              f"diff {v['max_diff_over_strict_vs_first']:.3g}")
