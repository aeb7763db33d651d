#!/bin/bash
# GPU tests, C3 Cholesky A/B, per-config timings (C2/C3/C4), bench line.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
MODES=${1:-0,9}
step() { local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc"; grep -v "amdgpu.ids" "gpurun_out/$name.log" | tail -3 | cut -c1-300
  case $rc in 0|1|5) ;; *) echo "stopping after $name"; exit $rc;; esac; }
step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step chol_ab 400 python scripts/chol_ab.py --rounds 5 --modes $MODES
step configs 400 python scripts/bench_configs.py --configs c2,c3,c4 --reps 3 --check 2
step bench 400 python bench.py --steps 20 --warmup 3 --cpu-seconds 10
