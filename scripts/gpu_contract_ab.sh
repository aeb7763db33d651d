#!/bin/bash
# GPU tests + varying-white-noise contraction A/B (mode 0: two samples per
# workgroup, mode 10: one) on C2 / C4.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc"; grep -v "amdgpu.ids" "gpurun_out/$name.log" | tail -4 | cut -c1-400
  case $rc in 0|1|5) ;; *) echo "stopping after $name"; exit $rc;; esac; }
step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step cfg_mode0 300 python scripts/bench_configs.py --configs c2,c4 --reps 3 --check 2 --mode 0
step cfg_mode10 300 python scripts/bench_configs.py --configs c2,c4 --reps 3 --check 2 --mode 10
