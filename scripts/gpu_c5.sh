#!/bin/bash
# GPU tests + C5 (HD-correlated) bench under rocprofv3 kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc"; grep -v "amdgpu.ids" "gpurun_out/$name.log" | tail -3 | cut -c1-300
  case $rc in 0|1|5) ;; *) echo "stopping after $name"; exit $rc;; esac; }
step pytest_gpu 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step bench_c5 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python bench.py --config c5 --steps 3 --warmup 1
