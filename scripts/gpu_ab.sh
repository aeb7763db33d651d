#!/bin/bash
# GPU tests, C3 Cholesky A/B over kernel modes, bench line.  Each GPU step
# has its own limit; a crash-class exit stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
MODES=${1:-0,8}
step() { local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log"
  case $rc in 0|1|5) ;; *) echo "stopping after $name"; exit $rc;; esac; }
step pytest_gpu 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
step chol_ab 400 python scripts/chol_ab.py --rounds 5 --modes $MODES
step bench 400 python bench.py --steps 20 --warmup 3 --cpu-seconds 10
