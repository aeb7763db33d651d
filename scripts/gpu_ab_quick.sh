#!/bin/bash
# C3 Cholesky A/B over kernel modes only (dev library), one GPU step.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
MODES=${1:-0,17}
timeout -k 10 400 python scripts/chol_ab.py --rounds 7 --modes $MODES > gpurun_out/chol_ab.log 2>&1; rc=$?
echo "chol_ab rc=$rc"; cat gpurun_out/chol_ab.log | tail -40
exit $rc
