#!/bin/bash
# fp64 issue probe, C3 Cholesky phase stamps (mode 21), A/B of the chol modes.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
MODES=${1:-0,17,20}
timeout -k 10 120 ./build/probes/fp64_issue_probe > gpurun_out/issue_probe3.log 2>&1; rc=$?; echo "probe rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python scripts/chol_stamps.py > gpurun_out/chol_stamps.log 2>&1; rc=$?; echo "stamps rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python scripts/chol_ab.py --rounds 7 --modes $MODES > gpurun_out/chol_ab.log 2>&1; rc=$?; echo "chol_ab rc=$rc"
exit $rc
