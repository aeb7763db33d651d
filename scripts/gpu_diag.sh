#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo pytest rc=$rc; grep -E "passed|failed|FAILED|max err|^E  " gpurun_out/pytest_gpu.log | tail -70
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python -u scripts/diag_precision.py c2_small,c4_small 0,1,4,5 > gpurun_out/diag1.log 2>&1; echo diag rc=$?; cat gpurun_out/diag1.log
timeout -k 10 300 python -u scripts/diag_precision.py c3_small,c3_freesp 0,6 > gpurun_out/diag2.log 2>&1; echo diag rc=$?; cat gpurun_out/diag2.log
