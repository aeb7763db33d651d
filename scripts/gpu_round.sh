#!/bin/bash
# One GPU session: GPU tests (verbose), smoke, bench (with CPU baseline + sampler latency).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -v -s -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo pytest rc=$rc; grep -E "passed|failed|FAILED|^E  " gpurun_out/pytest_gpu.log | tail -30
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; rc=$?; echo smoke rc=$rc; tail -2 gpurun_out/smoke.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; echo bench rc=$?; tail -1 gpurun_out/bench.log
