#!/bin/bash
# GPU parity suite (verbose, prints max err/strict per fixture), then a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo pytest rc=$rc; grep -E "passed|failed|max err" gpurun_out/pytest_gpu.log | tail -60
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1; echo bench rc=$?; tail -2 gpurun_out/bench.log
