#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -v -s -m gpu --timeout 600 --timeout-method thread -k "c5 or correlated or golden or multi_context" > gpurun_out/pytest_c5.log 2>&1; rc=$?
echo pytest rc=$rc; grep -E "passed|failed|FAILED|^E  |c5.*max err" gpurun_out/pytest_c5.log | tail -30
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python bench.py --config c5 --partition pulsars --steps 20 --warmup 3 > gpurun_out/bench_c5p.log 2>&1; echo c5p rc=$?; tail -1 gpurun_out/bench_c5p.log | cut -c1-400
timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/bench_c5.log 2>&1; echo c5 rc=$?; tail -1 gpurun_out/bench_c5.log | cut -c1-300
