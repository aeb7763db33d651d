#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -v -s -m "gpu or gpu_ab" --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo pytest rc=$rc; grep -E "passed|failed|FAILED|^E  " gpurun_out/pytest_gpu.log | tail -30
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python bench.py --config c5 --partition pulsars --steps 20 --warmup 3 > gpurun_out/bench_c5p.log 2>&1; echo c5p rc=$?; tail -1 gpurun_out/bench_c5p.log
timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/bench_c5.log 2>&1; echo c5 rc=$?; tail -1 gpurun_out/bench_c5.log
