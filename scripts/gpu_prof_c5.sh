#!/bin/bash
# rocprofv3 kernel trace of the C5 bench (B=512) and of the single-proposal path
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r02}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_$TAG -o run --output-format csv -- python bench.py --config c5 --steps 2 --warmup 1 > gpurun_out/prof_c5.log 2>&1; echo rc=$?
f=$(find gpurun_out/prof_c5_$TAG -name "*kernel_stats.csv" | head -1); echo $f; head -20 "$f" | cut -c1-220
