#!/bin/bash
# Varying-white-noise path (contract2_kernel): C2 / C4 throughput + parity,
# then a kernel-trace profile of the C2 and C4 batches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "c2 or c4 or chromvary or system" > gpurun_out/c2c4_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/c2c4_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_configs.py --configs c2,c4 --reps 5 > gpurun_out/c2c4_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/c2c4_bench.log | grep config
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2c4 -o run --output-format csv -- \
  python scripts/bench_configs.py --configs c2,c4 --reps 3 --check 0 > gpurun_out/c2c4_prof.log 2>&1
rc=$?; echo "prof rc=$rc"
f=$(ls gpurun_out/prof_c2c4/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -n "$f" ] && head -8 "$f"
exit $rc
