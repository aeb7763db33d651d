# latency kernel (theta first, parallel fold, B <= 8): tests, stamps, sweep
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_properties.py -x -v -s -m gpu -k "latency or graph or fixed_white" --timeout 250 --timeout-method thread > gpurun_out/pytest_lat.log 2>&1; rc=$?; echo lat rc=$rc; grep -E "latency vs|FAIL|Error|passed|failed" gpurun_out/pytest_lat.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/lat_stamps.py --B 1 > gpurun_out/lat_stamps_b1.log 2>&1; rc=$?; echo st1 rc=$rc; grep -v amdgpu gpurun_out/lat_stamps_b1.log | head -20
if crash $rc; then exit $rc; fi
timeout -k 10 300 python scripts/latency_sweep.py --batches 1,2,4,8,16 > gpurun_out/latency.log 2>&1; rc=$?; echo lat rc=$rc; grep -v amdgpu gpurun_out/latency.log | python -c "import json,sys; d=json.load(sys.stdin); [print(k, round(v['us_median'],1)) for k,v in d.items()]"
if crash $rc; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lat -o run --output-format csv -- python scripts/latency_sweep.py --reps 100 --batches 1,8 --modes 0 > gpurun_out/latency_prof.log 2>&1; rc=$?; echo latprof rc=$rc; grep -E "chol_lat|Name" gpurun_out/prof_lat/run_kernel_stats.csv | cut -c1-200
