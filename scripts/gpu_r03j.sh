# latency kernel + C5 right-looking first (short limit), then the GPU suite,
# then the round-3 baseline profile (probe, stamps, PMC, rocprof), the bench
# and the C5 one-proposal timing
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_properties.py -x -v -s -m gpu -k "latency or graph or right_looking" --timeout 250 --timeout-method thread > gpurun_out/pytest_lat.log 2>&1; rc=$?; echo lat rc=$rc; grep -E "latency vs|PASS|FAIL|Error" gpurun_out/pytest_lat.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c5 --partition pulsars --steps 20 --warmup 3 > gpurun_out/bench_c5_b1.log 2>&1; rc=$?; echo c5b1 rc=$rc; tail -c 700 gpurun_out/bench_c5_b1.log
if crash $rc; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20; tail -2 gpurun_out/pytest_gpu.log
if crash $rc; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1; echo bench rc=$?; tail -c 1200 gpurun_out/bench.log
bash scripts/gpu_r03i.sh
