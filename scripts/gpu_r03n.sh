# full GPU suite, smoke, bench on the round-3 tree
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20; tail -2 gpurun_out/pytest_gpu.log
if crash $rc; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo smoke rc=$rc; tail -1 gpurun_out/smoke.log
if crash $rc; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1; echo bench rc=$?; tail -c 1500 gpurun_out/bench.log
