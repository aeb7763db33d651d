set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/diag_fault.py c4_small C2 > gpurun_out/diag.log 2>&1; rc=$?; echo diag rc=$rc; tail -4 gpurun_out/diag.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20; tail -3 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo smoke rc=$rc; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1; echo bench rc=$?; tail -c 3000 gpurun_out/bench.log
