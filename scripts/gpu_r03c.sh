set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/accuracy_goldens.py > gpurun_out/acc.log 2>&1; rc=$?; echo acc rc=$rc; tail -14 gpurun_out/acc.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python scripts/chol_ab.py --rounds 7 --modes 0,17 > gpurun_out/chol_ab.log 2>&1; rc=$?; echo ab rc=$rc; grep -A1 "mode\|median" gpurun_out/chol_ab.log | grep -E "mode|median" | paste - - | head
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 1100 python -u -m pytest tests -v -m gpu --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | grep -v PASSED | head -20; tail -3 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1; echo bench rc=$?; tail -c 600 gpurun_out/bench.log
