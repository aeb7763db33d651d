set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/accuracy_goldens.py > gpurun_out/acc.log 2>&1; rc=$?; echo acc rc=$rc; tail -14 gpurun_out/acc.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; tail -5 gpurun_out/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1; echo bench rc=$?; tail -c 1500 gpurun_out/bench.log
