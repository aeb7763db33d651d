# Final-tree checks on one GPU: the -m gpu suite, the dev A/B
# suite (-m gpu_ab), the device debug build (-m gpu_debug), smoke, and the
# 2-rank launcher rehearsal in both C3 partitions (verify on by default with
# more than one rank: no --verify flag).  Outputs under gpurun_out/ tagged
# TAG; stops at a crash.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r06}
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
step() {  # step <name> <seconds> cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/${name}_$TAG.log"
  if crash $rc; then echo "crash-class exit $rc in $name: stopping"; exit $rc; fi
  return 0
}
step pytest_gpu 900 python -u -m pytest tests -v -rP -m gpu --timeout 300 --timeout-method thread
step pytest_gpu_ab 900 python -u -m pytest tests -v -m gpu_ab --timeout 600 --timeout-method thread
step pytest_gpu_debug 1000 python -u -m pytest tests -v -rP -m gpu_debug --timeout 1000 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step launch2 300 python bench.py --gpus 2 --dist-backend gloo --same-device --steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-secondary
step launch2s 300 python bench.py --gpus 2 --dist-backend gloo --same-device --c3-partition samples --steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-secondary
echo FINAL_DONE
