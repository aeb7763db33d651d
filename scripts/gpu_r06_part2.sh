# round-6 checks, part 2: dev A/B suite, device debug build, 2-rank
# launcher rehearsals (verify on by default).  Stops at a crash-class exit.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/${TAG:-r06g}; export TMPDIR=/tmp
step() {
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/${TAG:-r06g}/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 "gpurun_out/${TAG:-r06g}/$name.log"
  case $rc in 0|1) ;; *) echo "crash-class exit $rc in $name"; exit $rc;; esac
}
step pytest_gpu_ab 700 python -u -m pytest tests -v -m gpu_ab --timeout 600 --timeout-method thread
step pytest_gpu_debug 700 python -u -m pytest tests -v -rP -m gpu_debug --timeout 650 --timeout-method thread
step launch2 300 python bench.py --gpus 2 --dist-backend gloo --same-device --steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-secondary
step launch2s 300 python bench.py --gpus 2 --dist-backend gloo --same-device --c3-partition samples --steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-secondary
echo PART2_DONE
