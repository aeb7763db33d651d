#!/bin/bash
# One GPU session: smoke, GPU tests, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash-class exit (abort, segfault,
# timeout, kill) stops the script before anything else touches the GPU.
# Test failures (pytest exit 1) do not stop the bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
crash() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # run <name> <seconds> cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if crash $rc; then echo "crash-class exit $rc in $name: stopping"; exit $rc; fi
  return 0
}
run lane_ops 120 bash -c "hipcc --offload-arch=gfx950 -O2 -o /tmp/lane_ops_test tests/hip/lane_ops_test.hip && /tmp/lane_ops_test"
run smoke 400 python __graft_entry__.py smoke
run pytest_gpu 900 python -m pytest tests -q -m gpu -x
run bench 600 python bench.py --steps 10 --warmup 2
run chol_ab 600 python scripts/chol_ab.py --rounds 5 --modes 0,3,2
run configs 900 python scripts/bench_configs.py
run pmc 1500 bash scripts/gpu_pmc.sh $TAG
run rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline
echo ALL_DONE
