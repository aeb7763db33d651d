# Round-5 GPU pass on the current tree: the GPU suite, smoke, the bench
# (with the wide-basis secondary), the 2-rank launcher rehearsal on one card
# (gloo, same device, --verify) and rocprof kernel stats of the wide block.
# Outputs tagged TAG under gpurun_out/.  Stops at the first crash-class exit.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05a}
STEPS=${2:-all}
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
has() { case ",$STEPS," in *",all,"*|*",$1,"*) return 0;; *) return 1;; esac; }
if has pytest; then
  step pytest_gpu 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread
  grep -E "FAILED|ERROR" "gpurun_out/pytest_gpu_$TAG.log" | head -20
fi
has smoke && step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
has bench && step bench 700 python bench.py --steps 20 --warmup 3
has launch2 && step launch2 300 python bench.py --gpus 2 --dist-backend gloo --same-device --verify --steps 5 --warmup 2 --no-cpu-baseline --no-latency --no-secondary
has benchsec && step benchsec 500 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-latency --no-c5 --no-wide
has wideonly && step wideonly 400 python bench.py --only-wide
has wideprof && step wideprof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profwide_$TAG -o run --output-format csv -- python bench.py --only-wide
echo ROUND_DONE
