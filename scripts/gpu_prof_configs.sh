#!/bin/bash
# Kernel-trace stats (and contraction PMC) for the varying-white-noise configs
# C2 and C4.  Usage: bash scripts/gpu_prof_configs.sh <tag> [configs]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
CFG=${2:-c2,c4}
crash() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # run <name> <seconds> cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  if crash $rc; then echo "crash-class exit $rc in $name: stopping"; exit $rc; fi
  return 0
}
run cfg_$TAG 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cfg_$TAG -o run --output-format csv -- python scripts/bench_configs.py --configs $CFG --reps 2 --check 2
run cfgpmc1_$TAG 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_cfg_${TAG}_sq -o run --output-format csv -- python scripts/bench_configs.py --configs $CFG --reps 1 --check 1
run cfgpmc2_$TAG 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_cfg_${TAG}_fetch -o run --output-format csv -- python scripts/bench_configs.py --configs $CFG --reps 1 --check 1
echo CFG_DONE
