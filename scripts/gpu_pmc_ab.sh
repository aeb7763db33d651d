#!/bin/bash
# PMC passes over the Cholesky A/B script: per-kernel-variant instruction mix.
# Usage: bash scripts/gpu_pmc_ab.sh <tag> <modes>
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ab}
MODES=${2:-0,4,5}
crash() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
pass() {  # pass <name> counters...
  local name=$1; shift
  echo "== pmc $name: $*"
  timeout -k 10 -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/pmc_${TAG}_$name -o run --output-format csv -- python scripts/chol_ab.py --rounds 2 --modes $MODES > gpurun_out/pmc_${TAG}_$name.log 2>&1
  local rc=$?
  echo "== pmc $name rc=$rc"; tail -2 gpurun_out/pmc_${TAG}_$name.log
  if crash $rc; then echo "crash-class exit $rc: stopping"; exit $rc; fi
}
pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU
pass sq2 SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE
echo PMC_DONE
