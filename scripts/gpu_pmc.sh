#!/bin/bash
# PMC counter passes (one counter group per run, --kernel-trace only) on the
# C3 likelihood kernel; outputs under gpurun_out/pmc_<tag>_*.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
ARGS=${2:---rounds 2 --modes 0,3}
crash() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
pass() {  # pass <name> counters...
  local name=$1; shift
  echo "== pmc $name: $*"
  timeout -k 10 600 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/pmc_${TAG}_$name -o run --output-format csv -- python scripts/chol_ab.py $ARGS > gpurun_out/pmc_${TAG}_$name.log 2>&1
  local rc=$?
  echo "== pmc $name rc=$rc"; tail -3 gpurun_out/pmc_${TAG}_$name.log
  if crash $rc; then echo "crash-class exit $rc: stopping"; exit $rc; fi
}
pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_IFETCH
pass sq2 SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
echo PMC_DONE
