#!/bin/bash
# PMC passes on the C5 bench (one step): MFMA busy + fetch / write bytes per kernel
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r02}
crash() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
pass() {
  local name=$1; shift
  echo "== pmc $name: $*"
  timeout -k 10 600 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/pmcc5_${TAG}_$name -o run --output-format csv -- python bench.py --config c5 --steps 1 --warmup 0 > gpurun_out/pmcc5_${TAG}_$name.log 2>&1
  local rc=$?
  echo "== pmc $name rc=$rc"
  if crash $rc; then echo "crash-class exit $rc: stopping"; exit $rc; fi
}
pass sq SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES
pass fetch FETCH_SIZE
pass write WRITE_SIZE
python3 scripts/pmc_table.py gpurun_out/pmcc5_${TAG}_sq gpurun_out/pmcc5_${TAG}_fetch gpurun_out/pmcc5_${TAG}_write 2>&1 | tail -30
