#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
crash() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
pass() {
  local name=$1; shift
  timeout -k 10 600 rocprofv3 --pmc "$@" --kernel-include-regex "dchol_rowupdate" --kernel-trace -d gpurun_out/pmcru_$name -o run --output-format csv -- python bench.py --config c5 --steps 1 --warmup 0 > gpurun_out/pmcru_$name.log 2>&1
  local rc=$?; echo "== $name rc=$rc"
  if crash $rc; then exit $rc; fi
}
pass a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU
pass b SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
python3 scripts/pmc_table.py gpurun_out/pmcru_a gpurun_out/pmcru_b
