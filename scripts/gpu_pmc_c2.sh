#!/bin/bash
# PMC passes over the C2 (varying white noise) contraction kernel.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
crash() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
MODE=${MODE:-0}
pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "contract2" --kernel-trace -d gpurun_out/pmcc2_$name -o run --output-format csv -- python scripts/bench_configs.py --configs c2 --reps 2 --check 0 --mode $MODE > gpurun_out/pmcc2_$name.log 2>&1
  local rc=$?; echo "== $name rc=$rc"
  if crash $rc; then exit $rc; fi
}
pass a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU
pass b SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pass c SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_WAVES TCC_HIT_sum TCC_MISS_sum
python3 scripts/pmc_table.py gpurun_out/pmcc2_a gpurun_out/pmcc2_b gpurun_out/pmcc2_c
