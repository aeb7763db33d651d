# PMC passes on the wide batch-GEMM contraction (contract_xr_kernel, the
# 372-column 10k-TOA pulsar with white noise sampled, B = 1024).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-pmcxr}
W="scripts/wide_ab.py --cases w372_varwn --modes 0 --kinds prior --contract --rounds 1"
pass() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/${TAG}_$name -o run --output-format csv -- python $W > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAIT_ANY GRBM_GUI_ACTIVE
pass sq2 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum
echo PMC_DONE
