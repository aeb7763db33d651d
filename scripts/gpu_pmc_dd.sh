# PMC passes (one counter group per run) on the double-double factorisation
# (kernel mode 29, every unit in double-double) of the system model and the
# 372-column pulsar; the wide fp64 kernel (mode 27) in the same runs.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-pmcdd}
W="scripts/wide_ab.py --cases system,w372_fixed --modes 29,27 --kinds prior --rounds 1"
pass() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/${TAG}_$name -o run --output-format csv -- python $W > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAIT_ANY GRBM_GUI_ACTIVE
pass sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
echo PMC_DONE
