# PMC passes on the C2 / C4 contraction (contract2_kernel, prior draws):
# issue mix, LDS waits and bank conflicts, barrier waits.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-pmcc2}
W="scripts/wide_ab.py --cases c2,c4 --modes 0 --kinds prior --contract --rounds 1"
pass() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/${TAG}_$name -o run --output-format csv -- python $W > gpurun_out/${TAG}_$name.log 2>&1
  local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAIT_ANY GRBM_GUI_ACTIVE
pass sq2 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
echo PMC_DONE
