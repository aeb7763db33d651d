# One PMC pass on the C4 contraction (contract2_kernel<13, 8, BLOCKED, RSEP>):
# flat reads returning to registers vs to LDS (TA), VMEM instruction counts --
# the register-returning reads beyond wave 0's per-tile weight loads are the
# spill reloads.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc TA_FLAT_READ_WAVEFRONTS_sum TA_FLAT_READ_LDS_WAVEFRONTS_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_c4scr -o run --output-format csv -- python scripts/wide_ab.py --cases c4 --modes 0 --kinds prior --contract --rounds 1 > gpurun_out/pmc_c4scr.log 2>&1
echo rc=$?
