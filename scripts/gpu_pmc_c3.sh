# PMC passes on the C3 likelihood kernel only (the chol_ab part of
# gpu_final.sh), with the kernel-source sha recorded for bench.py's
# roofline.traffic.  Needs libewarp_hip_dev.so (make -C enterprise_warp_amd/csrc dev).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03i}
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
python -c "import bench; print(bench.kernel_sources_sha())" > gpurun_out/pmc_${TAG}_sha.txt
CH="scripts/chol_ab.py --rounds 1 --modes 0"
pmc() { local name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/pmc_${TAG}_$name -o run --output-format csv -- python $CH > gpurun_out/pmc_${TAG}_$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; if crash $rc; then exit $rc; fi; }
pmc sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU
pmc sq2 SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
pmc tc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum
pmc fetch FETCH_SIZE
pmc write WRITE_SIZE
echo PMC_DONE
