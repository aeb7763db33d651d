# Round profile of the current tree (TAG): GPU suite, smoke, bench (with the
# C2 / C4 / C5 secondaries), rocprof kernel stats of the bench, PMC passes on
# the C3 kernel (with the kernel-source sha recorded here, for bench.py's
# roofline.traffic) and on the C2 / C4 contraction.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03g}
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20; tail -1 gpurun_out/pytest_gpu.log
if crash $rc; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo smoke rc=$rc; tail -1 gpurun_out/smoke.log
if crash $rc; then exit $rc; fi
timeout -k 10 700 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1; rc=$?; echo bench rc=$rc; tail -c 300 gpurun_out/bench.log
if crash $rc; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-latency --no-secondary > gpurun_out/bench_prof.log 2>&1; rc=$?; echo rocprof rc=$rc
if crash $rc; then exit $rc; fi
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
CF="scripts/bench_configs.py --configs c2,c4 --reps 1 --check 0"
cpmc() { local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "contract2" --kernel-trace -d gpurun_out/cpmc_${TAG}_$name -o run --output-format csv -- python $CF > gpurun_out/cpmc_${TAG}_$name.log 2>&1
  local rc=$?; echo "cpmc $name rc=$rc"; if crash $rc; then exit $rc; fi; }
cpmc busy SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_WAVES
cpmc fetch FETCH_SIZE
cpmc write WRITE_SIZE
echo PROFILE_DONE
