# round-3 baseline profile of the two-level-panel C3 kernel: co-issue probe,
# phase stamps, PMC (SQ, TCP/TCC, HBM), rocprof stats of the bench, accuracy
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 120 ./build/fp64_issue_probe > gpurun_out/probe.log 2>&1; rc=$?; echo probe rc=$rc; tail -20 gpurun_out/probe.log
if crash $rc; then exit $rc; fi
timeout -k 10 300 python scripts/chol_stamps.py > gpurun_out/stamps.log 2>&1; rc=$?; echo stamps rc=$rc; head -30 gpurun_out/stamps.log
if crash $rc; then exit $rc; fi
CH="scripts/chol_ab.py --rounds 2 --modes 0"
pmc() { local name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/pmc_r03i_$name -o run --output-format csv -- python $CH > gpurun_out/pmc_r03i_$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; if crash $rc; then exit $rc; fi; }
pmc sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU
pmc sq2 SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
pmc tc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum
pmc fetch FETCH_SIZE
pmc write WRITE_SIZE
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03i -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-latency --no-secondary > gpurun_out/bench_prof.log 2>&1; rc=$?; echo rocprof rc=$rc; tail -c 600 gpurun_out/bench_prof.log
if crash $rc; then exit $rc; fi
timeout -k 10 300 python -u scripts/accuracy_goldens.py > gpurun_out/acc.log 2>&1; rc=$?; echo acc rc=$rc; cat gpurun_out/acc.log
