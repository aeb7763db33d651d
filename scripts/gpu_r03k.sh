# compact theta staging: parity subset, latency sweep (+ kernel trace), bench,
# PMC (SQ + HBM) of the C3 kernel, rocprof of the C5 step kernels
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu -k "latency or golden or bench_workload or mfma_vs_lds or units_sum" --timeout 300 --timeout-method thread > gpurun_out/pytest_sub.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "FAILED|ERROR" gpurun_out/pytest_sub.log | head; tail -2 gpurun_out/pytest_sub.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/latency_sweep.py > gpurun_out/latency.log 2>&1; rc=$?; echo lat rc=$rc; cat gpurun_out/latency.log | grep -v amdgpu.ids | python -c "import json,sys; d=json.load(sys.stdin); [print(k, round(v['us_median'],1)) for k,v in d.items()]"
if crash $rc; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lat -o run --output-format csv -- python scripts/latency_sweep.py --reps 100 --batches 1,16 > gpurun_out/latency_prof.log 2>&1; rc=$?; echo latprof rc=$rc
if crash $rc; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1; rc=$?; echo bench rc=$rc; tail -c 400 gpurun_out/bench.log
if crash $rc; then exit $rc; fi
CH="scripts/chol_ab.py --rounds 1 --modes 0"
pmc() { local name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/pmc_r03k_$name -o run --output-format csv -- python $CH > gpurun_out/pmc_r03k_$name.log 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; if crash $rc; then exit $rc; fi; }
pmc sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU
pmc sq2 SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
pmc tc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum
pmc fetch FETCH_SIZE
pmc write WRITE_SIZE
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03k -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-latency --no-secondary > gpurun_out/bench_prof.log 2>&1; rc=$?; echo rocprof rc=$rc
if crash $rc; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/bench_c5.log 2>&1; rc=$?; echo c5 rc=$rc; tail -c 300 gpurun_out/bench_c5.log
if crash $rc; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5b1 -o run --output-format csv -- python bench.py --config c5 --partition pulsars --steps 20 --warmup 3 > gpurun_out/bench_c5_b1.log 2>&1; rc=$?; echo c5b1 rc=$rc; tail -c 300 gpurun_out/bench_c5_b1.log
