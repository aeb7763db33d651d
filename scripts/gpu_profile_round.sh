#!/bin/bash
# Round profile on one GPU: bench line, rocprofv3 kernel stats of the bench,
# PMC passes on the C3 likelihood kernel (chol_ab, default mode) and on the
# varying-white-noise contraction (C2 / C4).  Outputs under gpurun_out/;
# copy the summaries into profiles/<tag>/ afterwards (scripts/collect_profiles.py).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
crash() { case "$1" in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # run <name> <seconds> cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 "gpurun_out/${name}_$TAG.log"
  if crash $rc; then echo "crash-class exit $rc in $name: stopping"; exit $rc; fi
  return 0
}
pmc() {  # pmc <name> <script args> -- counters...
  local name=$1; shift
  local sargs=$1; shift
  run pmc_$name 180 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/pmc_${TAG}_$name -o run --output-format csv -- python $sargs
}
# the PMC passes run scripts/chol_ab.py, which loads the dev library: build
# (or confirm up to date) both libraries first, so a stale or missing dev
# build stops the profile here instead of after the bench
# (SKIP_MAKE=1: use the libraries built in-tree before the upload -- build/obj
# does not travel, so make would rebuild both from scratch on the box)
[ "${SKIP_MAKE:-0}" = 1 ] || run make 600 make -C enterprise_warp_amd/csrc -j16 all dev
test -f enterprise_warp_amd/libewarp_hip_dev.so || { echo "dev library missing: stopping"; exit 1; }
python -c "import bench; print('kernel sources sha', bench.kernel_sources_sha())" > gpurun_out/kernel_sources_sha_$TAG.txt
cp gpurun_out/kernel_sources_sha_$TAG.txt gpurun_out/pmc_${TAG}_sha.txt   # (read by scripts/pmc_summary.py)
run bench 400 python bench.py --steps 20 --warmup 3 --cpu-seconds 10
run rocprof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-latency
run configs 400 rocprofv3 --kernel-trace --stats -d gpurun_out/profcfg_$TAG -o run --output-format csv -- python scripts/bench_configs.py --configs c2,c3,c4 --reps 3 --check 3
CH="scripts/chol_ab.py --rounds 2 --modes 0"
pmc sq1 "$CH" SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU
pmc sq2 "$CH" SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE
pmc fetch "$CH" FETCH_SIZE
pmc write "$CH" WRITE_SIZE
CF="scripts/bench_configs.py --configs c2,c4 --reps 1 --check 1"
pmc csq "$CF" SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pmc cfetch "$CF" FETCH_SIZE
pmc cwrite "$CF" WRITE_SIZE
# C5 (HD, 100 psr x 20k TOAs, B = 512): kernel stats and the pair kernel's counters
run c5prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profc5_$TAG -o run --output-format csv -- python scripts/c5_ab.py --modes 0 --rounds 2
C5="scripts/c5_ab.py --modes 0 --rounds 1"
pmc c5sq "$C5" SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
pmc c5fetch "$C5" FETCH_SIZE
pmc c5write "$C5" WRITE_SIZE
echo PROFILE_DONE
