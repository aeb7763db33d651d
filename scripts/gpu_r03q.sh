# latency kernel A/B: 0 = annealed block map + theta-first prologue,
# 24 = annealed map only, 25 = round-3 kernel; stamps of the new default;
# then the latency parity tests on the product library
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
EWARP_HIP_LIB=$PWD/enterprise_warp_amd/libewarp_hip_dev.so timeout -k 10 300 python scripts/latency_sweep.py --reps 600 --rounds 6 --batches 1,4,8 --modes 25,24,0 > gpurun_out/lat_ab.log 2>&1; rc=$?; echo sweep rc=$rc; grep -v amdgpu gpurun_out/lat_ab.log | python -c "import json,sys; d=json.load(sys.stdin); [print(k, round(v['us_median'],2), round(v['us_p10'],2), v['max_abs_diff_vs_first_mode']) for k,v in d.items()]"
if crash $rc; then exit $rc; fi
timeout -k 10 200 python scripts/lat_stamps.py --B 1 > gpurun_out/lat_stamps_b1.log 2>&1; rc=$?; echo stamps rc=$rc; grep -v amdgpu gpurun_out/lat_stamps_b1.log | head -30
if crash $rc; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "latency or graph or single or golden" --timeout 300 --timeout-method thread > gpurun_out/pytest_lat.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "FAILED|ERROR" gpurun_out/pytest_lat.log | head; tail -1 gpurun_out/pytest_lat.log
