# latency kernel, dataflow default (0) vs barrier form (24) vs round-3 (25):
# parity of the default against the batched path (dev lib), interleaved
# latency A/B, stamps of the default, then the product-library latency tests
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
DEV=$PWD/enterprise_warp_amd/libewarp_hip_dev.so
EWARP_HIP_LIB=$DEV timeout -k 10 240 python scripts/lat_variant_check.py --mode 0 > gpurun_out/lat_check0.log 2>&1; rc=$?; echo check rc=$rc; grep -v amdgpu gpurun_out/lat_check0.log | tr -d '\n '; echo
if [ $rc -ne 0 ]; then exit $rc; fi
EWARP_HIP_LIB=$DEV timeout -k 10 300 python scripts/latency_sweep.py --reps 600 --rounds 6 --batches 1,4,8 --modes 26,0 > gpurun_out/lat_ab3.log 2>&1; rc=$?; echo sweep rc=$rc; grep -v amdgpu gpurun_out/lat_ab3.log | python -c "import json,sys; d=json.load(sys.stdin); [print(k, round(v['us_median'],2), round(v['us_p10'],2), v['max_abs_diff_vs_first_mode']) for k,v in d.items()]"
if crash $rc; then exit $rc; fi
timeout -k 10 200 python scripts/lat_stamps.py --B 1 > gpurun_out/lat_stamps_b1.log 2>&1; rc=$?; echo stamps rc=$rc; grep -v amdgpu gpurun_out/lat_stamps_b1.log | tr -d '\n' | cut -c1-900; echo
if crash $rc; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "latency or graph or single or golden" --timeout 300 --timeout-method thread > gpurun_out/pytest_lat.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "FAILED|ERROR" gpurun_out/pytest_lat.log | head; tail -1 gpurun_out/pytest_lat.log
