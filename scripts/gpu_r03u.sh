# latency kernel: waits spinning without s_sleep (26) vs the default (0)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
export EWARP_HIP_LIB=$PWD/enterprise_warp_amd/libewarp_hip_dev.so
timeout -k 10 240 python scripts/lat_variant_check.py --mode 26 > gpurun_out/lat_check26.log 2>&1; rc=$?; echo check rc=$rc; grep -v amdgpu gpurun_out/lat_check26.log | tr -d '\n '; echo
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python scripts/latency_sweep.py --reps 600 --rounds 6 --batches 1,4,8 --modes 0,26 > gpurun_out/lat_ab26.log 2>&1; rc=$?; echo sweep rc=$rc; grep -v amdgpu gpurun_out/lat_ab26.log | python -c "import json,sys; d=json.load(sys.stdin); [print(k, round(v['us_median'],2), round(v['us_p10'],2), v['max_abs_diff_vs_first_mode']) for k,v in d.items()]"
exit $rc
