# theta staging: the probe (can the host store to fine-grained device
# memory; read latency and call round trip per kind), then, if it can, the
# latency path with theta there (dev mode 27) vs pinned host memory (0)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 ./build/theta_stage_probe > gpurun_out/theta_stage_probe.log 2>&1; rc=$?; echo probe rc=$rc; cat gpurun_out/theta_stage_probe.log
if [ $rc -ne 0 ]; then exit $rc; fi
if grep -q "device_finegrained: call" gpurun_out/theta_stage_probe.log; then
  export EWARP_HIP_LIB=$PWD/enterprise_warp_amd/libewarp_hip_dev.so
  timeout -k 10 240 python scripts/lat_variant_check.py --mode 27 > gpurun_out/lat_check27.log 2>&1; rc=$?; echo check rc=$rc; grep -v amdgpu gpurun_out/lat_check27.log | tr -d '\n '; echo
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -k 10 300 python scripts/latency_sweep.py --reps 600 --rounds 6 --batches 1,4,8 --modes 0,27 > gpurun_out/lat_ab27.log 2>&1; rc=$?; echo sweep rc=$rc; grep -v amdgpu gpurun_out/lat_ab27.log | python -c "import json,sys; d=json.load(sys.stdin); [print(k, round(v['us_median'],2), round(v['us_p10'],2), v['max_abs_diff_vs_first_mode']) for k,v in d.items()]"
fi
exit $rc
