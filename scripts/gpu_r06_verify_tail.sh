# the verify route's tail at strict/16 (product) and
# strict/64 on the system model's bench seed and three fresh seeds (dev
# library for EWARP_VERIFY_FRAC), then the wide / C4 parity tests on the
# product library.  Outputs under gpurun_out/r06h.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/r06h; export TMPDIR=/tmp
DEV=enterprise_warp_amd/libewarp_hip_dev.so
for F in 0.0625 0.015625; do
  EWARP_HIP_LIB=$DEV EWARP_VERIFY_FRAC=$F timeout -k 10 400 python -u scripts/verify_tail.py --offsets 0,1000,2000,3000 > gpurun_out/r06h/verify_tail_$F.log 2>&1 || exit $?
  cat gpurun_out/r06h/verify_tail_$F.log | grep -v amdgpu
done
timeout -k 10 600 python -u -m pytest -v -rP --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "verify_route or wide_prior or system_noise or c4_bench or headline" > gpurun_out/r06h/pytest.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/r06h/pytest.log
