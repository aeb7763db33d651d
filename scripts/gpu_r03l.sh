# latency-kernel phase stamps + co-issue probe (MFMA padding)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 200 python scripts/lat_stamps.py --B 1 > gpurun_out/lat_stamps_b1.log 2>&1; rc=$?; echo st1 rc=$rc; grep -v amdgpu gpurun_out/lat_stamps_b1.log
if crash $rc; then exit $rc; fi
timeout -k 10 200 python scripts/lat_stamps.py --B 16 > gpurun_out/lat_stamps_b16.log 2>&1; rc=$?; echo st16 rc=$rc; grep -v amdgpu gpurun_out/lat_stamps_b16.log | head -30
if crash $rc; then exit $rc; fi
timeout -k 10 120 ./build/fp64_issue_probe > gpurun_out/probe2.log 2>&1; rc=$?; echo probe rc=$rc; grep -E "pad|own fma" gpurun_out/probe2.log
