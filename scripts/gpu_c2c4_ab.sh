#!/bin/bash
# A/B of the pipelined contraction: 4 vs 8 waves per sample (dev library
# modes 15 / 16) on C2 and C4, then the product default with parity.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in 15 16; do
  EWARP_HIP_LIB=$PWD/enterprise_warp_amd/libewarp_hip_dev.so timeout -k 10 300 python scripts/bench_configs.py \
    --configs c2,c4 --reps 5 --mode $m > gpurun_out/ab_contract_$m.log 2>&1
  rc=$?; echo "mode $m rc=$rc"; grep config gpurun_out/ab_contract_$m.log | cut -c1-260
  [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_c2c4.sh
