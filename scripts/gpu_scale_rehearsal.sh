#!/bin/bash
# Rehearsal of bench.py's multi-rank path on a one-GPU box: two ranks on
# cuda:0 over gloo (RCCL takes one rank per GPU), overlapped all-reduce,
# --verify against the single-device entry; then the default N=1 line.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29631 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --same-device --verify \
  --no-latency > gpurun_out/rehearsal_n2.log 2>&1
rc=$?
echo "n2 rc=$rc"; tail -3 gpurun_out/rehearsal_n2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --verify --no-cpu-baseline --no-latency --no-secondary \
  > gpurun_out/rehearsal_n1.log 2>&1
rc=$?
echo "n1 rc=$rc"; tail -2 gpurun_out/rehearsal_n1.log
exit $rc
