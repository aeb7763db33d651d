# Interleaved A/B of the latency kernel across two builds (round 6: the
# diagonal chains' row replication by lane swaps, libewarp_hip_var.so built
# with -DEWH_LAT_REPL=2, against the product library): bit identity of the
# single-theta path on C3, then latency_sweep alternating A / B.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/latab; export TMPDIR=/tmp
A=enterprise_warp_amd/libewarp_hip.so; B=${1:-enterprise_warp_amd/libewarp_hip_var.so}
EWARP_HIP_LIB=$A timeout -k 10 200 python -u scripts/lat_values.py save gpurun_out/latab/a.npy > gpurun_out/latab/bitid.log 2>&1 || exit $?
EWARP_HIP_LIB=$B timeout -k 10 200 python -u scripts/lat_values.py compare gpurun_out/latab/a.npy >> gpurun_out/latab/bitid.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/latab/bitid.log
for r in 1 2 3; do
  for L in $A $B; do
    EWARP_HIP_LIB=$L timeout -k 10 200 python -u scripts/latency_sweep.py --reps 400 --batches 1,8,24 --modes 0 > gpurun_out/latab/sweep_$(basename $L .so)_$r.log 2>&1 || exit $?
    echo "$(basename $L .so) $r $(tail -1 gpurun_out/latab/sweep_$(basename $L .so)_$r.log)"
  done
done
