# Interleaved A/B of the headline kernel across two builds (round 6: the
# pivot-row broadcast by lane swaps, libewarp_hip_var.so, against the product
# library): bit identity of 4096 C3 prior draws + C3 near draws, then the
# bench line (headline only) alternating A / B.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/c3ab; export TMPDIR=/tmp
A=enterprise_warp_amd/libewarp_hip.so; B=${1:-enterprise_warp_amd/libewarp_hip_var.so}
EWARP_HIP_LIB=$A timeout -k 10 200 python -u scripts/c3_values.py save gpurun_out/c3ab/a.npy > gpurun_out/c3ab/bitid.log 2>&1 || exit $?
EWARP_HIP_LIB=$B timeout -k 10 200 python -u scripts/c3_values.py compare gpurun_out/c3ab/a.npy >> gpurun_out/c3ab/bitid.log 2>&1 || exit $?
cat gpurun_out/c3ab/bitid.log | grep -v amdgpu
for r in 1 2 3; do
  for L in $A $B; do
    EWARP_HIP_LIB=$L timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-latency --no-secondary > gpurun_out/c3ab/bench_$(basename $L .so)_$r.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/c3ab/bench_$(basename $L .so)_$r.log') if l.startswith('{')][-1]); print('$(basename $L .so)', $r, round(d['ms_per_step'],4), round(d['roofline']['launch_ms'],4), round(d['roofline']['frac'],4))"
  done
done
