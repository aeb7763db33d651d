# The double-double route's verify threshold on the bench's prior draws: for
# each fraction of strict the two fp64 orders must agree to, the refined
# share and the largest |route - every unit in double-double| in strict
# units (system model, 4096 draws; the 372-column pulsar, 1024).  Dev library
# (EWARP_VERIFY_FRAC is read there only).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for F in 0.25 0.0625 0.015625 0.00390625; do
  EWARP_VERIFY_FRAC=$F timeout -k 10 300 python -u scripts/wide_ab.py --cases system,w372_fixed --modes 29,0 --kinds prior --rounds 2 > gpurun_out/vfrac_$F.log 2>&1 || exit $?
  echo "== frac=$F"; python scripts/ab_table.py gpurun_out/vfrac_$F.log
done
