# The verify route on fresh prior draws beyond the bench's own batch: A/B
# against every unit in double-double (mode 29) for the system model and the
# 372-column pulsar (three more seeds), the 372-column pulsar with sampled
# white noise, and the blind-spot diagnosis (route / dd / enterprise order
# against the CPU double-double reference) on the system model's seeds.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-fresh}
timeout -k 10 300 python -u scripts/wide_ab.py --cases w372_varwn --modes 0,29 --kinds prior --rounds 1 > gpurun_out/${TAG}_varwn.log 2>&1 || exit $?
for off in 1000 2000 3000; do
  timeout -k 10 200 python -u scripts/wide_ab.py --cases system,w372_fixed --modes 0,29 --kinds prior --rounds 1 --seed-offset $off > gpurun_out/${TAG}_$off.log 2>&1 || exit $?
done
for off in 0 1000 2000 3000; do
  timeout -k 10 400 python -u scripts/diag_verify_blindspot.py system --max 8 --seed-offset $off > gpurun_out/${TAG}_diag_$off.log 2>&1 || exit $?
done
