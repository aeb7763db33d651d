# Wide / double-double route on one GPU: its parity tests, the bit-identity
# check against the round-5a schedule (dev mode 34) and the interleaved A/B
# timing (scripts/wide_ab.py).  Outputs under gpurun_out/ tagged TAG.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-wide}
MODES=${2:-0,34,27,29}
CASES=${3:-w372_fixed,system}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_properties.py tests/test_gpu_parity.py -m gpu -k "wide or dd_verify or system or golden" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/wide_variant_check.py > gpurun_out/${TAG}_variant.log 2>&1
rc=$?; cat gpurun_out/${TAG}_variant.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/wide_ab.py --cases $CASES --modes $MODES --rounds 4 > gpurun_out/${TAG}_ab.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_ab.log; exit $rc
