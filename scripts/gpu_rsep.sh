# r-separated contraction check on one GPU: the GPU suite, then the C4 / C2
# contraction A/B (mode 0 vs 36 = RSEP off) and the lnL batch A/B.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-rsep}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest.log; grep -E "FAILED|ERROR" gpurun_out/${TAG}_pytest.log | head; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u scripts/wide_ab.py --cases c4,c2 --modes 0,36 --kinds prior --contract --rounds 5 > gpurun_out/${TAG}_contract.log 2>&1 || exit $?
timeout -k 10 500 python -u scripts/wide_ab.py --cases c4 --modes 0,36 --kinds prior,near --rounds 3 > gpurun_out/${TAG}_lnl.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_lnl.log; exit $rc
