# Round-5 (r05h) A/B pass on one GPU: the wide route (its tests, bit identity
# against dev mode 34, interleaved timing) and the C2 / C4 contraction run
# order (modes 0 vs 35, contraction alone).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05h}
bash scripts/gpu_wide_ab.sh ${TAG}w 0,34,29 w372_fixed,system || exit $?
timeout -k 10 500 python -u scripts/wide_ab.py --cases c2,c4 --modes 0,35 --kinds prior --contract --rounds 5 > gpurun_out/${TAG}_c2c4.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_c2c4.log; exit $rc
