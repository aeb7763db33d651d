set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python scripts/chol_ab.py --rounds 7 --modes 0,17 > gpurun_out/chol_ab.log 2>&1; rc=$?; echo ab rc=$rc; cat gpurun_out/chol_ab.log | python -c "import json,sys; d=json.load(sys.stdin); [print(k, round(v['median_ms'],4), round(v['max_err_over_tol_vs_mode0'],3)) for k,v in d.items()]"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/chol_stamps.py > gpurun_out/chol_stamps.log 2>&1; rc=$?; echo stamps rc=$rc; head -40 gpurun_out/chol_stamps.log
