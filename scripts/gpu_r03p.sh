# A/B of the pivot log-det forms (0: rs-product PANEL_2L_LP, 23: lane-masked
# per-row log-det PANEL_2L), then the parity subset on the new default
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
crash() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
timeout -k 10 400 python scripts/chol_ab.py --rounds 9 --modes 0,23 > gpurun_out/chol_ab.log 2>&1; rc=$?; echo ab rc=$rc; grep -v amdgpu gpurun_out/chol_ab.log | python -c "import json,sys; d=json.load(sys.stdin); [print(k, round(v['median_ms'],4), round(v['min_ms'],4), v['max_err_over_tol_vs_mode0']) for k,v in d.items()]"
if crash $rc; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "golden or bench_workload or latency or mfma_vs_lds or units_sum" --timeout 300 --timeout-method thread > gpurun_out/pytest_sub.log 2>&1; rc=$?; echo pytest rc=$rc; grep -E "FAILED|ERROR" gpurun_out/pytest_sub.log | head; tail -1 gpurun_out/pytest_sub.log
