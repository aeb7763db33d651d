set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -v -s -m gpu --timeout 400 --timeout-method thread -k "graph or single_call or multi_context or set_fixed or golden" > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo pytest rc=$rc; grep -E "passed|failed|FAILED|^E  " gpurun_out/pytest_gpu.log | tail -20
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 > gpurun_out/bench.log 2>&1; echo bench rc=$?; python -c "import json;d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['sampler_latency'])"
