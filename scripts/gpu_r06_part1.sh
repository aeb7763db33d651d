set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/${TAG:-r06g}; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -v -rP -m gpu --timeout 300 --timeout-method thread > gpurun_out/${TAG:-r06g}/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -3 gpurun_out/${TAG:-r06g}/pytest_gpu.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG:-r06g}/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/${TAG:-r06g}/smoke.log
