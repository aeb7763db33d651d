# r05h pass 2: wide tests + bit identity (mode 34), the epoch-sum A/B on the
# sampled-white-noise wide pulsar (mode 0 vs 37), then smoke, the bench and
# rocprof kernel stats of the wide block (scripts/gpu_r05.sh steps).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05h2}
bash scripts/gpu_wide_ab.sh ${TAG}w 0,37 w372_varwn || exit $?
bash scripts/gpu_r05.sh $TAG smoke,bench,wideprof
