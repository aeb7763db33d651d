# Timing split of chol_dd_kernel (dev library, kernel mode 29 = every unit in
# double-double): the full kernel, then with its trailing update (1), panel
# solve (2) or wave-0 diagonal chain (4) skipped via EWARP_DD_SKIP -- results
# meaningless, times only.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for k in 0 1 2 4 7; do
  EWARP_DD_SKIP=$k timeout -k 10 300 python -u scripts/wide_ab.py --cases system,w372_fixed --modes 29 --kinds prior --rounds 3 > gpurun_out/ddskip_$k.log 2>&1 || exit $?
  echo "== skip $k"; python scripts/ab_table.py gpurun_out/ddskip_$k.log
done
