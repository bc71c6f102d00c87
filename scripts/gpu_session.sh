#!/bin/bash
# One GPU session: every -m gpu test + smoke (unless SKIP_TESTS), then gpu_pmc_cfg.sh for each
# "<config>:<traces>:<tag>[:extra bench args]" argument.  Each GPU step has its own time limit
# and a failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail 3 --timeout 300 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"} > $O/pytest_gpu.log 2>&1
  rc=$?
  grep -E "passed|failed" $O/pytest_gpu.log | tail -2
  [ $rc -ne 0 ] && { grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; exit 1; }
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
for spec in "$@"; do
  IFS=: read -r cfg tr tag extra <<< "$spec"
  bash scripts/gpu_pmc_cfg.sh $cfg $tr $tag $extra || exit 1
done
echo ALLDONE
