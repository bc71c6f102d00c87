#!/bin/bash
# Round-2 GPU session: every -m gpu test (no -x: collect all outcomes, stop after 6 failures),
# smoke, then the bench line.  Each GPU step has its own time limit; a fault or timeout ends
# the script (exit codes 124/134/137/139).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
K=${1:-}
ARGS=(-m gpu -v -s --maxfail 6 --timeout 900 --timeout-method thread)
if [ -n "$K" ]; then ARGS+=(-k "$K"); fi
timeout -k 10 1500 python -u -m pytest tests "${ARGS[@]}" > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -60
case $rc in 124|134|137|139) echo "pytest fatal rc=$rc"; exit $rc;; esac
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
echo "ALLDONE pytest_rc=$rc"
