#!/bin/bash
# Experiment session: a parity subset (pytest -k $1, default the parity file), then the perf
# probe of the product build and of every variants/*.so (diagnostic).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pinned.py -m gpu -x -v --timeout 300 --timeout-method thread ${1:+-k "$1"} > $O/pytest_try.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_try.log | tail -30
case $rc in 124|134|137|139) echo "pytest fatal rc=$rc"; exit $rc;; esac
[ $rc -ne 0 ] && { tail -60 $O/pytest_try.log; exit 1; }
timeout -k 10 120 python -u scripts/perf_probe.py --config C2 --reps 3 > $O/probe_main.log 2>&1 || { echo "probe failed"; tail -5 $O/probe_main.log; exit 1; }
echo "== main"; grep rerun $O/probe_main.log | tail -2
if ls variants/*.so >/dev/null 2>&1; then bash scripts/probe_variants.sh --config C2 --reps 3 || exit 1; fi
echo ALLDONE
