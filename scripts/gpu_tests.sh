#!/bin/bash
# GPU tests only (optionally a -k filter in $1), each run under its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
ARGS=(-m gpu -v -s --maxfail 4 --timeout 900 --timeout-method thread)
if [ -n "$1" ]; then ARGS+=(-k "$1"); fi
timeout -k 10 ${2:-1100} python -u -m pytest tests "${ARGS[@]}" > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -40
exit $rc
