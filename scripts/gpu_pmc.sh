#!/bin/bash
# Parity subset, then per-kernel PMC passes over a perf-probe run (diagnostic GPU session).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -x --timeout 600 --timeout-method thread -k "${1:-parity}" > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -10
case $rc in 124|134|137|139) echo "pytest fatal rc=$rc"; exit $rc;; esac
[ $rc -ne 0 ] && { tail -40 $O/pytest_gpu.log; exit 1; }
bash scripts/pmc_probe.sh --config C2 > $O/pmc_probe.txt 2>&1 || { tail -20 $O/pmc_probe.txt; exit 1; }
cat $O/pmc_probe.txt
for m in 2 4; do
  timeout -k 10 300 python -u scripts/perf_probe.py --config C2 --reps 3 --split $m > $O/split$m.log 2>&1 || { echo "split $m failed"; tail -5 $O/split$m.log; exit 1; }
  grep -E "rerun|split" $O/split$m.log | tail -3
done
echo ALLDONE
