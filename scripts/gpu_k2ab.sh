#!/bin/bash
# K2 A/B: the round-2 per-source kernel (RM_K2=1) against the block-expanded one (RM_K2=2) on C2
# and a C3 sample, then the parity tests that exercise K2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O/k2ab
cd $R
for cfg in "C2 0" "C3 125000"; do
  set -- $cfg
  for v in 1 2; do
    RM_K2=$v timeout -k 10 240 python -u scripts/perf_probe.py --config $1 --traces $2 --reps 3 > $O/k2ab/$1_v$v.log 2>&1 || { echo "probe $1 v$v failed"; tail -5 $O/k2ab/$1_v$v.log; exit 1; }
    echo "== $1 RM_K2=$v"; grep rerun $O/k2ab/$1_v$v.log | tail -1
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -k "parity or fullsize or pinned or balls" > $O/k2ab/pytest.log 2>&1
rc=$?
tail -3 $O/k2ab/pytest.log
exit $rc
