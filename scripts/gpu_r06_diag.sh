#!/bin/bash
# diagnostic variants (wrong results by design): timing only
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06_diag
mkdir -p $O
cd $R
for v in main "$@"; do
  lib=""; [ $v != main ] && lib=$R/variants/$v.so
  REPORTER_MATCH_LIB=$lib timeout -k 10 300 python -u scripts/perf_probe.py --config C2 --reps 3 $PROBE_ARGS > $O/C2_$v.log 2>&1 || { echo "probe $v failed"; tail -5 $O/C2_$v.log; exit 1; }
  echo "== $v"; grep rerun $O/C2_$v.log | tail -1
done
