#!/bin/bash
# A/B with bench-style timing (only the named stages timed; wall ms/step untimed): main vs variants
#   bash scripts/gpu_r06_ab.sh "<configs>" "<stages>" variant...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFGS=$1; ST=$2; shift 2
O=$R/gpurun_out/ab6
mkdir -p $O
cd $R
for c in $CFGS; do
  IFS=, read -r cfg tr <<< "$c"
  for rep in 1 2; do
    for v in main "$@"; do
      lib=""; [ $v != main ] && lib=$R/variants/$v.so
      REPORTER_MATCH_LIB=$lib timeout -k 10 300 python -u scripts/perf_probe.py --config $cfg ${tr:+--traces $tr} --reps 20 --only $ST $PROBE_ARGS > $O/${cfg}_${v}_$rep.log 2>&1 || { echo "probe $cfg $v failed"; tail -5 $O/${cfg}_${v}_$rep.log; exit 1; }
      echo "== $cfg $v ($rep) $(grep '^only' $O/${cfg}_${v}_$rep.log)"
    done
  done
done
echo ABDONE
