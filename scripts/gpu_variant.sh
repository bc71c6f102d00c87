#!/bin/bash
# A/B of experiment variants against the product build: parity tests with the variant library
# (K = "-": none), then perf_probe on each config.   bash scripts/gpu_variant.sh "<configs>" "<tests -k expr>" variant...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFGS=$1; K=$2; shift 2
O=$R/gpurun_out/ab
mkdir -p $O
export TMPDIR=/tmp
cd $R
for v in "$@"; do
  [ "$K" = "-" ] && break   # perf only
  REPORTER_MATCH_LIB=$R/variants/$v.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $O/pytest_$v.log 2>&1 || { echo "parity $v failed"; tail -30 $O/pytest_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $O/pytest_$v.log)"
done
for c in $CFGS; do
  IFS=, read -r cfg tr <<< "$c"
  for v in main "$@"; do
    lib=""; [ $v != main ] && lib=$R/variants/$v.so
    REPORTER_MATCH_LIB=$lib timeout -k 10 300 python -u scripts/perf_probe.py --config $cfg ${tr:+--traces $tr} --reps 3 $PROBE_ARGS > $O/${cfg}_$v.log 2>&1 || { echo "probe $cfg $v failed"; tail -5 $O/${cfg}_$v.log; exit 1; }
    echo "== $cfg $v"; grep rerun $O/${cfg}_$v.log | tail -1
  done
done
echo ABDONE
