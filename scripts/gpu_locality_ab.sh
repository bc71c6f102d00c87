#!/bin/bash
# Locality-order A/B (round 4): parity tests, then perf_probe --ab-locality on each config.
#   bash scripts/gpu_locality_ab.sh "<tests -k expr or ->" CFG,TRACES ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/loc
mkdir -p $O
export TMPDIR=/tmp
cd $R
K=$1; shift
if [ "$K" != "-" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -v --maxfail 2 --timeout 600 --timeout-method thread -k "$K" > $O/pytest.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -20
  [ $rc -ne 0 ] && { grep -E "Error|assert" $O/pytest.log | head -20; exit 1; }
fi
for c in "$@"; do
  IFS=, read -r cfg tr <<< "$c"
  timeout -k 10 500 python -u scripts/perf_probe.py --config $cfg ${tr:+--traces $tr} --reps 3 --ab-locality > $O/${cfg}.log 2>&1 || { echo "probe $cfg failed"; tail -5 $O/${cfg}.log; exit 1; }
  echo "== $cfg"; grep -E "locality=" $O/${cfg}.log
done
echo LOCDONE
