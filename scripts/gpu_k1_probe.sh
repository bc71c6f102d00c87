#!/bin/bash
# K1 grid-choice probe: CITY30 / C3 (100 m queries) and C2 stage times, default build vs one grid.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/k1p
mkdir -p $O
cd $R
for cfg in CITY30 C3; do
  timeout -k 10 300 python3 -u scripts/perf_probe.py --config $cfg --traces 100000 --reps 3 > $O/${cfg}_alt.log 2>&1 || exit 1
  RM_GRID_ALT=0 timeout -k 10 300 python3 -u scripts/perf_probe.py --config $cfg --traces 100000 --reps 3 > $O/${cfg}_one.log 2>&1 || exit 1
done
echo K1PDONE
