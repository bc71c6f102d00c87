#!/bin/bash
# K1 A/B: lane tier (default) vs every state in the wave tier (RM_K1_WAVE_ALL=1), CITY30 / C2 / C4-sized C2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/k1ab
mkdir -p $O
cd $R
for cfg in CITY30 C2; do
  for w in 0 1; do
    RM_K1_WAVE_ALL=$w timeout -k 10 300 python3 -u scripts/perf_probe.py --config $cfg --traces 10000 --reps 3 > $O/${cfg}_w$w.log 2>&1 || exit 1
  done
done
echo K1ABDONE
