#!/bin/bash
# K2 probe: C2 and C3 (125 k and 1 M traces) stage times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/k2p
mkdir -p $O
cd $R
timeout -k 10 200 python3 -u scripts/perf_probe.py --config C2 --reps 3 > $O/c2.log 2>&1 || exit 1
timeout -k 10 200 python3 -u scripts/perf_probe.py --config C3 --traces 125000 --reps 3 > $O/c3_125k.log 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/perf_probe.py --config C3 --reps 3 > $O/c3_1m.log 2>&1 || exit 1
echo K2PDONE
