#!/bin/bash
# K3 / latency probe: C1 single-trace latency, C2 lone trace, 38 traces, full C2 and C5 stage times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/k3p
mkdir -p $O
cd $R
timeout -k 10 200 python3 -u scripts/c1_probe.py > $O/c1.log 2>&1 || exit 1
for t in 1 38; do
  timeout -k 10 200 python3 -u scripts/perf_probe.py --config C2 --traces $t --reps 5 > $O/c2_t$t.log 2>&1 || exit 1
done
timeout -k 10 300 python3 -u scripts/perf_probe.py --config C2 --reps 3 > $O/c2.log 2>&1 || exit 1
timeout -k 10 300 python3 -u scripts/perf_probe.py --config C5 --reps 3 > $O/c5.log 2>&1 || exit 1
echo K3PDONE
