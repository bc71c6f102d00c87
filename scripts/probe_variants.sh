#!/bin/bash
# Time every variants/*.so with the perf probe (diagnostic; one process per variant).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/probe
cd $R
for lib in variants/*.so; do
  n=$(basename $lib .so)
  REPORTER_MATCH_LIB=$R/$lib timeout -k 10 120 python -u scripts/perf_probe.py "$@" > gpurun_out/probe/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/probe/$n.log; exit 1; }
  echo "== $n"; grep rerun gpurun_out/probe/$n.log | tail -1
done
