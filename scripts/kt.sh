#!/bin/bash
# Kernel-trace stats of the perf probe (per-kernel average durations), CSV under gpurun_out/kt.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kt -o run -- python3 -u $R/scripts/perf_probe.py "$@" > $R/gpurun_out/p.log 2>&1
