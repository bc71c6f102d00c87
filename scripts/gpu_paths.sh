#!/bin/bash
# Path-walk experiment: parity subset, C2 probe of every build, C3 probe (200k traces) of every build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
bash scripts/gpu_try.sh "$1" || exit 1
timeout -k 10 300 python -u scripts/perf_probe.py --config C3 --traces 200000 --reps 2 > $O/probe_c3.log 2>&1 || { tail -5 $O/probe_c3.log; exit 1; }
echo "== main C3"; grep rerun $O/probe_c3.log | tail -1
for lib in variants/*.so; do
  n=$(basename $lib .so)
  REPORTER_MATCH_LIB=$R/$lib timeout -k 10 300 python -u scripts/perf_probe.py --config C3 --traces 200000 --reps 2 > $O/probe_c3_$n.log 2>&1 || { tail -5 $O/probe_c3_$n.log; exit 1; }
  echo "== $n C3"; grep rerun $O/probe_c3_$n.log | tail -1
done
echo ALLDONE
