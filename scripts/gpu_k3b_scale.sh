#!/bin/bash
# K3 batch kernels at larger batches: 8 lanes per trace vs 16 (RM_VIT_LANES=16), C2 graph at 40 k
# traces and C3 at 125 k traces.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/k3s
mkdir -p $O
cd $R
for cfg in "C2 40000" "C3 125000"; do
  set -- $cfg
  for v in new p16; do
    if [ $v = p16 ]; then export RM_VIT_LANES=16; else unset RM_VIT_LANES; fi
    timeout -k 10 300 python3 -u scripts/perf_probe.py --config $1 --traces $2 --reps 3 > $O/$1_$2_$v.log 2>&1 || exit 1
    grep rerun $O/$1_$2_$v.log | tail -2 | sed "s/^/$v $1 $2 /"
  done
done
echo K3SDONE
