#!/bin/bash
# Round-6 evidence for the other configs: PMC passes + traffic-carrying bench lines at the sizes
# the PMC runs (C3 and C4 at 125 k traces, CITY30 at its 100 k), then default-size bench lines.
#   bash scripts/gpu_r06_cfgs.sh pmc|lines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
if [ "$1" = pmc ]; then
  for ct in ${CFGS:-C3:125000 C4:125000 CITY30:100000}; do
    c=${ct%%:*}; t=${ct##*:}; lc=$(echo $c | tr A-Z a-z)
    bash scripts/gpu_pmc_cfg.sh $c $t r06_$lc || exit 1
  done
else
  mkdir -p $R/gpurun_out/r06_cfgs
  for c in ${CFGS:-C3 C4 C5 CITY}; do
    lc=$(echo $c | tr A-Z a-z)
    timeout -k 10 600 python -u bench.py --config $c --no-extras > $R/gpurun_out/r06_cfgs/bench_${lc}_n1.json 2> $R/gpurun_out/r06_cfgs/bench_${lc}_n1.err || { echo "bench $c failed"; tail -20 $R/gpurun_out/r06_cfgs/bench_${lc}_n1.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$R/gpurun_out/r06_cfgs/bench_${lc}_n1.json'))
print('$c', round(d['value']/1e6,1), 'M points/s', round(d['ms_per_step'],2), 'ms/step', 'K2', round(d['roofline']['avg_launch_ms'],3), 'frac', d['roofline']['frac'])"
  done
fi
echo CFGSDONE
