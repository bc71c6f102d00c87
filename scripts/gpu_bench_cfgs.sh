#!/bin/bash
# bench.py lines for the other BASELINE configs (C3, C4 at the default radius); one GPU step each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
for C in ${@:-C3 C4}; do
  timeout -k 10 500 python -u bench.py --config $C --no-extras > $O/bench_$C.json 2> $O/bench_$C.err || { echo "bench $C failed"; tail -20 $O/bench_$C.err; exit 1; }
  python -c "
import json,sys; d=json.load(open('$O/bench_$C.json'))
print('$C', round(d['value']/1e6,1), 'Mpts/s', round(d['ms_per_step'],2), 'ms', d['kernels_ms_per_step'], d['roofline']['frac'], d['config']['route_balls'] if 'route_balls' in d['config'] else d['roofline'].get('route_balls'))
"
done
echo ALLDONE
