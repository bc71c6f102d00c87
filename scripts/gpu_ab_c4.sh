#!/bin/bash
# Parity subset, the C2 bench line, then C4 with GPU-built vs host-built route balls.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pinned.py tests/test_gpu_isolation.py tests/test_gpu_balls.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_ab.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest_ab.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAILED|ERROR|Error" $O/pytest_ab.log | head -20; exit 1; }
timeout -k 10 300 python -u bench.py --no-extras --no-cpu-baseline > $O/bench_ab_c2.json 2> $O/bench_ab_c2.err || { tail -20 $O/bench_ab_c2.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_ab_c2.json')); print('C2', round(d['value']/1e6,1), d['kernels_ms_per_step'])"
for how in ${AB_HOW:-gpu host}; do
  RM_BALL_BUILD=$how timeout -k 10 500 python -u bench.py --config C4 --no-extras > $O/bench_ab_c4_$how.json 2> $O/bench_ab_c4_$how.err || { tail -20 $O/bench_ab_c4_$how.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/bench_ab_c4_$how.json')); print('C4 $how', round(d['value']/1e6,1), d['kernels_ms_per_step'], d['roofline'].get('route_balls'))"
done
echo ALLDONE
