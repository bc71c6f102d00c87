#!/bin/bash
# Multi-stream check: equality test, then the C2 bench at 2 and 1 streams (diagnostic).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_multistream.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_ms.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" $O/pytest_ms.log | tail -8
[ $rc -ne 0 ] && { tail -30 $O/pytest_ms.log; exit $rc; }
for s in ${@:-2 1}; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-extras --streams $s > $O/b$s.json 2> $O/b$s.err || { tail -20 $O/b$s.err; exit 1; }
  python -c "
import json
d=json.load(open('$O/b$s.json')); print('streams $s', round(d['value']/1e6,1), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernels_ms_per_step'].items()}, round(d['roofline']['frac'],3))
"
done
echo ALLDONE
