#!/bin/bash
# JSON boundary check: drop-in / coalescing / isolation tests, then the full C2 bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_isolation.py -m gpu -x -v --timeout 300 --timeout-method thread -k "json or coalesc or isolation or global or fails" > $O/pytest_json.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|Error" $O/pytest_json.log | tail -10
[ $rc -ne 0 ] && { tail -30 $O/pytest_json.log; exit $rc; }
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json
d=json.load(open('$O/bench.json')); print(round(d['value']/1e6,1), d['json_boundary'], d['c1_latency']['median_ms'])
"
echo ALLDONE
