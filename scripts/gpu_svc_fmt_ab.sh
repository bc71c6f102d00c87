#!/bin/bash
# Service A/B: replies formatted by their callers (default) or by the dispatcher
# (RM_COALESCE_FORMAT=dispatcher); 60-point requests from the C client, then the service tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/svcfmt
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_small.py tests/test_gpu_isolation.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for f in callers dispatcher; do
    RM_COALESCE_FORMAT=$f timeout -k 10 200 python3 -u scripts/svc_client_probe.py --clients 1,64,256 --workers 2 > $O/${f}_rep$rep.log 2>&1 || exit 1
    echo "== $f rep $rep"; grep -E "clients|pts/s|points" $O/${f}_rep$rep.log | tail -4
  done
done
echo SVCFMTDONE
