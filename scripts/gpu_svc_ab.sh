#!/bin/bash
# Service A/B: lone-caller inline path on / off (RM_COALESCE_INLINE), 60-point requests, C client.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/svcab
mkdir -p $O
cd $R
for rep in 1 2; do
  for inl in 1 0; do
    RM_COALESCE_INLINE=$inl timeout -k 10 200 python3 -u scripts/svc_client_probe.py --clients 1,64 --workers 2 > $O/inl${inl}_rep$rep.log 2>&1 || exit 1
  done
done
echo SVCABDONE
