#!/bin/bash
# Service tail diagnosis: the C-ABI client at 256 clients on 60-point requests (bench.py's
# service_client_60pt_256 shape) with RM_COALESCE_TRACE printing every batch slower than 3 ms.
#   bash scripts/gpu_svc_tail.sh [clients] [points]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
CL=${1:-256}; PTS=${2:-60}
O=$R/gpurun_out/svctail
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u $R/scripts/svc_prep.py /tmp/svcprep --points $PTS --requests 20000 > $O/prep.log 2>&1 || { tail -5 $O/prep.log; exit 1; }
for i in 1 2; do
  RM_COALESCE_TRACE=${TRACE_MS:-3} timeout -k 10 120 $R/reporter_amd/bin/rm_svc_client /tmp/svcprep/conf.json /tmp/svcprep/reqs.txt $CL 20000 2048 > $O/run$i.json 2> $O/run$i.err || { tail -5 $O/run$i.err; exit 1; }
  echo "== run $i"; cat $O/run$i.json | tail -1 | cut -c1-400; grep -c coalesce $O/run$i.err; grep coalesce $O/run$i.err | sort -t' ' -k7 -n -r | head -8
done
echo SVCTAILDONE
