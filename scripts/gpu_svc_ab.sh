#!/bin/bash
# Service A/B on one box: the C-ABI client on 60-point requests at 64 and 256 clients, each
# variant (an environment assignment, e.g. RM_SMALL_GRAPH=0) twice, interleaved.
#   bash scripts/gpu_svc_ab.sh "RM_SMALL_GRAPH=0" "RM_SMALL_GRAPH=1"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/svcab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
PTS=${PTS:-60}
timeout -k 10 300 python3 -u $R/scripts/svc_prep.py /tmp/svcprep --points $PTS --requests 20000 > $O/prep.log 2>&1 || { tail -5 $O/prep.log; exit 1; }
for rep in 1 2; do
  for v in "$@"; do
    for cl in ${CLIENTS:-64 256}; do
      tag=$(echo "$v" | tr -c 'A-Za-z0-9=_\n' '_')_c${cl}_r$rep
      env $v RM_COALESCE_TRACE=${TRACE_MS:-20} timeout -k 10 120 $R/reporter_amd/bin/rm_svc_client /tmp/svcprep/conf.json /tmp/svcprep/reqs.txt $cl 20000 2048 > $O/$tag.json 2> $O/$tag.err || { echo "client failed: $v $cl"; tail -5 $O/$tag.err; exit 1; }
      python3 - "$O/$tag.json" "$v" "$cl" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("%-22s c%-4s %8.2f M pts/s  p50 %.3f p99 %.3f max %.2f ms  batch %.1f  engine %.4f ms  cpu %.2f s  throttled %s (%s ms)" % (
    sys.argv[2], sys.argv[3], d["points_per_s"] / 1e6, d["latency_ms"]["p50"], d["latency_ms"]["p99"], d["latency_ms"]["max"],
    d["requests_per_batch"], d["dispatcher_ms_per_batch"]["engine"], d.get("cpu_seconds", -1),
    d.get("cgroup_throttled_periods"), d.get("cgroup_throttled_ms")))
PY
    done
  done
done
echo SVCABDONE
