#!/bin/bash
# Where the 256-client service's CPU goes: the box's CPU quota, a CPU-only model of the
# coalescer's hand-offs (variants/cv_*: global-mutex vs per-request waits, 150 us per batch), and
# the real client at 256 clients with library variants / allocator switches (VARIANTS).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/svccpu
mkdir -p $O
echo "nproc $(nproc)  cpu.max $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"
if [ -x $R/variants/cv_global ]; then
  for b in cv_global cv_perreq; do for c in 64 256; do timeout -k 5 60 $R/variants/$b $c 20000 150 || exit 1; done; done
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u $R/scripts/svc_prep.py /tmp/svcprep --points 60 --requests 20000 > $O/prep.log 2>&1 || { tail -5 $O/prep.log; exit 1; }
VARIANTS=${VARIANTS:-"RM_X=0 LD_LIBRARY_PATH=$R/variants/zcoff LD_LIBRARY_PATH=$R/variants/old MALLOC_ARENA_MAX=2 RM_X=1 LD_LIBRARY_PATH=$R/variants/zcoff LD_LIBRARY_PATH=$R/variants/old"}
i=0
for v in $VARIANTS; do
  i=$((i+1))
  for cl in ${CLIENTS:-256}; do
    f=$O/v${i}_c$cl
    env $v timeout -k 10 120 $R/reporter_amd/bin/rm_svc_client /tmp/svcprep/conf.json /tmp/svcprep/reqs.txt $cl 20000 2048 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    python3 - $f.json "$v" $cl <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("%-48s c%-4s %6.2f M pts/s p50 %.3f p99 %6.2f engine %.4f cpu %.2f client %.2f cs %s thr %s" % (
    sys.argv[2][-48:], sys.argv[3], d["points_per_s"] / 1e6, d["latency_ms"]["p50"], d["latency_ms"]["p99"],
    d["dispatcher_ms_per_batch"]["engine"], d["cpu_seconds"], d.get("client_cpu_seconds", -1), d.get("context_switches"),
    d.get("cgroup_throttled_periods")))
PY
  done
done
echo SVCCPUDONE
