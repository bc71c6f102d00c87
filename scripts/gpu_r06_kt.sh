#!/bin/bash
# kernel stats of one perf_probe run (diagnostic): bash scripts/gpu_r06_kt.sh <tag> <probe args...>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
O=$R/gpurun_out/kt_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/scripts/perf_probe.py --reps 2 "$@" > $O/probe.log 2>&1 || { echo "kt $TAG failed"; tail -5 $O/probe.log; exit 1; }
python3 - $O <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:14]:
    n = r["Name"].replace("rm::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    print("%-28s calls %5s avg %9.1f us" % (n, r["Calls"], float(r["AverageNs"]) / 1e3))
PY
grep "route tiers" $O/probe.log
