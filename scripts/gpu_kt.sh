#!/bin/bash
# Stage timings (perf_probe) + rocprofv3 kernel trace of one config (diagnostic GPU session).
# $1: config (default C2); $2: output tag.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
C=${1:-C2}
TAG=${2:-kt}
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u scripts/perf_probe.py --config $C --reps 3 > $O/${TAG}_probe.txt 2>&1 || { echo "probe failed"; tail -20 $O/${TAG}_probe.txt; exit 1; }
cat $O/${TAG}_probe.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof -o run -- python $R/scripts/perf_probe.py --config $C --reps 3 > $O/${TAG}_prof.log 2>&1 || { echo "kt failed"; tail -5 $O/${TAG}_prof.log; exit 1; }
cd $R
python - "$O/${TAG}_prof" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"].replace("rm::(anonymous namespace)::", "").split("(")[0]
        print("%-50s calls=%-5s avg_us=%.1f" % (n[:50], r["Calls"], float(r["AverageNs"]) / 1e3))
    break
PY
echo ALLDONE
