#!/bin/bash
# Parity subset + variant timings + kernel trace of the product build (diagnostic GPU session).
# $1: pytest -k expression.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -x --timeout 600 --timeout-method thread -k "${1:-parity}" > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -30
case $rc in 124|134|137|139) echo "pytest fatal rc=$rc"; exit $rc;; esac
[ $rc -ne 0 ] && { tail -40 $O/pytest_gpu.log; exit 1; }
bash scripts/probe_variants.sh --config C2 || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python $R/scripts/perf_probe.py --config C2 --reps 3 > $O/prof_kt.log 2>&1 || { echo "kt failed"; tail -5 $O/prof_kt.log; exit 1; }
cd $R
python - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/prof_kt/**/run_kernel_stats.csv", recursive=True) + glob.glob("gpurun_out/prof_kt/run_kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Name"].replace("rm::(anonymous namespace)::", "").split("(")[0]
        print("%-40s calls=%-5s avg_us=%.1f" % (n[:40], r["Calls"], float(r["AverageNs"]) / 1e3))
    break
PY
echo ALLDONE
