#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration for K2's access shapes (scripts/calib/fetch_calib.hip):
# timed run, then one PMC pass per counter group.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/calib
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/scripts/bin/fetch_calib > $O/run.txt 2>&1 || { echo "calib failed"; cat $O/run.txt; exit 1; }
cat $O/run.txt
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $R/scripts/bin/fetch_calib > $O/fetch.log 2>&1 || { echo "pmc failed"; tail -5 $O/fetch.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $O/rdreq -o run -- $R/scripts/bin/fetch_calib > $O/rdreq.log 2>&1 || { echo "pmc2 failed"; tail -5 $O/rdreq.log; }
cd $R
python3 - $O <<'PY'
import csv, glob, sys
for d in ("fetch", "rdreq"):
    for f in glob.glob(sys.argv[1] + "/" + d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            print(d, r["Kernel_Name"].split("(")[0], r["Counter_Name"], r["Counter_Value"])
PY
echo ALLDONE
