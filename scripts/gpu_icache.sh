#!/bin/bash
# Instruction-cache counters per kernel over one C2 perf-probe run (diagnostic).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/icache
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_VALU SQ_WAVES --output-format csv -d $O/p1 -o run -- python3 $R/scripts/perf_probe.py --reps 1 --config C2 > $O/p1.log 2>&1 || { echo "pass failed"; tail -5 $O/p1.log; exit 1; }
cd $R
python3 - "$O" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
per = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(sys.argv[1], "p1", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("rm::(anonymous namespace)::", "").split("(")[0]
        per[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(per.items(), key=lambda kv: -sum(kv[1].get("SQ_INSTS_VALU", [0]))):
    e = {c: sum(v) / len(v) for c, v in cs.items()}
    h, m = e.get("SQC_ICACHE_HITS", 0), e.get("SQC_ICACHE_MISSES", 0)
    print("%-26s icache hit=%.4g miss=%.4g missrate=%.4f valu=%.4g waves=%.4g" % (k[:26], h, m, m / max(h + m, 1), e.get("SQ_INSTS_VALU", 0), e.get("SQ_WAVES", 0)))
PY
echo ALLDONE
