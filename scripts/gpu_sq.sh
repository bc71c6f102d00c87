#!/bin/bash
# SQ instruction-mix / stall counters of chosen kernels (two 8-counter passes, one rocprofv3 run
# each) for the product build and optional variants (variants/<name>.so):
#   bash scripts/gpu_sq.sh "<kernel regex>" <config> [variant...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
RX=$1; CFG=$2; shift 2
O=$R/gpurun_out/sq
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM"
for v in main "$@"; do
  lib=""; [ $v != main ] && lib=$R/variants/$v.so
  i=0
  for pass in "$P1" "$P2"; do
    i=$((i+1))
    REPORTER_MATCH_LIB=$lib timeout -s KILL 180 rocprofv3 --pmc $pass --kernel-include-regex "$RX" --output-format csv -d $O/${v}_p$i -o run -- python3 $R/scripts/perf_probe.py --reps 1 --config $CFG > $O/${v}_p$i.log 2>&1 || { echo "pass $v $i failed"; tail -5 $O/${v}_p$i.log; exit 1; }
  done
done
cd $R
python3 - "$O" main "$@" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
for v in sys.argv[2:]:
    per = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, v + "_p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("rm::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in sorted(per.items()):
        e = {c: sum(x) / len(x) for c, x in cs.items()}
        print(v, k, " ".join("%s=%.4g" % kv for kv in sorted(e.items())))
PY
echo SQDONE
