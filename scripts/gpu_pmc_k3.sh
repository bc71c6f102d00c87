#!/bin/bash
# K3 diagnostics: SQ counters of the product build and of variants/vit2.so, and the product
# build at 8,000 traces (one round of resident waves).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/k3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
P2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM"
for v in main vit2; do
  lib=""; [ $v = vit2 ] && lib=$R/variants/vit2.so
  i=0
  for pass in "$P1" "$P2"; do
    i=$((i+1))
    REPORTER_MATCH_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex "k_viterbi" --output-format csv -d $O/${v}_p$i -o run -- python3 $R/scripts/perf_probe.py --reps 1 --config C2 > $O/${v}_p$i.log 2>&1 || { echo "pass $v $i failed"; tail -5 $O/${v}_p$i.log; exit 1; }
  done
done
cd $R
python3 - "$O" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
for v in ("main", "vit2"):
    per = defaultdict(list)
    for f in glob.glob(os.path.join(d, v + "_p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "viterbi" in r["Kernel_Name"]:
                per[r["Counter_Name"]].append(float(r["Counter_Value"]))
    e = {k: sum(x) / len(x) for k, x in per.items()}
    print(v, " ".join("%s=%.4g" % kv for kv in sorted(e.items())))
PY
timeout -k 10 120 python -u scripts/perf_probe.py --config C2 --reps 3 --traces 8000 > $O/probe8k.log 2>&1 && grep rerun $O/probe8k.log | tail -1
timeout -k 10 120 python -u scripts/perf_probe.py --config C2 --reps 3 --traces 4000 > $O/probe4k.log 2>&1 && grep rerun $O/probe4k.log | tail -1
echo ALLDONE
