#!/bin/bash
# Round 6: K2 walk count (diagnostic build), K3 chunk-clamp parity + A/B + its HBM traffic.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06_k3
mkdir -p $O
cd $R
export TMPDIR=/tmp
REPORTER_MATCH_LIB=$R/variants/k2stats.so timeout -k 10 300 python -u scripts/perf_probe.py --config C2 --reps 1 --turn 200 > $O/k2stats_c2.log 2>&1 || { echo "k2stats failed"; tail -5 $O/k2stats_c2.log; exit 1; }
grep "route tiers" $O/k2stats_c2.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_turns.py tests/test_gpu_small.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "parity failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in C2 C5; do
  for v in main vitnoclamp; do
    lib=""; [ $v != main ] && lib=$R/variants/$v.so
    REPORTER_MATCH_LIB=$lib timeout -k 10 300 python -u scripts/perf_probe.py --config $c --reps 3 > $O/${c}_$v.log 2>&1 || { echo "probe $c $v failed"; exit 1; }
    echo "== $c $v"; grep rerun $O/${c}_$v.log | tail -1
  done
done
cd /tmp
for v in main vitnoclamp; do
  lib=""; [ $v != main ] && lib=$R/variants/$v.so
  REPORTER_MATCH_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$v -o run -- python3 $R/scripts/perf_probe.py --config C2 --reps 1 > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $O/pmc_$v.log; exit 1; }
  python3 - $O/pmc_$v <<'PY'
import csv, glob, sys
from collections import defaultdict
d = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "viterbi" in r["Kernel_Name"] or "routes_ball2" in r["Kernel_Name"]:
            d[r["Kernel_Name"].split("(")[0][-40:]].append(float(r["Counter_Value"]))
for k, v in d.items():
    print(sys.argv[1].split("/")[-1], k, "FETCH KB/launch %.0f (x2 = %.3f GB)" % (sum(v) / len(v), sum(v) / len(v) * 2048 / 1e9))
PY
done
echo K3DONE
