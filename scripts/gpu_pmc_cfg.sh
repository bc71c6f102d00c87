#!/bin/bash
# Kernel stats + PMC passes (FETCH_SIZE, WRITE_SIZE, TCC hit/miss, SQ instruction counts; one rocprofv3 run each) of
# one bench configuration, their per-stage summary, then the bench line carrying that traffic.
#   bash scripts/gpu_pmc_cfg.sh <config> <traces> <tag> [extra bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=$1; TR=$2; TAG=$3; shift 3
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
ARGS="--config $CFG --traces $TR --no-extras --parts-extra 0 $*"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python3 $R/bench.py $ARGS --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_kt.log 2>&1 || { echo "$TAG kt failed"; tail -5 $O/prof_kt.log; exit 1; }
echo "$TAG kt done"
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES"; do
  name=$(echo $pass | tr ' ' '_')
  timeout -s KILL 400 rocprofv3 --pmc $pass --output-format csv -d $O/pmc_$name -o run -- python3 $R/bench.py $ARGS --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_$name.log 2>&1 || { echo "$TAG pmc $pass failed"; tail -5 $O/pmc_$name.log; exit 1; }
  echo "$TAG pmc $name done"
done
cd $R
python scripts/pmc_summary.py $O $O/summary --config $CFG --traces $TR --streams 1 --tag $TAG --turn-penalty ${TURN:-0} --what "python bench.py $ARGS --steps 5 --warmup 1 --no-cpu-baseline" > $O/summary.log 2>&1 || { echo "$TAG summary failed"; tail -5 $O/summary.log; exit 1; }
timeout -k 10 600 python -u bench.py $ARGS --traffic-json $O/summary/pmc_$TAG.json > $O/bench.json 2> $O/bench.err || { echo "$TAG bench failed"; tail -20 $O/bench.err; exit 1; }
python - <<PY
import json; d = json.load(open("$O/bench.json"))
r = d["rooflines"]
print("$TAG", round(d["value"] / 1e6, 1), "Mpts/s", round(d["ms_per_step"], 2), "ms/step")
for k in ("K1", "K2", "K3", "paths", "K4"):
    x = r[k]
    print("  %-5s ms=%.3f frac=%s dram_frac=%s traffic=%s" % (k, x.get("avg_launch_ms") or 0, x.get("frac"), x.get("dram_frac"), x.get("traffic")))
PY
