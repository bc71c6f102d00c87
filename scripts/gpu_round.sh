#!/bin/bash
# One GPU session: smoke, bench, rocprofv3 kernel stats, PMC passes (each pass its own run).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_kt.log 2>&1 || { echo "kt failed"; exit 1; }
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  name=$(echo $pass | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d $O/pmc_$name -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_$name.log 2>&1 || { echo "pmc $pass failed"; exit 1; }
done
echo ALLDONE
