#!/bin/bash
# Profiles of the current build (no tests): rocprofv3 kernel stats of the bench, PMC passes
# (one counter group per run), their summary (engine sha), the C2 bench line carrying that
# traffic, then C3 and C4 bench lines.  $1: output dir under gpurun_out (default prof).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-prof}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras > $O/prof_kt.log 2>&1 || { echo "kt failed"; tail -5 $O/prof_kt.log; exit 1; }
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  name=$(echo $pass | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d $O/pmc_$name -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > $O/pmc_$name.log 2>&1 || { echo "pmc $pass failed"; tail -5 $O/pmc_$name.log; exit 1; }
done
cd $R
python3 scripts/pmc_summary.py $O $O/summary --config C2 --traces 10000 > $O/summary.log 2>&1 || { echo "summary failed"; tail -20 $O/summary.log; exit 1; }
timeout -k 10 300 python3 -u bench.py --traffic-json $O/summary/pmc_routes_c2.json > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench failed"; tail -20 $O/bench_c2.err; exit 1; }
cat $O/bench_c2.json
for C in C3 C4; do
  timeout -k 10 500 python3 -u bench.py --config $C --no-extras > $O/bench_$C.json 2> $O/bench_$C.err || { echo "bench $C failed"; tail -20 $O/bench_$C.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench_$C.json'))
print('$C', round(d['value']/1e6,1), 'Mpts/s', round(d['ms_per_step'],2), 'ms', d['kernels_ms_per_step'])"
done
echo ALLDONE
