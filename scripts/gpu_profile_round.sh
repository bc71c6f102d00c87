#!/bin/bash
# Round profile session: every -m gpu test, smoke, rocprofv3 kernel stats of the C2 bench, the
# PMC passes (each its own run) and their summary, the C2 bench line with the PMC traffic of
# this same build, then the C3 / C4 bench lines.  Every GPU step has its own time limit and a
# failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail 3 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?
  grep -E "passed|failed" $O/pytest_gpu.log | tail -2
  [ $rc -ne 0 ] && { grep -E "FAILED|ERROR" $O/pytest_gpu.log | head; exit 1; }
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-extras --parts-extra 0 > $O/prof_kt.log 2>&1 || { echo "kt failed"; tail -5 $O/prof_kt.log; exit 1; }
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  name=$(echo $pass | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d $O/pmc_$name -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras --parts-extra 0 > $O/pmc_$name.log 2>&1 || { echo "pmc $pass failed"; tail -5 $O/pmc_$name.log; exit 1; }
done
cd $R
python scripts/pmc_summary.py $O $O/summary --config C2 --traces 10000 --streams 1 > $O/summary.log 2>&1 || { echo "summary failed"; tail -5 $O/summary.log; exit 1; }
timeout -k 10 400 python -u bench.py --traffic-json $O/summary/pmc_routes_c2.json > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
[ -z "$SKIP_CFGS" ] && { bash scripts/gpu_bench_cfgs.sh C3 C4 || exit 1; }
echo ALLDONE
