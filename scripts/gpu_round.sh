#!/bin/bash
# One GPU session: parity tests, smoke, rocprofv3 kernel stats, PMC passes (each pass its
# own run), their summary, then the bench line with the PMC traffic of this same build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_kt -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_kt.log 2>&1 || { echo "kt failed"; exit 1; }
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  name=$(echo $pass | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d $O/pmc_$name -o run -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $O/pmc_$name.log 2>&1 || { echo "pmc $pass failed"; exit 1; }
done
cd $R
python scripts/pmc_summary.py $O $O/summary --config C2 --traces 10000 > $O/summary.log 2>&1 || { echo "summary failed"; exit 1; }
timeout -k 10 300 python -u bench.py --traffic-json $O/summary/pmc_routes_c2.json > $O/bench.json 2> $O/bench.err || { echo "bench failed"; exit 1; }
cat $O/bench.json
timeout -k 10 600 python -u bench.py --config C3 --traces 125000 --steps 5 --warmup 1 > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench C3 failed"; exit 1; }
timeout -k 10 900 python -u bench.py --config C4 --traces 125000 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || { echo "bench C4 failed"; exit 1; }
echo ALLDONE
