#!/bin/bash
# Round 6: the GPU suite, then the default bench line (C2 + turn costs + service extras).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06_suite
mkdir -p $O
cd $R
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "tests failed"; tail -30 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
  python - <<PY
import json; d = json.load(open("$O/bench.json"))
print("value %.1f M  step %.3f ms  K2 %.3f ms frac %.3f" % (d["value"] / 1e6, d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"]))
t = d.get("turn_costs") or {}
print("turn value %.1f M  step %.3f  K2 %s" % (t.get("value", 0) / 1e6, t.get("ms_per_step", 0), (t.get("roofline") or {}).get("avg_launch_ms")))
for k, v in d["kernels_ms_per_step"].items(): print("  ", k, round(v, 3))
s = d.get("service_throughput") or {}
print("service", json.dumps(s)[:600])
PY
fi
echo SUITEDONE
