#!/bin/bash
# Round-6 evidence of the final engine: the GPU suite, C2 kernel stats + PMC passes + the bench line
# carrying that traffic, the same at turn_penalty_factor 200, then the default bench line (which
# reads both PMC summaries from profiles/r06 -- copied here on the box first).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06_final
mkdir -p $O $R/profiles/r06
cd $R
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "tests failed"; tail -20 $O/pytest_gpu.txt; exit 1; }
  tail -1 $O/pytest_gpu.txt
fi
bash scripts/gpu_pmc_cfg.sh C2 10000 r06_c2 || exit 1
cp $R/gpurun_out/r06_c2/summary/pmc_r06_c2.json $R/profiles/r06/pmc_routes_c2.json
TURN=200 bash scripts/gpu_pmc_cfg.sh C2 10000 r06_c2_turn200 --turn-penalty 200 || exit 1
cp $R/gpurun_out/r06_c2_turn200/summary/pmc_r06_c2_turn200.json $R/profiles/r06/pmc_routes_c2_turn200.json
cd $R
timeout -k 10 900 python -u bench.py > $O/bench_c2_default.json 2> $O/bench_c2_default.err || { echo "bench failed"; tail -20 $O/bench_c2_default.err; exit 1; }
python - <<PY
import json; d = json.load(open("$O/bench_c2_default.json"))
r = d["roofline"]; t = d.get("turn_costs") or {}
print("C2 %.1f M points/s, %.3f ms/step; K2 %.3f ms frac %.3f dram %s traffic %s" % (d["value"] / 1e6, d["ms_per_step"], r["avg_launch_ms"], r["frac"], r.get("dram_frac"), r.get("traffic")))
tr = t.get("roofline") or {}
print("turn %.1f M points/s, %.3f ms/step; K2 %s frac %s dram %s" % (t.get("value", 0) / 1e6, t.get("ms_per_step", 0), tr.get("avg_launch_ms"), tr.get("frac"), tr.get("dram_frac")))
PY
echo FINALDONE
