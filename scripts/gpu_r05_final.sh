#!/bin/bash
# Round-5 evidence run: the GPU suite, C2 kernel stats + PMC passes + the bench line carrying that
# traffic (scripts/gpu_pmc_cfg.sh), the default bench line, the turn-cost bench line is part of
# the default run.  Outputs under gpurun_out/r05_final (copied into profiles/r05 afterwards).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05_final
mkdir -p $O
cd $R
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { echo "tests failed"; tail -20 $O/pytest_gpu.txt; exit 1; }
  echo "tests done"
fi
bash scripts/gpu_pmc_cfg.sh C2 10000 r05_c2 || exit 1
cd $R
timeout -k 10 900 python -u bench.py > $O/bench_c2_default.json 2> $O/bench_c2_default.err || { echo "bench failed"; tail -20 $O/bench_c2_default.err; exit 1; }
echo FINALDONE
