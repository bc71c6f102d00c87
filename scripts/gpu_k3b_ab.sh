#!/bin/bash
# K3 batch kernel A/B: parity with the batch kernel forced on every size (RM_VIT_WAVE_MAX=0), then
# C2 / C5 / C2-with-turn-costs stage times against round 4.s kernel (RM_VIT_R4=1 selected it until it
# was removed; the A/B logs under profiles/r05/k3b are from then).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/k3b
mkdir -p $O
cd $R
RM_VIT_WAVE_MAX=0 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_stages.py tests/test_gpu_turns.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in new r4 new r4; do
  if [ $v = r4 ]; then export RM_VIT_R4=1; else unset RM_VIT_R4; fi
  timeout -k 10 200 python3 -u scripts/perf_probe.py --config C2 --reps 3 > $O/c2_$v.log 2>&1 || exit 1
  grep rerun $O/c2_$v.log | tail -2 | sed "s/^/$v C2 /"
done
for v in new r4; do
  if [ $v = r4 ]; then export RM_VIT_R4=1; else unset RM_VIT_R4; fi
  timeout -k 10 200 python3 -u scripts/perf_probe.py --config C5 --reps 3 > $O/c5_$v.log 2>&1 || exit 1
  grep rerun $O/c5_$v.log | tail -2 | sed "s/^/$v C5 /"
  timeout -k 10 200 python3 -u scripts/perf_probe.py --config C2 --turn 200 --reps 3 > $O/c2t_$v.log 2>&1 || exit 1
  grep rerun $O/c2t_$v.log | tail -2 | sed "s/^/$v C2turn /"
done
echo K3BDONE
