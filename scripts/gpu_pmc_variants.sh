#!/bin/bash
# Two SQ PMC passes per variants/*.so over one C2 perf-probe run; prints the k_viterbi /
# named kernel rows (diagnostic).  $1: kernel-name filter for the summary (default all).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for lib in $R/variants/*.so; do
  n=$(basename $lib .so)
  O=$R/gpurun_out/pmcv/$n
  mkdir -p $O
  i=0
  for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
              "SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    REPORTER_MATCH_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $O/p$i -o run -- python3 $R/scripts/perf_probe.py --reps 1 --config C2 > $O/p$i.log 2>&1 || { echo "$n pass $i failed"; tail -5 $O/p$i.log; exit 1; }
  done
  echo "== $n"
  cd $R && python3 scripts/pmc_probe_summary.py $O | grep -A1 -E "${1:-.}" ; cd /tmp
done
echo ALLDONE
