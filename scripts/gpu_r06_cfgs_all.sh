#!/bin/bash
# Round-6 non-C2 evidence of the final engine in one call: PMC passes + traffic-carrying bench lines
# at the PMC sizes (C3 and C4 at 125 k traces, CITY30 at its 100 k), then the default-size lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash scripts/gpu_r06_cfgs.sh pmc || exit 1
bash scripts/gpu_r06_cfgs.sh lines || exit 1
echo CFGSALLDONE
