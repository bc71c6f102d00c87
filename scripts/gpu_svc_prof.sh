#!/bin/bash
# Kernel timeline of the coalesced service at the Java batcher's request size (60-point /report
# requests, 64 C-ABI clients): rocprofv3 kernel trace of rm_svc_client, CSV under gpurun_out/svcprof.
# Analyse with scripts/svc_timeline.py gpurun_out/svcprof.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
PTS=${1:-60}; CL=${2:-64}
mkdir -p $R/gpurun_out/svcprof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 -u $R/scripts/svc_prep.py /tmp/svcprep --points $PTS --requests 8000 --traces 1200 > $R/gpurun_out/svcprof/prep.log 2>&1 || exit 1
timeout -k 10 120 $R/reporter_amd/bin/rm_svc_client /tmp/svcprep/conf.json /tmp/svcprep/reqs.txt $CL 8000 2000 > $R/gpurun_out/svcprof/plain.json 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/svcprof -o run -- $R/reporter_amd/bin/rm_svc_client /tmp/svcprep/conf.json /tmp/svcprep/reqs.txt $CL 3000 1000 > $R/gpurun_out/svcprof/prof.json 2>&1
