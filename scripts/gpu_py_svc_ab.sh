#!/bin/bash
# Python 60-point service clients: valhalla._match vs the ctypes path (RM_PY_CTYPES=1), twice each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pysvc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -u $R/scripts/svc_prep.py /tmp/svcprep --points 60 --requests 20000 > $O/prep.log 2>&1 || { tail -5 $O/prep.log; exit 1; }
for rep in 1 2; do
  for v in "RM_X=fast" "RM_PY_CTYPES=1"; do
    env $v timeout -k 10 200 python3 -u $R/scripts/py_svc.py /tmp/svcprep 64 8192 > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -5 $O/${v}_$rep.err; exit 1; }
    echo "$v $rep $(cat $O/${v}_$rep.json)"
  done
done
echo PYSVCDONE
