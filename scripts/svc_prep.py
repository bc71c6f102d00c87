"""Write a C2 world, a Valhalla-style config and a file of /report requests (60- or 600-point
windows of C2 traces) for running reporter_amd/bin/rm_svc_client directly, e.g. under rocprofv3
(diagnostic; bench.py runs the contract lines).

    python scripts/svc_prep.py OUTDIR [--points 60] [--requests 20000]
    rocprofv3 --kernel-trace -d OUT -- reporter_amd/bin/rm_svc_client OUTDIR/conf.json OUTDIR/reqs.txt 64 4000 1000
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from reporter_amd import world  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("out")
ap.add_argument("--points", type=int, default=60)
ap.add_argument("--requests", type=int, default=20000)
ap.add_argument("--traces", type=int, default=2500)
ap.add_argument("--workers", type=int, default=None)
a = ap.parse_args()
os.makedirs(a.out, exist_ok=True)
import valhalla  # noqa: E402
c = world.CONFIGS["C2"]
g = os.path.join(a.out, "c2.rmg")
world.build_world(g, c["rows"], c["cols"], c["block_m"], seed=1, cell_m=c["cell_m"])
tr = world.generate_traces(g, a.traces, c["n_points"], 1.0, 5.0, seed=1000)
if a.points >= c["n_points"]:
    reqs, _ = bench.request_jsons(tr, a.requests)
else:
    reqs, _ = bench.window_requests(tr, a.requests, a.points)
with open(os.path.join(a.out, "reqs.txt"), "w") as f:
    for r in reqs:
        f.write((r.decode() if isinstance(r, bytes) else r) + "\n")
valhalla.write_config(os.path.join(a.out, "conf.json"), g, device=0, coalesce=True, coalesce_workers=a.workers)
print("wrote", len(reqs), "requests to", a.out)
