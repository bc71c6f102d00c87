"""Service ceiling probe: the C-ABI client (reporter_amd/bin/rm_svc_client) on C2 requests of
600 and 60 points at several client counts (diagnostic; bench.py reports the contract lines)."""
import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from reporter_amd import world  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--clients", default="1,16,64,256")
ap.add_argument("--traces", type=int, default=2000)
ap.add_argument("--n", type=int, default=4096)
ap.add_argument("--workers", default="1", help="coalescer dispatcher threads to try")
a = ap.parse_args()
tmp = tempfile.mkdtemp()
c = world.CONFIGS["C2"]
g = os.path.join(tmp, "c2.rmg")
world.build_world(g, c["rows"], c["cols"], c["block_m"], seed=1, cell_m=c["cell_m"])
tr = world.generate_traces(g, a.traces, c["n_points"], 1.0, 5.0, seed=1000)
r600, _ = bench.request_jsons(tr, a.traces)
r60, _ = bench.window_requests(tr, a.n * 2, 60)
for name, rq in (("600pt", r600), ("60pt", r60)):
    for wk in [int(x) for x in a.workers.split(",")]:
        for cl in [int(x) for x in a.clients.split(",")]:
            res = bench.client_service(g, tmp, rq, cl, a.n, min(2048, a.n // 2), workers=wk)
            keep = {k: res.get(k) for k in ("requests_per_s", "points_per_s", "requests_per_batch", "ms_per_batch",
                                            "latency_ms", "dispatcher_ms_per_batch", "error")}
            print(name, "workers", wk, "clients", cl, keep, flush=True)
