"""Small-batch latency (GPU): one C1 trace through an uncoalesced SegmentMatcher.MatchMany, 200
times; run under rocprofv3 --kernel-trace --stats to split the per-batch time into kernel time
and launch / synchronisation gaps."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import valhalla  # noqa: E402
from reporter_amd import world as W  # noqa: E402

tmp = os.environ.get("TMPDIR", "/tmp")
c1 = W.CONFIGS["C1"]
g = os.path.join(tmp, "small_batch_c1.rmg")
W.build_world(g, c1["rows"], c1["cols"], c1["block_m"], seed=1, cell_m=c1["cell_m"])
tr = W.generate_traces(g, 1, c1["n_points"], c1["rate_s"], c1["noise_m"], seed=1)
req = json.dumps(W.trace_to_request(tr, 0), separators=(",", ":"))
valhalla.Configure(valhalla.write_config(os.path.join(tmp, "small_batch.json"), g, device=0, coalesce=False))
sm = valhalla.SegmentMatcher()
for _ in range(20):
    sm.MatchMany([req])
lat = []
for _ in range(200):
    t = time.perf_counter()
    sm.MatchMany([req])
    lat.append((time.perf_counter() - t) * 1e3)
lat.sort()
print("one 1,000-point trace: median %.3f ms, p10 %.3f, p90 %.3f; library %s" % (
    lat[100], lat[20], lat[180], sm.last_timing()), flush=True)
