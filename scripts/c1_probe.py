"""C1 latency probe (diagnostic; bench.py reports the contract line): one 1,000-point 1 Hz trace
through valhalla.SegmentMatcher().Match, as bench.extras measures it, plus the engine's stage
times for the same batch.

    python scripts/c1_probe.py [--n 200]
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import valhalla  # noqa: E402
from reporter_amd import engine, world  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=200)
a = ap.parse_args()
tmp = tempfile.mkdtemp()
c1 = world.CONFIGS["C1"]
g = os.path.join(tmp, "c1.rmg")
world.build_world(g, c1["rows"], c1["cols"], c1["block_m"], seed=1, cell_m=c1["cell_m"])
tr = world.generate_traces(g, 1, c1["n_points"], c1["rate_s"], c1["noise_m"], seed=1)
req = json.dumps(world.trace_to_request(tr, 0), separators=(",", ":"))
res = {}
for coalesce in (True, False):
    valhalla.Configure(valhalla.write_config(os.path.join(tmp, "c1.json"), g, device=0, coalesce=coalesce))
    sm = valhalla.SegmentMatcher()
    for _ in range(10):
        sm.Match(req)
    lat = []
    for _ in range(a.n):
        t = time.perf_counter()
        sm.Match(req)
        lat.append((time.perf_counter() - t) * 1e3)
    lat.sort()
    res["coalesce" if coalesce else "direct"] = {"median_ms": lat[len(lat) // 2], "p90_ms": lat[int(len(lat) * 0.9)],
                                                  "min_ms": lat[0]}
    sm.close()
eng = engine.Engine(g, 0)
bm = engine.BatchMatcher(eng)
bm.set_timing(True)
for _ in range(5):
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"])
bm.reset_times()
lat = []
for _ in range(50):
    t = time.perf_counter()
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"])
    bm.segments()
    lat.append((time.perf_counter() - t) * 1e3)
lat.sort()
kt = bm.kernel_times()
res["runner_run_plus_segments_ms"] = lat[len(lat) // 2]
res["stage_ms_per_run"] = {k: round(ms / 50.0, 4) for k, (ms, n) in kt.items() if n}
print(json.dumps(res))
bm.close()
eng.close()
