"""The JSON boundary alone (bench.py's json_boundary line): C2 traces as /report JSON through
MatchMany without coalescing; prints the wall time and the library's own timing of each call."""
import argparse, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
import valhalla
from reporter_amd import world

ap = argparse.ArgumentParser()
ap.add_argument("--traces", type=int, default=10000)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
c = world.CONFIGS["C2"]
os.makedirs("/tmp/rmprobe", exist_ok=True)
gp = "/tmp/rmprobe/C2.rmg"
world.build_config_graph("C2", gp, seed=1)
tr = world.generate_traces(gp, a.traces, c["n_points"], c["rate_s"], c["noise_m"], seed=7)
reqs, P = bench.request_jsons(tr, a.traces)
print("requests %d, points %d, %.0f MB" % (len(reqs), P, sum(map(len, reqs)) / 1e6), flush=True)
valhalla.Configure(valhalla.write_config("/tmp/rmprobe/c2_nc.json", gp, device=0, coalesce=False))
sm = valhalla.SegmentMatcher()
t = time.perf_counter()
sm.MatchMany(reqs)
print("first %.1f ms %s" % ((time.perf_counter() - t) * 1e3, sm.last_timing()), flush=True)
for r in range(a.reps):
    t = time.perf_counter()
    outs = sm.MatchMany(reqs)
    dt = time.perf_counter() - t
    lt = sm.last_timing()
    print("call %.1f ms  %.1f M points/s  library %.1f ms (%.1f M/s)  %s" % (
        dt * 1e3, P / dt / 1e6, lt["total_ms"], P / lt["total_ms"] / 1e3,
        " ".join("%s=%.1f" % (k, v) for k, v in lt.items())), flush=True)
