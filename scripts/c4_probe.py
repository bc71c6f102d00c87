"""C4 (the 16.6 M-node country graph) beyond its bench line: the route-ball
radius each of auto / bicycle / pedestrian gets under the shared table budget when all three are
built, and the step throughput of 30 s traces (C3's sampling, bounds up to 2 km: beyond the 1000 m
tables, so the search tiers take those pairs) next to C4's own 5 s traces.  Diagnostic."""
import argparse, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from reporter_amd import engine, world

ap = argparse.ArgumentParser()
ap.add_argument("--traces", type=int, default=125000)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
cfg = world.CONFIGS["C4"]
os.makedirs("/tmp/rmprobe", exist_ok=True)
gp = "/tmp/rmprobe/C4.rmg"
t = time.time()
world.build_config_graph("C4", gp, seed=1)
print("C4 graph %.1fs" % (time.time() - t), world.graph_info(gp), flush=True)
eng = engine.Engine(gp, 0)


def run(name, tr, opts, trace_opt=None):
    bm = engine.BatchMatcher(eng)
    T = len(tr["trace_off"]) - 1
    t = time.time()
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts,
           trace_opt if trace_opt is not None else np.zeros(T, np.uint32))
    first = time.time() - t
    bm.set_timing(True)
    bm.reset_times()
    t = time.time()
    for _ in range(a.reps):
        bm.rerun()
    dt = (time.time() - t) / a.reps
    kt = bm.kernel_times()
    P = len(tr["lon"])
    print("%s: %d traces, %d points, first %.2fs, step %.2f ms, %.1f M points/s  %s  tiers %s" % (
        name, T, P, first, dt * 1e3, P / dt / 1e6, " ".join("%s=%.2f" % (k, v[0] / a.reps) for k, v in kt.items()),
        bm.route_tiers()), flush=True)
    bm.close()


# 1. three modes in one batch: the radius each gets under the shared budget
names = [("auto", 0), ("bicycle", 3), ("pedestrian", 4)]
sets = [world.generate_traces(gp, 20000, cfg["n_points"], cfg["rate_s"], cfg["noise_m"], seed=4200 + m, mode=nm)
        for nm, m in names]
tr3 = world.concat_traces(*sets)
opts3 = engine.default_options(3, search_radius=cfg["search_radius"])
for q, (_, m) in enumerate(names):
    opts3[q]["mode"] = m
run("three modes (20 k traces each, 5 s)", tr3, opts3, np.repeat(np.arange(3, dtype=np.uint32), 20000))
for nm, m in names:
    print("ball", nm, eng.ball_stats(m), flush=True)
# 2. 30 s traces on C4 (auto), and C4's own 5 s traces at the same trace count
c3 = world.CONFIGS["C3"]
tr30 = world.generate_traces(gp, a.traces, c3["n_points"], c3["rate_s"], c3["noise_m"], seed=77)
run("30 s traces (C3 sampling)", tr30, engine.default_options(1, search_radius=c3["search_radius"]))
tr5 = world.generate_traces(gp, a.traces, cfg["n_points"], cfg["rate_s"], cfg["noise_m"], seed=78)
run("5 s traces (C4 sampling)", tr5, engine.default_options(1, search_radius=cfg["search_radius"]))
