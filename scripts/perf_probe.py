"""Quick engine timing on a BASELINE config (diagnostic; bench.py is the contract)."""
import argparse, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from reporter_amd import engine, world

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C2")
ap.add_argument("--traces", type=int, default=0)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--split", type=int, default=0, help="also time M concurrent runners (streams) over sub-batches")
ap.add_argument("--ab-locality", action="store_true", help="also time the same batch with the locality order off / on")
ap.add_argument("--ab-modes", default="0,1,0,1", help="locality modes the A/B cycles through")
ap.add_argument("--ball-radius", type=float, default=None, help="route-ball radius in m (0: the search tiers alone)")
ap.add_argument("--turn", type=float, default=0.0, help="turn_penalty_factor of every trace (meili's auto default: 200)")
ap.add_argument("--only", default="", help="time only these stages (comma list, bench.py style: e.g. routes); "
                "with every stage timed the event pairs shift the stages by up to ~0.1 ms")
a = ap.parse_args()
c = dict(world.CONFIGS[a.config])
if a.traces:
    c["n_traces"] = a.traces
os.makedirs("/tmp/rmprobe", exist_ok=True)
gp = "/tmp/rmprobe/%s.rmg" % a.config
t = time.time()
world.build_config_graph(a.config, gp, seed=1)
print("world", world.graph_info(gp), "%.1fs" % (time.time() - t), flush=True)
t = time.time()
tr = world.generate_traces(gp, c["n_traces"], c["n_points"], c["rate_s"], c["noise_m"], seed=7)
print("traces %d pts %.1fs" % (len(tr["lon"]), time.time() - t), flush=True)
eng = engine.Engine(gp, 0)
if a.ball_radius is not None:
    eng.set_ball_radius(a.ball_radius)
bm = engine.BatchMatcher(eng)
opts = engine.default_options(1, search_radius=c["search_radius"], turn_penalty_factor=a.turn)
t = time.time()
bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts)
print("first run %.3fs" % (time.time() - t), bm.sizes(), flush=True)
print("route tiers", bm.route_tiers(), "balls", eng.ball_stats(0), flush=True)
if a.only:
    import time as _t
    for _ in range(3):
        bm.rerun()
    engine_sync = getattr(bm, "sync", None)
    bm.set_timing(False)
    t = _t.time()
    for _ in range(a.reps):
        bm.rerun()
    wall = (_t.time() - t) / a.reps
    bm.set_timing_stages(tuple(a.only.split(",")))
    bm.reset_times()
    for _ in range(a.reps):
        bm.rerun()
    kt = bm.kernel_times()
    bm.set_timing(False)
    print("only %.4f ms/step wall (untimed)  " % (wall * 1e3) +
          " ".join("%s=%.3fms" % (k, kt[k][0] / a.reps) for k in a.only.split(",")), flush=True)
    sys.exit(0)
bm.set_timing(True)
for r in range(a.reps):
    bm.reset_times()
    t = time.time()
    bm.rerun()
    dt = time.time() - t
    kt = bm.kernel_times()
    print("rerun %.4fs  %.1f Mpts/s  " % (dt, len(tr["lon"]) / dt / 1e6) +
          " ".join("%s=%.2fms" % (k, v[0]) for k, v in kt.items()), flush=True)

if a.ab_locality:
    for mode in [int(x) for x in a.ab_modes.split(",")]:
        bm.set_locality(mode)
        bm.rerun()
        bm.reset_times()
        t = time.time()
        for r in range(a.reps):
            bm.rerun()
        dt = (time.time() - t) / a.reps
        kt = bm.kernel_times()
        print("locality=%d used=%d %.4fs  %.1f Mpts/s  " % (mode, bm.locality_used(), dt, len(tr["lon"]) / dt / 1e6) +
              " ".join("%s=%.2fms" % (k, v[0] / a.reps) for k, v in kt.items()), flush=True)
if a.split > 1:
    import threading
    T = len(tr["trace_off"]) - 1
    bounds = np.linspace(0, T, a.split + 1).astype(int)
    bms = []
    for m in range(a.split):
        t0, t1 = bounds[m], bounds[m + 1]
        o0, o1 = int(tr["trace_off"][t0]), int(tr["trace_off"][t1])
        sub = {k: tr[k][o0:o1] for k in ("lon", "lat", "time", "accuracy")}
        off = tr["trace_off"][t0:t1 + 1] - o0
        b2 = engine.BatchMatcher(eng)
        b2.run(off, sub["lon"], sub["lat"], sub["time"], sub["accuracy"], opts)
        bms.append(b2)
    for r in range(a.reps + 1):
        ths = [threading.Thread(target=b2.rerun) for b2 in bms]
        t = time.time()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        dt = time.time() - t
        print("split %d: %.4fs  %.1f Mpts/s" % (a.split, dt, len(tr["lon"]) / dt / 1e6), flush=True)
