"""K3 at service batch sizes (diagnostic): per-stage ms of batches of T C2 traces (600 points)
through the engine API, T in 1..256, with the stage timers on."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
from reporter_amd import engine, world  # noqa: E402

tmp = os.environ.get("TMPDIR", "/tmp")
c = world.CONFIGS["C2"]
g = os.path.join(tmp, "k3_small_c2.rmg")
world.build_world(g, c["rows"], c["cols"], c["block_m"], seed=1, cell_m=c["cell_m"])
Ts = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1,8,38,150,256").split(",")]
full = world.generate_traces(g, max(Ts), c["n_points"], 1.0, 5.0, seed=1000)
eng = engine.Engine(g, 0)
for T in Ts:
    o = int(full["trace_off"][T])
    sub = {k: full[k][:o] for k in ("lon", "lat", "time", "accuracy")}
    bm = engine.BatchMatcher(eng)
    bm.run(full["trace_off"][:T + 1], sub["lon"], sub["lat"], sub["time"], sub["accuracy"])
    bm.set_timing(True)
    for _ in range(5):
        bm.rerun()
    bm.reset_times()
    reps = 50
    t = time.perf_counter()
    for _ in range(reps):
        bm.rerun()
    dt = (time.perf_counter() - t) / reps
    kt = bm.kernel_times()
    print("T=%d wall %.3f ms  " % (T, dt * 1e3) + " ".join("%s=%.3f" % (k, v[0] / reps) for k, v in kt.items()), flush=True)
    bm.close()
