"""Diagnostic: segments of the product library vs variants/segblocks.so on a C2 sample."""
import os
import subprocess
import sys
import json
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if len(sys.argv) > 1 and sys.argv[1] == "child":
    from reporter_amd import engine, world
    path = "/tmp/dbg_c2.rmg"
    cfg = world.CONFIGS["C2"]
    if not os.path.exists(path):
        world.build_world(path, cfg["rows"], cfg["cols"], cfg["block_m"], seed=1, cell_m=cfg["cell_m"])
    tr = world.generate_traces(path, 500, cfg["n_points"], cfg["rate_s"], cfg["noise_m"], seed=1000)
    eng = engine.Engine(path, 0)
    bm = engine.BatchMatcher(eng)
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], engine.default_options(1))
    soff, segs = bm.segments()
    poff, pcnt, pool, rdist = bm.paths()
    n_states, orig = bm.states()
    _, road, s, _ = bm.candidates()
    choice, cs = bm.viterbi()
    np.savez(sys.argv[2], soff=soff, segs=segs, pcnt=pcnt, rdist=rdist, poff=poff, pool=pool, n_states=n_states,
             orig=orig, road=road, s=s, choice=choice, cs=cs, time=tr["time"], trace_off=tr["trace_off"])
    sys.exit(0)
out = {}
for name, lib in (("new", os.path.join(ROOT, "reporter_amd", "libreporter_match.so")), ("old", os.path.join(ROOT, "variants", "segblocks.so"))):
    env = dict(os.environ, REPORTER_MATCH_LIB=lib)
    f = os.path.join(ROOT, "gpurun_out", "dbg_%s.npz" % name)
    subprocess.run([sys.executable, __file__, "child", f], env=env, check=True, timeout=300)
    out[name] = np.load(f)
a, b = out["new"], out["old"]
print("seg_off equal", np.array_equal(a["soff"], b["soff"]))
sa, sb = a["segs"], b["segs"]
for f in sa.dtype.names:
    x, y = sa[f], sb[f]
    if x.dtype.kind == "f":
        x, y = x.view(np.uint64), y.view(np.uint64)
    bad = np.nonzero(x != y)[0]
    print(f, len(bad), bad[:5])
    if len(bad) and f == "start_time":
        for i in bad[:6]:
            k = np.searchsorted(a["soff"], i, side="right") - 1
            print("  seg", i, "trace", k, "run", i - a["soff"][k], "of", a["soff"][k + 1] - a["soff"][k],
                  "new", sa[i], "\n   old", sb[i])
