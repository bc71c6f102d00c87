"""Route balls built on the GPU (k_ball_build) against the host build (GPU).

Country-scale graphs at moderate radii (C4: 16.6 M nodes, tens of nodes per ball) build
their route-ball tables on the device instead of 16 host threads (21 s for C4 at 700 m in
round 1).  Row order inside a table may differ from the host build, so the tables are
compared the way K2 uses them: every probed (node, road) pair returns the same two keys as
the host build (rm_balls_lookup), including "outside the ball" answers.
"""
import ctypes as C
import os
import time

import numpy as np
import pytest

from reporter_amd import _lib, engine, graphfile, world

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def slice_graph(built_lib, tmpdir_session):
    path = str(tmpdir_session / "balls_slice.rmg")
    world.build_world(path, 1000, 1000, 250.0, seed=1, cell_m=250.0)
    return path


def _pairs(g, n_from, seed):
    """(from node, road) pairs around random nodes: every road with an endpoint within two
    grid steps of the node (inside and just outside a 400-700 m ball)."""
    rng = np.random.default_rng(seed)
    cols = 1000
    r0, r1 = g["road_node0"].astype(np.int64), g["road_node1"].astype(np.int64)
    inc = {}
    for r, (a, b) in enumerate(zip(r0.tolist(), r1.tolist())):
        inc.setdefault(a, []).append(r)
        inc.setdefault(b, []).append(r)
    f, rd = [], []
    for _ in range(n_from):
        i, j = rng.integers(3, cols - 3, size=2)
        u = int(i * cols + j)
        for di in range(-3, 4):
            for dj in range(-3, 4):
                for r in inc.get(int((i + di) * cols + (j + dj)), []):
                    f.append(u)
                    rd.append(r)
    return np.array(f, np.uint32), np.array(rd, np.uint32)


@pytest.mark.parametrize("mode,radius", [(0, 700.0), (3, 400.0), (0, 1000.0)])   # 1000 m: C4's default
def test_gpu_built_balls_equal_host_build(slice_graph, mode, radius):
    g = graphfile.load(slice_graph)
    eng = engine.Engine(slice_graph, 0)
    eng.set_ball_radius(radius)
    tr = world.generate_traces(slice_graph, 16, 60, rate_s=5.0, noise_m=5.0, seed=3,
                               mode="bicycle" if mode == 3 else "auto")
    bm = engine.BatchMatcher(eng)
    t = time.time()
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], engine.default_options(1, mode=mode))
    st = eng.ball_stats(mode)
    print("mode", mode, "radius", radius, "first run (incl. ball build) %.2fs" % (time.time() - t), st, flush=True)
    assert st["built_on_gpu"] and st["keys"] > 0 and st["radius_m"] == radius
    f, rd = _pairs(g, 400, seed=mode)
    got, gpred = eng.ball_lookup(mode, f, rd, preds=True)
    want = np.empty((len(f), 2), np.uint64)
    wpred = np.empty((len(f), 2), np.uint8)
    _lib.check(_lib.lib().rm_balls_lookup(os.fsencode(slice_graph), mode, radius, len(f), f.ctypes.data,
                                          rd.ctypes.data, want.ctypes.data, wpred.ctypes.data))
    inside = (want != np.uint64(2**64 - 1)).any(axis=1)
    assert inside.sum() > 1000 and (~inside).sum() > 100, (inside.sum(), len(f))
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(gpred, wpred)   # the rows' canonical predecessors (path walk)
    assert int((wpred < 7).sum()) > 1000
    bm.close()
    eng.close()


def test_modes_share_the_table_budget(built_lib, tmpdir_session, monkeypatch):
    """VERDICT r02 / ADVICE r02 (route-ball memory): the tables of every mode a batch uses come
    out of ONE budget (RM_BALL_TOTAL_GB here, half the HBM by default).  auto and bus share one
    build; bicycle gets the next radius that fits what is left; pedestrian, with nothing left,
    gets no tables and runs in the search tiers.  A mixed batch matches the oracle bit for bit."""
    import meili_oracle as mo
    from parity_util import compare_all
    cfg = world.CONFIGS["C2"]
    path = str(tmpdir_session / "budget_c2.rmg")
    world.build_world(path, cfg["rows"], cfg["cols"], cfg["block_m"], seed=1, cell_m=cfg["cell_m"])
    sample = (C.c_double * 3)()
    _lib.check(_lib.lib().rm_graph_ball_sample(os.fsencode(path), 0, 2000.0, sample))
    auto_gib = sample[1] / float(1 << 30)
    # room for auto at 2000 m (+10 % sampling margin) and a little more
    monkeypatch.setenv("RM_BALL_TOTAL_GB", "%.4f" % (auto_gib * 1.1 + 0.25))
    eng = engine.Engine(path, 0)
    modes = [("auto", 0), ("bus", 1), ("bicycle", 3), ("pedestrian", 4)]
    sets = [world.generate_traces(path, 24, 200, rate_s=2.0, noise_m=5.0, seed=40 + m, mode=name) for name, m in modes]
    tr = world.concat_traces(*sets)
    opts = engine.default_options(4)
    for q, (_, m) in enumerate(modes):
        opts[q]["mode"] = m
    trace_opt = np.repeat(np.arange(4, dtype=np.uint32), 24)
    bm = engine.BatchMatcher(eng)
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, trace_opt)
    st = {m: eng.ball_stats(m) for _, m in modes}
    print("per-mode tables", st, flush=True)
    assert st[0]["radius_m"] == 2000.0 and st[0]["keys"] > 0
    assert st[1]["radius_m"] == 2000.0 and st[1]["entries"] == st[0]["entries"]   # shared build
    assert 0.0 < st[3]["radius_m"] < 2000.0 and st[3]["keys"] > 0
    assert st[4]["radius_m"] < 2000.0
    used_gib = (st[0]["entries"] + st[3]["entries"] + st[4]["entries"]) * 16 / float(1 << 30)
    assert used_gib <= auto_gib * 1.1 + 0.25
    ref = mo.match(graphfile.load(path), mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"],
                                                  opts, trace_opt))
    c = compare_all(bm, ref, tr["trace_off"])
    assert c["chained"] > 5000, c
    bm.close()
    eng.close()
    # a budget nothing fits: no mode gets tables, every transition runs in the search tiers
    monkeypatch.setenv("RM_BALL_TOTAL_GB", "0.0001")
    eng = engine.Engine(path, 0)
    bm = engine.BatchMatcher(eng)
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, trace_opt)
    assert all(eng.ball_stats(m)["radius_m"] == 0.0 for _, m in modes)
    compare_all(bm, ref, tr["trace_off"])
    bm.close()
    eng.close()
