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


@pytest.mark.parametrize("mode,radius", [(0, 700.0), (3, 400.0)])
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
    got = eng.ball_lookup(mode, f, rd)
    want = np.empty((len(f), 2), np.uint64)
    _lib.check(_lib.lib().rm_balls_lookup(os.fsencode(slice_graph), mode, radius, len(f), f.ctypes.data,
                                          rd.ctypes.data, want.ctypes.data))
    inside = (want != np.uint64(2**64 - 1)).any(axis=1)
    assert inside.sum() > 1000 and (~inside).sum() > 100, (inside.sum(), len(f))
    np.testing.assert_array_equal(got, want)
    bm.close()
    eng.close()
