"""Route balls (K2's lookup tier, reporter_amd/csrc/balls.cpp) on the CPU.

The table of node u must hold, for every road with an endpoint whose shortest
lexicographic (dist cm, time ms) key from u has distance <= radius, exactly those keys —
the values a bounded Dijkstra of the reference matcher (meili, simple_reporter.py:166)
settles the endpoints with when started at u with key 0 — and nothing beyond the radius.  Checked
here against an independent heapq Dijkstra over the graph file, per travel mode, through
the same probe sequence the GPU kernel uses (rm_balls_lookup).
"""
import ctypes as C
import heapq
import os

import numpy as np
import pytest

from reporter_amd import _lib, graphfile

KEY_INF = (1 << 64) - 1
ACCESS = {0: 1, 1: 1, 2: 1, 3: 2, 4: 4}     # rm_common.hpp mode_access
SPEED_CAP = {0: 0xFFFF, 1: 0xFFFF, 2: 450, 3: 180, 4: 51}   # mode_speed_dkph caps (0.1 km/h)


def _edge_keys(g, mode):
    e = g["edges"].reshape(-1, 4).astype(np.uint64)
    tgt, ln, info = e[:, 0], e[:, 1], e[:, 2]
    ok = ((info >> 16) & 7) & ACCESS[mode] != 0
    dk = np.minimum(info & 0xFFFF, SPEED_CAP[mode])
    t = (ln * 360) // np.maximum(dk, 1)
    return tgt.astype(np.int64), np.where(ok, (ln << np.uint64(32)) | t, np.uint64(KEY_INF))


def _dijkstra(g, tgt, key, u, radius_cm):
    off = g["node_off"]
    lab = {u: 0}
    pq = [(0, u)]
    done = {}
    while pq:
        k, x = heapq.heappop(pq)
        if x in done:
            continue
        done[x] = k
        for e in range(off[x], off[x + 1]):
            if int(key[e]) == KEY_INF:
                continue
            nk = k + int(key[e])
            if (nk >> 32) > radius_cm:
                continue
            v = int(tgt[e])
            if nk < lab.get(v, KEY_INF):
                lab[v] = nk
                heapq.heappush(pq, (nk, v))
    return done


def _lookup(path, mode, radius_m, fr, road, preds=False):
    fr = np.ascontiguousarray(fr, np.uint32)
    road = np.ascontiguousarray(road, np.uint32)
    out = np.empty(2 * len(fr), np.uint64)
    pr = np.empty(2 * len(fr), np.uint8)
    _lib.check(_lib.lib().rm_balls_lookup(os.fsencode(path), mode, radius_m, len(fr), fr.ctypes.data,
                                          road.ctypes.data, out.ctypes.data, pr.ctypes.data if preds else None))
    return (out.reshape(-1, 2), pr.reshape(-1, 2)) if preds else out.reshape(-1, 2)


def _pred_index(g, key, done, u, v):
    """Canonical predecessor of v in the search from u, as the index among v's in-edges in
    edge-id order (rm_common.hpp kBallRoadBits): the first usable edge x -> v with
    key(u -> x) + key(x -> v) == key(u -> v); 7 for u itself, outside the ball, or index >= 7."""
    if v == u or v not in done:
        return 7
    ins = _in_edges(g)[v]
    for i, (e, x) in enumerate(ins[:7]):
        if int(key[e]) != KEY_INF and x in done and done[x] + int(key[e]) == done[v]:
            return i
    return 7


_IN = {}


def _in_edges(g):
    k = id(g)
    if k not in _IN:
        off = g["node_off"]
        tgt = g["edges"].reshape(-1, 4)[:, 0]
        ins = {}
        for x in range(len(off) - 1):
            for e in range(off[x], off[x + 1]):
                ins.setdefault(int(tgt[e]), []).append((e, x))
        for v in ins:
            ins[v].sort()
        _IN.clear()
        _IN[k] = ins
    return _IN[k]


@pytest.mark.parametrize("mode,radius_m", [(0, 400.0), (0, 150.0), (3, 400.0), (4, 250.0), (0, 655.0), (0, 2000.0), (4, 2000.0)])
def test_ball_rows_match_dijkstra(small_world, mode, radius_m):
    """Row of road r in the table of node u = keys from u to r's node0 and node1."""
    g = graphfile.load(small_world)
    tgt, key = _edge_keys(g, mode)
    n0, n1 = g["road_node0"], g["road_node1"]
    R = len(n0)
    rng = np.random.default_rng(mode * 7 + int(radius_m))
    fr, roads, want, wpred = [], [], [], []
    for u in rng.choice(g.n_nodes, 50, replace=False):
        done = _dijkstra(g, tgt, key, int(u), int(radius_m * 100))
        near = np.nonzero(np.isin(n0, list(done)) | np.isin(n1, list(done)))[0]
        for r in np.concatenate([near, rng.choice(R, 20)]):
            fr.append(u)
            roads.append(r)
            want.append((done.get(int(n0[r]), KEY_INF), done.get(int(n1[r]), KEY_INF)))
            inside = any(int(x) in done for x in (n0[r], n1[r]))
            wpred.append((_pred_index(g, key, done, int(u), int(n0[r])) if inside else 7,
                          _pred_index(g, key, done, int(u), int(n1[r])) if inside else 7))
    got, pred = _lookup(small_world, mode, radius_m, fr, roads, preds=True)
    np.testing.assert_array_equal(got, np.array(want, np.uint64))
    assert int(np.sum(got != np.uint64(KEY_INF))) > 200
    # the rows' canonical predecessors (what the path walk follows)
    np.testing.assert_array_equal(pred, np.array(wpred, np.uint8))
    assert int(np.sum(pred < 7)) > 200


def test_ball_radius_zero_keeps_only_self(small_world):
    g = graphfile.load(small_world)
    r = int(np.nonzero(g["road_node0"] == 0)[0][0])
    other = int(g["road_node1"][r])
    got = _lookup(small_world, 0, 0.0, [0, other], [r, r])
    assert list(got[0]) == [0, KEY_INF] and list(got[1]) == [KEY_INF, 0]


def test_auto_radius_covers_default_breakage(small_world, tmpdir_session, monkeypatch):
    """A city graph gets 2000 m balls (meili's default breakage distance: every default
    bound is a probe); a graph too large for the table budget per mode (72 GiB, or
    RM_BALL_BUDGET_GB) gets a smaller radius."""
    import ctypes
    r = ctypes.c_double()
    _lib.check(_lib.lib().rm_graph_auto_ball_radius(os.fsencode(small_world), ctypes.byref(r)))
    assert r.value == 2000.0
    from reporter_amd import world
    big = str(tmpdir_session / "auto_r_big.rmg")
    world.build_world(big, 1400, 1400, 250.0, seed=2, cell_m=250.0)   # 2 M nodes
    _lib.check(_lib.lib().rm_graph_auto_ball_radius(os.fsencode(big), ctypes.byref(r)))
    assert r.value == 2000.0
    monkeypatch.setenv("RM_BALL_BUDGET_GB", "16")
    _lib.check(_lib.lib().rm_graph_auto_ball_radius(os.fsencode(big), ctypes.byref(r)))
    assert 400.0 <= r.value < 2000.0
    assert _lib.lib().rm_graph_auto_ball_radius(b"/nonexistent.rmg", ctypes.byref(r)) != 0


def test_ball_lookup_errors(small_world):
    one = np.zeros(1, np.uint32)
    out = np.zeros(2, np.uint64)
    L = _lib.lib()
    assert L.rm_balls_lookup(os.fsencode(small_world), 9, 100.0, 1, one.ctypes.data, one.ctypes.data, out.ctypes.data, None) != 0
    assert L.rm_balls_lookup(os.fsencode(small_world), 0, 20000.0, 1, one.ctypes.data, one.ctypes.data, out.ctypes.data, None) != 0
    big = np.array([10 ** 9], np.uint32)
    assert L.rm_balls_lookup(os.fsencode(small_world), 0, 100.0, 1, big.ctypes.data, one.ctypes.data, out.ctypes.data, None) != 0


def _sample(path, mode, radius_m):
    import ctypes
    out = (ctypes.c_double * 3)()
    _lib.check(_lib.lib().rm_graph_ball_sample(os.fsencode(path), mode, radius_m, out))
    return {"nodes": out[0], "table_bytes": out[1], "skipped_frac": out[2]}


def _fit(path, mode, start_m, avail_gb):
    import ctypes
    r = ctypes.c_double()
    _lib.check(_lib.lib().rm_graph_fit_ball_radius(os.fsencode(path), mode, start_m, avail_gb, ctypes.byref(r)))
    return r.value


def test_fit_ball_radius_steps_down_at_the_budget(tmpdir_session, built_lib):
    """VERDICT r02 (route-ball memory): a mode's tables are built at the largest radius whose
    sampled tables (+10 %) fit the memory left for them; a budget just below the 2000 m tables
    steps down instead of failing, and a budget nothing fits leaves the mode to the search tiers."""
    from reporter_amd import world
    path = str(tmpdir_session / "fit_c2.rmg")
    cfg = world.CONFIGS["C2"]
    world.build_world(path, cfg["rows"], cfg["cols"], cfg["block_m"], seed=1, cell_m=cfg["cell_m"])
    gib = float(1 << 30)
    for mode in (0, 3, 4):
        s2000 = _sample(path, mode, 2000.0)
        need = s2000["table_bytes"] * 1.1 / gib
        assert _fit(path, mode, 2000.0, need * 1.01) == 2000.0
        below = _fit(path, mode, 2000.0, need * 0.99)   # just above the cap: the next radius down
        assert 0.0 < below < 2000.0
        assert _sample(path, mode, below)["table_bytes"] * 1.1 / gib <= need * 0.99
        assert _fit(path, mode, 2000.0, 1e-6) == 0.0    # nothing fits: no tables for the mode
        assert _fit(path, mode, 0.0, 1.0) == 0.0        # radius 0: the search tiers by choice
    # a start radius off the ladder is tried first, then the ladder below it
    assert _fit(path, 0, 650.0, 64.0) == 650.0
    # each mode is sampled over its own edges (pedestrians: no highways, no one-way limits)
    assert _sample(path, 4, 1000.0)["table_bytes"] != _sample(path, 0, 1000.0)["table_bytes"]
    L = _lib.lib()
    import ctypes
    r = ctypes.c_double()
    assert L.rm_graph_fit_ball_radius(os.fsencode(path), 7, 100.0, 1.0, ctypes.byref(r)) != 0
    assert L.rm_graph_fit_ball_radius(os.fsencode(path), 0, 20000.0, 1.0, ctypes.byref(r)) != 0
