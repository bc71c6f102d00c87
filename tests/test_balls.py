"""Route balls (K2's lookup tier, reporter_amd/csrc/balls.cpp) on the CPU.

The tables must hold, for every node u and every node v whose shortest lexicographic
(dist cm, time ms) key from u has distance <= radius, exactly that key — the value a
bounded Dijkstra of the reference matcher (meili, simple_reporter.py:166) settles v
with when started at u with key 0 — and nothing for nodes beyond the radius.  Checked
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


def _lookup(path, mode, radius_m, fr, to):
    fr = np.ascontiguousarray(fr, np.uint32)
    to = np.ascontiguousarray(to, np.uint32)
    out = np.empty(len(fr), np.uint64)
    _lib.check(_lib.lib().rm_balls_lookup(os.fsencode(path), mode, radius_m, len(fr), fr.ctypes.data,
                                          to.ctypes.data, out.ctypes.data))
    return out


@pytest.mark.parametrize("mode,radius_m", [(0, 400.0), (0, 150.0), (3, 400.0), (4, 250.0)])
def test_ball_keys_match_dijkstra(small_world, mode, radius_m):
    g = graphfile.load(small_world)
    tgt, key = _edge_keys(g, mode)
    rng = np.random.default_rng(mode * 7 + int(radius_m))
    fr, to, want = [], [], []
    n = g.n_nodes
    for u in rng.choice(n, 60, replace=False):
        done = _dijkstra(g, tgt, key, int(u), int(radius_m * 100))
        inside = list(done.items())
        outside = rng.choice(n, 20)
        for v, k in inside:
            fr.append(u); to.append(v); want.append(k)
        for v in outside:
            if int(v) not in done:
                fr.append(u); to.append(v); want.append(KEY_INF)
    got = _lookup(small_world, mode, radius_m, fr, to)
    np.testing.assert_array_equal(got, np.array(want, np.uint64))
    assert sum(1 for k in want if k != KEY_INF) > 200


def test_ball_radius_zero_keeps_only_self(small_world):
    got = _lookup(small_world, 0, 0.0, [0, 0, 5], [0, 1, 5])
    assert list(got) == [0, KEY_INF, 0]


def test_ball_lookup_errors(small_world):
    one = np.zeros(1, np.uint32)
    out = np.zeros(1, np.uint64)
    assert _lib.lib().rm_balls_lookup(os.fsencode(small_world), 9, 100.0, 1, one.ctypes.data, one.ctypes.data,
                                      out.ctypes.data) != 0
    big = np.array([10 ** 9], np.uint32)
    assert _lib.lib().rm_balls_lookup(os.fsencode(small_world), 0, 100.0, 1, big.ctypes.data, one.ctypes.data,
                                      out.ctypes.data) != 0
