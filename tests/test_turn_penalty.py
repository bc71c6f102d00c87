"""meili's turn costs (DESIGN.md §3 rule 3b), CPU side.

The reference configures them: stock valhalla_build_config (reference Dockerfile:42-49) writes
meili's per-mode turn_penalty_factor (auto 200, bicycle 140, pedestrian 100), and the client
sends the field (py/generate_test_trace.py:37,47).  Configure accepts such a config, a negative or
infinite factor fails (meili's TransitionCostModel refuses a negative one), and the oracle's turn
weights are pinned here by an independent pure-Python restatement on small cases.
"""
import heapq
import json
import math

import numpy as np
import pytest

import meili_oracle as mo
from reporter_amd import engine, graphfile, world


def _conf(tmp_path, meili, ra=None):
    p = tmp_path / "conf.json"
    ra = dict(ra or {})
    ra.setdefault("graph", str(tmp_path / "missing.rmg"))
    p.write_text(json.dumps({"meili": meili, "reporter_amd": ra}))
    return str(p)


STOCK = {"default": {"turn_penalty_factor": 0, "sigma_z": 4.07, "beta": 3}, "auto": {"turn_penalty_factor": 200},
         "bicycle": {"turn_penalty_factor": 140}, "pedestrian": {"turn_penalty_factor": 100, "search_radius": 50}}


def test_configure_accepts_stock_turn_costs(built_lib, tmp_path):
    """Checked before the graph loads (no GPU needed): the stock per-mode factors get as far as
    the (missing) graph; a negative or infinite factor fails with its own message."""
    import valhalla
    with pytest.raises(RuntimeError, match="missing.rmg"):
        valhalla.Configure(_conf(tmp_path, STOCK))
    with pytest.raises(RuntimeError, match="missing.rmg"):
        valhalla.Configure(_conf(tmp_path, {"auto": {"turn_penalty_factor": 200}}, {"ignore_turn_penalty": True}))
    for bad in (-1, -1e-30, 1e39):
        with pytest.raises(RuntimeError, match="turn_penalty_factor must be non-negative"):
            valhalla.Configure(_conf(tmp_path, {"bicycle": {"turn_penalty_factor": bad}}))


# ---- an independent restatement of rule 3b (pure Python, small cases) ----

D2R = 0.017453292519943295


def _gc32(lon_a, lat_a, lon_b, lat_b):
    """PointLL::Distance with libm: law of cosines, rounded to float."""
    if lon_a == lon_b and lat_a == lat_b:
        return 0.0
    a, c = float(lat_a) * D2R, float(lat_b) * D2R
    dl = (float(lon_b) - float(lon_a)) * D2R
    cb = math.sin(a) * math.sin(c) + math.cos(a) * math.cos(c) * math.cos(dl)
    cb = min(1.0, max(-1.0, cb))
    return float(np.float32(math.acos(cb) * 6378160.187))


def _bearing(lon_a, lat_a, lon_b, lat_b):
    """PointLL::Heading with math.atan2 (the oracle uses its own deterministic series)."""
    if lon_a == lon_b and lat_a == lat_b:
        return 0.0
    p1, p2 = float(lat_a) * D2R, float(lat_b) * D2R
    dl = (float(lon_b) - float(lon_a)) * D2R
    y = math.sin(dl) * math.cos(p2)
    x = math.cos(p1) * math.sin(p2) - math.sin(p1) * math.cos(p2) * math.cos(dl)
    return math.degrees(math.atan2(y, x)) % 360.0


def _heading_along(xs, ys):
    """PointLL::HeadingAlongPolyline(shape, 30 m), then NodeInfo's 8-bit storage and back."""
    n = len(xs)
    if n == 2:
        h = _bearing(xs[0], ys[0], xs[1], ys[1])
    else:
        d, h = 0.0, None
        for i in range(n - 1):
            if d >= 30.0:
                break
            seg = _gc32(xs[i], ys[i], xs[i + 1], ys[i + 1])
            if d + seg > 30.0:
                f = (30.0 - d) / seg
                x = np.float32(float(xs[i]) + (float(xs[i + 1]) - float(xs[i])) * f)
                y = np.float32(float(ys[i]) + (float(ys[i + 1]) - float(ys[i])) * f)
                h = _bearing(xs[0], ys[0], x, y)
                break
            d += seg
        if h is None:
            h = _bearing(xs[0], ys[0], xs[-1], ys[-1])
    hd = int(math.floor(h + 0.5)) % 360
    h8 = int(math.floor(np.float32(hd) * (np.float32(255.0) / np.float32(359.0)) + np.float32(0.5)))
    return int(math.floor(np.float32(h8) * (np.float32(359.0) / np.float32(255.0)) + np.float32(0.5)))


def _road_heads(g):
    verts = g["verts"].reshape(-1, 4)
    lon, lat = verts[:, 0].view(np.float32), verts[:, 1].view(np.float32)
    off = g["road_vert_off"]
    h0 = np.empty(len(off) - 1, np.int64)
    h1 = np.empty(len(off) - 1, np.int64)
    for r in range(len(off) - 1):
        a, b = int(off[r]), int(off[r + 1])
        h0[r] = _heading_along(lon[a:b], lat[a:b])
        h1[r] = _heading_along(lon[a:b][::-1], lat[a:b][::-1])
    return h0, h1


def test_road_headings_match_atan2(built_lib, small_world):
    """The oracle's road headings (HeadingAlongPolyline at 30 m, 8-bit NodeInfo storage) against
    the libm restatement above on a generated world."""
    g = graphfile.load(small_world)
    h0, h1 = mo.road_heads(g)
    p0, p1 = _road_heads(g)
    for a, b in ((h0, p0), (h1, p1)):
        d = np.abs(a.astype(np.int64) - b)
        d = np.minimum(d, 360 - d)
        assert int(d.max()) <= 2, int(d.max())            # one 359/255-degree step at most
        assert (d == 0).mean() > 0.999
    # a grid: roads leave their nodes along the four compass directions (+-20 % jitter)
    q = np.concatenate([h0, h1]).astype(np.int64)
    near = np.minimum.reduce([np.minimum(np.abs(q - c), 360 - np.abs(q - c)) for c in (0, 90, 180, 270)])
    assert np.median(near) < 15


def _tu(d):
    return int(round(65536.0 * math.exp(-d / 45.0)))


def _turn(hb, hs):
    d = abs(int(hb) - int(hs))
    return _tu(360 - d if d > 180 else d)


def _py_route_turns(g, heads, ra, sa, rb, sb, mode_acc, speed_cap, bound):
    """Rule 3b by brute force: bounded Dijkstra from the source's exits on (dist, time) keys,
    canonical predecessors (smallest-id tight usable in-edge), the route's combination, and the
    turn weight along the walk.  Returns (route dist cm or None, U)."""
    E = g["edges"].reshape(-1, 4).astype(np.int64)
    node_off = g["node_off"].astype(np.int64)
    N = len(node_off) - 1
    src = np.repeat(np.arange(N), np.diff(node_off))
    h0, h1 = heads

    def ok(e):
        return e != 0xffffffff and ((int(E[e, 2]) >> 16) & 7) & mode_acc

    def tms(d, e):
        sp = min(int(E[e, 2]) & 0xffff, speed_cap)
        return (d * 360) // max(sp, 1)

    L = int(g["road_len_cm"][ra])
    ef, er = int(g["road_fwd"][ra]), int(g["road_rev"][ra])
    n0, n1 = int(g["road_node0"][ra]), int(g["road_node1"][ra])
    lab, root = {}, {}
    pq = []
    if ok(ef) and L - sa <= bound:
        k = ((L - sa) << 32) | tms(L - sa, ef)
        root[n1] = k
        lab[n1] = min(lab.get(n1, 1 << 64), k)
    if ok(er) and sa <= bound:
        k = (sa << 32) | tms(sa, er)
        root[n0] = k
        lab[n0] = min(lab.get(n0, 1 << 64), k)
    for v, k in lab.items():
        heapq.heappush(pq, (k, v))
    done = set()
    while pq:
        k, u = heapq.heappop(pq)
        if u in done or k != lab[u]:
            continue
        done.add(u)
        for e in range(node_off[u], node_off[u + 1]):
            if not ok(e):
                continue
            ln = int(E[e, 1])
            nk = k + ((ln << 32) | tms(ln, e))
            if (nk >> 32) > bound:
                continue
            v = int(E[e, 0])
            if nk < lab.get(v, 1 << 64):
                lab[v] = nk
                heapq.heappush(pq, (nk, v))
    Lb = int(g["road_len_cm"][rb])
    bf, br = int(g["road_fwd"][rb]), int(g["road_rev"][rb])
    best, combo = None, -1
    if ra == rb:
        if ok(bf) and sb >= sa:
            best, combo = ((sb - sa) << 32) | tms(sb - sa, bf), 0
        if ok(br) and sa >= sb:
            k = ((sa - sb) << 32) | tms(sa - sb, br)
            if best is None or k < best:
                best, combo = k, 1
    if ok(bf) and int(g["road_node0"][rb]) in lab:
        k = lab[int(g["road_node0"][rb])] + ((sb << 32) | tms(sb, bf))
        if best is None or k < best:
            best, combo = k, 2
    if ok(br) and int(g["road_node1"][rb]) in lab:
        k = lab[int(g["road_node1"][rb])] + (((Lb - sb) << 32) | tms(Lb - sb, br))
        if best is None or k < best:
            best, combo = k, 3
    if best is None or (best >> 32) > bound:
        return None, 0
    if combo < 2:
        return best >> 32, 0
    side = combo - 2
    hs = h0[rb] if side == 0 else h1[rb]
    v = int(g["road_node0"][rb]) if side == 0 else int(g["road_node1"][rb])
    U = 0
    while lab[v] != root.get(v):
        tight = [e for e in range(len(E)) if E[e, 0] == v and ok(e) and int(src[e]) in lab
                 and lab[int(src[e])] + ((int(E[e, 1]) << 32) | tms(int(E[e, 1]), e)) == lab[v]]
        e = min(tight)
        r2, rev = int(E[e, 3]) >> 1, int(E[e, 3]) & 1
        U += _turn(h0[r2] if rev else h1[r2], hs)
        hs = h1[r2] if rev else h0[r2]
        v = int(src[e])
    U += _turn(h1[ra] if v == n1 else h0[ra], hs)
    return best >> 32, U


def test_oracle_turn_weights_restated(built_lib, tmp_path):
    """The oracle's per-transition turn weights against the brute-force restatement above, on
    sampled transitions of 1 Hz and 30 s traces (every transition with a turn in a few traces)."""
    path = str(tmp_path / "w.rmg")
    world.build_world(path, 16, 16, 100.0, seed=3)
    g = graphfile.load(path)
    heads = mo.road_heads(g)
    rng = np.random.default_rng(0)
    checked = turned = 0
    for rate, radius in ((1.0, 50.0), (30.0, 100.0)):
        tr = world.generate_traces(path, n_traces=6, n_points=60 if rate == 1.0 else 16, rate_s=rate, noise_m=5.0, seed=4)
        opts = engine.default_options(1, turn_penalty_factor=200.0, search_radius=radius)
        T = len(tr["trace_off"]) - 1
        ref = mo.match(g, mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts,
                                   np.zeros(T, np.uint32)))
        for k in range(T):
            o = int(tr["trace_off"][k])
            for s in range(1, int(ref["n_states"][k])):
                la, lb = o + s - 1, o + s
                KA, KB = int(ref["cand_n"][la]), int(ref["cand_n"][lb])
                if not KA or not KB or rng.random() > 0.35:
                    continue
                gc = float(ref["gc"][lb])
                bound = min(int(math.floor(min(gc * 5.0, 2000.0) * 100.0)), 100000000)
                for i in range(KA):
                    for j in range(KB):
                        d, U = _py_route_turns(g, heads, int(ref["cand_road"][la][i]), int(ref["cand_s"][la][i]),
                                               int(ref["cand_road"][lb][j]), int(ref["cand_s"][lb][j]), 1, 0xffff, bound)
                        q = int(ref["trans_off"][lb]) + i * KB + j
                        if ref["route"][q] == 0xffffffff:
                            continue   # also beyond the time bound; no turn weight is used
                        assert d == int(ref["route"][q]), (k, s, i, j)
                        assert U == int(ref["route_turn"][q]), (k, s, i, j, U, int(ref["route_turn"][q]))
                        checked += 1
                        turned += U > 0
    assert checked > 300 and turned > 100, (checked, turned)


def test_turn_costs_change_some_choices_only(built_lib, small_world):
    """Factor 0 gives zero weights and the previous matcher's choices; 200 weighs most routes that
    leave their road and changes a few choices, never the routes themselves (rule 3b: turn costs
    weigh a transition, they do not change its route)."""
    g = graphfile.load(small_world)
    tr = world.generate_traces(small_world, n_traces=24, n_points=200, rate_s=1.0, noise_m=8.0, seed=6)
    T = len(tr["trace_off"]) - 1
    res = {}
    for f in (0.0, 200.0):
        opts = engine.default_options(1, turn_penalty_factor=f)
        res[f] = mo.match(g, mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts,
                                      np.zeros(T, np.uint32)))
    a, b = res[0.0], res[200.0]
    assert not a["route_turn"].any()
    np.testing.assert_array_equal(a["route"], b["route"])
    valid = b["route"] != 0xffffffff
    assert (b["route_turn"][valid] > 0).mean() > 0.2
    diff = int((a["choice"] != b["choice"]).sum())
    assert 0 < diff < 0.05 * len(a["choice"]), diff


CURVED = """<?xml version='1.0' encoding='UTF-8'?>
<osm version="0.6" generator="hand">
 <node id="1" lat="0.0000000" lon="0.0000000"/>
 <node id="2" lat="0.0000000" lon="0.0000449"/>
 <node id="3" lat="0.0009040" lon="0.0000449"/>
 <node id="4" lat="0.0013040" lon="0.0004449"/>
 <way id="7">
  <nd ref="1"/><nd ref="2"/><nd ref="3"/><nd ref="4"/>
  <tag k="highway" v="residential"/>
 </way>
</osm>
"""


def test_curved_way_headings_hand_derived(built_lib, tmp_path):
    """a way that leaves its node 5 m east and then runs north.  Valhalla's NodeInfo
    heading is taken 30 m along the shape (HeadingAlongPolyline), not toward the first vertex:
    H0 = atan2(5.0 m east, 25.0 m north) = 11.3 deg -> 11 -> 8 bits round(11 * 255/359) = 8 -> back
    round(8 * 359/255) = 11 (the first-vertex rule gave 90).  At the other end the first segment
    is 62.9 m long: the heading toward node 3, atan2(-44.5, -44.2) = 225.2 deg -> 225 -> 160 -> 225."""
    p = tmp_path / "curved.osm"
    p.write_text(CURVED)
    g = graphfile.load(world.import_osm(str(p), str(tmp_path / "curved.rmg"), cell_m=50.0))
    assert len(g["road_len_cm"]) == 1
    h0, h1 = mo.road_heads(g)
    n0 = int(g["road_node0"][0])
    lonn = g["node_lon"].view(np.float32) if g["node_lon"].dtype != np.float32 else g["node_lon"]
    first_is_1 = float(lonn[n0]) == 0.0
    at1, at4 = (h0[0], h1[0]) if first_is_1 else (h1[0], h0[0])
    assert (int(at1), int(at4)) == (11, 225)
    p0, p1 = _road_heads(g)
    assert (int(p0[0]), int(p1[0])) == (int(h0[0]), int(h1[0]))
