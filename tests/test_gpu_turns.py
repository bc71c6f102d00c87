"""GPU parity with meili's turn costs (DESIGN.md §3 rule 3b).

The reference's production config has them: stock valhalla_build_config (reference
Dockerfile:42-49) writes meili's per-mode turn_penalty_factor -- auto 200, bicycle 140,
pedestrian 100 -- and the Java batcher does not override it (Batch.java:58-65).  Every stage,
including every transition's turn weight, must equal the oracle bit for bit at those factors: on
the C2 graph (1 Hz, past 4,096 traces so the four-traces-per-wave K3 runs, and below it the
one-wave-per-trace K3), at 30 s sampling with bounds beyond the route-table radius, with the
search tiers alone, over the three modes x sigma_z, and on the generic OSM city at 1 Hz and 30 s.
"""
import json

import numpy as np
import pytest

import meili_oracle as mo
from parity_util import compare_all, match_and_compare
from reporter_amd import engine, graphfile, world

pytestmark = pytest.mark.gpu

STOCK = {0: 200.0, 1: 200.0, 2: 0.0, 3: 140.0, 4: 100.0}   # meili's per-mode defaults (mode id -> factor)


def _turned(c):
    """Transitions with a valid route and a non-zero turn weight (the _ref is dropped from c)."""
    ref = c.pop("_ref")
    valid = ref["route"] != 0xffffffff
    return int((ref["route_turn"][valid] > 0).sum())


@pytest.fixture(scope="module")
def c2_graph(built_lib, tmpdir_session):
    cfg = dict(world.CONFIGS["C2"])
    path = str(tmpdir_session / "turn_c2.rmg")
    world.build_world(path, cfg["rows"], cfg["cols"], cfg["block_m"], seed=1, cell_m=cfg["cell_m"])
    return path, cfg


@pytest.mark.timeout(400)
@pytest.mark.parametrize("n_traces,n_points", [(4200, 120), (600, 300)])
def test_c2_auto_200(c2_graph, n_traces, n_points):
    """C2 graph, 1 Hz, auto at 200: route tables with turn rows; 4,200 traces take the
    four-traces-per-wave K3, 600 the one-wave-per-trace K3."""
    path, cfg = c2_graph
    tr = world.generate_traces(path, n_traces, n_points, cfg["rate_s"], cfg["noise_m"], seed=1200)
    opts = engine.default_options(1, search_radius=cfg["search_radius"], turn_penalty_factor=200.0)
    c = match_and_compare(path, tr, opts, None, hist=True, keep_ref=True)
    assert _turned(c) > 10 * n_traces, c
    assert c["segments"] > 2 * n_traces and c["valid_reports"] > n_traces // 10, c
    print("C2 turn 200 parity", c)


@pytest.mark.parametrize("ball_radius", [0.0, 60.0, 500.0])
def test_search_tiers_and_mixed(built_lib, tmpdir_session, ball_radius):
    """30 s sampling (bounds up to 2 km): the search tiers alone (radius 0), mostly them (60 m),
    and 500 m tables whose answers beyond the radius are used when exact -- the turn weights of
    the search tiers' canonical-path walks and of the turn rows agree with the oracle."""
    path = str(tmpdir_session / "turn_30s.rmg")
    world.build_world(path, 60, 60, 150.0, seed=8, cell_m=150.0)
    tr = world.generate_traces(path, 400, 30, rate_s=30.0, noise_m=5.0, seed=81)
    opts = engine.default_options(1, search_radius=100.0, turn_penalty_factor=200.0)
    c = match_and_compare(path, tr, opts, None, hist=True, ball_radius=ball_radius, keep_ref=True)
    assert _turned(c) > 5_000 and c["chained"] > 5_000, c
    print("30 s turn parity", ball_radius, c)


def test_modes_stock_factors_sigma(c2_graph):
    """auto 200 / bicycle 140 / pedestrian 100 (and bus 200 sharing auto's tables and turn rows,
    motor_scooter without turn costs) over sigma_z 2..16 m, per-trace options in one batch."""
    path, cfg = c2_graph
    modes = [0, 3, 4, 1, 2]
    sig = [2.0, 4.07, 8.0, 16.0]
    n = 400
    tr = world.generate_traces(path, n, 200, 1.0, 6.0, seed=1300)
    opts = engine.default_options(len(modes) * len(sig))
    q = 0
    for m in modes:
        for s in sig:
            opts[q]["mode"] = m
            opts[q]["sigma_z"] = s
            opts[q]["search_radius"] = max(50.0, 3.0 * s)
            opts[q]["turn_penalty_factor"] = STOCK[m]
            q += 1
    trace_opt = (np.arange(n) % len(opts)).astype(np.uint32)
    c = match_and_compare(path, tr, opts, trace_opt, hist=True, keep_ref=True)
    assert _turned(c) > 5_000, c
    print("modes x sigma turn parity", c)


@pytest.fixture(scope="module")
def city(built_lib, tmp_path_factory):
    d = tmp_path_factory.mktemp("turn_city")
    return world.build_city(str(d / "city.rmg"), rows=40, cols=40, seed=7)


@pytest.mark.parametrize("rate,radius,n,pts", [(1.0, 50.0, 300, 240), (30.0, 100.0, 500, 40)])
def test_city_stock_factors(city, rate, radius, n, pts):
    """The generic OSM city (hubs of 9 roads, curved ways, roundabouts, one-way pairs): its
    headings are those of real shapes, and the canonical paths enter nodes at in-edge index >= 7
    (the turn rows' scan); auto at 200, every stage bit-exact."""
    tr = world.generate_traces(city, n, pts, rate_s=rate, noise_m=5.0, seed=91)
    opts = engine.default_options(1, search_radius=radius, turn_penalty_factor=200.0)
    c = match_and_compare(city, tr, opts, None, hist=True, keep_ref=True)
    assert _turned(c) > 2_000, c
    print("city turn parity", rate, c)


def test_turn_rows_built_once(c2_graph):
    """A batch with turn costs builds the mode's turn rows once (8 bytes per table slot); a batch
    without them takes the plain kernels and gives the factor-0 answers."""
    path, cfg = c2_graph
    g = graphfile.load(path)
    eng = engine.Engine(path, 0)
    tr = world.generate_traces(path, 64, 200, 1.0, 5.0, seed=1400)
    T = 64
    for f in (200.0, 0.0, 140.0):
        opts = engine.default_options(1, turn_penalty_factor=f)
        bm = engine.BatchMatcher(eng)
        bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, np.zeros(T, np.uint32))
        ref = mo.match(g, mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts,
                                   np.zeros(T, np.uint32)))
        compare_all(bm, ref, tr["trace_off"])
        assert (bm.route_terms() is not None) == (f > 0)
        bm.close()
    eng.close()


def test_dropin_request_with_turn_costs(small_world, tmp_path):
    """Through valhalla.SegmentMatcher().Match: a request with turn_penalty_factor 200 is answered
    (the segments the oracle forms at 200), one with a negative factor fails alone (the
    service's 500) and does not disturb its coalesced neighbour."""
    import valhalla
    conf = valhalla.write_config(str(tmp_path / "tp.json"), small_world, device=0, coalesce=True)
    valhalla.Configure(conf)
    sm = valhalla.SegmentMatcher()
    tr = world.generate_traces(small_world, n_traces=2, n_points=160, rate_s=1.0, noise_m=5.0, seed=5)
    ok = json.dumps(world.trace_to_request(tr, 0, turn_penalty_factor=200), separators=(",", ":"))
    bad = json.dumps(world.trace_to_request(tr, 1, turn_penalty_factor=-5), separators=(",", ":"))
    with pytest.raises(RuntimeError, match="turn_penalty_factor must be non-negative"):
        sm.Match(bad)
    got = json.loads(sm.Match(ok))
    sm.close()
    g = graphfile.load(small_world)
    opts = engine.default_options(1, turn_penalty_factor=200.0)
    ref = mo.match(g, mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts,
                               np.zeros(2, np.uint32)))
    want = engine.segment_dicts(ref["segs"][ref["seg_off"][0]:ref["seg_off"][1]])
    assert got["segments"] == want and len(want) > 3
    # a config as stock valhalla_build_config writes it (per-mode sections): a request that names
    # no factor gets its mode's (auto: 200)
    stock = {"meili": {"default": {"turn_penalty_factor": 0, "sigma_z": 4.07, "beta": 3},
                       "auto": {"turn_penalty_factor": 200, "search_radius": 50},
                       "bicycle": {"turn_penalty_factor": 140}, "pedestrian": {"turn_penalty_factor": 100}},
             "reporter_amd": {"graph": small_world, "device": 0, "coalesce": True}}
    (tmp_path / "stock.json").write_text(json.dumps(stock))
    valhalla.Configure(str(tmp_path / "stock.json"))
    sm = valhalla.SegmentMatcher()
    plain = json.dumps(world.trace_to_request(tr, 0), separators=(",", ":"))
    assert json.loads(sm.Match(plain))["segments"] == want
    sm.close()
