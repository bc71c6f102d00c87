"""GPU parity on a graph the engine did not generate.

osm_city.cpp writes an irregular city as generic OSM PBF (no reporter:* tags) and
rm_graph_import_osm ingests it the way it would an extract (reference Dockerfile:42-49 builds
Valhalla's tiles from one; py/get_tiles.py:30-102, py/simple_reporter.py:36-49 name their tiles
and OSMLR ids).  Every stage of every trajectory must equal the oracle bit for bit on it, with
report() and the speed histogram / duration sums, at 1 Hz and at 30 s sampling, in the route-ball
tier and in the search tiers alone, and for the three travel modes.  The city has what the grid
never has: hubs with 9 in-edges (the path walk's predecessor scan past the rows' 3-bit index),
curved ways over many cells, roundabouts, one-way carriageway pairs, dead ends, two roads between
one node pair, a bridged trunk road, and roads without OSMLR coverage.
"""
import numpy as np
import pytest

import meili_oracle as mo
from parity_util import compare_all, match_and_compare
from reporter_amd import engine, graphfile, world

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def city(built_lib, tmp_path_factory):
    d = tmp_path_factory.mktemp("gpu_city")
    return world.build_city(str(d / "city.rmg"), rows=48, cols=48, seed=7)


def _scan_walked_edges(path, ref):
    """Chosen path edges entering a node at in-edge index >= 7 (in edge-id order): the walk back
    from such a node cannot take the predecessor the route-ball row stores (3 bits, 7 = none)
    and scans the node's in-edges instead (rm_common.hpp ball_pred, k_paths_ball)."""
    g = graphfile.load(path)
    tgt = g["edges"].reshape(-1, 4)[:, 0].astype(np.int64)
    order = np.argsort(tgt, kind="stable")
    first = np.searchsorted(tgt[order], tgt[order])
    rank = np.empty(len(tgt), np.int64)
    rank[order] = np.arange(len(tgt)) - first
    pool = ref["path_pool"][: int(ref["path_off"].max() + ref["path_cnt"].max())]
    return int((rank[pool.astype(np.int64)] >= 7).sum())


@pytest.mark.parametrize("ball_radius", [None, 0.0])
def test_city_1hz_auto(city, ball_radius):
    """1 Hz auto traces, radius 50 m: the ball tier (2 km tables) and the search tiers alone."""
    tr = world.generate_traces(city, 400, 300, rate_s=1.0, noise_m=5.0, seed=71)
    opts = engine.default_options(1, search_radius=50.0)
    c = match_and_compare(city, tr, opts, None, hist=True, ball_radius=ball_radius, keep_ref=True)
    ref = c.pop("_ref")
    assert c["segments"] > 2_000 and c["valid_reports"] > 500, c
    if ball_radius is None:
        assert c["route_tiers"]["ball_to_search"] == 0, c
    print("city 1 Hz parity", ball_radius, c, "scan-walked edges", _scan_walked_edges(city, ref))


@pytest.mark.parametrize("ball_radius", [None, 0.0])
def test_city_30s_auto(city, ball_radius):
    """30 s sampling, radius 100 m: route bounds up to the 2 km breakage distance, long paths
    through the hubs (some entered at in-edge index >= 7)."""
    tr = world.generate_traces(city, 600, 40, rate_s=30.0, noise_m=5.0, seed=72)
    opts = engine.default_options(1, search_radius=100.0)
    c = match_and_compare(city, tr, opts, None, hist=True, ball_radius=ball_radius, keep_ref=True)
    ref = c.pop("_ref")
    scans = _scan_walked_edges(city, ref)
    assert c["chained"] > 15_000 and scans > 0, (c, scans)
    print("city 30 s parity", ball_radius, c, "scan-walked edges", scans)


def test_city_modes_sigma(city):
    """auto / bicycle / pedestrian (footways, cycleways, one-way streets walked both ways)
    x sigma_z {2, 4.07, 8}, radius max(50, 3 sigma)."""
    parts, opts = [], []
    per = 60
    for mi, mode in enumerate(("auto", "bicycle", "pedestrian")):
        for si, sz in enumerate((2.0, 4.07, 8.0)):
            parts.append(world.generate_traces(city, per, 300, rate_s=1.0, noise_m=sz, seed=7300 + mi * 10 + si,
                                               mode=mode))
            opts.append(engine.default_options(1, mode=world.MODES[mode], sigma_z=sz,
                                               search_radius=max(50.0, 3 * sz))[0])
    tr = world.concat_traces(*parts)
    trace_opt = np.repeat(np.arange(len(parts), dtype=np.uint32), per)
    c = match_and_compare(city, tr, np.array(opts, engine.OPTIONS_DTYPE), trace_opt, rl=(0, 1, 2), tl=(0, 1, 2),
                          hist=True)
    assert c["traces"] == 9 * per and c["segments"] > 1_000, c
    print("city modes parity", c)


def test_second_k1_grid_for_wide_queries(built_lib, city, monkeypatch):
    """K1's grid is chosen per batch radius.  On the city the 50 m default
    and 100 m queries prefer different splits, so the engine keeps both; a 100 m batch takes the
    second one and every stage still equals the oracle (and the one-grid engine, RM_GRID_ALT=0)."""
    g = graphfile.load(city)
    tr = world.generate_traces(city, 300, 40, rate_s=30.0, noise_m=5.0, seed=95)
    T = len(tr["trace_off"]) - 1
    opts = engine.default_options(1, search_radius=100.0)
    ref = mo.match(g, mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts,
                               np.zeros(T, np.uint32)))
    eng = engine.Engine(city, 0)
    f_alt, r_alt = eng.grid_alt()
    assert f_alt not in (0, eng.grid_split()) and 50.0 < r_alt <= 100.0, (eng.grid_split(), f_alt, r_alt)
    bm = engine.BatchMatcher(eng)
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts)
    c = compare_all(bm, ref, tr["trace_off"])
    assert c["segments"] > 200, c
    bm.close()
    eng.close()
    monkeypatch.setenv("RM_GRID_ALT", "0")
    eng = engine.Engine(city, 0)
    assert eng.grid_alt() == (0, 0.0)
    bm = engine.BatchMatcher(eng)
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts)
    compare_all(bm, ref, tr["trace_off"])
    bm.close()
    eng.close()
