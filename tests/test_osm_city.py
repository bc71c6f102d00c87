"""An irregular city as generic OSM, ingested by the importer (CPU).

The engine's own world (world.cpp) lays out a perturbed grid.  Valhalla's tiles come from OSM
extracts (reference Dockerfile:42-49, py/get_tiles.py:30-102), whose topology that grid never
has.  osm_city.cpp writes such a city as plain OSM (no reporter:* tags). rm_graph_import_osm
ingests it generically, and the oracle matches on the result.  The GPU parity test on the same
graphs is tests/test_gpu_osm_city.py.
"""
import numpy as np
import pytest

import meili_oracle as mo
from parity_util import truth_recovery
from reporter_amd import engine, graphfile, world


@pytest.fixture(scope="module")
def city(tmp_path_factory):
    d = tmp_path_factory.mktemp("city")
    pbf = str(d / "city.osm.pbf")
    path = world.build_city(str(d / "city.rmg"), pbf_path=pbf, rows=40, cols=40, seed=3)
    return path, pbf, d


def test_city_is_generic_osm(built_lib, city):
    """The writer's XML and PBF carry the same elements (identical graphs), nothing engine-specific,
    and the same seed gives the same file."""
    path, pbf, d = city
    xml = world.write_city_osm(str(d / "city.osm"), pbf=False, rows=40, cols=40, seed=3)
    text = open(xml).read()
    assert "reporter:" not in text and 'k="junction" v="roundabout"' in text and 'k="bridge" v="yes"' in text
    assert 'k="type" v="osmlr"' in text and 'role="backward"' in text
    back = world.import_osm(xml, str(d / "city_xml.rmg"))
    assert open(back, "rb").read() == open(path, "rb").read()
    again = world.write_city_osm(str(d / "again.osm.pbf"), rows=40, cols=40, seed=3)
    assert open(again, "rb").read() == open(pbf, "rb").read()
    other = world.write_city_osm(str(d / "other.osm.pbf"), rows=40, cols=40, seed=4)
    assert open(other, "rb").read() != open(pbf, "rb").read()


def test_city_topology(built_lib, city):
    """What the grid generator never produces is in the ingested graph."""
    g = graphfile.load(city[0])
    E = g["edges"].reshape(-1, 4)
    N = len(g["node_lon"])
    indeg = np.bincount(E[:, 0], minlength=N)
    outdeg = np.diff(g["node_off"].astype(np.int64))
    acc = (E[:, 2] >> 16) & 7
    # more than 7 in-edges: beyond the route-ball rows' 3-bit predecessor index
    assert (indeg > 7).sum() >= 10 and indeg.max() >= 9
    assert 5 <= outdeg.max() <= 31
    # dead ends, and pairs of roads between the same two nodes (service loops)
    assert (outdeg == 1).sum() >= 20
    r0, r1 = g["road_node0"].astype(np.int64), g["road_node1"].astype(np.int64)
    _, cnt = np.unique(np.minimum(r0, r1) * N + np.maximum(r0, r1), return_counts=True)
    assert (cnt > 1).sum() >= 10
    # one-way for vehicles (roundabouts, carriageways, one-way streets): one direction auto,
    # the other pedestrian only
    fwd, rev = g["road_fwd"], g["road_rev"]
    oneway = ((acc[fwd] & 1) != (acc[rev] & 1)).sum()
    assert oneway >= 200
    # paths for pedestrians / cyclists only, auto-only trunk, link ramps (internal)
    assert (acc == 4).sum() > 0 and (acc == 2).sum() > 0 and (acc == 1).sum() > 0
    assert ((E[:, 2] >> 19) & 1).sum() > 0 and ((E[:, 2] >> 20) & 1).sum() > 0
    # curved multi-vertex roads, some longer than several grid cells
    nv = np.diff(g["road_vert_off"].astype(np.int64))
    assert nv.max() >= 8 and (g["road_len_cm"] > 150_00).sum() > 100 and g["road_len_cm"].max() > 500_00
    # OSMLR coverage on part of the roads only, ids in the level | tile << 3 | index << 25 layout
    has = g["edge_seg"] != 0xFFFFFFFF
    assert 0.2 < has.mean() < 0.9
    lv = g["seg_id"] & 7
    assert set(lv.tolist()) == {0, 1, 2}
    # segments of two member ways: the segment's edges are contiguous in offset order
    s = g["edge_seg"][has]
    off = g["edge_seg_off"][has]
    ln = E[has, 1]
    order = np.lexsort((off, s))
    s, off, ln = s[order], off[order], ln[order]
    same = s[1:] == s[:-1]
    np.testing.assert_array_equal(off[1:][same], (off + ln)[:-1][same])
    np.testing.assert_array_equal(np.bincount(s, weights=ln, minlength=len(g["seg_id"])).astype(np.int64),
                                  g["seg_len_cm"].astype(np.int64))


@pytest.mark.parametrize("mode,rate,radius,floor", [("auto", 1.0, 50.0, 0.93), ("auto", 30.0, 100.0, 0.88),
                                                      ("bicycle", 1.0, 50.0, 0.92), ("pedestrian", 1.0, 50.0, 0.90)])
def test_oracle_matches_on_the_city(built_lib, city, mode, rate, radius, floor):
    """The oracle recovers the driven roads on the ingested city (floors a little under its
    own rates, as tests/test_gpu_pinned.py sets them) and the paths pass through the hubs."""
    g = graphfile.load(city[0])
    npts = 300 if rate == 1.0 else 40
    tr = world.generate_traces(city[0], 60, npts, rate_s=rate, noise_m=5.0, seed=21, mode=mode)
    opts = engine.default_options(1, search_radius=radius, mode=world.MODES[mode])
    ref = mo.match(g, mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts,
                               np.zeros(60, np.uint32)))
    frac, matched, states = truth_recovery(tr["trace_off"], ref["n_states"], ref["state_orig"], ref["cand_road"],
                                           ref["choice"], tr["truth_edge"], g["edges"])
    assert matched == states and frac >= floor, (frac, matched, states)
    assert len(ref["segs"]) > 100
