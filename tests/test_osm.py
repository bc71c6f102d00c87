"""OpenStreetMap exchange of the road graph (CPU).

The reference's graph is Valhalla tiles built from an OSM extract (tile hierarchy
py/get_tiles.py:30-102, OSMLR id layout py/simple_reporter.py:36-49).  The engine's .rmg
world round-trips through OSM XML bit for bit, so the same synthetic world can be handed
to a tile builder wherever one exists, and a generic OSM file can be ingested.
"""
import numpy as np

import meili_oracle as mo
from reporter_amd import engine, graphfile, world


def test_export_import_is_bit_identical(built_lib, tmp_path):
    for name, (rows, cols, block, cell) in {"c1": (40, 40, 100.0, 100.0), "c3": (30, 30, 200.0, 200.0)}.items():
        src = str(tmp_path / (name + ".rmg"))
        world.build_world(src, rows, cols, block, seed=3, cell_m=cell)
        osm = world.export_osm(src, str(tmp_path / (name + ".osm")))
        back = world.import_osm(osm, str(tmp_path / (name + "_back.rmg")))
        assert open(src, "rb").read() == open(back, "rb").read(), name
        text = open(osm).read()
        assert text.count("<way ") == world.graph_info(src)["roads"]
        assert 'k="type" v="osmlr"' in text and 'k="highway"' in text and 'k="maxspeed"' in text


def test_matching_on_the_reingested_graph_is_identical(built_lib, tmp_path):
    src = str(tmp_path / "m.rmg")
    world.build_world(src, 30, 30, 100.0, seed=4)
    back = world.import_osm(world.export_osm(src, str(tmp_path / "m.osm")), str(tmp_path / "m_back.rmg"))
    tr = world.generate_traces(src, 8, 200, rate_s=1.0, noise_m=5.0, seed=9)
    runs = []
    for p in (src, back):
        b = mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], engine.default_options(1),
                     np.zeros(8, np.uint32))
        runs.append(mo.match(graphfile.load(p), b))
    assert len(runs[0]["segs"]) > 20
    assert runs[0]["segs"].tobytes() == runs[1]["segs"].tobytes()
    np.testing.assert_array_equal(runs[0]["path_pool"], runs[1]["path_pool"])


GENERIC = """<?xml version='1.0' encoding='UTF-8'?>
<osm version="0.6" generator="hand">
 <node id="10" lat="47.0000" lon="8.0000"/>
 <node id="11" lat="47.0000" lon="8.0020"/>
 <node id="12" lat="47.0000" lon="8.0040"/>
 <node id="20" lat="46.9990" lon="8.0020"/>
 <node id="21" lat="47.0010" lon="8.0020"/>
 <node id="30" lat="47.0005" lon="8.0030"/>
 <way id="100">
  <nd ref="10"/><nd ref="11"/><nd ref="12"/>
  <tag k="highway" v="primary"/><tag k="maxspeed" v="50"/><tag k="name" v="A &amp; B"/>
 </way>
 <way id="200">
  <nd ref="20"/><nd ref="11"/><nd ref="21"/>
  <tag k="highway" v="residential"/><tag k="oneway" v="yes"/>
 </way>
 <way id="300">
  <nd ref="21"/><nd ref="30"/><nd ref="12"/>
  <tag k="highway" v="footway"/>
 </way>
 <way id="400">
  <nd ref="10"/><nd ref="20"/>
  <tag k="building" v="yes"/>
 </way>
</osm>
"""


def test_generic_osm_is_split_at_intersections(built_lib, tmp_path):
    p = tmp_path / "g.osm"
    p.write_text(GENERIC)
    out = world.import_osm(str(p), str(tmp_path / "g.rmg"), cell_m=50.0)
    g = graphfile.load(out)
    info = world.graph_info(out)
    # way 100 and way 200 cross at node 11; way 300 ends at 21 and 12; 30 is a shape vertex;
    # way 400 has no highway tag
    assert info["nodes"] == 5 and info["roads"] == 5 and info["edges"] == 10 and info["segments"] == 0
    e = g["edges"].reshape(-1, 4)
    speed = e[:, 2] & 0xFFFF
    acc = (e[:, 2] >> 16) & 7
    assert sorted(set(speed.tolist())) == [50, 300, 500]
    ways = g["edge_way"]
    # way 200 is one-way for vehicles: its reverse edges keep pedestrian access only
    rev200 = [(int(a), int(w)) for a, w, r in zip(acc, ways, e[:, 3]) if w == 200 and (r & 1)]
    assert rev200 and all(a == 4 for a, _ in rev200)
    # the footway is pedestrian-only both ways
    assert set(acc[ways == 300].tolist()) == {4}


def test_roundabout_oneway_tags(built_lib, tmp_path):
    """A roundabout is one-way in its drawing direction unless tagged: oneway=no keeps both
    directions, and an explicit oneway=-1 wins over the implied direction."""
    for tagv, fwd_auto, rev_auto in ((None, True, False), ("no", True, True), ("-1", False, True), ("yes", True, False)):
        ow = '' if tagv is None else '<tag k="oneway" v="%s"/>' % tagv
        x = tmp_path / ("r%s.osm" % tagv)
        x.write_text(GENERIC.replace('<tag k="highway" v="residential"/><tag k="oneway" v="yes"/>',
                                     '<tag k="highway" v="residential"/><tag k="junction" v="roundabout"/>' + ow))
        g = graphfile.load(world.import_osm(str(x), str(tmp_path / ("r%s.rmg" % tagv)), cell_m=50.0))
        e = g["edges"].reshape(-1, 4)
        acc = (e[:, 2] >> 16) & 7
        for a, w, r in zip(acc, g["edge_way"], e[:, 3]):
            if w != 200:
                continue
            assert bool(a & 1) == (rev_auto if (r & 1) else fwd_auto), (tagv, int(a), int(r))
            assert a & 4   # pedestrians both ways


def test_pbf_export_import_is_bit_identical(built_lib, tmp_path):
    """the world as OSM PBF — the input valhalla_build_tiles reads — comes back
    bit-identical, and carries the same elements as the XML export."""
    for name, (rows, cols, block, cell) in {"c1": (40, 40, 100.0, 100.0), "c3": (30, 30, 200.0, 200.0)}.items():
        src = str(tmp_path / (name + ".rmg"))
        world.build_world(src, rows, cols, block, seed=3, cell_m=cell)
        pbf = world.export_pbf(src, str(tmp_path / (name + ".osm.pbf")))
        back = world.import_osm(pbf, str(tmp_path / (name + "_pbf.rmg")))
        assert open(src, "rb").read() == open(back, "rb").read(), name
        data = open(pbf, "rb").read()
        assert data[4:5] == b"\x0a" and b"OSMHeader" in data[:32] and b"OSMData" in data
        xml = world.export_osm(src, str(tmp_path / (name + ".osm")))
        assert len(data) < len(open(xml, "rb").read()) / 5   # deflated, delta-coded


def test_pbf_keeps_floats_near_the_origin(built_lib, tmp_path):
    """Coordinates whose float nanodegrees would not survive (floats near 0 degrees that are not
    the nearest float of a nanodegree) travel as exact hex floats (reporter:ll): XML -> .rmg ->
    PBF -> .rmg is bit-identical."""
    x = tmp_path / "o.osm"
    x.write_text(GENERIC.replace('lat="47.0000" lon="8.0000"', 'lat="0.000123456789" lon="-0.0000987654321"')
                 .replace('lat="47.0000" lon="8.0020"', 'lat="0.0001" lon="0.0002"')
                 .replace('lat="47.0000" lon="8.0040"', 'lat="0.0001" lon="0.0004"')
                 .replace('lat="46.9990" lon="8.0020"', 'lat="0.0" lon="0.0002"')
                 .replace('lat="47.0010" lon="8.0020"', 'lat="0.0002" lon="0.0002"')
                 .replace('lat="47.0005" lon="8.0030"', 'lat="0.00015" lon="0.0003"'))
    a = world.import_osm(str(x), str(tmp_path / "o.rmg"), cell_m=10.0)
    g = graphfile.load(a)
    lat = g["node_lat"]
    lost = (np.round(lat.astype(np.float64) * 1e9) * 1e-9).astype(np.float32) != lat
    assert lost.any()   # nanodegrees alone would not bring these floats back
    pbf = world.export_pbf(a, str(tmp_path / "o.osm.pbf"))
    back = world.import_osm(pbf, str(tmp_path / "o_back.rmg"))
    assert open(a, "rb").read() == open(back, "rb").read()


def test_pbf_rejects_damage(built_lib, tmp_path):
    import pytest
    src = str(tmp_path / "d.rmg")
    world.build_world(src, 10, 10, 100.0, seed=6)
    pbf = world.export_pbf(src, str(tmp_path / "d.osm.pbf"))
    data = open(pbf, "rb").read()
    for cut in (len(data) - 7, len(data) // 2, 30):
        p = tmp_path / ("cut%d.pbf" % cut)
        p.write_bytes(data[:cut])
        with pytest.raises(RuntimeError):
            world.import_osm(str(p), str(tmp_path / "cut.rmg"))


SPLIT_OSMLR = """<?xml version='1.0' encoding='UTF-8'?>
<osm version="0.6" generator="hand">
 <node id="1" lat="47.0000" lon="8.0000"/>
 <node id="2" lat="47.0000" lon="8.0020"/>
 <node id="3" lat="47.0000" lon="8.0040"/>
 <node id="4" lat="46.9990" lon="8.0020"/>
 <way id="100"><nd ref="1"/><nd ref="2"/><nd ref="3"/><tag k="highway" v="primary"/></way>
 <way id="200"><nd ref="4"/><nd ref="2"/><tag k="highway" v="residential"/></way>
 <relation id="7"><member type="way" ref="100" role="forward"/>
  <tag k="type" v="osmlr"/><tag k="osmlr:id" v="%d"/></relation>
 <relation id="8"><member type="way" ref="100" role="backward"/>
  <tag k="type" v="osmlr"/><tag k="osmlr:id" v="%d"/></relation>
</osm>
"""


def test_osmlr_member_split_at_an_intersection_keeps_every_piece(built_lib, tmp_path):
    """way 100 is split at node 2 (way 200 joins there); the osmlr segments naming it
    cover both of its roads in travel order, with contiguous offsets, not the first piece alone."""
    p = tmp_path / "s.osm"
    p.write_text(SPLIT_OSMLR % (2 | (5 << 3), 2 | (6 << 3)))
    g = graphfile.load(world.import_osm(str(p), str(tmp_path / "s.rmg"), cell_m=50.0))
    e = g["edges"].reshape(-1, 4)
    for s in (0, 1):
        mine = np.nonzero(g["edge_seg"] == s)[0]
        assert len(mine) == 2, (s, mine)
        order = mine[np.argsort(g["edge_seg_off"][mine])]
        offs = g["edge_seg_off"][order]
        assert offs[0] == 0 and offs[1] == e[order[0], 1]          # contiguous
        assert g["seg_len_cm"][s] == e[order, 1].sum()
        # forward: from node 1 towards node 3; backward: the reverse edges, from node 3
        assert all(((e[order, 3] & 1) == s).tolist())


def test_implausible_grid_is_rejected(built_lib, tmp_path):
    import pytest
    src = str(tmp_path / "gr.rmg")
    world.build_world(src, 8, 8, 100.0, seed=7)
    osm = world.export_osm(src, str(tmp_path / "gr.osm"))
    text = open(osm).read()
    import re
    bad = re.sub(r'(k="reporter:grid" v="[^"]*?) \d+ \d+"', r'\1 4000000 4000000"', text)
    assert bad != text
    (tmp_path / "bad.osm").write_text(bad)
    with pytest.raises(RuntimeError, match="implausible"):
        world.import_osm(str(tmp_path / "bad.osm"), str(tmp_path / "bad.rmg"))


def test_valhalla_tile_files(built_lib, tmp_path):
    """The tiles the world's OSMLR ids name, and their file paths as get_tiles.py:79-102 forms
    them (level 2 ids have 7 digits padded to 9: 2/000/756/425.gph)."""
    assert world.valhalla_tile_file(2, 756425) == "2/000/756/425.gph"
    assert world.valhalla_tile_file(1, 37741) == "1/037/741.gph"
    assert world.valhalla_tile_file(0, 3015) == "0/003/015.gph"
    src = str(tmp_path / "t.rmg")
    world.build_world(src, 40, 40, 100.0, seed=1)
    tiles = world.valhalla_tiles(src)
    assert {lv for lv, _ in tiles} <= {0, 1, 2} and any(lv == 2 for lv, _ in tiles)
    for (lv, tl), f in tiles.items():
        assert f.startswith("%d/" % lv) and f.endswith(".gph")
