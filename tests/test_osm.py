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
