"""The one Match input the reference itself holds: the Manila trace of README.md:269
(tests/golden/manila_readme_trace.json, made by tests/golden/make_manila_fixture.py).

It is the reference's own /report example: 14 points, no `accuracy`, no match_options, and
irregular 7-29 s sampling.  The reference gives no expected output for it, so the reply is
checked two ways: segment for segment against the oracle on a world centred on the trace, and
against the reply schema README.md:270-301 documents (segment_id omitted without OSMLR coverage,
internal true only without a segment_id, -1 for times / lengths not known, shape indices into
the trace).  report() (reporter_service.py:79-179, restated in oracle/report_oracle.py) then
turns it into the datastore output README.md:271-273 shows."""
import json
import os

import numpy as np
import pytest

import meili_oracle as mo
import report_oracle
from reporter_amd import engine, graphfile, world

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _fixture():
    with open(os.path.join(HERE, "golden", "manila_readme_trace.json")) as f:
        return json.load(f)["request"]


def manila_world(path):
    req = _fixture()
    lat = [p["lat"] for p in req["trace"]]
    lon = [p["lon"] for p in req["trace"]]
    world.build_world(path, 40, 40, 100.0, seed=11, cell_m=100.0, center_lat=0.5 * (min(lat) + max(lat)),
                      center_lon=0.5 * (min(lon) + max(lon)))
    return req


def oracle_segments(path, req):
    n = len(req["trace"])
    tr = dict(trace_off=np.array([0, n], np.uint32),
              lon=np.array([p["lon"] for p in req["trace"]], np.float64),
              lat=np.array([p["lat"] for p in req["trace"]], np.float64),
              time=np.array([p["time"] for p in req["trace"]], np.float64),
              accuracy=np.full(n, -1.0, np.float32))   # the request carries no accuracy
    ref = mo.match(graphfile.load(path), mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"],
                                                  engine.default_options(1), np.zeros(1, np.uint32)))
    return engine.segment_dicts(ref["segs"])


def check_schema(segs, n_points):
    keys = {"way_ids", "start_time", "end_time", "queue_length", "length", "internal", "begin_shape_index",
            "end_shape_index"}
    for s in segs:
        assert keys <= set(s) <= keys | {"segment_id"}, s
        assert isinstance(s["way_ids"], list) and 1 <= len(s["way_ids"]) <= 2
        assert all(isinstance(w, int) and w >= 0 for w in s["way_ids"])
        if "segment_id" in s:
            assert not s["internal"]                       # internal only without a segment id
            assert 0 < s["segment_id"] < 0x3fffffffffff    # INVALID_SEGMENT_ID never appears
            assert (s["segment_id"] & 7) in (0, 1, 2)      # level bits (simple_reporter.py:37-49)
        for k in ("start_time", "end_time"):
            assert s[k] == -1 or (isinstance(s[k], float) and 1000.0 <= s[k] <= 1167.0), s
        if s["start_time"] != -1 and s["end_time"] != -1:
            assert s["start_time"] <= s["end_time"]
        # an OSMLR segment's length only when it was entered and left at its ends (README.md:298);
        # a run without OSMLR coverage (internal / unassociated) reports the metres it covered
        if "segment_id" in s:
            assert (s["length"] == -1) == (s["start_time"] == -1 or s["end_time"] == -1), s
        else:
            assert s["length"] >= 0
        assert isinstance(s["queue_length"], int) and s["queue_length"] >= 0
        assert 0 <= s["begin_shape_index"] <= s["end_shape_index"] < n_points
    for a, b in zip(segs, segs[1:]):
        assert a["begin_shape_index"] <= b["begin_shape_index"]


def test_manila_readme_trace(built_lib, tmp_path):
    import valhalla
    path = str(tmp_path / "manila.rmg")
    req = manila_world(path)
    want = oracle_segments(path, req)
    assert len(want) >= 3
    conf = valhalla.write_config(str(tmp_path / "manila.json"), path, device=0)
    valhalla.Configure(conf)
    sm = valhalla.SegmentMatcher()
    got = json.loads(sm.Match(json.dumps(req, separators=(",", ":"))))
    assert set(got) == {"segments"}
    assert got["segments"] == want
    check_schema(got["segments"], len(req["trace"]))
    assert any("segment_id" in s for s in got["segments"])
    # the service's post-processing (reporter_service.py:240-242), levels as the README run
    trace = dict(req, match_options={"report_levels": [0, 1], "transition_levels": [0, 1]})
    rep = report_oracle.report(got, trace, 15, {0, 1}, {0, 1})
    assert rep["segment_matcher"]["mode"] == "auto" and rep["datastore"]["mode"] == "auto"
    for r in rep["datastore"]["reports"]:
        assert set(r) <= {"id", "next_id", "t0", "t1", "length", "queue_length"}
    print("manila", len(got["segments"]), "segments;", len(rep["datastore"]["reports"]), "reports;",
          "shape_used", rep.get("shape_used"))
    sm.close()
