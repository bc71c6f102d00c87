"""rm_match_batch's device JSON path (round 4): the trace arrays of compact requests are parsed on
the GPU (engine.hip k_parse_json, rules in json_points.hpp), everything else on the host.

The replies must not depend on which parser read a request.  The same requests through Match (the
coalescer parses every request on the host) and through MatchMany without coalescing (the device
path) give identical replies; batches that mix compact requests with requests the device rejects
(whitespace, 17-digit numbers, extra keys, nested values) too; a failing request fails the call
with the host reader's message.  tests/cpp/trace_json_test.cpp checks the same rules against the
DOM reader on the host over ~30k documents.
"""
import json

import numpy as np
import pytest

from reporter_amd import world

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _device_parse_for_small_batches(monkeypatch):
    """These batches are ~1 MB of JSON, below the size from which rm_match_batch parses on the
    device (RM_JSON_DEVICE_MIN_MB, 8 MB): force the device path."""
    monkeypatch.setenv("RM_JSON_DEVICE_MIN_MB", "0")


def _compact(tr, k, fmt="%.6f", order=("lat", "lon", "time", "accuracy")):
    o0, o1 = int(tr["trace_off"][k]), int(tr["trace_off"][k + 1])
    pts = []
    for i in range(o0, o1):
        v = {"lat": fmt % float(tr["lat"][i]), "lon": fmt % float(tr["lon"][i]), "time": "%d" % int(tr["time"][i]),
             "accuracy": "%g" % float(tr["accuracy"][i])}
        pts.append("{" + ",".join('"%s":%s' % (key, v[key]) for key in order) + "}")
    return ('{"uuid":"%d","trace":[%s],"match_options":{"mode":"auto","report_levels":[0,1],'
            '"transition_levels":[0,1]}}' % (k, ",".join(pts)))


@pytest.fixture(scope="module")
def requests(small_world):
    tr = world.generate_traces(small_world, n_traces=48, n_points=300, rate_s=1.0, noise_m=5.0, seed=61)
    reqs = []
    for k in range(48):
        kind = k % 8
        if kind in (0, 1, 2):
            reqs.append(_compact(tr, k))                                   # the bench layout
        elif kind == 3:
            reqs.append(_compact(tr, k, order=("time", "accuracy", "lon", "lat")))
        elif kind == 4:
            reqs.append(json.dumps(world.trace_to_request(tr, k)))         # ", " / ": " separators
        elif kind == 5:   # float32 widened to double: 16-17 digits (host reader only)
            reqs.append(json.dumps(world.trace_to_request(tr, k), separators=(",", ":")))
        elif kind == 6:   # an extra key in one point
            s = _compact(tr, k)
            reqs.append(s.replace('},{', ',"speed":3},{', 1))
        else:             # a nested value in a point (the device's '{' count is not the point count)
            s = _compact(tr, k)
            reqs.append(s.replace('},{', ',"x":{"y":[1,{"z":2}]}},{', 2))
    return reqs


def test_device_path_replies_equal_host_path(small_world, tmp_path, requests):
    import valhalla
    valhalla.Configure(valhalla.write_config(str(tmp_path / "c.json"), small_world, device=0, coalesce=True))
    sm = valhalla.SegmentMatcher()
    want = [sm.Match(r) for r in requests]   # host reader (coalesced batches)
    sm.close()
    valhalla.Configure(valhalla.write_config(str(tmp_path / "nc.json"), small_world, device=0, coalesce=False))
    sm = valhalla.SegmentMatcher()
    assert sum(len(json.loads(w)["segments"]) for w in want) > 100
    # compact requests alone (all on the device), the mixed batch, and the mixed batch without the
    # nested-value requests (no whole-batch fall-back)
    compact = [k for k in range(len(requests)) if k % 8 in (0, 1, 2, 3)]
    assert sm.MatchMany([requests[k] for k in compact]) == [want[k] for k in compact]
    assert sm.MatchMany(requests) == want
    no_nested = [k for k in range(len(requests)) if k % 8 != 7]
    assert sm.MatchMany([requests[k] for k in no_nested]) == [want[k] for k in no_nested]
    assert sm.MatchMany(requests[:1]) == want[:1]
    # twice more: the grow-only buffers and a smaller batch after a larger one
    assert sm.MatchMany(requests[:7]) == want[:7]
    assert sm.MatchMany(requests) == want
    sm.close()


@pytest.mark.parametrize("bad", [
    '{"lat":95.0,"lon":8.0,"time":1,"accuracy":5}',       # compact, out of range
    '{"lat":47.0,"time":1,"accuracy":5}',                  # compact-looking, lon missing
    '{"lat":47.0,"lon":8.0,"time":1,"accuracy":5,}',       # syntax error inside the trace
])
def test_device_path_errors_are_the_host_readers(small_world, tmp_path, requests, bad):
    import valhalla
    valhalla.Configure(valhalla.write_config(str(tmp_path / "c2.json"), small_world, device=0, coalesce=True))
    sm = valhalla.SegmentMatcher()
    doc = requests[0].replace('"trace":[', '"trace":[' + bad + ",", 1)
    with pytest.raises(RuntimeError) as host_err:
        sm.Match(doc)
    sm.close()
    valhalla.Configure(valhalla.write_config(str(tmp_path / "nc2.json"), small_world, device=0, coalesce=False))
    sm = valhalla.SegmentMatcher()
    with pytest.raises(RuntimeError) as dev_err:
        sm.MatchMany([requests[1], doc, requests[2]])
    assert str(host_err.value) in str(dev_err.value) or str(dev_err.value) in str(host_err.value), (host_err.value,
                                                                                                   dev_err.value)
    # the matcher still serves afterwards
    assert len(sm.MatchMany(requests[:3])) == 3
    sm.close()


def test_device_path_many_threads(small_world, tmp_path, monkeypatch):
    """2,000 compact requests: every host pool thread fills and uploads its own arena (uploads
    from 16 threads on one stream, overlapping the parse); the replies equal the host path's."""
    import valhalla
    tr = world.generate_traces(small_world, n_traces=2000, n_points=40, rate_s=1.0, noise_m=5.0, seed=71)
    reqs = [_compact(tr, k) for k in range(2000)]
    valhalla.Configure(valhalla.write_config(str(tmp_path / "nc3.json"), small_world, device=0, coalesce=False))
    sm = valhalla.SegmentMatcher()
    monkeypatch.setenv("RM_JSON_DEVICE_MIN_MB", "100000")   # host parse
    want = sm.MatchMany(reqs)
    monkeypatch.setenv("RM_JSON_DEVICE_MIN_MB", "0")        # device parse
    got = sm.MatchMany(reqs)
    assert got == want
    assert sum(len(json.loads(w)["segments"]) for w in want) > 1000
    assert sm.MatchMany(reqs[:1500]) == want[:1500]
    sm.close()
