"""turn_penalty_factor is refused, not dropped.

meili adds turn costs to the transition cost when turn_penalty_factor > 0.  The reference's
client sends the field (py/generate_test_trace.py:37,47).  The stock valhalla_build_config
(reference Dockerfile:42-49) configures it per mode.  This matcher has no turn costs (DESIGN.md
§3).  So a request asking for them fails: reporter_service.py:244-245 answers 500 and
simple_reporter.py:169-173 skips the window.  A configured non-zero value fails Configure unless
reporter_amd.ignore_turn_penalty accepts zero turn costs.  It used to be parsed and ignored.
"""
import json

import numpy as np
import pytest

from reporter_amd import engine, world


def _conf(tmp_path, meili, ra=None):
    p = tmp_path / "conf.json"
    ra = dict(ra or {})
    ra.setdefault("graph", str(tmp_path / "missing.rmg"))
    p.write_text(json.dumps({"meili": meili, "reporter_amd": ra}))
    return str(p)


def test_configure_refuses_turn_costs(built_lib, tmp_path):
    """Checked before the graph loads (no GPU needed): the message names the mode and the fix."""
    import valhalla
    for meili in ({"auto": {"turn_penalty_factor": 200}}, {"default": {"turn_penalty_factor": 5}},
                  {"pedestrian": {"turn_penalty_factor": 100, "search_radius": 50}}):
        with pytest.raises(RuntimeError, match="turn_penalty_factor"):
            valhalla.Configure(_conf(tmp_path, meili))
    # accepted as zero with the opt-in: Configure gets as far as the (missing) graph
    with pytest.raises(RuntimeError, match="missing.rmg"):
        valhalla.Configure(_conf(tmp_path, {"auto": {"turn_penalty_factor": 200}}, {"ignore_turn_penalty": True}))
    with pytest.raises(RuntimeError, match="missing.rmg"):
        valhalla.Configure(_conf(tmp_path, {"auto": {"turn_penalty_factor": 0}}))


@pytest.mark.gpu
def test_request_with_turn_costs_fails_alone(small_world, tmp_path):
    """Through the drop-in: a request with turn_penalty_factor 200 raises (the service's 500),
    the same request with 0 is answered, and coalesced neighbours are unaffected; the batch API
    refuses it too."""
    import valhalla
    conf = valhalla.write_config(str(tmp_path / "tp.json"), small_world, device=0, coalesce=True)
    valhalla.Configure(conf)
    sm = valhalla.SegmentMatcher()
    tr = world.generate_traces(small_world, n_traces=2, n_points=120, rate_s=1.0, noise_m=5.0, seed=5)
    ok = json.dumps(world.trace_to_request(tr, 0, turn_penalty_factor=0), separators=(",", ":"))
    bad = json.dumps(world.trace_to_request(tr, 1, turn_penalty_factor=200), separators=(",", ":"))
    with pytest.raises(RuntimeError, match="turn_penalty_factor must be 0"):
        sm.Match(bad)
    assert json.loads(sm.Match(ok))["segments"]
    sm.close()
    eng = engine.Engine(small_world, 0)
    bm = engine.BatchMatcher(eng)
    opts = engine.default_options(1)
    opts[0]["turn_penalty_factor"] = 140.0
    with pytest.raises(RuntimeError, match="turn_penalty_factor must be 0"):
        bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, np.zeros(2, np.uint32))
    bm.close()
    eng.close()
