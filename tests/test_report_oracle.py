"""report() oracles against the reference's own golden vectors (CPU).

tests/golden/report_golden.json was produced by running the reference's
report() (py/reporter_service.py:79-179) — see tests/golden/make_report_golden.py.
"""
import copy
import json
import os

import numpy as np
import pytest

import report_oracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "report_golden.json")


@pytest.fixture(scope="module")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


def test_python_oracle_matches_reference_goldens(golden):
    assert len(golden) >= 400
    for i, rec in enumerate(golden):
        c = rec["input"]
        trace = {"trace": [{"time": c["trace_end_time"]}]}
        out = report_oracle.report(copy.deepcopy(c["match"]), trace, c["threshold_sec"], set(c["report_levels"]),
                                   set(c["transition_levels"]))
        assert json.loads(json.dumps(out)) == rec["output"], "case %d" % i


def _to_records(segs):
    from reporter_amd.engine import SEGMENT_DTYPE
    a = np.zeros(len(segs), SEGMENT_DTYPE)
    for i, s in enumerate(segs):
        has = "segment_id" in s and s["segment_id"] is not None
        a[i]["segment_id"] = s["segment_id"] if has else 0x3FFFFFFFFFFF
        a[i]["start_time"] = s["start_time"]
        a[i]["end_time"] = s["end_time"]
        a[i]["length"] = s["length"]
        a[i]["queue_length"] = s["queue_length"]
        a[i]["flags"] = (1 if s.get("internal", False) else 0) | (2 if has else 0)
        a[i]["begin_shape_index"] = s["begin_shape_index"]
        a[i]["end_shape_index"] = s["end_shape_index"]
        a[i]["seg_dense"] = 0xFFFFFFFF
    return a


def test_c_oracle_report_matches_reference_goldens(golden, built_lib):
    import meili_oracle as mo
    from reporter_amd.engine import levels_mask
    for i, rec in enumerate(golden):
        c, want = rec["input"], rec["output"]
        segs = _to_records(c["match"]["segments"])
        reps, st = mo.report_trace(segs, c["trace_end_time"], c["threshold_sec"], levels_mask(c["report_levels"]),
                                   levels_mask(c["transition_levels"]))
        wr = want["datastore"]["reports"]
        assert len(reps) == len(wr), "case %d" % i
        for r, w in zip(reps, wr):
            assert int(r["id"]) == w["id"] and float(r["t0"]) == w["t0"] and float(r["t1"]) == w["t1"]
            assert int(r["length"]) == w["length"] and int(r["queue_length"]) == w["queue_length"]
            assert (int(r["next_id"]) if int(r["next_id"]) != 0x3FFFFFFFFFFF else None) == w.get("next_id")
        ws = want["stats"]
        assert st["successful_count"] == ws["successful_matches"]["count"]
        assert st["unreported_count"] == ws["unreported_matches"]["count"]
        km = lambda m: 0 if m < 0 else round(m * 0.001, 3)
        assert km(st["successful_length_m"]) == ws["successful_matches"]["length"]
        assert km(st["unreported_length_m"]) == ws["unreported_matches"]["length"]
        assert st["discontinuities"] == ws["match_errors"]["discontinuities"]
        assert st["invalid_speeds"] == ws["match_errors"]["invalid_speeds"]
        assert st["invalid_times"] == ws["match_errors"]["invalid_times"]
        assert st["unassociated"] == ws["unassociated_segments"]
        assert (st["shape_used"] if st["shape_used"] >= 0 else None) == want.get("shape_used")
