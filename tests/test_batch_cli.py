"""Host side of the GPU batch reporter (reporter_amd/batch.py): trace-file parsing in
the reference's format (py/simple_reporter.py:113,139-140), vehicle ids, config, output."""
import json

import numpy as np

from reporter_amd import batch


def test_trace_files_and_ids(tmp_path):
    p = tmp_path / "abc"
    p.write_text("veh1,1483228800,47.1,8.2,5\nveh2,1483228801,47.2,8.3,7\n\nveh1,1483228790,47.0,8.1,4\n")
    uuids, pts = batch.read_trace_files([str(p)])
    assert uuids == ["veh1", "veh2", "veh1"]
    np.testing.assert_array_equal(pts["time"], [1483228800, 1483228801, 1483228790])
    np.testing.assert_array_equal(pts["accuracy"], np.array([5, 7, 4], np.float32))
    idx, names = batch.dense_ids(uuids)
    assert names == ["veh1", "veh2"] and list(idx) == [0, 1, 0]


def test_config_and_output(built_lib, tmp_path):
    conf = tmp_path / "conf.json"
    conf.write_text(json.dumps({"meili": {"default": {"sigma_z": 5.0, "beta": 4.0}, "bicycle": {"search_radius": 30}},
                                "reporter_amd": {"graph": "g.rmg"}}))
    o, g = batch.options_from_config(str(conf), "bicycle")
    assert float(o["sigma_z"][0]) == 5.0 and float(o["beta"][0]) == 4.0 and float(o["search_radius"][0]) == 30.0
    assert int(o["mode"][0]) == 3 and g == str(tmp_path / "g.rmg")
    batch.write_tiles({"0_3599/1/5": "h\nx\n"}, str(tmp_path / "out"))
    assert (tmp_path / "out" / "0_3599" / "1" / "5").read_text() == "h\nx\n"
