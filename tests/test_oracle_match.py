"""CPU oracle sanity (no GPU): the restated matcher recovers the generator's true
roads, is deterministic, and its segments obey the reply schema invariants of
README.md:288-301 that report() relies on (py/reporter_service.py:79-179)."""
import numpy as np

import meili_oracle as mo
from reporter_amd import engine, graphfile, world


def _run(path, tr, **opt):
    g = graphfile.load(path)
    T = len(tr["trace_off"]) - 1
    b = mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], engine.default_options(1, **opt),
                 np.zeros(T, np.uint32))
    return g, mo.match(g, b)


def test_truth_recovery_low_noise(small_world):
    tr = world.generate_traces(small_world, 16, 300, rate_s=1.0, noise_m=2.0, seed=5)
    g, out = _run(small_world, tr)
    edges = g["edges"].reshape(-1, 4)
    ok = tot = 0
    for k in range(16):
        o = tr["trace_off"][k]
        for s in range(out["n_states"][k]):
            c = out["choice"][o + s]
            if c < 0:
                continue
            tot += 1
            ok += (edges[tr["truth_edge"][o + out["state_orig"][o + s]], 3] >> 1) == out["cand_road"][o + s, c]
    assert tot > 1000 and ok / tot > 0.95


def test_deterministic(small_world):
    tr = world.generate_traces(small_world, 8, 200, rate_s=1.0, noise_m=5.0, seed=6)
    _, a = _run(small_world, tr)
    _, b = _run(small_world, tr)
    for k in ("route", "choice", "path_pool"):
        np.testing.assert_array_equal(a[k], b[k])
    assert a["segs"].tobytes() == b["segs"].tobytes()


def test_segment_invariants(small_world):
    tr = world.generate_traces(small_world, 24, 300, rate_s=1.0, noise_m=5.0, seed=7)
    g, out = _run(small_world, tr)
    segs = out["segs"]
    assert len(segs) > 50
    has_id = (segs["flags"] & 2) > 0
    internal = (segs["flags"] & 1) > 0
    assert not np.any(has_id & internal)                      # internal runs carry no id (README.md:297)
    complete = has_id & (segs["start_time"] != -1) & (segs["end_time"] != -1)
    assert np.all(segs["length"][complete] > 0)
    assert np.all(segs["length"][has_id & ~complete] == -1)   # partial -> -1 (README.md:296)
    both = (segs["start_time"] != -1) & (segs["end_time"] != -1)
    assert np.all(segs["end_time"][both] >= segs["start_time"][both])
    assert np.all(segs["begin_shape_index"] <= segs["end_shape_index"])
    ids = segs["segment_id"][has_id]
    assert set(np.unique(ids & 7).tolist()) <= {0, 1, 2}
    assert np.all(segs["queue_length"] >= 0)


def test_sparse_routes_use_long_searches(built_lib, tmp_path):
    p = str(tmp_path / "sparse.rmg")
    world.build_world(p, 40, 40, 200.0, seed=2, cell_m=200.0)
    tr = world.generate_traces(p, 16, 30, rate_s=30.0, noise_m=5.0, seed=8)
    mo.reset_counters()
    _, out = _run(p, tr, search_radius=100.0)
    c = mo.counters()
    assert c["settled"] / max(c["searches"], 1) > 20   # long bounded searches (C3 regime)
    assert (out["choice"] >= 0).sum() > 300


def test_truth_recovery_sparse_and_sigma_sweep(built_lib, tmp_path):
    """The oracle's spec recovers the driven road in the C3 regime (30 s sampling, 100 m
    radius) and across C5's modes x sigma_z (CPU, small samples; the GPU test
    tests/test_gpu_pinned.py asserts the same on the GPU's own choices at full size)."""
    from parity_util import truth_recovery
    p = str(tmp_path / "c3like.rmg")
    world.build_world(p, 60, 60, 200.0, seed=3, cell_m=200.0)
    tr = world.generate_traces(p, 200, 40, rate_s=30.0, noise_m=5.0, seed=9)
    g, out = _run(p, tr, search_radius=100.0)
    frac, n, _ = truth_recovery(tr["trace_off"], out["n_states"], out["state_orig"], out["cand_road"], out["choice"],
                                tr["truth_edge"], g["edges"])
    assert n > 5000 and frac > 0.93, (frac, n)
    p2 = str(tmp_path / "c5like.rmg")
    world.build_world(p2, 60, 60, 100.0, seed=1)
    floors = {2.0: 0.95, 8.0: 0.87, 16.0: 0.72}
    for mode in ("auto", "bicycle", "pedestrian"):
        for sz, floor in floors.items():
            tr = world.generate_traces(p2, 12, 300, rate_s=1.0, noise_m=sz, seed=11, mode=mode)
            g, out = _run(p2, tr, mode=world.MODES[mode], sigma_z=sz, search_radius=max(50.0, 3 * sz))
            frac, n, _ = truth_recovery(tr["trace_off"], out["n_states"], out["state_orig"], out["cand_road"],
                                        out["choice"], tr["truth_edge"], g["edges"])
            assert n > 300 and frac > floor, (mode, sz, frac, n)


def test_oracle_on_the_readme_manila_trace(tmp_path, built_lib):
    """The README.md:269 trace (no accuracy, 7-29 s sampling) on a world centred on it: the
    oracle's segments follow the reply schema README.md:270-301 (the GPU test compares the
    engine against these)."""
    from test_gpu_manila import check_schema, manila_world, oracle_segments
    path = str(tmp_path / "manila.rmg")
    req = manila_world(path)
    segs = oracle_segments(path, req)
    assert len(segs) >= 3 and any("segment_id" in s for s in segs)
    check_schema(segs, len(req["trace"]))
