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


def test_pipeline_duration_sums_and_histogram(small_world):
    """og_pipeline2's per-segment duration sums (reduced with the histogram)
    equal sum(int(round(t1 - t0))) of the reports the histogram counts, recomputed here from
    the oracle's segments through report() and the batch filter of py/simple_reporter.py:177-179
    (Python round() of a positive float > 0.5 = floor(x + 0.5) up to the exact-half ties, which
    Python 2 rounds away from zero: np.floor(x + 0.5) matches both)."""
    tr = world.generate_traces(small_world, 24, 300, rate_s=1.0, noise_m=5.0, seed=17)
    g, out = _run(small_world, tr)
    nseg = len(g["seg_id"])
    T = len(tr["trace_off"]) - 1
    b = mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], engine.default_options(1),
                 np.zeros(T, np.uint32))
    hist = np.zeros(nseg * 16, np.uint32)
    dur = np.zeros(nseg, np.uint64)
    nvalid = mo.pipeline(g, b, 15.0, 0x6, 0x6, hist, dur)
    want_h = np.zeros(nseg * 16, np.uint64)
    want_d = np.zeros(nseg, np.uint64)
    n = 0
    for k in range(T):
        segs = out["segs"][out["seg_off"][k]:out["seg_off"][k + 1]]
        end = tr["time"][tr["trace_off"][k + 1] - 1]
        reps, _ = mo.report_trace(segs, end, 15.0, 0x6, 0x6)
        for r in reps:
            dt = r["t1"] - r["t0"]
            if not (r["t0"] > 0 and r["t1"] > 0 and dt > 0.5 and r["length"] > 0 and r["queue_length"] >= 0):
                continue
            n += 1
            if r["seg_dense"] == 0xFFFFFFFF:
                continue
            want_h[r["seg_dense"] * 16 + min(15, max(0, int(r["length"] / dt * 3.6 / 10.0)))] += 1
            want_d[r["seg_dense"]] += int(np.floor(dt + 0.5))
    assert nvalid == n and n > 50
    np.testing.assert_array_equal(hist, want_h.astype(np.uint32))
    np.testing.assert_array_equal(dur, want_d)


def test_path_walk_counters(small_world):
    """Counters behind bench.py's paths roofline: after prepare_path_counters, every walked
    node visits at least its canonical in-edge, and each visited usable in-edge reads at most
    two route-ball rows."""
    tr = world.generate_traces(small_world, 16, 300, rate_s=1.0, noise_m=5.0, seed=18)
    g = graphfile.load(small_world)
    T = len(tr["trace_off"]) - 1
    b = mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], engine.default_options(1),
                 np.zeros(T, np.uint32))
    mo.reset_counters()
    mo.match(g, b)
    assert mo.counters()["path_in_edges"] == 0          # not prepared: not counted
    mo.prepare_path_counters(g)
    mo.reset_counters()
    out = mo.match(g, b)
    c = mo.counters()
    walked = int(np.maximum(out["path_cnt"][out["path_cnt"] > 2].astype(np.int64) - 2, 0).sum())
    assert c["chained"] > 1000 and walked > 0
    assert c["path_in_edges"] >= walked
    assert c["path_rows"] <= 2 * c["path_in_edges"] + 4 * c["chained"]
    assert mo.paths_algorithmic_bytes(c) > 116 * c["chained"]


def test_target_stopped_counters(small_world):
    """Counters 17-19 (the search roofline's formulation since round 4): the settles, scans and label
    writes of the same searches stopped at their targets are a prefix of the full searches', and at
    sparse sampling (bounds far beyond the targets) a small part of them."""
    tr = world.generate_traces(small_world, 40, 40, rate_s=30.0, noise_m=5.0, seed=9)
    mo.reset_counters()
    _run(small_world, tr, search_radius=100.0)
    c = mo.counters()
    assert c["searches"] > 1000
    for a, b in (("settled_to_targets", "settled"), ("scanned_to_targets", "scanned"),
                 ("label_writes_to_targets", "label_writes")):
        assert 0 < c[a] <= c[b], (a, c)
    assert c["settled_to_targets"] < 0.6 * c["settled"], c
    assert mo.routes_targets_algorithmic_bytes(c) < mo.routes_algorithmic_bytes(c)
