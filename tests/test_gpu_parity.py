"""GPU parity: the HIP engine against the CPU oracle, bit-exact at every stage.

Inputs are seeded synthetic worlds/traces (BASELINE.json configs, scaled so
the oracle finishes in seconds).  Exactness bar: integer/index outputs equal,
fp32/fp64 outputs equal bit for bit (the engine and the oracle share one
written arithmetic spec; -ffp-contract=off on both sides).
"""
import json
import os

import numpy as np
import pytest

import meili_oracle as mo
import report_oracle
from parity_util import check_reports as _check_reports, compare_all
from reporter_amd import engine, graphfile, world

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c1(small_world):
    eng = engine.Engine(small_world, 0)
    return small_world, graphfile.load(small_world), eng


def _run_both(graph_path, g, eng, tr, opts, trace_opt, **rp):
    bm = engine.BatchMatcher(eng)
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, trace_opt, **rp)
    ref = mo.match(g, mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, trace_opt))
    return bm, ref


def test_c1_dense_1hz(c1):
    path, g, eng = c1
    tr = world.generate_traces(path, n_traces=64, n_points=400, rate_s=1.0, noise_m=5.0, seed=11)
    opts = engine.default_options(1)
    bm, ref = _run_both(path, g, eng, tr, opts, np.zeros(64, np.uint32))
    c = compare_all(bm, ref, tr["trace_off"])
    assert c["chained"] > 1000 and c["segments"] > 100
    nrep = _check_reports(bm, ref, tr)
    assert nrep > 0
    print("C1 parity", c, "reports", nrep)


@pytest.mark.parametrize("radius_m", [0.0, 60.0, 400.0])
def test_route_ball_tier_radius(small_world, radius_m):
    """K2 answered by the route balls (table probes), by the bounded searches (radius 0),
    and by both (a radius most bounds exceed): routes identical to the oracle's searches."""
    g = graphfile.load(small_world)
    eng = engine.Engine(small_world, 0)
    eng.set_ball_radius(radius_m)
    tr = world.generate_traces(small_world, n_traces=48, n_points=300, rate_s=2.0, noise_m=5.0, seed=21)
    opts = engine.default_options(2)
    opts[1]["mode"] = 3   # bicycle: a second mode's tables
    trace_opt = (np.arange(48) % 2).astype(np.uint32)
    bm, ref = _run_both(small_world, g, eng, tr, opts, trace_opt)
    c = compare_all(bm, ref, tr["trace_off"])
    assert c["chained"] > 500
    tiers = bm.route_tiers()
    st = eng.ball_stats(0)
    if radius_m == 0.0:
        assert st["keys"] == 0
    else:
        assert st["keys"] > 0 and eng.ball_stats(3)["keys"] > 0
    if radius_m == 60.0:
        assert tiers["ball_to_search"] > 0    # the mixed case really mixes
    print("ball radius", radius_m, tiers, st)
    bm.close()
    eng.close()


def test_route_ball_beyond_radius(built_lib, tmpdir_session):
    """Pairs whose bound exceeds the ball radius (30 s sampling: bounds up to 2 km, tables of
    500 m) are answered by the tables when every route of the item is provably exact
    (ball_exact_limit: distance <= exit key + radius), else by the search tiers.  Routes, paths
    and segments equal the oracle's (full bounded searches), and the tables decide most items."""
    path = str(tmpdir_session / "beyond.rmg")
    world.build_world(path, 80, 80, 200.0, seed=5, cell_m=200.0)
    g = graphfile.load(path)
    eng = engine.Engine(path, 0)
    eng.set_ball_radius(500.0)
    tr = world.generate_traces(path, n_traces=400, n_points=40, rate_s=30.0, noise_m=5.0, seed=25)
    opts = engine.default_options(1, search_radius=100.0)
    bm, ref = _run_both(path, g, eng, tr, opts, np.zeros(400, np.uint32))
    c = compare_all(bm, ref, tr["trace_off"])
    tiers = bm.route_tiers()
    items = int(sum(np.asarray(ref["cand_n"][:-1], np.int64)))   # an upper bound of the (pair, source) items
    assert c["chained"] > 5000
    assert 0 < tiers["ball_to_search"] < items // 2, (tiers, items)
    assert tiers["paths_ball_to_search"] > 0
    print("beyond radius", tiers, "items <=", items, c)
    bm.close()
    eng.close()


def test_route_ball_nodes_without_table(small_world, monkeypatch):
    """Nodes whose ball is too large get no table; transitions leaving through them are
    handed to the search tiers (K2 and paths) with identical results."""
    monkeypatch.setenv("RM_BALL_MAX_KEYS", "8")   # 200 m balls hold ~5-13 nodes on this grid: a mix
    g = graphfile.load(small_world)
    eng = engine.Engine(small_world, 0)
    eng.set_ball_radius(200.0)
    tr = world.generate_traces(small_world, n_traces=32, n_points=300, rate_s=1.0, noise_m=5.0, seed=23)
    bm, ref = _run_both(small_world, g, eng, tr, engine.default_options(1), np.zeros(32, np.uint32))
    c = compare_all(bm, ref, tr["trace_off"])
    st, tiers = eng.ball_stats(0), bm.route_tiers()
    assert st["nodes_without_table"] > 0 and st["keys"] > 0
    assert tiers["ball_to_search"] > 0 and tiers["paths_ball_to_search"] > 0
    assert c["chained"] > 500
    print("no-table nodes", st, tiers)
    bm.close()
    eng.close()


def test_sparse_30s_large_radius(built_lib, tmpdir_session):
    """C3-like: 30 s sampling, 200 m blocks, radius 100 m -> long bounded searches (retry tier)."""
    path = str(tmpdir_session / "c3s.rmg")
    world.build_world(path, 60, 60, 200.0, seed=3, cell_m=200.0)
    g = graphfile.load(path)
    eng = engine.Engine(path, 0)
    tr = world.generate_traces(path, n_traces=64, n_points=40, rate_s=30.0, noise_m=5.0, seed=5)
    opts = engine.default_options(1, search_radius=100.0)
    bm, ref = _run_both(path, g, eng, tr, opts, np.zeros(64, np.uint32))
    c = compare_all(bm, ref, tr["trace_off"])
    _check_reports(bm, ref, tr)
    print("sparse parity", c)


def test_mixed_modes_sigma_sweep(c1):
    """C5-like: auto/bicycle/pedestrian traces, sigma_z in {2, 4.07, 8, 16}, noise = sigma."""
    path, g, eng = c1
    parts, opts = [], []
    for mi, mode in enumerate(("auto", "bicycle", "pedestrian")):
        for si, sz in enumerate((2.0, 4.07, 8.0, 16.0)):
            tr = world.generate_traces(path, n_traces=4, n_points=200, rate_s=1.0, noise_m=sz, seed=100 + mi * 10 + si,
                                       mode=mode)
            parts.append(tr)
            opts.append(engine.default_options(1, mode=world.MODES[mode], sigma_z=sz,
                                               search_radius=max(50.0, 3 * sz))[0])
    tr = {k: np.concatenate([p[k] for p in parts]) for k in ("lon", "lat", "time", "accuracy")}
    tr["trace_off"] = (np.arange(len(parts) * 4 + 1) * 200).astype(np.uint32)
    trace_opt = np.repeat(np.arange(len(parts), dtype=np.uint32), 4)
    opts = np.array(opts, engine.OPTIONS_DTYPE)
    bm, ref = _run_both(path, g, eng, tr, opts, trace_opt, report_levels=(0, 1, 2), transition_levels=(0, 1, 2))
    c = compare_all(bm, ref, tr["trace_off"])
    _check_reports(bm, ref, tr, rl=(0, 1, 2), tl=(0, 1, 2))
    print("mixed parity", c)


def test_edge_cases(c1):
    """Points off the graph (no candidates -> chain breaks), duplicates (interpolation),
    a 1-point trace, non-increasing times, a long gap (breakage)."""
    path, g, eng = c1
    tr = world.generate_traces(path, n_traces=6, n_points=120, rate_s=1.0, noise_m=3.0, seed=77)
    lon, lat, tm = tr["lon"].copy(), tr["lat"].copy(), tr["time"].copy()
    lon[130:135] += 1.0                     # trace 1: 5 points far away
    lon[250:260] = lon[249]; lat[250:260] = lat[249]  # trace 2: stationary
    tm[370:380] = tm[369]                    # trace 3: frozen clock
    lat[540:600] += 0.02                     # trace 4: jump > breakage in the middle
    off = list(tr["trace_off"])
    # append a single-point trace
    lon = np.append(lon, lon[0]); lat = np.append(lat, lat[0]); tm = np.append(tm, tm[0])
    acc = np.append(tr["accuracy"], -1.0).astype(np.float32)
    off.append(off[-1] + 1)
    trd = dict(lon=lon, lat=lat, time=tm, accuracy=acc, trace_off=np.array(off, np.uint32))
    opts = engine.default_options(1)
    bm, ref = _run_both(path, g, eng, trd, opts, np.zeros(len(off) - 1, np.uint32))
    compare_all(bm, ref, trd["trace_off"])
    _check_reports(bm, ref, trd)
    choice, cs = bm.viterbi()
    assert cs.sum() > 7  # breaks happened


def test_histogram_matches_cpu_pipeline(c1):
    path, g, eng = c1
    tr = world.generate_traces(path, n_traces=128, n_points=300, rate_s=1.0, noise_m=5.0, seed=21)
    opts = engine.default_options(1)
    nseg = eng.n_segments
    import ctypes
    from reporter_amd import _lib
    dptr = ctypes.c_void_p()
    _lib.check(_lib.lib().rm_device_alloc(nseg * 16 * 4, ctypes.byref(dptr)))
    try:
        _lib.check(_lib.lib().rm_device_memset(dptr, 0, nseg * 16 * 4))
        bm = engine.BatchMatcher(eng)
        bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts,
               np.zeros(128, np.uint32), hist_dev=dptr.value, report_levels=(0, 1, 2), transition_levels=(0, 1, 2))
        hist = np.empty(nseg * 16, np.uint32)
        _lib.check(_lib.lib().rm_device_download(hist.ctypes.data, dptr, hist.nbytes))
    finally:
        _lib.lib().rm_device_free(dptr)
    want = np.zeros(nseg * 16, np.uint32)
    nvalid = mo.pipeline(g, mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts,
                                     np.zeros(128, np.uint32)), 15.0, 0xE, 0xE, want)
    np.testing.assert_array_equal(hist, want)
    assert int(hist.sum()) == nvalid > 0


def test_valhalla_dropin_json(c1, tmpdir_session):
    """The drop-in module: Configure + SegmentMatcher().Match, then the reference's
    report() restatement on the reply, as reporter_service.py:240-242 does."""
    path, g, eng = c1
    import valhalla
    conf = valhalla.write_config(str(tmpdir_session / "conf.json"), path, device=0)
    valhalla.Configure(conf)
    sm = valhalla.SegmentMatcher()
    tr = world.generate_traces(path, n_traces=8, n_points=150, rate_s=1.0, noise_m=5.0, seed=31)
    opts = engine.default_options(1)
    ref = mo.match(g, mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts,
                               np.zeros(8, np.uint32)))
    reqs = [world.trace_to_request(tr, k) for k in range(8)]
    outs = [sm.Match(json.dumps(r, separators=(",", ":"))) for r in reqs]
    outs2 = sm.MatchMany([json.dumps(r) for r in reqs])
    for k in range(8):
        got = json.loads(outs[k])
        assert got == json.loads(outs2[k])
        want = engine.segment_dicts(ref["segs"][ref["seg_off"][k]:ref["seg_off"][k + 1]])
        assert got["segments"] == want
        rep = report_oracle.report(got, reqs[k], 15, {0, 1}, {0, 1})
        assert "datastore" in rep and rep["segment_matcher"]["mode"] == "auto"
    # error path -> RuntimeError (service answers 500, reporter_service.py:244-245)
    with pytest.raises(RuntimeError):
        sm.Match('{"uuid":"x","trace":[]}')
    with pytest.raises(RuntimeError):
        sm.Match('{"uuid":"x","trace":[{"lat":1.0}]}')
    with pytest.raises(RuntimeError):
        sm.Match("not json")
    # the packed batch path without coalescing: the same replies, one failing trace fails the call
    sm.close()
    conf = valhalla.write_config(str(tmpdir_session / "conf_nc.json"), path, device=0, coalesce=False)
    valhalla.Configure(conf)
    sm = valhalla.SegmentMatcher()
    assert sm.MatchMany([json.dumps(r) for r in reqs]) == outs2
    assert sm.MatchMany([json.dumps(reqs[0])]) == outs2[:1]
    assert sm.MatchMany([]) == []
    with pytest.raises(RuntimeError):
        sm.MatchMany([json.dumps(reqs[0]), '{"uuid":"x","trace":[]}'])
    sm.close()


def test_rerun_is_deterministic(c1):
    path, g, eng = c1
    tr = world.generate_traces(path, n_traces=32, n_points=200, rate_s=1.0, noise_m=5.0, seed=41)
    bm = engine.BatchMatcher(eng)
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"])
    o1, s1 = bm.segments()
    for _ in range(3):
        bm.rerun()
        o2, s2 = bm.segments()
        np.testing.assert_array_equal(o1, o2)
        assert s1.tobytes() == s2.tobytes()


def test_coalesced_match_from_threads(c1, tmpdir_session):
    """The service's threading model (one SegmentMatcher per worker thread,
    py/reporter_service.py:28-64) over the coalescing drop-in: concurrent Match calls
    are served by shared GPU batches and every caller gets its own exact reply."""
    import threading
    import valhalla
    path, g, eng = c1
    conf = valhalla.write_config(str(tmpdir_session / "conf_coalesce.json"), path, device=0, coalesce=True,
                                 coalesce_window_ms=3.0)
    valhalla.Configure(conf)
    before = valhalla.coalesce_stats()
    n = 96
    tr = world.generate_traces(path, n_traces=n, n_points=120, rate_s=1.0, noise_m=5.0, seed=61)
    ref = mo.match(g, mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"],
                               engine.default_options(1), np.zeros(n, np.uint32)))
    reqs = [json.dumps(world.trace_to_request(tr, k), separators=(",", ":")) for k in range(n)]
    out = [None] * n
    errors = []

    def worker(tid):
        try:
            sm = valhalla.SegmentMatcher()
            for k in range(tid, n, 12):
                out[k] = sm.Match(reqs[k])
            with pytest.raises(RuntimeError):   # a bad request fails alone (HTTP 500 path)
                sm.Match('{"uuid":"x","trace":[]}')
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(12)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errors, errors
    for k in range(n):
        want = engine.segment_dicts(ref["segs"][ref["seg_off"][k]:ref["seg_off"][k + 1]])
        assert json.loads(out[k])["segments"] == want
    st = valhalla.coalesce_stats()
    served = st["requests"] - before["requests"]
    assert served == n
    assert st["batches"] - before["batches"] < served and st["max_batch"] > 1
    print("coalescing", st)


def test_coalesced_large_batch(c1, tmpdir_session):
    """80 requests released at once into a 200 ms coalescing window form batches larger than the
    32 traces one host thread assembles, so the batch is gathered into the dispatcher's pinned
    staging by several pool threads; every caller still gets its exact reply."""
    import threading
    import valhalla
    path, g, eng = c1
    conf = valhalla.write_config(str(tmpdir_session / "conf_coalesce_big.json"), path, device=0, coalesce=True,
                                 coalesce_window_ms=200.0)
    valhalla.Configure(conf)
    n = 80
    tr = world.generate_traces(path, n_traces=n, n_points=100, rate_s=1.0, noise_m=5.0, seed=62)
    ref = mo.match(g, mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"],
                               engine.default_options(1), np.zeros(n, np.uint32)))
    reqs = [json.dumps(world.trace_to_request(tr, k), separators=(",", ":")) for k in range(n)]
    out, errors = [None] * n, []
    gate = threading.Barrier(n)

    def worker(k):
        try:
            sm = valhalla.SegmentMatcher()
            gate.wait()
            out[k] = sm.Match(reqs[k])
            sm.close()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(k,)) for k in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errors, errors
    for k in range(n):
        want = engine.segment_dicts(ref["segs"][ref["seg_off"][k]:ref["seg_off"][k + 1]])
        assert json.loads(out[k])["segments"] == want
    st = valhalla.coalesce_stats()
    assert st["max_batch"] > 32, st


def test_randomised_options_per_trace(c1):
    """Every MatchOptions field varied per trace (one option row per trace), with mixed sampling
    rates and noise: the GPU against the oracle at every stage, and report() on top."""
    path, g, eng = c1
    rng = np.random.default_rng(2024)
    parts, opts = [], []
    modes = list(world.MODES)
    for q in range(48):
        mode = modes[q % len(modes)]
        rate = float(rng.choice([1.0, 2.0, 5.0, 15.0, 30.0, 60.0]))
        noise = float(rng.uniform(2.0, 20.0))
        n_pts = int(rng.integers(2, 400))
        parts.append(world.generate_traces(path, 1, n_pts, rate, noise, seed=int(rng.integers(1 << 30)), mode=mode))
        opts.append(engine.default_options(
            1, mode=world.MODES[mode], sigma_z=float(rng.uniform(1.0, 25.0)), beta=float(rng.uniform(0.3, 12.0)),
            search_radius=float(rng.uniform(5.0, 220.0)), gps_accuracy=float(rng.uniform(1.0, 60.0)),
            breakage_distance=float(rng.uniform(150.0, 4000.0)),
            interpolation_distance=float(rng.uniform(0.0, 40.0)),
            max_route_distance_factor=float(rng.uniform(1.0, 8.0)),
            max_route_time_factor=float(rng.uniform(1.0, 6.0)))[0])
    tr = {k: np.concatenate([p[k] for p in parts]) for k in ("lon", "lat", "time", "accuracy")}
    tr["trace_off"] = np.concatenate([[0], np.cumsum([len(p["lon"]) for p in parts])]).astype(np.uint32)
    trace_opt = np.arange(len(parts), dtype=np.uint32)
    bm, ref = _run_both(path, g, eng, tr, np.array(opts, engine.OPTIONS_DTYPE), trace_opt)
    c = compare_all(bm, ref, tr["trace_off"])
    assert c["segments"] > 50 and c["chained"] > 1000, c
    bm.close()
