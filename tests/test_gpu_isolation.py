"""Per-trace failure isolation and the global-memory search tier (GPU).

The reference answers each /report on its own thread: an exception in one Match is one
HTTP 500 (py/reporter_service.py:244-245), and the batch reporter logs and skips one
window (py/simple_reporter.py:169-173).  Here many requests share one GPU batch, so a
failure must stay with its own trace:
  * searches that outgrow the LDS tiers (kilometre route bounds) finish in the
    global-memory tier with the oracle's exact answer;
  * a trace that fails on its own (more than 192 roads inside its radius) gets its error
    while every co-batched request gets its exact reply.
"""
import json
import threading

import numpy as np
import pytest

import meili_oracle as mo
from parity_util import compare_all
from reporter_amd import engine, graphfile, world

pytestmark = pytest.mark.gpu


def _c2(tmpdir_session):
    cfg = world.CONFIGS["C2"]
    path = str(tmpdir_session / "iso_c2.rmg")
    world.build_world(path, cfg["rows"], cfg["cols"], cfg["block_m"], seed=1, cell_m=cfg["cell_m"])
    return path


def _dense(tmpdir_session):
    """60x60 grid of 20 m blocks: a 200 m radius holds several hundred roads."""
    path = str(tmpdir_session / "iso_dense.rmg")
    world.build_world(path, 60, 60, 20.0, seed=2, cell_m=20.0)
    return path


def _ref_segments(g, tr, opts, trace_opt):
    return mo.match(g, mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, trace_opt))


def test_global_tier_kilometre_bounds(built_lib, tmpdir_session):
    """200 s sampling with breakage_distance 10 km on the C2 graph: route bounds of up to
    10 km (tens of thousands of nodes) outgrow the 4096-slot LDS hash and finish in the
    global-memory tier; every stage equals the oracle's unbounded heap Dijkstra."""
    path = _c2(tmpdir_session)
    g = graphfile.load(path)
    tr = world.generate_traces(path, n_traces=12, n_points=6, rate_s=200.0, noise_m=5.0, seed=71)
    opts = engine.default_options(1, breakage_distance=10000.0)
    eng = engine.Engine(path, 0)
    bm = engine.BatchMatcher(eng)
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts)
    tiers = bm.route_tiers()
    assert tiers["wave_to_global"] > 0, tiers
    ref = _ref_segments(g, tr, opts, np.zeros(12, np.uint32))
    c = compare_all(bm, ref, tr["trace_off"])
    assert c["chained"] > 20, c
    # a second run on the same matcher runs the global tier in line (scratch already there)
    bm.rerun()
    compare_all(bm, ref, tr["trace_off"])
    print("global tier", tiers, c)
    bm.close()
    eng.close()


def test_runner_isolation_fails_only_the_overflowing_traces(built_lib, tmpdir_session):
    """Traces whose 200 m radius holds > 192 roads fail alone; the others match exactly."""
    path = _dense(tmpdir_session)
    g = graphfile.load(path)
    T = 16
    tr = world.generate_traces(path, n_traces=T, n_points=80, rate_s=1.0, noise_m=3.0, seed=73)
    opts = engine.default_options(2, search_radius=30.0)
    opts[1]["search_radius"] = 200.0
    trace_opt = np.zeros(T, np.uint32)
    bad = [3, 9]
    trace_opt[bad] = 1
    eng = engine.Engine(path, 0)
    bm = engine.BatchMatcher(eng)
    with pytest.raises(RuntimeError, match="candidate roads"):   # strict by default
        bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, trace_opt)
    bm.set_isolation(True)
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, trace_opt)
    errs = bm.trace_errors()
    assert sorted(np.nonzero(errs)[0].tolist()) == bad and all(errs[b] & 1 for b in bad), errs
    soff, segs = bm.segments()
    roff, reps, stats = bm.reports()
    good = [k for k in range(T) if k not in bad]
    sub = {k: tr[k] for k in ("lon", "lat", "time", "accuracy", "truth_edge")}
    o = tr["trace_off"]
    sel = np.concatenate([np.arange(o[k], o[k + 1]) for k in good])
    sub = {k: v[sel] for k, v in sub.items()}
    sub["trace_off"] = np.concatenate([[0], np.cumsum([o[k + 1] - o[k] for k in good])]).astype(np.uint32)
    ref = _ref_segments(g, sub, opts[:1], np.zeros(len(good), np.uint32))
    for i, k in enumerate(good):
        a = segs[soff[k]:soff[k + 1]]
        b = ref["segs"][ref["seg_off"][i]:ref["seg_off"][i + 1]]
        assert a.tobytes() == b.tobytes(), "trace %d" % k
    for b in bad:
        assert soff[b + 1] == soff[b] and roff[b + 1] == roff[b]
    assert len(segs) > 50
    bm.close()
    eng.close()


def _threaded(sm_factory, reqs, n_threads=12):
    out, err = [None] * len(reqs), [None] * len(reqs)

    def worker(tid):
        sm = sm_factory()
        for k in range(tid, len(reqs), n_threads):
            try:
                out[k] = sm.Match(reqs[k])
            except RuntimeError as e:
                err[k] = str(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(n_threads)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    return out, err


def test_coalesced_breakage_10km_request_among_95(built_lib, tmpdir_session):
    """one coalesced /report with breakage_distance 10000 on the C2 grid among 95
    ordinary ones: it matches exactly (global tier) and so do the 95."""
    import valhalla
    path = _c2(tmpdir_session)
    g = graphfile.load(path)
    conf = valhalla.write_config(str(tmpdir_session / "iso_c2.json"), path, device=0, coalesce=True,
                                 coalesce_window_ms=5.0)
    valhalla.Configure(conf)
    n = 95
    tr = world.generate_traces(path, n_traces=n, n_points=90, rate_s=1.0, noise_m=5.0, seed=75)
    sp = world.generate_traces(path, n_traces=1, n_points=6, rate_s=200.0, noise_m=5.0, seed=76)
    opts = engine.default_options(1)
    ref = _ref_segments(g, tr, opts, np.zeros(n, np.uint32))
    ref_sp = _ref_segments(g, sp, engine.default_options(1, breakage_distance=10000.0), np.zeros(1, np.uint32))
    reqs = [json.dumps(world.trace_to_request(tr, k), separators=(",", ":")) for k in range(n)]
    reqs.insert(40, json.dumps(world.trace_to_request(sp, 0, breakage_distance=10000), separators=(",", ":")))
    out, err = _threaded(valhalla.SegmentMatcher, reqs)
    assert not any(err), [e for e in err if e]
    got_sp = json.loads(out.pop(40))["segments"]
    assert got_sp == engine.segment_dicts(ref_sp["segs"]) and len(got_sp) > 0
    for k in range(n):
        want = engine.segment_dicts(ref["segs"][ref["seg_off"][k]:ref["seg_off"][k + 1]])
        assert json.loads(out[k])["segments"] == want, k


def test_coalesced_failing_request_fails_alone(built_lib, tmpdir_session):
    """A request whose radius holds > 192 roads gets its own error (HTTP 500 in the service)
    while the 95 requests co-batched with it get their exact replies."""
    import valhalla
    path = _dense(tmpdir_session)
    g = graphfile.load(path)
    conf = valhalla.write_config(str(tmpdir_session / "iso_dense.json"), path, device=0, coalesce=True,
                                 coalesce_window_ms=5.0)
    valhalla.Configure(conf)
    n = 95
    tr = world.generate_traces(path, n_traces=n + 1, n_points=60, rate_s=1.0, noise_m=3.0, seed=77)
    opts = engine.default_options(1, search_radius=30.0)
    ref = _ref_segments(g, tr, opts, np.zeros(n + 1, np.uint32))
    reqs = [json.dumps(world.trace_to_request(tr, k, search_radius=30), separators=(",", ":")) for k in range(n)]
    reqs.insert(17, json.dumps(world.trace_to_request(tr, n, search_radius=200), separators=(",", ":")))
    before = valhalla.coalesce_stats()
    out, err = _threaded(valhalla.SegmentMatcher, reqs)
    assert err[17] and "candidate roads" in err[17], err[17]
    assert sum(e is not None for e in err) == 1, [e for e in err if e]
    out.pop(17)
    for k in range(n):
        want = engine.segment_dicts(ref["segs"][ref["seg_off"][k]:ref["seg_off"][k + 1]])
        assert json.loads(out[k])["segments"] == want, k
    st = valhalla.coalesce_stats()
    assert st["batches"] - before["batches"] < n + 1   # they really shared batches
    print("isolation", st)


def test_download_buffer_failure_then_retry(built_lib, small_world, monkeypatch):
    """a segment download whose buffer cannot be allocated fails as a batch too
    large for the device (the coalescer's split signal, serve_policy.hpp) and leaves the matcher
    usable; the next call on the same matcher allocates again and returns the exact segments."""
    tr = world.generate_traces(small_world, n_traces=16, n_points=200, rate_s=1.0, noise_m=5.0, seed=77)
    eng = engine.Engine(small_world, 0)
    want = engine.BatchMatcher(eng)
    want.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"])
    o_want, s_want = want.segments()
    want.close()
    bm = engine.BatchMatcher(eng)
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"])
    monkeypatch.setenv("RM_TEST_DOWNLOAD_ALLOC_LIMIT", "64")
    with pytest.raises(RuntimeError, match="does not fit in HBM"):
        bm.segments()
    monkeypatch.delenv("RM_TEST_DOWNLOAD_ALLOC_LIMIT")
    o, s = bm.segments()
    np.testing.assert_array_equal(o, o_want)
    assert s.tobytes() == s_want.tobytes() and len(s) > 50
    bm.close()
    eng.close()


def test_workspace_exact_size_fallback(built_lib, small_world, monkeypatch):
    """the workspace grows to 1.5x its last capacity, and when that does not fit but
    the batch's own size does, it allocates the exact size instead of failing the batch (the
    hook RM_TEST_WS_POINTS_LIMIT makes larger workspaces fail as out of memory)."""
    g = graphfile.load(small_world)
    small = world.generate_traces(small_world, n_traces=8, n_points=125, rate_s=1.0, noise_m=5.0, seed=78)
    big = world.generate_traces(small_world, n_traces=10, n_points=125, rate_s=1.0, noise_m=5.0, seed=79)
    eng = engine.Engine(small_world, 0)
    bm = engine.BatchMatcher(eng)
    bm.run(small["trace_off"], small["lon"], small["lat"], small["time"], small["accuracy"])   # 1,000 points
    # 1,250 points: the grown size is 1,000 * 1.5 + 64 points, the exact one 1,250 + 64
    monkeypatch.setenv("RM_TEST_WS_POINTS_LIMIT", "1400")
    bm.run(big["trace_off"], big["lon"], big["lat"], big["time"], big["accuracy"])
    ref = mo.match(g, mo.Batch(big["trace_off"], big["lon"], big["lat"], big["time"], big["accuracy"],
                               engine.default_options(1), np.zeros(10, np.uint32)))
    compare_all(bm, ref, big["trace_off"])
    # a batch whose own size does not fit (1,750 points) still fails as too large for the device,
    # and the matcher works again once memory allows
    bigger = world.generate_traces(small_world, n_traces=14, n_points=125, rate_s=1.0, noise_m=5.0, seed=80)
    with pytest.raises(RuntimeError, match="does not fit in HBM"):
        bm.run(bigger["trace_off"], bigger["lon"], bigger["lat"], bigger["time"], bigger["accuracy"])
    monkeypatch.delenv("RM_TEST_WS_POINTS_LIMIT")
    bm.run(big["trace_off"], big["lon"], big["lat"], big["time"], big["accuracy"])
    compare_all(bm, ref, big["trace_off"])
    bm.close()
    eng.close()
