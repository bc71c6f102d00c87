"""Small batches (Matcher::run_small), GPU.

A coalesced service batch holds a few to a few thousand requests.  run_small runs it with its
pools sized from upper bounds instead of read-back totals, one input upload, fused scans and the
reply's segments compacted before the one read-back.  It must give the ordinary path's answers
bit for bit (both against the oracle), and a batch an upper bound cannot cover -- the path pool
overflowing, a search handed to the global tier before its scratch exists -- must come out
exact through the ordinary path it falls back to.
"""
import json

import numpy as np
import pytest

import meili_oracle as mo
from parity_util import compare_all
from reporter_amd import engine, graphfile, world

pytestmark = pytest.mark.gpu


def _ref(g, tr, opts):
    T = len(tr["trace_off"]) - 1
    return mo.match(g, mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts,
                                np.zeros(T, np.uint32)))


@pytest.mark.parametrize("turn", [0.0, 200.0])
def test_small_and_ordinary_runs_agree(built_lib, small_world, monkeypatch, turn):
    """40 requests of 60 points (the Java batcher's size): every stage equals the oracle on the
    small path and on the ordinary one (RM_SMALL_BATCH_POINTS=0), with and without turn costs."""
    g = graphfile.load(small_world)
    tr = world.generate_traces(small_world, n_traces=40, n_points=60, rate_s=1.0, noise_m=5.0, seed=301)
    opts = engine.default_options(1, turn_penalty_factor=turn)
    ref = _ref(g, tr, opts)
    eng = engine.Engine(small_world, 0)
    bm = engine.BatchMatcher(eng)
    got = {}
    for limit in (None, "0", None):
        if limit is None:
            monkeypatch.delenv("RM_SMALL_BATCH_POINTS", raising=False)
        else:
            monkeypatch.setenv("RM_SMALL_BATCH_POINTS", limit)
        bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts)
        c = compare_all(bm, ref, tr["trace_off"])
        off, segs = bm.segments()
        got.setdefault(limit, (off, segs.tobytes()))
        assert c["segments"] > 40, c
    assert got[None][1] == got["0"][1]
    np.testing.assert_array_equal(got[None][0], got["0"][0])
    bm.close()
    eng.close()


def test_small_run_path_pool_overflow_falls_back(built_lib, tmpdir_session):
    """120 s sampling on a fresh matcher: the chosen paths' pooled edges exceed the path pool a
    first run allocates, so the small run gates itself off and the ordinary path (which grows the
    pool) gives the oracle's answer; the same matcher's next run fits and stays small."""
    path = str(tmpdir_session / "small_sparse.rmg")
    world.build_world(path, 48, 48, 100.0, seed=12, cell_m=100.0)
    g = graphfile.load(path)
    tr = world.generate_traces(path, n_traces=40, n_points=12, rate_s=120.0, noise_m=5.0, seed=302)
    opts = engine.default_options(1, search_radius=60.0)
    ref = _ref(g, tr, opts)
    P = int(tr["trace_off"][-1])
    cp = P + 64
    n = cp // 8 + 1024
    first_pool = n + n // 4 + 1024          # Matcher::alloc_points -> ensure_path_raw on a fresh matcher
    cnt = ref["path_cnt"].astype(np.int64)
    pooled = int(cnt[cnt > 8].sum())      # kInlinePath edges per slot stay in line
    assert pooled > first_pool, (pooled, first_pool)
    eng = engine.Engine(path, 0)
    bm = engine.BatchMatcher(eng)
    for _ in range(2):
        bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts)
        c = compare_all(bm, ref, tr["trace_off"])
        assert c["chained"] > 100, c
    bm.close()
    eng.close()


def test_service_replies_through_small_runs(built_lib, small_world, tmp_path):
    """Through SegmentMatcher().Match with the coalescer (the replies come from the segments
    run_small compacts before its read-back) and MatchMany: every reply equals the oracle's."""
    import valhalla
    g = graphfile.load(small_world)
    tr = world.generate_traces(small_world, n_traces=48, n_points=60, rate_s=1.0, noise_m=5.0, seed=303)
    ref = _ref(g, tr, engine.default_options(1))
    conf = valhalla.write_config(str(tmp_path / "small.json"), small_world, device=0, coalesce=True)
    valhalla.Configure(conf)
    sm = valhalla.SegmentMatcher()
    reqs = [json.dumps(world.trace_to_request(tr, k), separators=(",", ":")) for k in range(48)]
    outs = [sm.Match(r) for r in reqs[:8]]
    outs += sm.MatchMany(reqs[8:])
    sm.close()
    for k in range(48):
        want = engine.segment_dicts(ref["segs"][ref["seg_off"][k]:ref["seg_off"][k + 1]])
        assert json.loads(outs[k])["segments"] == want, k


def test_lone_caller_runs_inline(built_lib, small_world, tmp_path):
    """A caller that sends one request at a time: after a streak of single-request batches the
    coalescer runs each request on its caller's thread (Coalescer::submit); the replies stay the
    oracle's, and the batch count still counts every request."""
    import valhalla
    g = graphfile.load(small_world)
    tr = world.generate_traces(small_world, n_traces=24, n_points=60, rate_s=1.0, noise_m=5.0, seed=304)
    ref = _ref(g, tr, engine.default_options(1))
    conf = valhalla.write_config(str(tmp_path / "lone.json"), small_world, device=0, coalesce=True)
    valhalla.Configure(conf)
    sm = valhalla.SegmentMatcher()
    before = valhalla.coalesce_stats()
    for k in range(24):
        got = json.loads(sm.Match(json.dumps(world.trace_to_request(tr, k), separators=(",", ":"))))["segments"]
        want = engine.segment_dicts(ref["segs"][ref["seg_off"][k]:ref["seg_off"][k + 1]])
        assert got == want, k
    st = valhalla.coalesce_stats()
    assert st["requests"] - before["requests"] == 24 and st["batches"] - before["batches"] == 24, (before, st)
    sm.close()


@pytest.mark.parametrize("rate,turn", [(15.0, 0.0), (30.0, 200.0)])
def test_small_run_short_chain_hand_overs(built_lib, small_world, monkeypatch, rate, turn):
    """Round 6: a ball-covered small run hands the K2 / path ball tiers' leftovers straight to the
    16-lane group tier and its leftovers to the 4096-slot tier (RM_SMALL_SHORT_CHAIN, default on).
    With 100 m route balls and sparse sampling most searches are handed over; the short chain, the
    full five-tier chain (RM_SMALL_SHORT_CHAIN=0) and the oracle agree at every stage."""
    g = graphfile.load(small_world)
    tr = world.generate_traces(small_world, n_traces=40, n_points=16, rate_s=rate, noise_m=5.0, seed=305)
    opts = engine.default_options(1, turn_penalty_factor=turn)
    ref = _ref(g, tr, opts)
    eng = engine.Engine(small_world, 0)
    eng.set_ball_radius(100.0)
    bm = engine.BatchMatcher(eng)
    got, tiers = {}, {}
    # (the first run may outgrow a fresh matcher's path pool and take the ordinary path, which
    # sizes it: the short chain's own run is the second)
    for short in ("1", "1", "0"):
        monkeypatch.setenv("RM_SMALL_SHORT_CHAIN", short)
        bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts)
        tiers[short] = bm.route_tiers()
        c = compare_all(bm, ref, tr["trace_off"])
        assert c["segments"] > 40, c
        off, segs = bm.segments()
        got[short] = (off, segs.tobytes())
    print(tiers)
    assert tiers["1"]["ball_to_search"] > 100 and tiers["1"]["paths_ball_to_search"] > 20, tiers
    assert tiers["1"]["lane_to_tier2"] == 0, tiers   # the lane tier did not run
    assert got["1"][1] == got["0"][1]
    np.testing.assert_array_equal(got["1"][0], got["0"][0])
    bm.close()
    eng.close()
