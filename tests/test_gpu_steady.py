"""Steady runs (Matcher::run_steady), GPU.

Once an ordinary run has sized a matcher's pools, a later batch runs without the two mid-run
read-backs: K2's grid covers the previous run's sources and an eighth more, and a batch that
outgrows the pools or that grid is gated off on the device and run again the ordinary way.  Both
must give the oracle's answers bit for bit.  RM_SMALL_BATCH_POINTS=0 keeps these small test
batches off the small-batch path, so they take the ordinary / steady one.
"""
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


def _run(bm, tr, opts):
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts)
    off, segs = bm.segments()
    return off.tobytes(), segs.tobytes()


@pytest.mark.parametrize("turn", [0.0, 200.0])
def test_steady_runs_match_the_oracle(built_lib, small_world, monkeypatch, turn):
    """The same batch three times on one matcher (an ordinary run, then steady ones), then a batch
    four times larger (more sources than the steady grid covers: gated off, run the ordinary way),
    then that batch again (steady): every stage equals the oracle each time."""
    monkeypatch.setenv("RM_SMALL_BATCH_POINTS", "0")
    g = graphfile.load(small_world)
    opts = engine.default_options(1, turn_penalty_factor=turn)
    small = world.generate_traces(small_world, n_traces=20, n_points=60, rate_s=1.0, noise_m=5.0, seed=311)
    large = world.generate_traces(small_world, n_traces=80, n_points=60, rate_s=1.0, noise_m=5.0, seed=312)
    ref_s, ref_l = _ref(g, small, opts), _ref(g, large, opts)
    eng = engine.Engine(small_world, 0)
    bm = engine.BatchMatcher(eng)
    first = None
    for tr, ref in ((small, ref_s), (small, ref_s), (small, ref_s), (large, ref_l), (large, ref_l), (small, ref_s)):
        got = _run(bm, tr, opts)
        c = compare_all(bm, ref, tr["trace_off"])
        assert c["segments"] > 20, c
        if tr is small:
            first = first or got
            assert got == first
    bm.close()
    eng.close()


def test_steady_and_ordinary_agree(built_lib, small_world, monkeypatch):
    """RM_STEADY=0 (every run the ordinary way) gives the same segments and reports."""
    monkeypatch.setenv("RM_SMALL_BATCH_POINTS", "0")
    tr = world.generate_traces(small_world, n_traces=40, n_points=60, rate_s=1.0, noise_m=5.0, seed=313)
    opts = engine.default_options(1)
    outs = {}
    for steady in ("1", "0"):
        monkeypatch.setenv("RM_STEADY", steady)
        eng = engine.Engine(small_world, 0)
        bm = engine.BatchMatcher(eng)
        for _ in range(3):
            outs.setdefault(steady, []).append(_run(bm, tr, opts))
        bm.close()
        eng.close()
    assert outs["1"] == outs["0"]
