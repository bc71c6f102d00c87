"""K1's split grid (engine.hip choose_grid_split / Engine::Engine; numpy mirror
graphfile.split_grid): the same bounding-box rule as the graph builder, and the oracle finds
exactly the same candidates (and everything downstream) on it while reading fewer items.
CPU only."""
import sys
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def test_split_rule_matches_builder(built_lib, tmp_path):
    from reporter_amd import graphfile, world
    gp = str(tmp_path / "g.rmg")
    world.build_world(gp, 30, 30, 100.0, seed=4)
    g = graphfile.load(gp)
    r = graphfile.split_grid(g, 1, rebuild=True)
    assert np.array_equal(r["cell_off"], g["cell_off"])
    assert np.array_equal(r["cell_item"], g["cell_item"])


def test_oracle_identical_on_split_grid(built_lib, tmp_path):
    import meili_oracle as mo
    from reporter_amd import engine, graphfile, world
    gp = str(tmp_path / "g.rmg")
    world.build_world(gp, 40, 40, 100.0, seed=1)
    g = graphfile.load(gp)
    tr = world.generate_traces(gp, 40, 300, 1.0, 5.0, seed=3)
    T = len(tr["trace_off"]) - 1
    opts = engine.default_options(1)
    out = []
    for f in (1, 2, 3):
        mo.reset_counters()
        res = mo.match(graphfile.split_grid(g, f), mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"],
                                                          tr["accuracy"], opts, np.zeros(T, np.uint32)))
        out.append((res, mo.counters()["cand_items"]))
    for res, _ in out[1:]:
        for k, v in out[0][0].items():
            if isinstance(v, np.ndarray):
                assert np.array_equal(v, res[k]), k
    assert out[1][1] < 0.8 * out[0][1]   # f = 2 reads fewer grid items on a 100 m-block grid


def test_double_quotient_time_is_exact():
    """engine.hip time_ms_dev: trunc((double)(d*360) / (double)D) == floor for d*360 < 2^32 and
    every 16-bit speed D (exact multiples, their neighbours and random distances)."""
    rng = np.random.default_rng(5)
    D = np.arange(1, 65536, dtype=np.uint64)
    for _ in range(4):
        k = (rng.integers(0, 2**32, len(D), dtype=np.uint64) // D)
        for dd in (-1, 0, 1):
            N = (k * D).astype(np.int64) + dd
            d = np.clip(N // 360, 0, 11930464).astype(np.uint64)
            num = d * 360
            ref = num // D
            got = np.trunc(num.astype(np.float64) / D.astype(np.float64)).astype(np.uint64)
            assert np.array_equal(ref, got)


def test_split_by_points_balances_and_covers():
    """engine.split_by_points (MultiMatcher's parts): contiguous, covering, balanced by points."""
    from reporter_amd import engine
    rng = np.random.default_rng(2)
    for parts in (1, 2, 3, 7):
        lens = rng.integers(1, 400, 500)
        off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint32)
        cuts = engine.split_by_points(off, parts)
        assert cuts[0] == 0 and cuts[-1] == 500 and cuts == sorted(set(cuts))
        pts = [int(off[b] - off[a]) for a, b in zip(cuts[:-1], cuts[1:])]
        assert sum(pts) == int(off[-1])
        assert max(pts) - min(pts) <= 2 * 400   # within two traces of even
    assert engine.split_by_points(np.array([0, 5], np.uint32), 4) == [0, 1]
