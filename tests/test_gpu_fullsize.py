"""GPU parity at BASELINE.json's full graph sizes.

test_gpu_parity.py covers the configs on graphs scaled so every corner case is
cheap; here the graphs are the configs' own (C2/C5: 200x200 @100 m, C3:
500x500 @200 m, C4: a 1000x1000 @250 m country slice of the 4000x4000 graph —
the full one takes a minute to generate on the host), and the C2 batch is the
bench's exact rank-0 workload (10,000 traces x 600 points, seed 1000): every
stage of every trajectory must equal the oracle bit for bit, and the speed
histogram and the per-segment duration sums must equal the
CPU pipeline's.  C3/C4/C5 check bounded trace
samples (the oracle's long 30 s searches run ~8k points/s on one core).
"""
import numpy as np
import pytest

from parity_util import match_and_compare
from reporter_amd import engine, world

pytestmark = pytest.mark.gpu


def _world(tmpdir_session, name, rows=None, cols=None):
    cfg = dict(world.CONFIGS[name])
    path = str(tmpdir_session / ("full_%s_%s.rmg" % (name, rows or cfg["rows"])))
    world.build_world(path, rows or cfg["rows"], cols or cfg["cols"], cfg["block_m"], seed=1, cell_m=cfg["cell_m"])
    return path, cfg


@pytest.mark.timeout(400)
def test_c2_full_bench_workload(built_lib, tmpdir_session):
    """C2 exactly as bench.py rank 0 runs it: all 10,000 trajectories bit-exact."""
    path, cfg = _world(tmpdir_session, "C2")
    tr = world.generate_traces(path, cfg["n_traces"], cfg["n_points"], cfg["rate_s"], cfg["noise_m"], seed=1000)
    opts = engine.default_options(1, search_radius=cfg["search_radius"])
    c = match_and_compare(path, tr, opts, None, hist=True)
    assert c["points"] == 6_000_000 and c["segments"] > 200_000 and c["valid_reports"] > 50_000, c
    print("C2 full parity", c)


@pytest.mark.parametrize("ball_radius", [400.0, 2000.0])
def test_c3_full_graph_sample(built_lib, tmpdir_session, ball_radius):
    """C3 graph (500x500 @200 m), 30 s sampling, radius 100 m: route bounds up to the 2 km
    breakage distance, answered by the search tiers (400 m balls) or by the ball tier (2 km)."""
    path, cfg = _world(tmpdir_session, "C3")
    tr = world.generate_traces(path, 1500, cfg["n_points"], cfg["rate_s"], cfg["noise_m"], seed=3000)
    opts = engine.default_options(1, search_radius=cfg["search_radius"])
    c = match_and_compare(path, tr, opts, None, hist=True, ball_radius=ball_radius)
    assert c["chained"] > 40_000, c
    assert (c["route_tiers"]["ball_to_search"] == 0) == (ball_radius >= 2000.0), c
    print("C3 sample parity", c)


def test_c4_country_slice_sample(built_lib, tmpdir_session):
    """C4 block size and sampling (250 m, 5 s) on a 1000x1000 slice (1 M nodes)."""
    path, cfg = _world(tmpdir_session, "C4", rows=1000, cols=1000)
    tr = world.generate_traces(path, 2000, cfg["n_points"], cfg["rate_s"], cfg["noise_m"], seed=4000)
    opts = engine.default_options(1, search_radius=cfg["search_radius"])
    c = match_and_compare(path, tr, opts, None, hist=True, ball_radius=cfg["ball_radius_m"])
    assert c["segments"] > 20_000, c
    print("C4 slice parity", c)


def test_c5_full_graph_modes_sigma(built_lib, tmpdir_session):
    """C5: C2 graph, auto/bicycle/pedestrian x sigma_z {2, 4.07, 8, 16}, radius max(50, 3 sigma)."""
    path, cfg = _world(tmpdir_session, "C5")
    parts, opts = [], []
    per = 100
    for mi, mode in enumerate(("auto", "bicycle", "pedestrian")):
        for si, sz in enumerate((2.0, 4.07, 8.0, 16.0)):
            parts.append(world.generate_traces(path, n_traces=per, n_points=cfg["n_points"], rate_s=1.0, noise_m=sz,
                                               seed=5000 + mi * 10 + si, mode=mode))
            opts.append(engine.default_options(1, mode=world.MODES[mode], sigma_z=sz,
                                               search_radius=max(50.0, 3 * sz))[0])
    tr = {k: np.concatenate([p[k] for p in parts]) for k in ("lon", "lat", "time", "accuracy")}
    tr["trace_off"] = (np.arange(len(parts) * per + 1) * cfg["n_points"]).astype(np.uint32)
    trace_opt = np.repeat(np.arange(len(parts), dtype=np.uint32), per)
    opts = np.array(opts, engine.OPTIONS_DTYPE)
    c = match_and_compare(path, tr, opts, trace_opt, rl=(0, 1, 2), tl=(0, 1, 2), hist=True)
    assert c["traces"] == 1200 and c["segments"] > 10_000, c
    print("C5 parity", c)
