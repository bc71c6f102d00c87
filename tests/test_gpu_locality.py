"""Locality order (round 4): K1 / K2 / the path stage take their work sorted by region.

The state slots are sorted each step by the Morton code of their point's ~500 m grid cell
(engine.hip k_locality_keys). K1 reads states, K2 (pair, source) items and the path stage
chosen transitions in that order, so one region's cell records and route-ball tables meet in
one XCD's L2. Results still go to their own slots. Every stage's output must be byte-identical
to the slot-order run and equal to the oracle. The engine's default turns it on for large
graphs (C3 / C4), so the C3 and C4 parity tests already run it. Here it is forced on and off on
the same batches.
"""
import numpy as np
import pytest

import meili_oracle as mo
from parity_util import check_reports, compare_all
from reporter_amd import engine, graphfile, world

pytestmark = pytest.mark.gpu


def _same(a, b):
    if isinstance(a, (tuple, list)):
        return all(_same(x, y) for x, y in zip(a, b)) and len(a) == len(b)
    return np.asarray(a).tobytes() == np.asarray(b).tobytes()


@pytest.mark.parametrize("kind", ["grid30s", "city1hz", "city30s"])
def test_locality_order_is_invisible(built_lib, tmpdir_session, kind):
    if kind == "grid30s":
        path = str(tmpdir_session / "loc_grid.rmg")
        world.build_world(path, 120, 120, 200.0, seed=3, cell_m=200.0)
        tr = world.generate_traces(path, 1500, 40, rate_s=30.0, noise_m=5.0, seed=81)
        opts = engine.default_options(1, search_radius=100.0)
    else:
        path = str(tmpdir_session / "loc_city.rmg")
        world.build_city(path, rows=60, cols=60, seed=9)
        rate = 1.0 if kind == "city1hz" else 30.0
        tr = world.generate_traces(path, 600 if rate == 1.0 else 1500, 300 if rate == 1.0 else 40, rate_s=rate,
                                   noise_m=5.0, seed=82)
        opts = engine.default_options(1, search_radius=50.0 if rate == 1.0 else 100.0)
    eng = engine.Engine(path, 0)
    T = len(tr["trace_off"]) - 1
    ref = mo.match(graphfile.load(path), mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"],
                                                  opts, np.zeros(T, np.uint32)))
    outs = {}
    for mode in (0, 1, 2):   # 1: K1 and K2 in locality order, 2: the path stage too
        bm = engine.BatchMatcher(eng)
        bm.set_locality(mode)
        bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, np.zeros(T, np.uint32))
        assert bm.locality_used() == bool(mode)
        if mode:
            bm.rerun()   # the bench's steady state: the order is rebuilt every run
        # every stage of every state slot equals the oracle's (slots without a state hold
        # nothing, so whole arrays are not compared), the compacted outputs byte for byte
        c = compare_all(bm, ref, tr["trace_off"])
        c["reports"] = check_reports(bm, ref, tr)
        outs[mode] = (bm.segments(), bm.reports())
        assert c["chained"] > 10_000, c
        bm.close()
    for mode in (1, 2):
        assert _same(outs[0], outs[mode]), mode
    eng.close()
    print(kind, c)
