"""C4 at its full size and the native RCCL path (GPU).

C4 (BASELINE.json configs[3]): the 4000 x 4000 @250 m country graph — 16.6 M nodes,
65 M directed edges, 19.4 M OSMLR segments — replicated in HBM, traces at 5 s.  Sampled
traces are matched at the product default (automatic ball radius, 1000 m on this graph,
tables built on the GPU) and at 400 m (5 s bounds beyond the radius go to the search tiers), every stage compared bit for bit with the oracle, and the full
19.4 M x 16 speed histogram compared with the CPU pipeline's.

RCCL: the histogram exchange that replaces the keyed "id next_id" repartition
(BatchingProcessor.java:126) runs through the library's own communicator
(rm_comm_init / rm_comm_allreduce, no PyTorch) on that 1.24 GB histogram, and the tile
stage runs its all-reduce + all-gather path with a communicator.  One GPU means one rank;
the multi-rank semantics are covered by tests/test_dist_gloo.py.
"""
import ctypes
import os
import time

import numpy as np
import pytest

from reporter_amd import _lib, dist, engine, world
from parity_util import match_and_compare

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def c4_graph(built_lib, tmpdir_session):
    cfg = dict(world.CONFIGS["C4"])
    path = str(tmpdir_session / "c4_full.rmg")
    t = time.time()
    world.build_world(path, cfg["rows"], cfg["cols"], cfg["block_m"], seed=1, cell_m=cfg["cell_m"])
    print("C4 graph built in %.1fs" % (time.time() - t), world.graph_info(path), flush=True)
    yield path, cfg
    os.remove(path)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("ball_radius", [None, 400.0])
def test_c4_full_graph(c4_graph, ball_radius):
    path, cfg = c4_graph
    auto = ctypes.c_double()
    _lib.check(_lib.lib().rm_graph_auto_ball_radius(os.fsencode(path), ctypes.byref(auto)))
    assert auto.value == 1000.0
    tr = world.generate_traces(path, 3000, cfg["n_points"], cfg["rate_s"], cfg["noise_m"], seed=4000)
    opts = engine.default_options(1, search_radius=cfg["search_radius"])
    t = time.time()
    c = match_and_compare(path, tr, opts, None, hist=True, ball_radius=ball_radius)
    assert c["ball_stats"]["radius_m"] == (ball_radius or auto.value)
    assert c["segments"] > 30_000 and c["valid_reports"] > 10_000, c
    print("C4 full graph, radius", ball_radius or "auto", "%.1fs" % (time.time() - t), c, flush=True)


@pytest.mark.timeout(900)
def test_c4_three_modes_fit_hbm(c4_graph):
    """VERDICT r02 (route-ball memory): auto, bicycle and pedestrian on the full C4 graph in one
    batch.  Their tables come out of one budget (half of the HBM): auto keeps its 1000 m tables
    (68 GB), the others step down as far as the remaining budget needs, nothing runs out of
    memory, and every stage equals the oracle's."""
    import meili_oracle as mo
    from parity_util import compare_all
    from reporter_amd import graphfile
    path, cfg = c4_graph
    eng = engine.Engine(path, 0)
    names = [("auto", 0), ("bicycle", 3), ("pedestrian", 4)]
    sets = [world.generate_traces(path, 400, cfg["n_points"], cfg["rate_s"], cfg["noise_m"], seed=4200 + m, mode=nm)
            for nm, m in names]
    tr = world.concat_traces(*sets)
    opts = engine.default_options(3, search_radius=cfg["search_radius"])
    for q, (_, m) in enumerate(names):
        opts[q]["mode"] = m
    trace_opt = np.repeat(np.arange(3, dtype=np.uint32), 400)
    bm = engine.BatchMatcher(eng)
    t = time.time()
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, trace_opt)
    st = {m: eng.ball_stats(m) for _, m in names}
    print("C4 three modes: first run %.1fs" % (time.time() - t), st, flush=True)
    assert st[0]["radius_m"] == 1000.0
    total = sum(s["entries"] for s in st.values()) * 16
    assert total <= 0.5 * 288e9 * 1.05, total
    ref = mo.match(graphfile.load(path), mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"],
                                                  opts, trace_opt))
    c = compare_all(bm, ref, tr["trace_off"])
    assert c["chained"] > 100_000, c
    bm.close()
    eng.close()


@pytest.mark.timeout(900)
def test_rccl_comm_on_c4_histogram(c4_graph, tmpdir_session):
    path, cfg = c4_graph
    eng = engine.Engine(path, 0)
    nseg = eng.n_segments
    assert nseg > 19_000_000
    hist = dist.DeviceBuffer(nseg * 16 * 4)   # 1.24 GB of u32 bins
    bm = engine.BatchMatcher(eng)
    tr = world.generate_traces(path, 2000, cfg["n_points"], cfg["rate_s"], cfg["noise_m"], seed=4100)
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"],
           engine.default_options(1, search_radius=cfg["search_radius"]), None, hist_dev=hist.ptr, zero_hist=True)
    before = hist.download()
    assert before.sum() > 5000
    comm = dist.Comm(0, 1, 0, rdzv_dir=str(tmpdir_session), token="c4test")
    try:
        for op in (dist.SUM, dist.MAX):
            t = time.time()
            comm.allreduce(hist.ptr, nseg * 16, dist.U32, op)
            print("rm_comm_allreduce u32 op %d on %.2f GB: %.1f ms" % (op, nseg * 64 / 1e9, (time.time() - t) * 1e3))
            np.testing.assert_array_equal(hist.download(), before)
        for dt, npdt in ((dist.U64, np.uint64), (dist.F64, np.float64)):
            buf = dist.DeviceBuffer(1 << 20)
            x = (np.arange((1 << 20) // 8) * 3 + 1).astype(npdt)
            buf.upload(x)
            for op in (dist.SUM, dist.MAX):
                comm.allreduce(buf.ptr, len(x), dt, op)
                np.testing.assert_array_equal(buf.download(npdt), x)
            buf.close()
        assert comm.allreduce_host(7.5, dist.SUM) == 7.5 and comm.allreduce_host(3.0, dist.MAX) == 3.0
        comm.barrier()
        # tile stage: the communicator path (all-reduce of the row count, all-gather of rows,
        # ownership filter) gives exactly the local files with one rank
        local = bm.tiles()
        shared = bm.tiles(comm=comm)
        assert shared == local and len(local) > 10
        print("tiles via RCCL path", len(shared), "files", flush=True)
    finally:
        comm.close()
        hist.close()
        bm.close()
        eng.close()
