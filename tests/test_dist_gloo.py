"""N>1 path on CPU: uuid sharding + histogram all-reduce with gloo, world_size 2.

On the GPU the same reduction runs over RCCL (reporter_amd.dist.Comm); here each
rank matches its shard with the CPU oracle and the reduced histogram must equal
the single-process histogram of the whole trace set (the reference's keyed
repartition, BatchingProcessor.java:126, is a sum over vehicles).
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sub(tr, idx):
    off = tr["trace_off"].astype(np.int64)
    parts = {k: [] for k in ("lon", "lat", "time", "accuracy")}
    new_off = [0]
    for k in idx:
        for f in parts:
            parts[f].append(tr[f][off[k]:off[k + 1]])
        new_off.append(new_off[-1] + int(off[k + 1] - off[k]))
    out = {f: np.concatenate(v) if v else np.zeros(0) for f, v in parts.items()}
    out["trace_off"] = np.array(new_off, np.uint32)
    return out


def _hist(graph_path, tr):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import meili_oracle as mo
    from reporter_amd import engine, graphfile
    g = graphfile.load(graph_path)
    T = len(tr["trace_off"]) - 1
    h = np.zeros(len(g["seg_id"]) * 16, np.uint32)
    if T:
        b = mo.Batch(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], engine.default_options(1),
                     np.zeros(T, np.uint32))
        mo.pipeline(g, b, 15.0, 0xE, 0xE, h)
    return h


def _rank_main(rank, world, port, graph_path, npz, out):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from reporter_amd.dist import shard_by_uuid
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = np.load(npz)
    tr = {k: d[k] for k in d.files}
    uuids = ["veh-%d" % k for k in range(len(tr["trace_off"]) - 1)]
    pts = np.diff(tr["trace_off"].astype(np.int64))
    shards = shard_by_uuid(uuids, pts, world)
    h = _hist(graph_path, _sub(tr, shards[rank]))
    t = torch.from_numpy(h.astype(np.int64))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    if rank == 0:
        np.save(out, t.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_shard_invariants():
    sys.path.insert(0, ROOT)
    from reporter_amd.dist import shard_by_uuid, split
    uuids = ["u%d" % (i % 37) for i in range(200)]   # repeated vehicles
    pts = np.random.default_rng(0).integers(10, 1000, 200)
    for world in (1, 2, 3, 8):
        sh = shard_by_uuid(uuids, pts, world)
        allidx = np.sort(np.concatenate(sh))
        np.testing.assert_array_equal(allidx, np.arange(200))
        owner = {}
        for r, s in enumerate(sh):
            for i in s:
                assert owner.setdefault(uuids[i], r) == r  # a vehicle never straddles ranks
        loads = [pts[s].sum() for s in sh]
        assert max(loads) <= 1.6 * (sum(loads) / world) + pts.max()
    # split() reproduces py/simple_reporter.py:70-79
    assert [len(x) for x in split(list(range(10)), 3)] == [4, 3, 3]
    assert [len(x) for x in split(list(range(9)), 3)] == [3, 3, 3]


@pytest.mark.timeout(300)
def test_gloo_world2_histogram_equals_single_process(small_world, tmp_path):
    import multiprocessing as mp
    from reporter_amd import world
    tr = world.generate_traces(small_world, n_traces=48, n_points=200, rate_s=1.0, noise_m=5.0, seed=123)
    npz = str(tmp_path / "tr.npz")
    np.savez(npz, **{k: tr[k] for k in ("lon", "lat", "time", "accuracy", "trace_off")})
    out = str(tmp_path / "hist.npy")
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, small_world, npz, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
        assert p.exitcode == 0
    got = np.load(out)
    want = _hist(small_world, tr)
    np.testing.assert_array_equal(got, want.astype(np.int64))
    assert want.sum() > 0
