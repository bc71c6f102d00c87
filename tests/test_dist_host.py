"""The product's multi-rank code at world size 2 on CPU (gloo as the host transport).

On the GPU box the ranks talk RCCL over xGMI (dist.Comm, rm_comm_init); here the same
rm_comm object runs over an injected host all-gather (rm_comm_init_host, backed by
torch.distributed gloo in the test), so these CPU processes drive:

* dist.rendezvous — rank 0 hands the communicator id to the other ranks through a file;
* rm_comm_allreduce_host_f64 / rm_comm_barrier — bench.timed's barrier + max-over-ranks clock;
* bench.shard_ids — one seeded workload split by uuid with no trace on two ranks;
* the tile exchange of rm_runner_tiles (stages.hip): every rank's rows are all-gathered
  (padded to the largest rank's count, as the device path pads), each rank keeps the files
  rm_tile_file_owner assigns it (the same function the device filter k_tile_own calls) and
  culls them; the union of both ranks' files must be byte-identical to one process's.
  Rows and culling are the CPU restatement (tiles_oracle, pinned by the reference's own
  report() goldens); tests/test_gpu_stages.py runs the device side of the same exchange.

The reference's counterpart is the keyed Kafka repartition of "id next_id" reports
(BatchingProcessor.java:126) feeding one anonymiser per tile (AnonymisingProcessor.java:155-175).
"""
import json
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


def _points(path):
    from test_gpu_stages import _stream
    return _stream(path, n_veh=24, n_pts=200, seed=11)


def _tile_rows(g, pts, keep):
    """Tile lines {file: [rows]} of the vehicles in `keep` (CPU restatement)."""
    import tiles_oracle as to
    from test_gpu_stages import _oracle, _oracle_tiles  # noqa: F401
    import meili_oracle as mo
    from reporter_amd import engine
    sel = np.isin(pts["uuid"], keep)
    sub = {k: v[sel] for k, v in pts.items()}
    wins, tr, ref = _oracle(g, sub)
    rmask = tmask = engine.levels_mask((0, 1))
    files = {}
    for k in range(len(tr["trace_off"]) - 1):
        s0, s1 = ref["seg_off"][k], ref["seg_off"][k + 1]
        o0, o1 = tr["trace_off"][k], tr["trace_off"][k + 1]
        reps, _ = mo.report_trace(ref["segs"][s0:s1], tr["time"][o1 - 1], 15.0, rmask, tmask)
        rd = [{"id": int(r["id"]), "next_id": int(r["next_id"]), "t0": float(r["t0"]), "t1": float(r["t1"]),
               "length": int(r["length"]), "queue_length": int(r["queue_length"])} for r in reps]
        for name, ls in to.tile_lines(rd, int(tr["time"][o0]), int(tr["time"][o1 - 1])).items():
            files.setdefault(name, []).extend(ls)
    return files


def _owner(name, nranks):
    """rm_tile_file_owner of a file named "<start>_<end>/<level>/<tile index>" (3600 s tiles)."""
    from reporter_amd import _lib
    span, level, index = name.split("/")
    bucket = int(span.split("_")[0]) // 3600
    return _lib.lib().rm_tile_file_owner(bucket, int(level) | (int(index) << 3), nranks)


def _rank_main(rank, world, port, graph_path, rdzv, out_dir):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import time

    import torch
    import torch.distributed as tdist

    import bench
    import tiles_oracle as to
    from reporter_amd import dist, graphfile
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)

    def gloo_allgather(b):
        t = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(world)]
        tdist.all_gather(out, t)
        return [o.numpy().tobytes() for o in out]

    res = {}
    # rendezvous: rank 0's id reaches every rank -- rank 0 comes late, so rank 1 first finds the
    # stale id file the test planted (another launch's nonce) and must wait for the fresh one
    if rank == 0:
        time.sleep(1.0)
    res["rdzv"] = dist.rendezvous(rank, rdzv, lambda: os.urandom(128), 128, timeout_s=60).hex()
    # host communicator without a GPU: barrier + max-over-ranks timing exactly as bench.py times
    comm = dist.Comm(rank, world, -1, allgather=gloo_allgather)
    res["sum"] = comm.allreduce_host(rank + 1.0, dist.SUM)
    res["max"] = comm.allreduce_host(10.0 * rank, dist.MAX)
    res["timed"] = bench.timed(lambda: time.sleep(0.05 * (rank + 1)), 3, comm, lambda: None)
    # the data path of the exchange over the host transport (device -1: host buffers): the
    # histogram all-reduce and the optional reduce-scatter by segment-id range
    h = (np.arange(37, dtype=np.uint32) * 7 + rank * 1000).astype(np.uint32)
    comm.allreduce(h.ctypes.data, h.size, dist.U32, dist.SUM)
    res["ar"] = h.tolist()
    d = (np.arange(2 * 5, dtype=np.uint64) * (rank + 3)).astype(np.uint64)
    comm.reduce_scatter(d.ctypes.data, 5, dist.U64, dist.SUM)
    res["rs"] = d[5 * rank:5 * rank + 5].tolist()
    m = np.array([1.5 * rank, -2.0 * rank, 3.0], np.float64)
    comm.allreduce(m.ctypes.data, 3, dist.F64, dist.MAX)
    res["mx"] = m.tolist()
    # the tile exchange
    g = graphfile.load(graph_path)
    pts = _points(graph_path)
    veh = np.unique(pts["uuid"])
    shard = dist.shard_by_uuid([str(v) for v in veh], [int((pts["uuid"] == v).sum()) for v in veh], world)[rank]
    mine = _tile_rows(g, pts, veh[shard])
    blob = json.dumps(sorted((n, ls) for n, ls in mine.items())).encode()
    longest = int(comm.allreduce_host(len(blob), dist.MAX))                 # TileComm::max_u64
    parts = gloo_allgather(blob + b" " * (longest - len(blob)))             # TileComm::allgather, padded
    gathered = {}
    for p in parts:
        for name, ls in json.loads(p.decode().rstrip()):
            gathered.setdefault(name, []).extend(ls)
    owned = {}
    for name, ls in gathered.items():
        if _owner(name, world) == rank:
            body = to.tile_body(ls, 2)
            if body is not None:
                owned[name] = body
    res["files"] = owned
    res["rows_mine"] = sum(len(v) for v in mine.values())
    comm.barrier()
    comm.close()
    with open(os.path.join(out_dir, "rank%d.json" % rank), "w") as f:
        json.dump(res, f)
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.timeout(300)
def test_world2_host_comm_timing_and_tile_exchange(small_world, tmp_path, built_lib):
    import multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from reporter_amd import graphfile
    from test_gpu_stages import _oracle, _oracle_tiles
    port = _free_port()
    ctx = mp.get_context("spawn")
    rdzv = str(tmp_path / "rdzv.id")
    from reporter_amd import dist
    stale = os.urandom(128)
    with open(rdzv, "wb") as f:   # what a crashed earlier launch at the same path left behind
        f.write(stale + b"1234:5678".ljust(dist.NONCE_BYTES, b"\0"))
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, small_world, rdzv, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(280)
        assert p.exitcode == 0
    r0, r1 = (json.load(open(str(tmp_path / ("rank%d.json" % r)))) for r in range(2))
    assert r0["rdzv"] == r1["rdzv"] and len(r0["rdzv"]) == 256 and r0["rdzv"] != stale.hex()
    assert r0["sum"] == r1["sum"] == 3.0 and r0["max"] == r1["max"] == 10.0
    want_ar = (np.arange(37, dtype=np.uint64) * 14 + 1000).tolist()
    assert r0["ar"] == r1["ar"] == want_ar
    full = np.arange(10, dtype=np.uint64) * 3 + np.arange(10, dtype=np.uint64) * 4   # ranks 0 and 1
    assert r0["rs"] == full[:5].tolist() and r1["rs"] == full[5:].tolist()
    assert r0["mx"] == r1["mx"] == [1.5, 0.0, 3.0]
    # max over ranks: rank 1 sleeps 3 x 0.1 s, and both ranks report its clock
    assert r0["timed"] == r1["timed"] and 0.3 <= r0["timed"] < 2.0
    assert r0["rows_mine"] > 0 and r1["rows_mine"] > 0
    # tile files: disjoint between the ranks, their union byte-identical to one process's
    assert not set(r0["files"]) & set(r1["files"])
    union = dict(r0["files"], **r1["files"])
    g = graphfile.load(small_world)
    wins, tr, ref = _oracle(g, _points(small_world))
    want = _oracle_tiles(ref, tr, 2)
    assert len(want) > 3 and r0["files"] and r1["files"]
    assert union == want


def test_rendezvous_ignores_a_stale_id(tmp_path):
    """an id file at the launch's path written by another launch (a crashed
    run whose pid and port recur) is not accepted; the fresh one is, and rank 0 replaces it."""
    from reporter_amd import dist
    path = str(tmp_path / "rm_rdzv_x.id")
    stale = os.urandom(128)
    with open(path, "wb") as f:
        f.write(stale + b"old-launch".ljust(dist.NONCE_BYTES, b"\0"))
    with pytest.raises(TimeoutError):
        dist.rendezvous(1, path, None, 128, timeout_s=0.3, nonce="this-launch")
    with open(path, "wb") as f:   # a round-4 file (no nonce at all)
        f.write(stale)
    with pytest.raises(TimeoutError):
        dist.rendezvous(1, path, None, 128, timeout_s=0.3, nonce="this-launch")
    fresh = dist.rendezvous(0, path, lambda: os.urandom(128), 128, nonce="this-launch")
    assert fresh != stale and dist.rendezvous(1, path, None, 128, timeout_s=5, nonce="this-launch") == fresh
    # the default nonce: the parent process named by pid and start time (shared by sibling ranks)
    assert dist.launch_nonce().startswith("%d:" % os.getppid()) and dist.launch_nonce() != "%d:0" % os.getppid()


def test_rendezvous_nonce_changes_across_elastic_restarts(monkeypatch, tmp_path):
    """under torchrun --max-restarts the agent (the ranks' parent) survives a restart,
    so the nonce and the rendezvous file name also carry TORCHELASTIC_RUN_ID / _RESTART_COUNT: a
    crashed attempt's id file is not accepted by the next attempt's ranks."""
    from reporter_amd import dist
    monkeypatch.delenv("RM_RDZV_NONCE", raising=False)
    monkeypatch.delenv("RM_RDZV_TOKEN", raising=False)
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "job7")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "0")
    n0, p0 = dist.launch_nonce(), dist.rendezvous_path(str(tmp_path))
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")
    n1, p1 = dist.launch_nonce(), dist.rendezvous_path(str(tmp_path))
    assert n0 != n1 and p0 != p1 and n1.endswith(":job7:1")
    # attempt 0's file at attempt 1's path (same pid, port) is ignored until rank 0 replaces it
    dist.rendezvous(0, p1, lambda: os.urandom(128), 128, nonce=n0)
    with pytest.raises(TimeoutError):
        dist.rendezvous(1, p1, None, 128, timeout_s=0.3, nonce=n1)
    fresh = dist.rendezvous(0, p1, lambda: os.urandom(128), 128, nonce=n1)
    assert dist.rendezvous(1, p1, None, 128, timeout_s=5, nonce=n1) == fresh


def test_shard_ids_partition_one_workload():
    """bench.shard_ids: every trace of the seeded N x n set on exactly one rank."""
    sys.path.insert(0, ROOT)
    import bench
    for world in (1, 2, 4):
        ids = [bench.shard_ids("C2", 64, 600, world, r) for r in range(world)]
        allids = np.sort(np.concatenate(ids))
        np.testing.assert_array_equal(allids, np.arange(64 * world))
        assert min(len(x) for x in ids) > 0


def test_tile_owner_rule():
    """rm_tile_file_owner: a pure function of (bucket, tile, nranks) in [0, nranks), the same
    file always on the same rank, and files spread over the ranks."""
    from reporter_amd import _lib
    L = _lib.lib()
    for n in (1, 2, 3, 8):
        owners = [L.rm_tile_file_owner(b, t, n) for b in range(412000, 412040) for t in range(0, 800, 8)]
        assert set(owners) == set(range(n))
        assert owners == [L.rm_tile_file_owner(b, t, n) for b in range(412000, 412040) for t in range(0, 800, 8)]


def _tcp_rank(rank, world, port, out_dir):
    sys.path.insert(0, ROOT)
    from reporter_amd import dist
    ag = dist.TcpAllgather(rank, world, "127.0.0.1", port, timeout_s=60)
    res = {"parts": [p.hex() for p in ag(bytes([rank + 1]) * (3 + 0))]}
    big = ag(bytes([rank]) * 100000)
    res["big_ok"] = all(p == bytes([r]) * 100000 for r, p in enumerate(big))
    comm = dist.Comm(rank, world, -1, allgather=ag)   # the product's communicator, host values only
    res["sum"] = comm.allreduce_host(2.0 ** rank, dist.SUM)
    res["max"] = comm.allreduce_host(float(rank), dist.MAX)
    comm.barrier()
    comm.close()
    ag.close()
    with open(os.path.join(out_dir, "tcp%d.json" % rank), "w") as f:
        json.dump(res, f)


@pytest.mark.timeout(120)
def test_tcp_allgather_world3(tmp_path, built_lib):
    """dist.TcpAllgather (bench.py --comm host: ranks sharing a GPU, no framework) at world 3."""
    import multiprocessing as mp
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_tcp_rank, args=(r, 3, port, str(tmp_path))) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(100)
        assert p.exitcode == 0
    res = [json.load(open(str(tmp_path / ("tcp%d.json" % r)))) for r in range(3)]
    for r in res:
        assert r["parts"] == ["010101", "020202", "030303"]
        assert r["big_ok"] and r["sum"] == 7.0 and r["max"] == 2.0


def _stall_rank(rank, world, port, exit_mode, out_dir):
    """Rank 1 joins one all-reduce, then stops (never joins the second); rank 0 must fail within
    RM_COMM_TIMEOUT_S -- by exiting with status 3 (exit mode) or with an error (library mode)."""
    sys.path.insert(0, ROOT)
    import datetime
    import time

    import torch
    import torch.distributed as tdist

    from reporter_amd import _lib, dist
    os.environ["RM_COMM_TIMEOUT_S"] = "3"
    os.environ["RM_COMM_TIMEOUT_EXIT"] = "1" if exit_mode else "0"
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=120))

    def gloo_allgather(b):
        t = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(world)]
        tdist.all_gather(out, t)
        return [o.numpy().tobytes() for o in out]

    comm = dist.Comm(rank, world, -1, allgather=gloo_allgather)
    h = np.arange(8, dtype=np.uint32) + rank
    comm.allreduce(h.ctypes.data, h.size, dist.U32, dist.SUM)   # both ranks: completes
    res = {"first": h.tolist()}
    if rank == 1:
        time.sleep(10)   # stopped: the second all-reduce never sees this rank
        os._exit(0)
    t0 = time.time()
    try:
        comm.allreduce(h.ctypes.data, h.size, dist.U32, dist.SUM)
        res["second"] = "completed"
    except _lib.RmError as e:
        res["second"] = str(e)
    res["elapsed"] = time.time() - t0
    t1 = time.time()
    try:   # the broken communicator fails at once
        comm.allreduce_host(1.0, dist.SUM)
        res["third"] = "completed"
    except _lib.RmError as e:
        res["third"] = str(e)
    res["third_elapsed"] = time.time() - t1
    with open(os.path.join(out_dir, "stall%d.json" % rank), "w") as f:
        json.dump(res, f)
    os._exit(0)   # the stuck helper thread and process group are left behind


@pytest.mark.timeout(120)
@pytest.mark.parametrize("exit_mode", [True, False])
def test_collective_bounded_when_a_rank_stops(tmp_path, built_lib, exit_mode):
    """every collective (not only the init) runs under RM_COMM_TIMEOUT_S.  A
    rank whose peer stops mid-run fails within the bound: status 3 by default (a failed rank for
    the launcher, never a re-exec), or with RM_COMM_TIMEOUT_EXIT=0 (library hosts) an error from
    the call, after which the communicator refuses every call at once."""
    import multiprocessing as mp
    import time
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_stall_rank, args=(r, 2, port, exit_mode, str(tmp_path))) for r in range(2)]
    t0 = time.time()
    for p in procs:
        p.start()
    procs[0].join(60)
    elapsed = time.time() - t0
    assert procs[0].exitcode is not None, "rank 0 did not fail within the bound"
    if exit_mode:
        assert procs[0].exitcode == 3 and elapsed < 45
        assert not os.path.exists(str(tmp_path / "stall0.json"))
    else:
        assert procs[0].exitcode == 0
        r0 = json.load(open(str(tmp_path / "stall0.json")))
        assert r0["first"] == (np.arange(8) * 2 + 1).tolist()
        assert "RM_COMM_TIMEOUT_S" in r0["second"] and 2.5 < r0["elapsed"] < 15, r0
        assert "unusable" in r0["third"] and r0["third_elapsed"] < 1.0, r0
    procs[1].join(20)
    if procs[1].exitcode is None:
        procs[1].kill()
