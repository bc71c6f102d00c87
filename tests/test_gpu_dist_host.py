"""The product's multi-rank exchange on the GPU at world size 2 (two ranks sharing one GPU).

RCCL refuses two ranks on one device, so the ranks talk over the host transport of
rm_comm_init_host (torch.distributed gloo here); everything else is the product path:
rm_runner_run_points on each rank's uuid shard, rm_runner_tiles with the communicator
(rows padded to the largest rank's count, all-gathered, filtered by k_tile_own /
tile_file_owner, culled and formatted on the device), and rm_comm_allreduce of the
device speed histogram and duration sums.  The union of the two ranks' tile files must
be byte-identical to one process's, and the reduced histogram equal one process's.
"""
import json
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _match(path, pts, keep, comm=None):
    """run_points over the vehicles in `keep`; (tile files, histogram, duration sums)."""
    from reporter_amd import dist, engine
    sel = np.isin(pts["uuid"], keep)
    eng = engine.Engine(path, 0)
    bm = engine.BatchMatcher(eng)
    nseg = eng.n_segments
    hist, dur = dist.DeviceBuffer(nseg * 16 * 4), dist.DeviceBuffer(nseg * 8)
    bm.run_points(pts["uuid"][sel], pts["time"][sel], pts["lon"][sel], pts["lat"][sel], pts["accuracy"][sel],
                  inactivity=120, n_uuids=int(pts["uuid"].max()) + 1, hist_dev=hist.ptr, dur_dev=dur.ptr,
                  zero_hist=True)
    files = bm.tiles(privacy=2, comm=comm)
    rs = None
    if comm is not None:
        # the reduce-scatter exchange of the same counts: this rank's padded segment-id range
        w = comm.world_size
        ch = 16 * -(-nseg // w)   # whole segments per rank
        part = dist.DeviceBuffer(ch * w * 4)
        part.upload(hist.download())
        comm.reduce_scatter(part.ptr, ch, dist.U32, dist.SUM)
        rs = part.download()[comm.rank * ch:(comm.rank + 1) * ch]
        part.close()
        comm.allreduce(hist.ptr, nseg * 16, dist.U32, dist.SUM)
        comm.allreduce(dur.ptr, nseg, dist.U64, dist.SUM)
    h, d = hist.download(), dur.download(np.uint64)
    for x in (hist, dur, bm, eng):
        x.close()
    if rs is not None:   # the range equals the all-reduced histogram's (zero past the last segment)
        w = comm.world_size
        ch = 16 * -(-nseg // w)   # whole segments per rank
        want = np.zeros(ch * w, np.uint32)
        want[:nseg * 16] = h
        np.testing.assert_array_equal(rs, want[comm.rank * ch:(comm.rank + 1) * ch])
    return files, h, d


def _rank_main(rank, world, port, path, out_dir):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as tdist
    from reporter_amd import dist
    from test_gpu_stages import _stream
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)

    def gloo_allgather(b):
        t = torch.frombuffer(bytearray(b), dtype=torch.uint8)
        out = [torch.empty_like(t) for _ in range(world)]
        tdist.all_gather(out, t)
        return [o.numpy().tobytes() for o in out]

    pts = _stream(path, n_veh=30, n_pts=240, seed=21)
    veh = np.unique(pts["uuid"])
    shard = dist.shard_by_uuid([str(v) for v in veh], [int((pts["uuid"] == v).sum()) for v in veh], world)[rank]
    comm = dist.Comm(rank, world, 0, allgather=gloo_allgather)
    files, h, d = _match(path, pts, veh[shard], comm)
    comm.close()
    with open(os.path.join(out_dir, "rank%d.json" % rank), "w") as f:
        json.dump(files, f)
    if rank == 0:
        np.save(os.path.join(out_dir, "hist.npy"), h)
        np.save(os.path.join(out_dir, "dur.npy"), d)
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_ranks_one_gpu_tiles_and_histogram(small_world, tmp_path):
    import multiprocessing as mp
    from test_gpu_stages import _stream
    port = _free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, small_world, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
        assert p.exitcode == 0
    f0, f1 = (json.load(open(str(tmp_path / ("rank%d.json" % r)))) for r in range(2))
    pts = _stream(small_world, n_veh=30, n_pts=240, seed=21)
    want, wh, wd = _match(small_world, pts, np.unique(pts["uuid"]))
    assert f0 and f1 and not set(f0) & set(f1)
    assert dict(f0, **f1) == want
    np.testing.assert_array_equal(np.load(str(tmp_path / "hist.npy")), wh)
    np.testing.assert_array_equal(np.load(str(tmp_path / "dur.npy")), wd)
    assert wh.sum() > 0 and wd.sum() > 0


_LONE_RANK = r"""
import os, sys, time
sys.path.insert(0, os.environ["RM_ROOT"])
from reporter_amd import dist
t0 = time.time()
try:
    dist.Comm(0, 2, 0, rdzv_dir=os.environ["RM_RDZV_DIR"], token="lone", timeout_s=5)
except Exception as e:   # the library's RuntimeError, raised by the ctypes shim
    print("FAILED after %.1f s: %s" % (time.time() - t0, e))
    sys.exit(3)
sys.exit(0)
"""


def test_comm_init_without_peers_fails_in_bounded_time(built_lib, tmp_path):
    """rank 0 of a world of 2 whose peer never starts fails (exit status 3,
    a message naming the timeout) after RM_COMM_TIMEOUT_S instead of blocking in RCCL's init."""
    import subprocess
    env = dict(os.environ, RM_ROOT=ROOT, RM_RDZV_DIR=str(tmp_path), RM_COMM_TIMEOUT_S="4")
    r = subprocess.run([sys.executable, "-c", _LONE_RANK], env=env, capture_output=True, text=True, timeout=90)
    assert r.returncode == 3, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "RM_COMM_TIMEOUT_S" in r.stderr and "did not join" in r.stderr, r.stderr[-2000:]
