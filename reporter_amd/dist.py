"""Multi-GPU plumbing: one process per GPU, uuid sharding, RCCL histogram reduce.

The reference distributes only by vehicle: Kafka partitions keyed by uuid
(README.md:169-173), ``sha1(uuid)[0:3]`` files in the batch reporter
(py/simple_reporter.py:116) and a static block split over processes
(py/simple_reporter.py:70-79).  Its one exchange step is the keyed
repartition of ``"id next_id"`` reports (BatchingProcessor.java:126) into
time-tile histograms.  Here: traces shard by uuid across ranks with no
data-path collective; the per-OSMLR-segment speed histogram is combined with
one RCCL all-reduce over xGMI (``Comm``), bound natively in
libreporter_match.so (no PyTorch in the process).
"""
import ctypes as C
import hashlib
import os
import time

import numpy as np

from . import _lib

U32, U64, F64 = 0, 1, 2
SUM, MAX = 0, 1


def split(items, n):
    """Contiguous block split, remainder to the first blocks (py/simple_reporter.py:70-79)."""
    size = -(-len(items) // n) if n else 0
    cutoff = len(items) % n
    out, pos = [], 0
    for i in range(n):
        end = pos + size if cutoff == 0 or i < cutoff else pos + size - 1
        out.append(items[pos:end])
        pos = end
    return out


def uuid_bucket(uuid, n_buckets):
    """Stable bucket of a vehicle id (sha1 prefix, as py/simple_reporter.py:116 does)."""
    h = hashlib.sha1(str(uuid).encode("utf-8")).digest()
    return int.from_bytes(h[:8], "big") % n_buckets


def shard_by_uuid(uuids, points, world_size, buckets_per_rank=16):
    """Greedy point-count balancing of hash(uuid) buckets over ranks.

    Returns a list (per rank) of trace index arrays in input order.  Pure
    hashing leaves heavy tails; balancing whole buckets keeps every trace of a
    vehicle on one rank while evening out the points."""
    nb = max(1, world_size * buckets_per_rank)
    b = np.array([uuid_bucket(u, nb) for u in uuids], np.int64)
    load = np.bincount(b, weights=np.asarray(points, np.float64), minlength=nb)
    owner = np.empty(nb, np.int64)
    rank_load = np.zeros(world_size)
    for bucket in sorted(range(nb), key=lambda x: (-load[x], x)):
        r = int(np.argmin(rank_load))  # lowest rank on ties
        owner[bucket] = r
        rank_load[r] += load[bucket]
    return [np.nonzero(owner[b] == r)[0] for r in range(world_size)]


def _stdout_to_stderr(fn):
    """Run fn with file descriptor 1 pointed at stderr: RCCL prints a version banner on
    stdout at communicator init, and bench.py's stdout must hold exactly one JSON line."""
    import sys
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        return fn()
    finally:
        os.dup2(saved, 1)
        os.close(saved)


class Comm:
    """RCCL communicator for one rank (one process per GPU, single node)."""

    def __init__(self, rank, world_size, device, rdzv_dir=None, token=None, timeout_s=300.0):
        self.rank, self.world_size, self.device = rank, world_size, device
        L = _lib.lib()
        rdzv_dir = rdzv_dir or os.environ.get("RM_RDZV_DIR", "/tmp")
        token = token or "%s_%s" % (os.environ.get("MASTER_PORT", "0"), os.getppid())
        path = os.path.join(rdzv_dir, "rm_rdzv_%s.id" % token)
        uid = (C.c_uint8 * 128)()
        if rank == 0:
            _lib.check(L.rm_comm_unique_id(uid))
            tmp = path + ".tmp"
            with open(tmp, "wb") as f:
                f.write(bytes(uid))
            os.replace(tmp, path)
        else:
            t0 = time.time()
            while True:
                try:
                    with open(path, "rb") as f:
                        data = f.read()
                    if len(data) == 128:
                        break
                except FileNotFoundError:
                    pass
                if time.time() - t0 > timeout_s:
                    raise TimeoutError("rank %d: no RCCL id at %s" % (rank, path))
                time.sleep(0.05)
            C.memmove(uid, data, 128)
        self._h = _stdout_to_stderr(lambda: L.rm_comm_init(world_size, rank, uid, device))
        if not self._h:
            raise _lib.RmError(_lib.last_error())
        self._path = path

    def allreduce(self, dev_ptr, count, dtype=U32, op=SUM):
        _lib.check(_lib.lib().rm_comm_allreduce(self._h, dev_ptr, count, dtype, op))

    def allreduce_host(self, value, op=SUM):
        v = C.c_double(float(value))
        _lib.check(_lib.lib().rm_comm_allreduce_host_f64(self._h, C.byref(v), op))
        return v.value

    def barrier(self):
        _lib.check(_lib.lib().rm_comm_barrier(self._h))

    def close(self):
        if getattr(self, "_h", None):
            self.barrier()
            _lib.lib().rm_comm_destroy(self._h)
            self._h = None
            if self.rank == 0:
                try:
                    os.remove(self._path)
                except OSError:
                    pass


class DeviceBuffer:
    """Plain device allocation (no framework)."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        _lib.check(_lib.lib().rm_device_alloc(self.nbytes, C.byref(p)))
        self.ptr = p.value
        self.zero()

    def zero(self):
        _lib.check(_lib.lib().rm_device_memset(self.ptr, 0, self.nbytes))

    def download(self, dtype=np.uint32):
        out = np.empty(self.nbytes // np.dtype(dtype).itemsize, dtype)
        _lib.check(_lib.lib().rm_device_download(out.ctypes.data, self.ptr, self.nbytes))
        return out

    def upload(self, arr):
        arr = np.ascontiguousarray(arr)
        if arr.nbytes > self.nbytes:
            raise ValueError("array larger than the buffer")
        _lib.check(_lib.lib().rm_device_upload(self.ptr, arr.ctypes.data, arr.nbytes))

    def close(self):
        if getattr(self, "ptr", None):
            _lib.lib().rm_device_free(self.ptr)
            self.ptr = None
