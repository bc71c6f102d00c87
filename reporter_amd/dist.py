"""Multi-GPU plumbing: one process per GPU, uuid sharding, RCCL histogram reduce.

The reference distributes only by vehicle: Kafka partitions keyed by uuid
(README.md:169-173), ``sha1(uuid)[0:3]`` files in the batch reporter
(py/simple_reporter.py:116) and a static block split over processes
(py/simple_reporter.py:70-79).  Its one exchange step is the keyed
repartition of ``"id next_id"`` reports (BatchingProcessor.java:126) into
time-tile histograms.  Here: traces shard by uuid across ranks with no
data-path collective; the per-OSMLR-segment speed histogram is combined with
one RCCL all-reduce over xGMI (``Comm``), bound natively in
libreporter_match.so (no PyTorch in the process).  The same collectives can run
over a host transport the caller injects (``Comm(..., allgather=fn)``,
rm_comm_init_host): a multi-rank job that already has one (e.g. gloo), several
ranks sharing one GPU, or a CPU-only test of the exchange logic.
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


def _proc_start_ticks(pid):
    """Start time of process `pid` in clock ticks since boot (/proc/<pid>/stat field 22): with
    the pid it names one process instance, even after the pid is reused."""
    try:
        with open("/proc/%d/stat" % pid) as f:
            return f.read().rsplit(")", 1)[1].split()[19]
    except (OSError, IndexError):
        return "0"


def launch_nonce():
    """What every rank of one launch agrees on and no other launch has: the launcher's
    RM_RDZV_NONCE (bench.py self_launch sets a random one), else the parent process (torchrun's
    agent, or whatever started the ranks) named by pid and start time -- plus torchrun's run id and
    restart count when present: with --max-restarts the elastic agent is the same process across
    restarts, so a crashed attempt's file would otherwise carry the restarted attempt's nonce."""
    n = os.environ.get("RM_RDZV_NONCE")
    if n:
        return n
    ppid = os.getppid()
    return "%d:%s%s" % (ppid, _proc_start_ticks(ppid), _elastic_attempt())


def _elastic_attempt():
    """':<run id>:<restart count>' under torch.distributed.run (TORCHELASTIC_*), else ''."""
    run = os.environ.get("TORCHELASTIC_RUN_ID")
    cnt = os.environ.get("TORCHELASTIC_RESTART_COUNT")
    if run is None and cnt is None:
        return ""
    return ":%s:%s" % (run or "", cnt or "0")


def rendezvous_path(rdzv_dir=None, token=None):
    """Node-local file through which rank 0 hands its RCCL unique id to the other ranks."""
    rdzv_dir = rdzv_dir or os.environ.get("RM_RDZV_DIR", "/tmp")
    token = token or os.environ.get("RM_RDZV_TOKEN") or "%s_%s%s" % (
        os.environ.get("MASTER_PORT", "0"), os.getppid(),
        "_r" + os.environ["TORCHELASTIC_RESTART_COUNT"] if os.environ.get("TORCHELASTIC_RESTART_COUNT") else "")
    return os.path.join(rdzv_dir, "rm_rdzv_%s.id" % token)


NONCE_BYTES = 64


def rendezvous(rank, path, make_id, size=128, timeout_s=300.0, nonce=None):
    """Rank 0 writes make_id() (`size` bytes) and the launch nonce atomically to `path`; every
    other rank polls until a complete id carrying the same nonce is there.  A file a crashed
    earlier launch left at the same path (same port, a reused pid) carries another nonce and is
    ignored until rank 0 replaces it.  Returns the id on every rank."""
    tag = (nonce if nonce is not None else launch_nonce()).encode()[:NONCE_BYTES].ljust(NONCE_BYTES, b"\0")
    if rank == 0:
        data = bytes(make_id())
        if len(data) != size:
            raise ValueError("rendezvous id must be %d bytes" % size)
        try:
            os.remove(path)   # whatever an earlier launch left
        except FileNotFoundError:
            pass
        tmp = "%s.%d.tmp" % (path, os.getpid())
        with open(tmp, "wb") as f:
            f.write(data + tag)
        os.replace(tmp, path)
        return data
    t0 = time.time()
    while True:
        try:
            with open(path, "rb") as f:
                data = f.read()
            if len(data) == size + NONCE_BYTES and data[size:] == tag:
                return data[:size]
        except FileNotFoundError:
            pass
        if time.time() - t0 > timeout_s:
            raise TimeoutError("rank %d: no rendezvous id of this launch at %s" % (rank, path))
        time.sleep(0.05)


HOST_ALLGATHER = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p)


class TcpAllgather:
    """A host all-gather over TCP with no framework (for rm_comm_init_host): rank 0 listens on
    (addr, port), every other rank connects once; each call sends this rank's bytes to rank 0,
    which returns every rank's bytes in rank order to all.  Lets several ranks share one GPU
    (RCCL refuses two ranks on one device) with the product's exchange code unchanged."""

    def __init__(self, rank, world_size, addr="127.0.0.1", port=29555, timeout_s=300.0):
        import socket
        self.rank, self.world = rank, world_size
        self.peers = {}
        if world_size == 1:
            return
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(world_size)
            srv.settimeout(timeout_s)
            while len(self.peers) < world_size - 1:
                conn, _ = srv.accept()
                conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                r = int.from_bytes(self._recv(conn, 4), "little")
                self.peers[r] = conn
            srv.close()
        else:
            t0 = time.time()
            while True:
                try:
                    conn = socket.create_connection((addr, port), timeout=timeout_s)
                    break
                except OSError:
                    if time.time() - t0 > timeout_s:
                        raise
                    time.sleep(0.05)
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            conn.sendall(rank.to_bytes(4, "little"))
            self.peers[0] = conn

    @staticmethod
    def _recv(conn, n):
        buf = bytearray(n)
        view, got = memoryview(buf), 0
        while got < n:
            k = conn.recv_into(view[got:], n - got)
            if k == 0:
                raise ConnectionError("peer closed")
            got += k
        return bytes(buf)

    def __call__(self, data):
        if self.world == 1:
            return [data]
        n = len(data)
        if self.rank == 0:
            parts = [data] + [self._recv(self.peers[r], n) for r in range(1, self.world)]
            blob = b"".join(parts)
            for r in range(1, self.world):
                self.peers[r].sendall(blob)
            return parts
        self.peers[0].sendall(data)
        blob = self._recv(self.peers[0], n * self.world)
        return [blob[r * n:(r + 1) * n] for r in range(self.world)]

    def close(self):
        for c in self.peers.values():
            c.close()
        self.peers = {}


class Comm:
    """Communicator for one rank (one process per GPU, single node): RCCL over xGMI, or, with
    `allgather`, a host transport — a callable taking this rank's bytes and returning every
    rank's bytes in rank order (rm_comm_init_host).  device -1 (host transport only): host
    values and barriers without a GPU."""

    def __init__(self, rank, world_size, device, rdzv_dir=None, token=None, timeout_s=300.0, allgather=None):
        self.rank, self.world_size, self.device = rank, world_size, device
        L = _lib.lib()
        self._path = None
        if allgather is not None:
            def gather(_ctx, send, nbytes, recv):
                try:
                    parts = allgather(C.string_at(send, nbytes) if nbytes else b"")
                    if len(parts) != world_size or any(len(p) != nbytes for p in parts):
                        return 1
                    if nbytes:
                        C.memmove(recv, b"".join(parts), nbytes * world_size)
                    return 0
                except Exception:  # noqa: BLE001 -- reported to the library as a failed collective
                    return 1
            self._cb = HOST_ALLGATHER(gather)   # kept alive as long as the communicator
            self._h = L.rm_comm_init_host(world_size, rank, self._cb, None, device)
        else:
            path = rendezvous_path(rdzv_dir, token)

            def make_id():
                uid = (C.c_uint8 * 128)()
                _lib.check(L.rm_comm_unique_id(uid))
                return bytes(uid)
            uid = (C.c_uint8 * 128).from_buffer_copy(rendezvous(rank, path, make_id, 128, timeout_s))
            self._h = _stdout_to_stderr(lambda: L.rm_comm_init(world_size, rank, uid, device))
            self._path = path
        if not self._h:
            raise _lib.RmError(_lib.last_error())

    def allreduce(self, dev_ptr, count, dtype=U32, op=SUM):
        """In place on a device buffer (host memory on a device -1 host-transport Comm)."""
        _lib.check(_lib.lib().rm_comm_allreduce(self._h, dev_ptr, count, dtype, op))

    def reduce_scatter(self, ptr, count_per_rank, dtype=U32, op=SUM):
        """ptr holds world_size chunks of count_per_rank elements; chunk `rank` receives the
        reduction of every rank's chunk `rank` (each rank owns one segment-id range)."""
        _lib.check(_lib.lib().rm_comm_reduce_scatter(self._h, ptr, count_per_rank, dtype, op))

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
            if self.rank == 0 and self._path:
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
