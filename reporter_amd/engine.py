"""Batched array API over the HIP engine (rm_engine / rm_runner of the C-ABI).

This is the high-throughput path the bench and the batch pipeline use: traces
go in as flat numpy arrays (CSR offsets per trace), every stage runs on the GPU,
and stage outputs can be downloaded for parity checks.  Requires a GPU.
"""
import ctypes as C
import os

import numpy as np

from . import _lib

SEGMENT_DTYPE = np.dtype([
    ("segment_id", "<u8"), ("start_time", "<f8"), ("end_time", "<f8"), ("length", "<i4"),
    ("queue_length", "<i4"), ("flags", "<u4"), ("begin_shape_index", "<u4"), ("end_shape_index", "<u4"),
    ("seg_dense", "<u4"), ("way_first", "<u4"), ("way_last", "<u4")])
assert SEGMENT_DTYPE.itemsize == 56

REPORT_DTYPE = np.dtype([
    ("id", "<u8"), ("next_id", "<u8"), ("t0", "<f8"), ("t1", "<f8"), ("length", "<i4"),
    ("queue_length", "<i4"), ("seg_dense", "<u4"), ("pad", "<u4")])
assert REPORT_DTYPE.itemsize == 48

STATS_DTYPE = np.dtype([
    ("successful_count", "<i4"), ("unreported_count", "<i4"), ("successful_length_m", "<i4"),
    ("unreported_length_m", "<i4"), ("discontinuities", "<i4"), ("invalid_speeds", "<i4"),
    ("invalid_times", "<i4"), ("unassociated", "<i4"), ("shape_used", "<i4"), ("n_reports", "<i4")])
assert STATS_DTYPE.itemsize == 40

OPTIONS_DTYPE = np.dtype([
    ("mode", "<i4"), ("sigma_z", "<f4"), ("beta", "<f4"), ("search_radius", "<f4"), ("gps_accuracy", "<f4"),
    ("breakage_distance", "<f4"), ("interpolation_distance", "<f4"), ("max_route_distance_factor", "<f4"),
    ("max_route_time_factor", "<f4"), ("turn_penalty_factor", "<f4")])
assert OPTIONS_DTYPE.itemsize == 40

MAX_CAND = 16
INVALID_SEGMENT_ID = 0x3FFFFFFFFFFF  # Segment.java:16, simple_reporter.py:43


def default_options(n=1, **over):
    o = _lib.RmOptions()
    _lib.lib().rm_default_options(C.byref(o))
    a = np.zeros(n, OPTIONS_DTYPE)
    for name, _ in _lib.RmOptions._fields_:
        a[name] = getattr(o, name)
    for k, v in over.items():
        a[k] = v
    return a


def levels_mask(levels):
    """bit (level+1) per level, as the kernels and the oracle expect."""
    m = 0
    for lv in levels:
        if 0 <= int(lv) <= 7:
            m |= 1 << (int(lv) + 1)
    return m


class Engine:
    """The road graph resident in one GPU's HBM."""

    def __init__(self, graph_path, device=0):
        self._h = _lib.lib().rm_engine_create(os.fsencode(graph_path), int(device))
        if not self._h:
            raise _lib.RmError(_lib.last_error())
        self.graph_path = graph_path
        self.device = device

    @property
    def n_segments(self):
        return int(_lib.lib().rm_engine_n_segments(self._h))

    def segment_ids(self):
        ids = np.empty(self.n_segments, np.uint64)
        _lib.check(_lib.lib().rm_engine_segment_ids(self._h, ids.ctypes.data))
        return ids

    def set_ball_radius(self, meters):
        """Radius of the route balls (K2 lookup tier; 0 disables it).  Call before the first run."""
        _lib.check(_lib.lib().rm_engine_set_ball_radius(self._h, float(meters)))

    def ball_stats(self, mode=0):
        out = np.zeros(6, np.float64)
        _lib.check(_lib.lib().rm_engine_ball_stats(self._h, int(mode), out.ctypes.data))
        d = dict(zip(("radius_m", "keys", "entries", "nodes_without_table", "build_ms"), out[:5].tolist()))
        d["built_on_gpu"] = bool(out[5])
        return d

    def turn_rows(self):
        """Turn rows built so far (rule 3b): {mode name: build ms}."""
        mask = C.c_uint32(0)
        ms = np.zeros(5, np.float64)
        _lib.check(_lib.lib().rm_engine_turn_rows(self._h, C.byref(mask), ms.ctypes.data))
        names = ("auto", "bus", "motor_scooter", "bicycle", "pedestrian")
        return {names[m]: float(ms[m]) for m in range(5) if (mask.value >> m) & 1}

    def grid_split(self):
        """K1 grid refinement f (each graph-file cell split f x f)."""
        out = np.zeros(1, np.uint32)
        _lib.check(_lib.lib().rm_engine_grid_split(self._h, out.ctypes.data))
        return int(out[0])

    def grid_alt(self):
        """K1's second grid: (split f, batch radius in m from which it is used); (0, 0) if none."""
        f = np.zeros(1, np.uint32)
        r = np.zeros(1, np.float32)
        _lib.check(_lib.lib().rm_engine_grid_alt(self._h, f.ctypes.data, r.ctypes.data))
        return int(f[0]), float(r[0])

    def ball_lookup(self, mode, from_nodes, roads, preds=False):
        """Keys (n, 2) from each node to the two endpoints of each road through the engine's
        device tables of `mode` (all-ones outside the ball / without a table); with preds, also
        the rows' canonical predecessor indices (n, 2) (7: none stored)."""
        f = _c(from_nodes, np.uint32)
        r = _c(roads, np.uint32)
        keys = np.empty((len(f), 2), np.uint64)
        pr = np.empty((len(f), 2), np.uint8)
        _lib.check(_lib.lib().rm_engine_ball_lookup(self._h, int(mode), len(f), f.ctypes.data, r.ctypes.data,
                                                    keys.ctypes.data, pr.ctypes.data if preds else None))
        return (keys, pr) if preds else keys

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().rm_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


def _c(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


class BatchMatcher:
    """One HIP stream + device workspace; runs whole batches of traces."""

    def __init__(self, engine):
        self.engine = engine
        self._h = _lib.lib().rm_runner_create(engine._h)
        if not self._h:
            raise _lib.RmError(_lib.last_error())
        self._keep = None

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().rm_runner_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    @staticmethod
    def run_params(threshold_sec=15.0, report_levels=(0, 1), transition_levels=(0, 1), hist_dev=None,
                   do_report=True, zero_hist=False, dur_dev=None):
        rp = _lib.RmRunParams()
        rp.threshold_sec = threshold_sec
        rp.report_mask = levels_mask(report_levels)
        rp.transition_mask = levels_mask(transition_levels)
        rp.hist_dev = hist_dev or None
        rp.do_report = 1 if do_report else 0
        rp.zero_hist = 1 if zero_hist else 0
        rp.dur_dev = dur_dev or None
        return rp

    def run(self, trace_off, lon, lat, time, accuracy=None, opts=None, trace_opt=None, **rp_kw):
        """Upload a batch and run every stage (blocks until done)."""
        trace_off = _c(trace_off, np.uint32)
        T = len(trace_off) - 1
        P = int(trace_off[-1])
        lon = _c(lon, np.float32)
        lat = _c(lat, np.float32)
        time = _c(time, np.float64)
        accuracy = _c(np.full(P, -1.0, np.float32) if accuracy is None else accuracy, np.float32)
        opts = default_options(1) if opts is None else _c(opts, OPTIONS_DTYPE)
        trace_opt = np.zeros(T, np.uint32) if trace_opt is None else _c(trace_opt, np.uint32)
        if not (len(lon) == len(lat) == len(time) == len(accuracy) == P):
            raise ValueError("point arrays must all have trace_off[-1] elements")
        if len(trace_opt) != T:
            raise ValueError("trace_opt must have one entry per trace")
        d = _lib.RmBatchDesc(T, trace_off.ctypes.data, lon.ctypes.data, lat.ctypes.data, time.ctypes.data,
                             accuracy.ctypes.data, len(opts), opts.ctypes.data, trace_opt.ctypes.data)
        self._keep = (trace_off, lon, lat, time, accuracy, opts, trace_opt)
        rp = self.run_params(**rp_kw)
        _lib.check(_lib.lib().rm_runner_run(self._h, C.byref(d), C.byref(rp)))
        return self

    def run_points(self, uuid, time, lon, lat, accuracy=None, inactivity=120.0, opts=None, uuid_opt=None, n_uuids=None,
                   **rp_kw):
        """Raw per-vehicle points (any order) -> device time sort + inactivity windows of
        >= 2 points (reference py/simple_reporter.py:137-164) -> every matching stage.
        `uuid` is a dense vehicle index per point.  Blocks until done."""
        uuid = _c(uuid, np.uint32)
        n = len(uuid)
        time = _c(time, np.float64)
        lon = _c(lon, np.float32)
        lat = _c(lat, np.float32)
        accuracy = None if accuracy is None else _c(accuracy, np.float32)
        if not (len(time) == len(lon) == len(lat) == n) or (accuracy is not None and len(accuracy) != n):
            raise ValueError("point arrays must have equal lengths")
        nu = int(n_uuids if n_uuids is not None else (int(uuid.max()) + 1 if n else 0))
        opts = default_options(1) if opts is None else _c(opts, OPTIONS_DTYPE)
        uuid_opt = None if uuid_opt is None else _c(uuid_opt, np.uint32)
        if uuid_opt is not None and len(uuid_opt) != nu:
            raise ValueError("uuid_opt must have one entry per vehicle")
        d = _lib.RmPointsDesc(n, uuid.ctypes.data, time.ctypes.data, lon.ctypes.data, lat.ctypes.data,
                              accuracy.ctypes.data if accuracy is not None else None, float(inactivity), nu, len(opts),
                              opts.ctypes.data, uuid_opt.ctypes.data if uuid_opt is not None else None)
        self._keep = (uuid, time, lon, lat, accuracy, opts, uuid_opt)
        rp = self.run_params(**rp_kw)
        _lib.check(_lib.lib().rm_runner_run_points(self._h, C.byref(d), C.byref(rp)))
        return self

    def trace_uuid(self):
        """Vehicle index of every matched window of the last run_points."""
        out = np.empty(self.sizes()["traces"], np.uint32)
        _lib.check(_lib.lib().rm_runner_get_trace_uuid(self._h, out.ctypes.data))
        return out

    def batch(self):
        """The batch the last run matched (after run_points: the device-built windows)."""
        sz = self.sizes()
        P, T = sz["points"], sz["traces"]
        off = np.empty(T + 1, np.uint32)
        lon, lat, acc = (np.empty(P, np.float32) for _ in range(3))
        time = np.empty(P, np.float64)
        _lib.check(_lib.lib().rm_runner_get_batch(self._h, off.ctypes.data, lon.ctypes.data, lat.ctypes.data,
                                                  time.ctypes.data, acc.ctypes.data))
        return dict(trace_off=off, lon=lon, lat=lat, time=time, accuracy=acc)

    def tiles(self, quantisation=3600, privacy=2, source="smpl_rprt", mode="auto", comm=None):
        """Time tiles of the last run's reports: {"<start>_<end>/<level>/<index>": CSV text}
        exactly as the reference's report phase uploads them (py/simple_reporter.py:176-254).
        With a dist.Comm, rows of every rank are all-gathered and this rank's files returned."""
        tp = _lib.RmTileParams(int(quantisation), int(privacy), source.encode(), mode.encode())
        blob = C.c_void_p()
        n = C.c_size_t()
        _lib.check(_lib.lib().rm_runner_tiles(self._h, C.byref(tp), comm._h if comm is not None else None,
                                              C.byref(blob), C.byref(n)))
        try:
            raw = C.string_at(blob.value, n.value) if n.value else b""
        finally:
            _lib.lib().rm_free(blob)
        parts = raw.split(b"\0")
        return {parts[i].decode(): parts[i + 1].decode() for i in range(0, len(parts) - 1, 2)}

    def rerun(self, **rp_kw):
        """Run every stage again over the batch already in HBM."""
        rp = self.run_params(**rp_kw)
        _lib.check(_lib.lib().rm_runner_rerun(self._h, C.byref(rp)))

    def sizes(self):
        out = (C.c_uint64 * 10)()
        _lib.check(_lib.lib().rm_runner_sizes(self._h, out))
        return dict(zip(("points", "traces", "transitions", "path_edges", "segments", "reports", "routes_tier2",
                         "routes_tier3", "paths_tier2", "cand_tier2"), [int(x) for x in out]))

    def route_tiers(self):
        """Hand-overs of the last run: K2 ball tier -> search, register tier -> tier 2, tier 2 -> the
        LDS tiers (16-lane groups, then 512- and 4096-slot waves), wave -> global; the same for the
        path stage."""
        out = (C.c_uint64 * 10)()
        _lib.check(_lib.lib().rm_runner_route_tiers(self._h, out))
        return dict(zip(("ball_to_search", "lane_to_tier2", "tier2_to_wave", "paths_ball_to_search",
                         "wave_to_global", "paths_wave_to_global", "group_to_wave512", "paths_group_to_wave512",
                         "wave512_to_wave4096", "paths_wave512_to_wave4096"), [int(x) for x in out]))

    # ---- stage outputs (parity tests) ----
    def states(self):
        s = self.sizes()
        n_states = np.empty(s["traces"], np.uint32)
        orig = np.empty(s["points"], np.uint32)
        _lib.check(_lib.lib().rm_runner_get_states(self._h, n_states.ctypes.data, orig.ctypes.data))
        return n_states, orig

    def candidates(self):
        P = self.sizes()["points"]
        n = np.empty(P, np.uint8)
        road = np.empty(P * MAX_CAND, np.uint32)
        s = np.empty(P * MAX_CAND, np.uint32)
        sq = np.empty(P * MAX_CAND, np.float32)
        _lib.check(_lib.lib().rm_runner_get_candidates(self._h, n.ctypes.data, road.ctypes.data, s.ctypes.data,
                                                       sq.ctypes.data))
        return n, road.reshape(P, MAX_CAND), s.reshape(P, MAX_CAND), sq.reshape(P, MAX_CAND)

    def routes(self):
        sz = self.sizes()
        off = np.empty(sz["points"], np.uint32)
        gc = np.empty(sz["points"], np.float64)
        route = np.empty(max(sz["transitions"], 1), np.uint32)
        _lib.check(_lib.lib().rm_runner_get_routes(self._h, off.ctypes.data, gc.ctypes.data, route.ctypes.data))
        return off, gc, route[: sz["transitions"]]

    def route_terms(self):
        """With turn costs (DESIGN.md §3 rule 3b): every transition's distance term turn_m +
        |route_m - gc| (metres, inf when invalid) as the Viterbi adds it; None when the last run
        had no turn costs."""
        n = self.sizes()["transitions"]
        out = np.empty(max(n, 1), np.float64)
        present = C.c_int(0)
        _lib.check(_lib.lib().rm_runner_get_route_terms(self._h, out.ctypes.data, C.byref(present)))
        return out[:n] if present.value else None

    def viterbi(self):
        P = self.sizes()["points"]
        choice = np.empty(P, np.int8)
        cs = np.empty(P, np.uint8)
        _lib.check(_lib.lib().rm_runner_get_viterbi(self._h, choice.ctypes.data, cs.ctypes.data))
        return choice, cs

    def paths(self):
        sz = self.sizes()
        off = np.empty(sz["points"], np.uint32)
        cnt = np.empty(sz["points"], np.uint32)
        pool = np.empty(max(sz["path_edges"], 1), np.uint32)
        dist = np.empty(sz["points"], np.uint32)
        _lib.check(_lib.lib().rm_runner_get_paths(self._h, off.ctypes.data, cnt.ctypes.data, pool.ctypes.data,
                                                  dist.ctypes.data))
        return off, cnt, pool, dist

    def segments(self):
        sz = self.sizes()
        off = np.empty(sz["traces"] + 1, np.uint32)
        segs = np.empty(max(sz["segments"], 1), SEGMENT_DTYPE)
        _lib.check(_lib.lib().rm_runner_get_segments(self._h, off.ctypes.data, segs.ctypes.data))
        return off, segs[: sz["segments"]]

    def reports(self):
        sz = self.sizes()
        off = np.empty(sz["traces"] + 1, np.uint32)
        reps = np.empty(max(sz["reports"], 1), REPORT_DTYPE)
        stats = np.empty(sz["traces"], STATS_DTYPE)
        _lib.check(_lib.lib().rm_runner_get_reports(self._h, off.ctypes.data, reps.ctypes.data, stats.ctypes.data))
        return off, reps[: sz["reports"]], stats

    def set_isolation(self, on=True):
        """Per-trace failure isolation (rm_runner_set_isolation): a failing trace gets no output
        instead of failing the run; see trace_errors()."""
        _lib.check(_lib.lib().rm_runner_set_isolation(self._h, 1 if on else 0))

    def set_locality(self, mode):
        """Locality order of K1 / K2 / paths (rm_runner_set_locality): -1 engine default, 0 slot
        order, 1 sorted by region.  Results are identical either way."""
        _lib.check(_lib.lib().rm_runner_set_locality(self._h, int(mode)))

    def locality_used(self):
        v = C.c_int(0)
        _lib.check(_lib.lib().rm_runner_locality_used(self._h, C.byref(v)))
        return bool(v.value)

    def trace_errors(self):
        """Error bits per trace of the last run (1 candidates, 2 route search, 8 path rebuild)."""
        out = np.zeros(self.sizes()["traces"], np.uint32)
        _lib.check(_lib.lib().rm_runner_trace_errors(self._h, out.ctypes.data))
        return out

    # ---- timing ----
    def set_timing(self, on=True):
        _lib.check(_lib.lib().rm_runner_set_timing(self._h, 1 if on else 0))

    def set_timing_stages(self, names):
        """Time only the named stages (rm_kernel_name), e.g. ("routes",)."""
        n = _lib.lib().rm_num_kernels()
        idx = {_lib.lib().rm_kernel_name(i).decode(): i for i in range(n)}
        mask = 0
        for nm in names:
            mask |= 1 << idx[nm]
        _lib.check(_lib.lib().rm_runner_set_timing_mask(self._h, mask))

    def reset_times(self):
        _lib.check(_lib.lib().rm_runner_reset_times(self._h))

    def kernel_times(self):
        n = _lib.lib().rm_num_kernels()
        ms = np.zeros(n, np.float64)
        la = np.zeros(n, np.uint64)
        _lib.check(_lib.lib().rm_runner_kernel_times(self._h, ms.ctypes.data, la.ctypes.data, n))
        names = [_lib.lib().rm_kernel_name(i).decode() for i in range(n)]
        return {names[i]: (float(ms[i]), int(la[i])) for i in range(n)}


def split_by_points(trace_off, parts):
    """Trace index cuts [0, ..., T] of `parts` contiguous ranges with about equal point counts
    (a cut where the running point count crosses k * P / parts); empty ranges are dropped."""
    trace_off = np.asarray(trace_off, np.uint64)
    T = len(trace_off) - 1
    P = int(trace_off[-1]) if T >= 0 else 0
    cuts = [0] + [int(np.searchsorted(trace_off, P * k / parts)) for k in range(1, max(1, int(parts)))] + [T]
    return sorted(set(min(max(c, 0), T) for c in cuts))


class MultiMatcher:
    """One batch as `parts` contiguous trace ranges (balanced by points), each on its own
    BatchMatcher (HIP stream + workspace).  rerun() runs every part at once
    (rm_runners_rerun: one host thread per part), so one part's gather-latency-bound stages
    (K2 route probes, the path walk) overlap another part's issue-bound ones (K1, K3).  Every
    point of the batch is matched once per rerun; a shared histogram is zeroed once."""

    def __init__(self, engine, parts=2):
        self.engine = engine
        self.parts = max(1, int(parts))
        self.bms = []

    def run(self, trace_off, lon, lat, time, accuracy=None, opts=None, trace_opt=None, **rp_kw):
        trace_off = np.asarray(trace_off, np.uint64)
        T = len(trace_off) - 1
        P = int(trace_off[-1])
        accuracy = np.full(P, -1.0, np.float32) if accuracy is None else np.asarray(accuracy, np.float32)
        trace_opt = np.zeros(T, np.uint32) if trace_opt is None else np.asarray(trace_opt, np.uint32)
        cuts = split_by_points(trace_off, self.parts)
        for bm in self.bms:
            bm.close()
        self.bms = []
        zero = rp_kw.pop("zero_hist", False)
        if zero and rp_kw.get("hist_dev"):
            _lib.check(_lib.lib().rm_device_memset(rp_kw["hist_dev"], 0, self.engine.n_segments * 16 * 4))
        if zero and rp_kw.get("dur_dev"):
            _lib.check(_lib.lib().rm_device_memset(rp_kw["dur_dev"], 0, self.engine.n_segments * 8))
        for t0, t1 in zip(cuts[:-1], cuts[1:]):
            if t1 <= t0:
                continue
            o0, o1 = int(trace_off[t0]), int(trace_off[t1])
            bm = BatchMatcher(self.engine)
            bm.run(trace_off[t0:t1 + 1] - o0, lon[o0:o1], lat[o0:o1], time[o0:o1], accuracy[o0:o1], opts,
                   trace_opt[t0:t1], **rp_kw)
            self.bms.append(bm)
        return self

    def rerun(self, **rp_kw):
        rp = BatchMatcher.run_params(**rp_kw)
        hs = (C.c_void_p * len(self.bms))(*[bm._h for bm in self.bms])
        _lib.check(_lib.lib().rm_runners_rerun(hs, len(self.bms), C.byref(rp)))

    def set_timing(self, on=True):
        for bm in self.bms:
            bm.set_timing(on)

    def set_timing_stages(self, names):
        for bm in self.bms:
            bm.set_timing_stages(names)

    def reset_times(self):
        for bm in self.bms:
            bm.reset_times()

    def kernel_times(self):
        """Per stage: (ms summed over the parts' launches, launches) — each launch timed by HIP
        events on its own stream while the other parts run."""
        out = {}
        for bm in self.bms:
            for k, (ms, n) in bm.kernel_times().items():
                a, b = out.get(k, (0.0, 0))
                out[k] = (a + ms, b + n)
        return out

    def sizes(self):
        out = {}
        for bm in self.bms:
            for k, v in bm.sizes().items():
                out[k] = out.get(k, 0) + v
        return out

    def set_locality(self, mode):
        for bm in self.bms:
            bm.set_locality(mode)

    def locality_used(self):
        return any(bm.locality_used() for bm in self.bms)

    def route_tiers(self):
        out = {}
        for bm in self.bms:
            for k, v in bm.route_tiers().items():
                out[k] = out.get(k, 0) + v
        return out

    def close(self):
        for bm in self.bms:
            bm.close()
        self.bms = []


def report_segments(seg_off, segs, trace_end_time, threshold_sec, report_mask, transition_mask):
    """The device report() epilogue (rm_report_segments) over host segment lists.
    seg_off: n+1 offsets into segs (SEGMENT_DTYPE); per-trace end time, threshold and level
    masks (scalars broadcast).  Returns (rep_off, reports REPORT_DTYPE, stats STATS_DTYPE)."""
    seg_off = _c(seg_off, np.uint32)
    n = len(seg_off) - 1
    segs = np.ascontiguousarray(segs, SEGMENT_DTYPE)
    bc = lambda x, dt: _c(np.broadcast_to(np.asarray(x, dt), (n,)), dt)
    end, thr = bc(trace_end_time, np.float64), bc(threshold_sec, np.float64)
    rm, tm = bc(report_mask, np.uint32), bc(transition_mask, np.uint32)
    d = _lib.RmReportDesc(n, seg_off.ctypes.data, segs.ctypes.data if len(segs) else None, end.ctypes.data,
                          thr.ctypes.data, rm.ctypes.data, tm.ctypes.data)
    rep_off = np.zeros(n + 1, np.uint32)
    reps = np.empty(max(int(seg_off[-1]) if n else 0, 1), REPORT_DTYPE)
    stats = np.empty(max(n, 1), STATS_DTYPE)
    _lib.check(_lib.lib().rm_report_segments(C.byref(d), rep_off.ctypes.data, reps.ctypes.data, stats.ctypes.data))
    return rep_off, reps[: rep_off[-1]], stats[:n]


def segment_dicts(segs):
    """Match-reply segments (README.md:288-301 schema) from SEGMENT_DTYPE records."""
    out = []
    for r in segs:
        d = {}
        if int(r["flags"]) & 2:
            d["segment_id"] = int(r["segment_id"])
        ways = [int(r["way_first"])]
        if int(r["way_last"]) != int(r["way_first"]):
            ways.append(int(r["way_last"]))
        d["way_ids"] = ways
        d["start_time"] = float(r["start_time"]) if r["start_time"] != -1 else -1
        d["end_time"] = float(r["end_time"]) if r["end_time"] != -1 else -1
        d["queue_length"] = int(r["queue_length"])
        d["length"] = int(r["length"])
        d["internal"] = bool(int(r["flags"]) & 1)
        d["begin_shape_index"] = int(r["begin_shape_index"])
        d["end_shape_index"] = int(r["end_shape_index"])
        out.append(d)
    return out
