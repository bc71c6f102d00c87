"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py
cpu_baseline).  ctypes bridge to liboracle_meili.so (oracle/meili_oracle.c).

Parity status (see meili_oracle.h): real meili UNPINNED (not available
offline); report() PINNED by tests/golden/report_golden.json.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle_meili.so")
K = 16


class OgGraph(C.Structure):
    _fields_ = [("n_nodes", C.c_uint32), ("n_edges", C.c_uint32), ("n_roads", C.c_uint32), ("n_verts", C.c_uint32),
                ("n_segments", C.c_uint32)] + [(n, C.c_void_p) for n in (
                    "node_off", "edges", "edge_seg", "edge_seg_off", "edge_way", "road_node0", "road_node1",
                    "road_fwd", "road_rev", "road_len_cm", "road_vert_off", "verts", "seg_id", "seg_len_cm")] + [
                ("lon0", C.c_double), ("lat0", C.c_double), ("dlon", C.c_double), ("dlat", C.c_double),
                ("ncx", C.c_uint32), ("ncy", C.c_uint32), ("cell_off", C.c_void_p), ("cell_item", C.c_void_p)]


class OgBatch(C.Structure):
    _fields_ = [("n_traces", C.c_uint32)] + [(n, C.c_void_p) for n in (
        "trace_off", "lon", "lat", "time", "accuracy", "opts", "trace_opt")]


class OgStats(C.Structure):
    _fields_ = [(n, C.c_int32) for n in ("successful_count", "unreported_count", "successful_length_m",
                                         "unreported_length_m", "discontinuities", "invalid_speeds",
                                         "invalid_times", "unassociated", "shape_used", "n_reports")]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", HERE], check=True, capture_output=True)
        h = C.CDLL(LIB)
        h.og_match.restype = C.c_void_p
        h.og_match.argtypes = [C.POINTER(OgGraph), C.POINTER(OgBatch)]
        h.og_free.argtypes = [C.c_void_p]
        h.og_sizes.argtypes = [C.c_void_p] + [C.POINTER(C.c_uint64)] * 4
        for n, k in (("og_get_states", 2), ("og_get_candidates", 4), ("og_get_routes", 3), ("og_get_viterbi", 2),
                     ("og_get_paths", 4), ("og_get_segments", 2), ("og_get_route_turns", 1),
                     ("og_get_route_terms", 1)):
            getattr(h, n).argtypes = [C.c_void_p] + [C.c_void_p] * k
        h.og_report_trace.restype = C.c_int
        h.og_report_trace.argtypes = [C.c_void_p, C.c_uint32, C.c_double, C.c_double, C.c_uint32, C.c_uint32,
                                      C.c_void_p, C.POINTER(OgStats)]
        h.og_pipeline.restype = C.c_uint64
        h.og_pipeline.argtypes = [C.POINTER(OgGraph), C.POINTER(OgBatch), C.c_double, C.c_uint32, C.c_uint32,
                                  C.c_void_p]
        h.og_pipeline2.restype = C.c_uint64
        h.og_pipeline2.argtypes = [C.POINTER(OgGraph), C.POINTER(OgBatch), C.c_double, C.c_uint32, C.c_uint32,
                                   C.c_void_p, C.c_void_p]
        h.og_prepare_path_counters.argtypes = [C.POINTER(OgGraph)]
        h.og_road_heads.argtypes = [C.POINTER(OgGraph), C.c_void_p, C.c_void_p]
        h.og_reset_counters.argtypes = []
        h.og_get_counters.argtypes = [C.c_void_p]
        _lib = h
    return _lib


COUNTER_NAMES = ("searches", "settled", "scanned", "label_writes", "target_lookups", "route_writes",
                 "cand_items", "states", "ball_rows", "desc_reads", "cands", "grid_rows", "chained", "path_edges",
                 "segments", "path_in_edges", "path_rows", "settled_to_targets", "scanned_to_targets",
                 "label_writes_to_targets", "turn_rows", "turn_nodes")


def road_heads(graph):
    """(H0, H1) per road: the headings at node0 / node1 into the road (DESIGN.md §3 rule 3b)."""
    og = make_graph(graph)
    n = og.n_roads
    h0, h1 = np.empty(n, np.uint16), np.empty(n, np.uint16)
    lib().og_road_heads(C.byref(og), h0.ctypes.data, h1.ctypes.data)
    return h0, h1


def prepare_path_counters(graph):
    """Build the in-edge index the path-walk counters need (call outside timed regions; the
    graph's arrays must stay alive while matching on it)."""
    lib().og_prepare_path_counters(C.byref(make_graph(graph)))


def reset_counters():
    lib().og_reset_counters()


def counters():
    out = np.zeros(len(COUNTER_NAMES), np.uint64)
    lib().og_get_counters(out.ctypes.data)
    return dict(zip(COUNTER_NAMES, (int(x) for x in out)))


def routes_algorithmic_bytes(c):
    """K2 algorithmic bytes: 8 B CSR offsets per settled node, 16 B edge record per
    scanned edge, 12 B per label write, 8 B per target label lookup, 4 B per route write,
    24 B per search (source candidate + its road record)."""
    return (8 * c["settled"] + 16 * c["scanned"] + 12 * c["label_writes"] + 8 * c["target_lookups"]
            + 4 * c["route_writes"] + 24 * c["searches"])


def routes_targets_algorithmic_bytes(c):
    """routes_algorithmic_bytes of the same searches stopped at their targets (the formulation the
    search tiers run since round 4, engine.hip SearchTargets): the settles, scans and label writes
    up to the largest target route key of each search (counters 17-19)."""
    return (8 * c["settled_to_targets"] + 16 * c["scanned_to_targets"] + 12 * c["label_writes_to_targets"]
            + 8 * c["target_lookups"] + 4 * c["route_writes"] + 24 * c["searches"])


def routes_ball_algorithmic_bytes(c):
    """K2 algorithmic bytes of the route-ball formulation: 16 B table row per
    (source exit, target) probe, per layer pair a 32 B descriptor per source (KA = the searches)
    and 24 B per target (KB: road, offset, length, speeds + the two entry times; round 6 reads no
    more of it), 16 B per source for its two exits' table headers, 4 B per route write."""
    targets = c["desc_reads"] - c["searches"]
    return 16 * c["ball_rows"] + 32 * c["searches"] + 24 * targets + 16 * c["searches"] + 4 * c["route_writes"]


def routes_ball_turn_algorithmic_bytes(c):
    """routes_ball_algorithmic_bytes with turn costs (DESIGN.md §3 rule 3b, k_routes_ball2<true>):
    + 8 B turn row per transition that enters its target road from a node, + 4 B heading word
    of each source road, + 8 B distance term written per transition (route_d, read by K3 instead
    of the 4 B route)."""
    return routes_ball_algorithmic_bytes(c) + 8 * c["turn_rows"] + 4 * c["searches"] + 8 * c["route_writes"]


def candidates_algorithmic_bytes(c):
    """K1 algorithmic bytes of the formulation k_candidates_lane runs: per state
    16 B (point lon/lat, slot, options index) + 1 B candidate count; 8 B item range per grid
    row visited; 32 B self-contained cell record per cell item tested (both shape vertices,
    road, access); per candidate kept 32 B road record read + 32 B descriptor + 4 B sq written."""
    return 17 * c["states"] + 8 * c["grid_rows"] + 32 * c["cand_items"] + 68 * c["cands"]


def viterbi_algorithmic_bytes(c):
    """K3 algorithmic bytes (in the layout k_viterbi reads): 4 B route per
    transition, 4 B emission (sq) per candidate, per layer 8 B gc + 12 B layer descriptor
    (cand count, route offset, state) + 16 B back-pointer row written and read back + 2 B
    choice / chain flag."""
    return 4 * c["route_writes"] + 4 * c["cands"] + (8 + 12 + 32 + 2) * c["states"]


def segments_algorithmic_bytes(c):
    """K4 algorithmic bytes (matched edges x 16 B + segments x 48 B, in this
    build's layout): per path edge 4 B edge id + 16 B edge record + 12 B OSMLR association
    (segment, offset, way); per chained transition 64 B (two candidate offsets, two state
    indices, two times, route length, path header); per segment 56 B written."""
    return 32 * c["path_edges"] + 64 * c["chained"] + 56 * c["segments"]


def paths_algorithmic_bytes(c):
    """Path stage (k_paths_ball) algorithmic bytes: per chained transition 64 B of the chosen
    candidates' descriptors + 16 B pair constants + 16 B of exit table headers + 20 B written
    (route length, both offsets, path count and offset); 16 B per route-ball row read (the
    target road's rows, then per walked node the rows of its predecessor's road); 20 B per
    in-edge record read (the 16 B record + the node's 4 B in-edge offset, or its access word on
    a scan); 4 B per path edge written.  Needs the counters of prepare_path_counters."""
    return 116 * c["chained"] + 16 * c["path_rows"] + 20 * c["path_in_edges"] + 4 * c["path_edges"]


def make_graph(g):
    """OgGraph from reporter_amd.graphfile.load() arrays (arrays must stay alive)."""
    og = OgGraph()
    og.n_nodes = len(g["node_lon"])
    og.n_edges = len(g["edges"]) // 4
    og.n_roads = len(g["road_len_cm"])
    og.n_verts = len(g["verts"]) // 4
    og.n_segments = len(g["seg_id"])
    for n in ("node_off", "edges", "edge_seg", "edge_seg_off", "edge_way", "road_node0", "road_node1", "road_fwd",
              "road_rev", "road_len_cm", "road_vert_off", "verts", "seg_id", "seg_len_cm", "cell_off", "cell_item"):
        setattr(og, n, g[n].ctypes.data)
    og.lon0, og.lat0, og.dlon, og.dlat = g.lon0, g.lat0, g.dlon, g.dlat
    og.ncx, og.ncy = g.ncx, g.ncy
    return og


class Batch:
    """Keeps the numpy inputs alive for the C side."""

    def __init__(self, trace_off, lon, lat, time, accuracy, opts, trace_opt):
        self.arrays = dict(
            trace_off=np.ascontiguousarray(trace_off, np.uint32), lon=np.ascontiguousarray(lon, np.float32),
            lat=np.ascontiguousarray(lat, np.float32), time=np.ascontiguousarray(time, np.float64),
            accuracy=np.ascontiguousarray(accuracy, np.float32), opts=np.ascontiguousarray(opts),
            trace_opt=np.ascontiguousarray(trace_opt, np.uint32))
        a = self.arrays
        self.c = OgBatch(len(a["trace_off"]) - 1, *(a[n].ctypes.data for n in (
            "trace_off", "lon", "lat", "time", "accuracy", "opts", "trace_opt")))


def match(graph, batch):
    """Run the oracle matcher; returns every stage output as numpy arrays."""
    h = lib()
    og = make_graph(graph)
    r = h.og_match(C.byref(og), C.byref(batch.c))
    if not r:
        raise MemoryError("oracle allocation failed")
    try:
        P, NT, NP, NS = (C.c_uint64() for _ in range(4))
        h.og_sizes(r, C.byref(P), C.byref(NT), C.byref(NP), C.byref(NS))
        P, NT, NP, NS = P.value, NT.value, NP.value, NS.value
        T = batch.c.n_traces
        out = {}
        out["n_states"] = np.empty(T, np.uint32)
        out["state_orig"] = np.empty(P, np.uint32)
        h.og_get_states(r, out["n_states"].ctypes.data, out["state_orig"].ctypes.data)
        out["cand_n"] = np.empty(P, np.uint8)
        out["cand_road"] = np.empty((P, K), np.uint32)
        out["cand_s"] = np.empty((P, K), np.uint32)
        out["cand_sq"] = np.empty((P, K), np.float32)
        h.og_get_candidates(r, out["cand_n"].ctypes.data, out["cand_road"].ctypes.data, out["cand_s"].ctypes.data,
                            out["cand_sq"].ctypes.data)
        out["trans_off"] = np.empty(P, np.uint32)
        out["gc"] = np.empty(P, np.float64)
        out["route"] = np.empty(max(NT, 1), np.uint32)
        h.og_get_routes(r, out["trans_off"].ctypes.data, out["gc"].ctypes.data, out["route"].ctypes.data)
        out["route"] = out["route"][:NT]
        out["route_turn"] = np.empty(max(NT, 1), np.uint32)
        h.og_get_route_turns(r, out["route_turn"].ctypes.data)
        out["route_turn"] = out["route_turn"][:NT]
        out["route_d"] = np.empty(max(NT, 1), np.float64)
        h.og_get_route_terms(r, out["route_d"].ctypes.data)
        out["route_d"] = out["route_d"][:NT]
        out["choice"] = np.empty(P, np.int8)
        out["chain_start"] = np.empty(P, np.uint8)
        h.og_get_viterbi(r, out["choice"].ctypes.data, out["chain_start"].ctypes.data)
        out["path_off"] = np.empty(P, np.uint32)
        out["path_cnt"] = np.empty(P, np.uint32)
        out["path_pool"] = np.empty(max(NP, 1), np.uint32)
        out["route_dist"] = np.empty(P, np.uint32)
        h.og_get_paths(r, out["path_off"].ctypes.data, out["path_cnt"].ctypes.data, out["path_pool"].ctypes.data,
                       out["route_dist"].ctypes.data)
        from reporter_amd.engine import SEGMENT_DTYPE  # record layout only (numpy dtype)
        out["seg_off"] = np.empty(T + 1, np.uint32)
        out["segs"] = np.empty(max(NS, 1), SEGMENT_DTYPE)
        h.og_get_segments(r, out["seg_off"].ctypes.data, out["segs"].ctypes.data)
        out["segs"] = out["segs"][:NS]
        return out
    finally:
        h.og_free(r)


def report_trace(segs, trace_end_time, threshold_sec, report_mask, transition_mask):
    """og_report_trace on SEGMENT_DTYPE records -> (reports array, stats dict)."""
    from reporter_amd.engine import REPORT_DTYPE
    segs = np.ascontiguousarray(segs)
    out = np.empty(max(len(segs), 1), REPORT_DTYPE)
    st = OgStats()
    n = lib().og_report_trace(segs.ctypes.data if len(segs) else None, len(segs), float(trace_end_time),
                              float(threshold_sec), report_mask, transition_mask, out.ctypes.data, C.byref(st))
    return out[:n], {f: getattr(st, f) for f, _ in OgStats._fields_}


def pipeline(graph, batch, threshold_sec=15.0, report_mask=0x6, transition_mask=0x6, hist=None, dur=None):
    """Whole CPU pipeline (match + report + histogram [+ per-segment u64 duration sums]);
    returns #valid reports."""
    og = make_graph(graph)
    hp = hist.ctypes.data if hist is not None else None
    dp = dur.ctypes.data if dur is not None else None
    return int(lib().og_pipeline2(C.byref(og), C.byref(batch.c), threshold_sec, report_mask, transition_mask, hp, dp))
