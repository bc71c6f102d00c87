"""Synthetic world + trace generation (host side; no GPU required).

Configurations follow BASELINE.json ``configs`` / SURVEY.md §8d:

  C1  1 trace x 1,000 pts @1 Hz, 40x40 grid @100 m
  C2  10,000 traces x 600 pts @1 Hz, 200x200 grid @100 m   (the bench workload)
  C3  1,000,000 traces x 40 pts @30 s, 500x500 grid @200 m, radius 100 m
  C4  4,000x4,000 grid @250 m, 1,000,000 traces x 120 pts @5 s
  C5  C2 graph, auto/bicycle/pedestrian, sigma_z in {2, 4.07, 8, 16}

The trace generator restates reference py/generate_test_trace.py:35-104 and
:120-149 (see reporter_amd/csrc/world.cpp).
"""
import ctypes as C
import os

import numpy as np

from . import _lib

CONFIGS = {
    "C1": dict(rows=40, cols=40, block_m=100.0, n_traces=1, n_points=1000, rate_s=1.0, noise_m=5.0,
               search_radius=50.0, cell_m=100.0, ball_radius_m=None),
    "C2": dict(rows=200, cols=200, block_m=100.0, n_traces=10000, n_points=600, rate_s=1.0, noise_m=5.0,
               search_radius=50.0, cell_m=100.0, ball_radius_m=None),
    "C3": dict(rows=500, cols=500, block_m=200.0, n_traces=1000000, n_points=40, rate_s=30.0, noise_m=5.0,
               search_radius=100.0, cell_m=200.0, ball_radius_m=None),
    "C4": dict(rows=4000, cols=4000, block_m=250.0, n_traces=1000000, n_points=120, rate_s=5.0, noise_m=5.0,
               search_radius=50.0, cell_m=250.0, ball_radius_m=None),
    "C5": dict(rows=200, cols=200, block_m=100.0, n_traces=10000, n_points=600, rate_s=1.0, noise_m=5.0,
               search_radius=50.0, cell_m=100.0, ball_radius_m=None),
    # SURVEY §8(f)3 / VERDICT r03: C2's and C3's workloads on an irregular city written as generic
    # OSM PBF and ingested by rm_graph_import_osm (osm_city.cpp: 170x170 junctions @120 m, ~38 k
    # nodes, about the C2 graph's size)
    "CITY": dict(rows=170, cols=170, block_m=120.0, n_traces=10000, n_points=600, rate_s=1.0, noise_m=5.0,
                 search_radius=50.0, cell_m=100.0, ball_radius_m=None, city=True),
    "CITY30": dict(rows=170, cols=170, block_m=120.0, n_traces=100000, n_points=40, rate_s=30.0, noise_m=5.0,
                   search_radius=100.0, cell_m=100.0, ball_radius_m=None, city=True),
}


def build_config_graph(name, path, seed=1):
    """The graph of a CONFIGS entry at ``path``: the synthetic grid world, or (city configs) the
    OSM city ingested from PBF."""
    cfg = CONFIGS[name]
    if cfg.get("city"):
        return build_city(path, cell_m=cfg["cell_m"], rows=cfg["rows"], cols=cfg["cols"], block_m=cfg["block_m"],
                          seed=seed)
    return build_world(path, cfg["rows"], cfg["cols"], cfg["block_m"], seed=seed, cell_m=cfg["cell_m"])

MODES = {"auto": 0, "bus": 1, "motor_scooter": 2, "bicycle": 3, "pedestrian": 4}


def world_params(rows, cols, block_m=100.0, seed=1, cell_m=None, **kw):
    p = _lib.RmWorldParams()
    _lib.lib().rm_default_world_params(C.byref(p))
    p.rows, p.cols, p.block_m, p.seed = rows, cols, block_m, seed
    p.cell_m = cell_m if cell_m is not None else block_m
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def build_world(path, rows, cols, block_m=100.0, seed=1, cell_m=None, **kw):
    """Write a synthetic .rmg graph to ``path`` and return the path."""
    p = world_params(rows, cols, block_m, seed, cell_m, **kw)
    _lib.check(_lib.lib().rm_world_build(C.byref(p), os.fsencode(path)))
    return path


def export_osm(graph_path, osm_path):
    """The .rmg graph as OSM XML (routing tags + exact reporter:* tags + osmlr relations)."""
    _lib.check(_lib.lib().rm_graph_export_osm(os.fsencode(graph_path), os.fsencode(osm_path)))
    return osm_path


def export_pbf(graph_path, pbf_path):
    """The .rmg graph as OSM PBF (the same elements as export_osm; the tile builder's input)."""
    _lib.check(_lib.lib().rm_graph_export_pbf(os.fsencode(graph_path), os.fsencode(pbf_path)))
    return pbf_path


def import_osm(osm_path, graph_path, cell_m=100.0):
    """OSM XML or PBF -> .rmg (bit-identical for an export_osm / export_pbf file; generic OSM split
    at intersections)."""
    _lib.check(_lib.lib().rm_graph_import_osm(os.fsencode(osm_path), os.fsencode(graph_path), float(cell_m)))
    return graph_path


def write_city_osm(path, pbf=True, **kw):
    """A seeded irregular city as generic OSM PBF (or XML) at ``path`` (osm_city.cpp): curved
    multi-vertex ways, 9-road hubs, roundabouts, one-way carriageway pairs, dead ends, service
    loops, paths, a bridged trunk road, OSMLR relations on part of the ways.  Keyword arguments
    are rm_city_params fields (rows, cols, block_m, seed, ...)."""
    p = _lib.RmCityParams()
    _lib.lib().rm_default_city_params(C.byref(p))
    for k, v in kw.items():
        if not hasattr(p, k):
            raise TypeError("unknown city parameter " + k)
        setattr(p, k, v)
    _lib.check(_lib.lib().rm_osm_city_write(C.byref(p), os.fsencode(path), 1 if pbf else 0))
    return path


def build_city(graph_path, cell_m=100.0, pbf_path=None, **kw):
    """The city written as OSM PBF, then ingested by rm_graph_import_osm into ``graph_path``
    (the generic import path: nothing in the file is specific to this engine)."""
    pbf_path = pbf_path or graph_path + ".osm.pbf"
    write_city_osm(pbf_path, pbf=True, **kw)
    return import_osm(pbf_path, graph_path, cell_m=cell_m)


def graph_info(path):
    out = (C.c_uint64 * 7)()
    _lib.check(_lib.lib().rm_graph_info(os.fsencode(path), out))
    keys = ("nodes", "edges", "roads", "verts", "segments", "cells", "cell_items")
    return dict(zip(keys, [int(x) for x in out]))


def generate_traces(graph_path, n_traces, n_points, rate_s=1.0, noise_m=5.0, seed=1, mode="auto",
                    start_epoch=1483228800, threads=0, ids=None):
    """Seeded GPS traces on the graph.  Returns a dict of numpy arrays:
    lon/lat (6-dp degrees, f64), time (epoch s, f64), accuracy (f32),
    trace_off (u32, n_traces+1), truth_edge / truth_off_cm (u32).
    With ``ids``, trace k is trace ids[k] of the seeded set (n_traces = len(ids))."""
    if ids is not None:
        ids = np.ascontiguousarray(ids, np.uint32)
        n_traces = len(ids)
    p = _lib.RmTraceParams()
    _lib.lib().rm_default_trace_params(C.byref(p))
    p.n_traces, p.n_points, p.rate_s, p.noise_m = n_traces, n_points, rate_s, noise_m
    p.seed, p.mode, p.start_epoch, p.threads = seed, MODES[mode] if isinstance(mode, str) else int(mode), start_epoch, threads
    n = n_traces * n_points
    out = {k: np.empty(n, np.float64) for k in ("lon", "lat", "time")}
    out["accuracy"] = np.empty(n, np.float32)
    out["truth_edge"] = np.empty(n, np.uint32)
    out["truth_off_cm"] = np.empty(n, np.uint32)
    _lib.check(_lib.lib().rm_traces_generate_ids(
        os.fsencode(graph_path), C.byref(p), ids.ctypes.data if ids is not None else None,
        out["lon"].ctypes.data, out["lat"].ctypes.data,
        out["time"].ctypes.data, out["accuracy"].ctypes.data, out["truth_edge"].ctypes.data,
        out["truth_off_cm"].ctypes.data))
    out["trace_off"] = (np.arange(n_traces + 1, dtype=np.uint64) * n_points).astype(np.uint32)
    return out


def trace_to_request(tr, k, uuid=None, mode="auto", report_levels=(0, 1), transition_levels=(0, 1), **opts):
    """The /report JSON request for trace k (reporter_service.py:184-235 contract)."""
    o0, o1 = int(tr["trace_off"][k]), int(tr["trace_off"][k + 1])
    pts = [{"lat": float(tr["lat"][i]), "lon": float(tr["lon"][i]), "time": int(tr["time"][i]),
            "accuracy": float(tr["accuracy"][i])} for i in range(o0, o1)]
    mo = {"mode": mode, "report_levels": list(report_levels), "transition_levels": list(transition_levels)}
    mo.update(opts)
    return {"uuid": uuid or str(k), "trace": pts, "match_options": mo}


def concat_traces(*sets):
    """One trace set of several (each a generate_traces dict), in order."""
    out = {k: np.concatenate([s[k] for s in sets]) for k in ("lon", "lat", "time", "accuracy", "truth_edge", "truth_off_cm")}
    off, base = [np.zeros(1, np.uint64)], 0
    for s in sets:
        off.append(s["trace_off"][1:].astype(np.uint64) + base)
        base += int(s["trace_off"][-1])
    out["trace_off"] = np.concatenate(off).astype(np.uint32)
    return out


# Valhalla's tile hierarchy (reference py/get_tiles.py:30-39: world bbox, tile sizes 4 / 1 /
# 0.25 degrees for levels 0 / 1 / 2) and its tile file naming (GetFile, :79-102)
_TILE_SIZE = {0: 4.0, 1: 1.0, 2: 0.25}


def valhalla_tile_file(level, tile_id, suffix="gph"):
    """Path of a Valhalla tile file, as get_tiles.py:79-102 GetFile forms it: the id (with the
    level in front) zero-padded to a multiple of three digits, split into 3-digit directories."""
    size = _TILE_SIZE[level]
    ncols, nrows = int(np.ceil(360.0 / size)), int(np.ceil(180.0 / size))
    max_id = ncols * nrows - 1
    digits = len(str(max_id))
    if digits % 3:
        digits += 3 - digits % 3
    s = "{:,}".format(level * 10 ** digits + tile_id if level else 10 ** digits + tile_id).replace(",", "/")
    if level == 0:
        s = "0" + s[1:]
    return s + "." + suffix


def valhalla_tiles(graph_path):
    """{(level, tile id): tile file} of every tile the graph's OSMLR segment ids name
    (id layout level:3 | tile:22 | index:21, reference py/simple_reporter.py:37-49) — the tiles a
    Valhalla build of the exported OSM would have to produce for the two paths to agree."""
    from . import graphfile
    ids = graphfile.load(graph_path)["seg_id"].astype(np.uint64)
    out = {}
    for lv, tl in set(zip((ids & np.uint64(7)).tolist(), ((ids >> np.uint64(3)) & np.uint64(0x3FFFFF)).tolist())):
        out[(int(lv), int(tl))] = valhalla_tile_file(int(lv), int(tl))
    return out
