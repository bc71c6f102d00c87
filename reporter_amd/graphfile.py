"""numpy view of an ".rmg" graph file (layout: reporter_amd/csrc/graph.cpp).

Pure data reading — usable without the shared library or a GPU.
"""
import numpy as np

_SEC = np.dtype([("name", "S24"), ("offset", "<u8"), ("bytes", "<u8")])
_TYPES = {
    "node_lon": "<f4", "node_lat": "<f4", "node_off": "<u4", "edges": "<u4", "edge_seg": "<u4",
    "edge_seg_off": "<u4", "edge_way": "<u4", "road_node0": "<u4", "road_node1": "<u4", "road_fwd": "<u4",
    "road_rev": "<u4", "road_len_cm": "<u4", "road_vert_off": "<u4", "verts": "<u4", "seg_id": "<u8",
    "seg_len_cm": "<u4", "grid_meta": "<u1", "cell_off": "<u4", "cell_item": "<u4",
}


class GraphArrays(dict):
    """dict of numpy arrays plus grid metadata attributes."""

    @property
    def n_nodes(self):
        return len(self["node_lon"])

    @property
    def n_edges(self):
        return len(self["edges"]) // 4

    @property
    def n_segments(self):
        return len(self["seg_id"])


def load(path):
    with open(path, "rb") as f:
        raw = f.read()
    if raw[:8] != b"RMGRAPH1":
        raise ValueError("not an .rmg graph file: %s" % path)
    version, ns = np.frombuffer(raw, "<u4", 2, 8)
    if version != 1:
        raise ValueError("unsupported .rmg version %d" % version)
    hdr = np.frombuffer(raw, _SEC, int(ns), 16)
    g = GraphArrays()
    for h in hdr:
        name = h["name"].rstrip(b"\0").decode()
        dt = np.dtype(_TYPES.get(name, "<u1"))
        g[name] = np.frombuffer(raw, dt, int(h["bytes"]) // dt.itemsize, int(h["offset"])).copy()
    meta = g.pop("grid_meta")
    d = np.frombuffer(meta.tobytes(), "<f8", 4)
    u = np.frombuffer(meta.tobytes(), "<u4", 2, 32)
    g.lon0, g.lat0, g.dlon, g.dlat = (float(x) for x in d)
    g.ncx, g.ncy = int(u[0]), int(u[1])
    return g


def split_grid(g, f, rebuild=False):
    """Copy of ``g`` whose grid has every cell split f x f: the spatial index the engine's K1
    reads (Engine::Engine, choose_grid_split in engine.hip), built by the same bounding-box rule
    as build_grid_index (world.cpp).  Which roads a query finds does not depend on it.
    f = 1 returns ``g`` itself unless ``rebuild``.  engine_grid_split(path) gives the engine's f."""
    if f == 1 and not rebuild:
        return g
    out = GraphArrays(g)
    for k in ("lon0", "lat0"):
        setattr(out, k, getattr(g, k))
    out.dlon, out.dlat, out.ncx, out.ncy = g.dlon / f, g.dlat / f, g.ncx * f, g.ncy * f
    v = g["verts"].reshape(-1, 4)
    lon, lat = v[:, 0].view(np.float32).astype(np.float64), v[:, 1].view(np.float32).astype(np.float64)
    road = v[:, 3]
    piece = np.nonzero(road[:-1] != 0xFFFFFFFF)[0].astype(np.uint32)
    a, b = piece, piece + 1
    x0 = np.floor((np.minimum(lon[a], lon[b]) - out.lon0) / out.dlon).astype(np.int64)
    x1 = np.minimum(np.floor((np.maximum(lon[a], lon[b]) - out.lon0) / out.dlon).astype(np.int64), out.ncx - 1)
    y0 = np.floor((np.minimum(lat[a], lat[b]) - out.lat0) / out.dlat).astype(np.int64)
    y1 = np.minimum(np.floor((np.maximum(lat[a], lat[b]) - out.lat0) / out.dlat).astype(np.int64), out.ncy - 1)
    nx, ny = x1 - x0 + 1, y1 - y0 + 1
    n = nx * ny
    rep = np.repeat(np.arange(len(piece)), n)                 # one row per (piece, cell), piece order
    k = np.arange(len(rep)) - np.repeat(np.cumsum(n) - n, n)  # index of the cell within the piece's box
    cx = x0[rep] + k % nx[rep]
    cy = y0[rep] + k // nx[rep]
    cell = cy * out.ncx + cx
    order = np.argsort(cell, kind="stable")                   # pieces ascending within a cell
    out["cell_item"] = piece[rep[order]].astype(np.uint32)
    cnt = np.bincount(cell, minlength=out.ncx * out.ncy)
    out["cell_off"] = np.concatenate([[0], np.cumsum(cnt)]).astype(np.uint32)
    return out


def engine_grid_split(path):
    """The f the engine chooses for the graph file at ``path`` (host only, no GPU)."""
    import ctypes
    from reporter_amd import _lib
    f = ctypes.c_uint32(0)
    _lib.check(_lib.lib().rm_graph_grid_split(path.encode() if isinstance(path, str) else path, ctypes.byref(f)))
    return int(f.value)
