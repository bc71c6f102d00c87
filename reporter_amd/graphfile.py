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
