"""GPU batch reporter: the match and report phases of reference py/simple_reporter.py
on local files, with every stage on the MI355X.

    python -m reporter_amd.batch --trace-dir traces/ --match-config conf.json --dest-dir out/
    python -m torch.distributed.run --nproc-per-node 8 -m reporter_amd.batch ...   (one rank per GPU)

Input: the trace files simple_reporter's download phase writes (one point per line,
``uuid,time,lat,lon,accuracy``, py/simple_reporter.py:113; files named by a uuid hash,
:116).  Output: one file per time tile at ``<dest>/<start>_<end>/<level>/<tile index>``
holding exactly the text the reference's report phase would upload for that tile
(header + privacy-culled rows in string order, :211-254).

Reference phases and what replaces them:
  match()   :131-209  group by uuid, sort, inactivity windows      -> rm_runner_run_points
                      Match + report() per window                   -> the matcher kernels + k_report
                      valid-report filter, hour buckets, rows       -> rm_runner_tiles (rows)
  report()  :211-254  sort, privacy cull, CSV, upload               -> rm_runner_tiles (cull + CSV)
Multi-GPU: trace files are block-split over ranks (simple_reporter.split, :70-79, the
reference's process split); rows of every rank are all-gathered over RCCL and each rank
writes the tile files it owns.  There is no CPU path: the library raises without a GPU.
"""
import argparse
import json
import logging
import os
import sys

import numpy as np


def read_trace_files(paths):
    """Points of simple_reporter trace files -> (uuid strings, arrays).  Lines are
    ``uuid,time,lat,lon,accuracy`` (:113, parsed as :139-140: int time, float lat/lon,
    int accuracy)."""
    uuids, tm, lat, lon, acc = [], [], [], [], []
    for p in paths:
        with open(p, "r") as f:
            for line in f:
                line = line.strip()
                if not line:
                    continue
                u, t, la, lo, a = line.split(",")
                uuids.append(u)
                tm.append(int(t))
                lat.append(float(la))
                lon.append(float(lo))
                acc.append(int(a))
    return uuids, dict(time=np.asarray(tm, np.float64), lat=np.asarray(lat, np.float64),
                       lon=np.asarray(lon, np.float64), accuracy=np.asarray(acc, np.float32))


def dense_ids(uuids):
    """Dense vehicle index per point, in first-seen order; returns (index array, names)."""
    table = {}
    idx = np.empty(len(uuids), np.uint32)
    for k, u in enumerate(uuids):
        idx[k] = table.setdefault(u, len(table))
    return idx, list(table)


def options_from_config(conf_path, mode):
    """meili defaults (+ the mode's section) of a Valhalla-style config, as rm_configure reads it."""
    from . import engine
    from .world import MODES
    o = engine.default_options(1, mode=MODES[mode])
    with open(conf_path) as f:
        conf = json.load(f)
    meili = conf.get("meili", {})
    for section in (meili.get("default", {}), meili.get(mode, {})):
        for k, v in section.items():
            if k in o.dtype.names and k != "mode":
                o[k] = v
    graph = conf.get("reporter_amd", {}).get("graph") or conf.get("mjolnir", {}).get("tile_extract")
    if not graph:
        raise ValueError("config names no graph (reporter_amd.graph or mjolnir.tile_extract)")
    if not os.path.isabs(graph):
        graph = os.path.join(os.path.dirname(os.path.abspath(conf_path)), graph)
    return o, graph


def write_tiles(files, dest_dir):
    """{tile name: text} -> files under dest_dir (one file per tile, as uploaded)."""
    for name, body in files.items():
        path = os.path.join(dest_dir, name)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            f.write(body)


def run(trace_files, conf, dest_dir, mode="auto", report_levels=(0, 1), transition_levels=(0, 1), quantisation=3600,
        inactivity=120, privacy=2, source="smpl_rprt", rank=0, world=1, device=0, comm=None):
    from . import dist, engine
    mine = dist.split(sorted(trace_files), world)[rank] if world > 1 else sorted(trace_files)
    opts, graph = options_from_config(conf, mode)
    uuids, pts = read_trace_files(mine)
    idx, names = dense_ids(uuids)
    eng = engine.Engine(graph, device)
    with open(conf) as f:
        radius = json.load(f).get("reporter_amd", {}).get("ball_radius")
    if radius is not None:
        eng.set_ball_radius(float(radius))
    bm = engine.BatchMatcher(eng)
    bm.set_isolation(True)   # a failing window is logged and skipped (py/simple_reporter.py:169-173)
    try:
        bm.run_points(idx, pts["time"], pts["lon"], pts["lat"], pts["accuracy"], inactivity=inactivity, opts=opts,
                      n_uuids=len(names), report_levels=report_levels, transition_levels=transition_levels)
        errs = bm.trace_errors()
        if errs.any():
            owner = bm.trace_uuid()
            for k in np.nonzero(errs)[0]:
                logging.error("%s window %d failed to match (error bits %d); skipped", names[owner[k]], k, int(errs[k]))
        files = bm.tiles(quantisation=quantisation, privacy=privacy, source=source, mode=mode, comm=comm)
        write_tiles(files, dest_dir)
        return files
    finally:
        bm.close()
        eng.close()


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--trace-dir", required=True, help="directory of parsed trace files (simple_reporter --trace-dir)")
    ap.add_argument("--match-config", required=True)
    ap.add_argument("--dest-dir", required=True)
    ap.add_argument("--mode", default="auto")
    ap.add_argument("--report-levels", default="0,1")
    ap.add_argument("--transition-levels", default="0,1")
    ap.add_argument("--quantisation", type=int, default=3600)
    ap.add_argument("--inactivity", type=int, default=120)
    ap.add_argument("--privacy", type=int, default=2)
    ap.add_argument("--source-id", default="smpl_rprt")
    a = ap.parse_args(argv)
    files = []
    for root, _, fs in os.walk(a.trace_dir):
        files += [os.path.join(root, f) for f in fs]
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    comm = None
    if world > 1:
        from . import dist
        comm = dist.Comm(rank, world, local)
    levels = lambda s: tuple(int(x) for x in s.split(",") if x != "")
    try:
        out = run(files, a.match_config, a.dest_dir, a.mode, levels(a.report_levels), levels(a.transition_levels),
                  a.quantisation, a.inactivity, a.privacy, a.source_id, rank, world, local, comm)
    finally:
        if comm is not None:
            comm.close()
    print(json.dumps({"rank": rank, "tiles": len(out), "rows": sum(b.count("\n") - 1 for b in out.values())}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
