#!/usr/bin/env python3
"""bench.py — GPS points map-matched per second on MI355X (BASELINE.json metric).

One step = the whole hot path over one resident batch: state selection,
candidate search (K1), bounded route search (K2), Viterbi (K3), path recovery
and OSMLR segment forming (K4), the reference's report() epilogue and the
per-segment speed histogram — i.e. what valhalla.SegmentMatcher().Match +
reporter_service.report() do for every trace (reference py/reporter_service.py:
240-242), batched.  With N>1 ranks each GPU matches its own uuid shard (weak
scaling) and the histograms are all-reduced over RCCL every step.

    python bench.py                       # N=1, C2 (configs[1]): 10k x 600 pts @1 Hz
    python bench.py --gpus 8              # self-launches 8 ranks (or run under torch.distributed.run)

Prints ONE JSON line (rank 0).  No PyTorch is loaded: RCCL is bound natively
by libreporter_match.so and ranks rendezvous through a node-local file.
"""
import argparse
import json
import multiprocessing as mp
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GPS points map-matched/sec (node) at 1/2/4/8 MI355X; % of HBM peak"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
HBM_MEASURED_GBS = 6290.0      # float4 copy ceiling from the same guide


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2", help="C1..C5 (BASELINE.json configs); C2 is the metric's workload")
    ap.add_argument("--traces", type=int, default=0, help="override traces per rank")
    ap.add_argument("--cpu-procs", type=int, default=0, help="CPU baseline processes (default min(16, cpus))")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ball-radius", type=float, default=None,
                    help="route-ball radius in m (default: the config's, else the engine's automatic radius)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r01", "pmc_routes_c2.json"),
                    help="rocprofv3 PMC summary giving HBM bytes per routes launch (optional)")
    return ap.parse_args()


# ---------------------------------------------------------------- CPU baseline leg (oracle)
_CPU = {}  # inherited by forked workers (copy-on-write); set before the pool starts


def _cpu_worker(block):
    lo, hi = block
    import numpy as np
    import meili_oracle as mo
    from reporter_amd.engine import default_options
    g, tr, radius = _CPU["graph"], _CPU["traces"], _CPU["radius"]
    off = tr["trace_off"].astype(np.int64)
    o0, o1 = off[lo], off[hi]
    sub_off = (off[lo:hi + 1] - o0).astype(np.uint32)
    opts = default_options(1, search_radius=radius)
    b = mo.Batch(sub_off, tr["lon"][o0:o1], tr["lat"][o0:o1], tr["time"][o0:o1], tr["accuracy"][o0:o1], opts,
                 np.zeros(hi - lo, np.uint32))
    hist = np.zeros(len(g["seg_id"]) * 16, np.uint32)
    mo.reset_counters()
    t = time.perf_counter()
    nrep = mo.pipeline(g, b, 15.0, 0x6, 0x6, hist)
    dt = time.perf_counter() - t
    return dt, int(o1 - o0), nrep, mo.counters()


def cpu_baseline_leg(graph_path, tr, search_radius, procs):
    """The oracle (a C port of the matcher + report()) run as `procs` single-threaded
    processes over contiguous trace blocks (simple_reporter.split, py/simple_reporter.py:70-79).
    Must run before this process initialises the GPU (workers are forked)."""
    import meili_oracle as mo
    from reporter_amd import graphfile
    from reporter_amd.dist import split
    _CPU.update(graph=graphfile.load(graph_path), traces=tr, radius=search_radius)
    mo.lib()  # load once in the parent; children inherit it
    T = len(tr["trace_off"]) - 1
    blocks = [(b[0], b[-1] + 1) for b in split(list(range(T)), procs) if len(b)]
    ctx = mp.get_context("fork")
    with ctx.Pool(len(blocks)) as pool:
        res = pool.map(_cpu_worker, blocks)
    wall = max(r[0] for r in res)
    pts = sum(r[1] for r in res)
    counts = {}
    for r in res:
        for k, v in r[3].items():
            counts[k] = counts.get(k, 0) + v
    return dict(value=pts / wall, seconds=wall, points=pts, reports=sum(r[2] for r in res), cores=len(blocks),
                counts=counts)


# ---------------------------------------------------------------- launcher for --gpus N without torchrun
def self_launch(n):
    port = str(29500 + (os.getpid() % 1000))
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, RM_RDZV_TOKEN="%s_%s" % (port, os.getpid()))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = p.wait() or rc
    return rc


def main():
    a = parse()
    if a.gpus > 1 and "RANK" not in os.environ:
        sys.exit(self_launch(a.gpus))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit("--gpus %d but WORLD_SIZE=%d" % (a.gpus, world))

    import numpy as np
    from reporter_amd import dist, engine, world as W
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import meili_oracle as mo  # cpu_baseline leg only (algorithmic byte counts + CPU timing)

    cfg = dict(W.CONFIGS[a.config])
    n_traces = a.traces or cfg["n_traces"]
    gdir = os.environ.get("TMPDIR", "/tmp")
    gpath = os.path.join(gdir, "reporter_bench_%s_%d_%d.rmg" % (a.config, os.getpid(), rank))
    W.build_world(gpath, cfg["rows"], cfg["cols"], cfg["block_m"], seed=1, cell_m=cfg["cell_m"])
    tr = W.generate_traces(gpath, n_traces, cfg["n_points"], cfg["rate_s"], cfg["noise_m"], seed=1000 + rank)
    P = int(tr["trace_off"][-1])

    # CPU leg first, before this process touches the GPU (forked workers never inherit a HIP context)
    cpu = None
    if rank == 0 and not a.no_cpu_baseline:
        procs = a.cpu_procs or min(16, os.cpu_count() or 1)
        cpu = cpu_baseline_leg(gpath, tr, cfg["search_radius"], procs)

    comm = dist.Comm(rank, world, local, token=os.environ.get("RM_RDZV_TOKEN")) if world > 1 else None
    eng = engine.Engine(gpath, local)
    radius = a.ball_radius if a.ball_radius is not None else cfg.get("ball_radius_m")
    if radius is not None:
        eng.set_ball_radius(radius)   # else the engine's automatic radius (balls.hpp auto_ball_radius_cm)
    bm = engine.BatchMatcher(eng)
    nseg = eng.n_segments
    hist = dist.DeviceBuffer(nseg * 16 * 4)
    opts = engine.default_options(1, search_radius=cfg["search_radius"])
    rp = dict(hist_dev=hist.ptr, zero_hist=True)
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, None, **rp)

    def step():
        bm.rerun(**rp)
        if comm is not None:
            comm.allreduce(hist.ptr, nseg * 16, dist.U32, dist.SUM)

    for _ in range(a.warmup):
        step()
    _lib_sync()
    if comm is not None:
        comm.barrier()
    bm.set_timing(True)
    bm.reset_times()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    _lib_sync()
    if comm is not None:
        comm.barrier()
    elapsed = time.perf_counter() - t0
    kt = bm.kernel_times()
    if comm is not None:
        elapsed = comm.allreduce_host(elapsed, dist.MAX)
        total_points = comm.allreduce_host(P, dist.SUM)
    else:
        total_points = P
    sizes = bm.sizes()
    hist_sum = int(hist.download().sum())

    if rank == 0:
        steps = max(a.steps, 1)
        routes_ms = kt["routes"][0] / steps
        counts = cpu["counts"] if cpu else {}
        balls = eng.ball_stats(0)
        tiers = bm.route_tiers()
        ball_tier = balls["radius_m"] > 0 and balls["keys"] > 0
        # bytes of the formulation the launch runs: route-ball probes (every item answered by
        # the tables when nothing was handed over), else the bounded searches
        if counts and ball_tier and tiers["ball_to_search"] == 0:
            abytes, formulation = mo.routes_ball_algorithmic_bytes(counts), "route-ball table probes"
        elif counts:
            abytes, formulation = mo.routes_algorithmic_bytes(counts), "bounded searches"
        else:
            abytes, formulation = None, None
        achieved = abytes / (routes_ms * 1e-3) / 1e9 if abytes else None
        traffic = None
        if os.path.exists(a.traffic_json):
            try:
                with open(a.traffic_json) as f:
                    tj = json.load(f)
                if tj.get("config") == a.config and tj.get("traces") == n_traces:
                    traffic = tj.get("hbm_bytes_per_launch")
            except (OSError, ValueError):
                traffic = None
        out = {
            "metric": METRIC,
            "value": total_points * a.steps / elapsed,
            "unit": "points/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 geometry / f64 Viterbi + times / u64 (dist,time) route keys",
            "data": "synthetic (seeded perturbed-grid world + generate_test_trace.py-style noisy traces)",
            "config": {
                "workload": "%s: %d traces x %d pts @%gs per GPU, %dx%d grid @%gm, radius %gm" % (
                    a.config, n_traces, cfg["n_points"], cfg["rate_s"], cfg["rows"], cfg["cols"], cfg["block_m"],
                    cfg["search_radius"]),
                "points_per_gpu": P,
                "traces_per_gpu": n_traces,
                "graph": W.graph_info(gpath),
                "parallelism": "uuid shard x%d, graph replicated, RCCL all-reduce of %d x 16 u32 speed histogram"
                               % (world, nseg),
            },
            "roofline": {
                "kernel": "K2 route stage: k_src_items + k_routes_ball + search tiers for hand-overs (one launch "
                          "each per step)",
                "formulation": formulation,
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "frac_vs_measured_copy": (achieved / HBM_MEASURED_GBS) if achieved else None,
                "traffic": traffic,
                "traffic_source": (os.path.relpath(a.traffic_json, ROOT) + " (rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE "
                                   "passes of this bench, read side x2 per MI355X_MICROARCH.md)") if traffic else None,
                "algorithmic_bytes_per_launch": abytes,
                "search_equivalent_bytes_per_launch": mo.routes_algorithmic_bytes(counts) if counts else None,
                "avg_launch_ms": routes_ms,
                "counts": counts,
                "route_tiers": tiers,
                "route_balls": balls,
            },
            "kernels_ms_per_step": {k: v[0] / steps for k, v in kt.items()},
            "sizes_per_gpu": sizes,
            "histogram_total": hist_sum,
        }
        if cpu and world == 1:
            out["cpu_baseline"] = {
                "value": cpu["value"], "unit": "points/s", "cores": cpu["cores"], "kind": "port",
                "sample": "full %s workload (%d pts, %d traces) split into %d contiguous blocks, one "
                          "single-threaded oracle process each (match + report() + histogram); %.2fs wall"
                          % (a.config, cpu["points"], n_traces, cpu["cores"], cpu["seconds"]),
            }
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
    hist.close()
    bm.close()
    eng.close()
    try:
        os.remove(gpath)
    except OSError:
        pass


def _lib_sync():
    from reporter_amd import _lib
    _lib.check(_lib.lib().rm_device_synchronize())


if __name__ == "__main__":
    main()
