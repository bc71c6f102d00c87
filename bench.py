#!/usr/bin/env python3
"""bench.py — GPS points map-matched per second on MI355X (BASELINE.json metric).

One step = the whole hot path over one resident batch: state selection,
candidate search (K1), bounded route search (K2), Viterbi (K3), path recovery
and OSMLR segment forming (K4), the reference's report() epilogue, the
per-segment speed histogram and its RCCL all-reduce — i.e. what
valhalla.SegmentMatcher().Match + reporter_service.report() do for every trace
(reference py/reporter_service.py:240-242), batched, plus the exchange that
replaces the keyed "id next_id" repartition (BatchingProcessor.java:126).

Workload: ONE seeded set of N x 10,000 C2 trajectories (uuids "C2-veh-0000000"...),
sharded over the N ranks by dist.shard_by_uuid (hash(uuid) buckets balanced by point
count, py/simple_reporter.py:116); each rank generates exactly its shard.  Weak
scaling: 10k trajectories per GPU.

    python bench.py                       # N=1, C2 (configs[1]): 10k x 600 pts @1 Hz
    python bench.py --gpus 8              # self-launches 8 ranks (or run under torch.distributed.run)

Prints ONE JSON line (rank 0).  No PyTorch is loaded: RCCL is bound natively
by libreporter_match.so and ranks rendezvous through a node-local file.
"""
import argparse
import ctypes as C
import hashlib
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
# VALU issue ceiling: 256 CUs x 4 SIMDs, one wave64 VALU instruction per SIMD every 4 cycles
# (16 lanes per cycle for 32-bit and fp64 ops alike on CDNA4) at 2.4 GHz
VALU_PEAK_WAVE_INSTR_S = 256 * 4 * 2.4e9 / 4
ENGINE_SRC = os.path.join(ROOT, "reporter_amd", "csrc", "engine.hip")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="C2", help="C1..C5 (BASELINE.json configs; C2 is the metric's workload), CITY / "
                    "CITY30 (C2 / C3 workloads on the OSM-ingested city)")
    ap.add_argument("--traces", type=int, default=0, help="override traces per rank")
    ap.add_argument("--cpu-procs", type=int, default=0, help="CPU baseline processes (default min(16, cpus))")
    ap.add_argument("--streams", type=int, default=1,
                    help="the batch runs as this many concurrent parts, one HIP stream each (1 = one stream)")
    ap.add_argument("--parts-extra", type=int, default=2,
                    help="also time the batch as this many concurrent parts (engine.MultiMatcher), reported "
                         "beside the value as concurrent_parts (0 = skip; batches <= 20 M points)")
    ap.add_argument("--exchange", choices=("allreduce", "reduce_scatter"), default="allreduce",
                    help="allreduce: every rank ends with the whole histogram and duration sums; reduce_scatter: "
                         "each rank ends with its segment-id range of them (SURVEY 8(e)'s option; half the bytes)")
    ap.add_argument("--comm", choices=("rccl", "host"), default="rccl",
                    help="rccl: one rank per GPU over xGMI (the measured configuration); host: the same "
                         "collectives over TCP on the host (rm_comm_init_host), ranks may share a GPU -- a "
                         "functional run of the multi-rank path on fewer GPUs, not a scaling measurement")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the C1 latency and JSON-boundary lines")
    ap.add_argument("--json-traces", type=int, default=10000, help="traces sent through rm_match_batch as JSON")
    ap.add_argument("--ball-radius", type=float, default=None,
                    help="route-ball radius in m (default: the config's, else the engine's automatic radius)")
    ap.add_argument("--turn-penalty", type=float, default=0.0,
                    help="turn_penalty_factor of every trace (meili's stock auto default is 200; DESIGN.md rule 3b); "
                         "the default C2 run also measures the workload at 200 beside the value (turn_costs)")
    ap.add_argument("--traffic-json", default=None,
                    help="rocprofv3 PMC summary giving HBM bytes per stage launch (scripts/pmc_summary.py; default "
                         "profiles/r03/pmc_routes_<config>.json; used only when it was measured on this engine.hip "
                         "with the same config and trace count)")
    return ap.parse_args()


def engine_sha():
    with open(ENGINE_SRC, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


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
    if _CPU.get("opts") is not None:   # per-trace options (C5)
        opts, topt = _CPU["opts"], np.ascontiguousarray(_CPU["trace_opt"][lo:hi], np.uint32)
    else:
        opts, topt = default_options(1, search_radius=radius), np.zeros(hi - lo, np.uint32)
    b = mo.Batch(sub_off, tr["lon"][o0:o1], tr["lat"][o0:o1], tr["time"][o0:o1], tr["accuracy"][o0:o1], opts, topt)
    hist = np.zeros(len(g["seg_id"]) * 16, np.uint32)
    dur = np.zeros(len(g["seg_id"]), np.uint64)
    mo.prepare_path_counters(g)   # in-edge index of the path-walk counters, outside the timed region
    mo.reset_counters()
    t = time.perf_counter()
    nrep = mo.pipeline(g, b, 15.0, 0x6, 0x6, hist, dur)
    dt = time.perf_counter() - t
    return dt, int(o1 - o0), nrep, mo.counters()


def cpu_baseline_leg(graph_path, tr, search_radius, procs, opts=None, trace_opt=None):
    """The oracle (a C port of the matcher + report()) run as `procs` single-threaded
    processes over contiguous trace blocks (simple_reporter.split, py/simple_reporter.py:70-79).
    Must run before this process initialises the GPU (workers are forked)."""
    import meili_oracle as mo
    from reporter_amd import graphfile
    from reporter_amd.dist import split
    # the engine's K1 grid (each file cell split f x f): same results, the item counts it reads
    g = graphfile.split_grid(graphfile.load(graph_path), graphfile.engine_grid_split(graph_path))
    _CPU.update(graph=g, traces=tr, radius=search_radius, opts=opts, trace_opt=trace_opt)
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
    return dict(value=pts / wall, seconds=wall, cpu_seconds=sum(r[0] for r in res), points=pts,
                reports=sum(r[2] for r in res), cores=len(blocks), counts=counts)


# ---------------------------------------------------------------- launcher for --gpus N without torchrun
def self_launch(n):
    port = str(29500 + (os.getpid() % 1000))
    nonce = os.urandom(12).hex()
    procs = []
    for r in range(n):
        # the rendezvous token names this launch and its nonce tells its id from one a crashed
        # earlier launch with a reused pid left behind (dist.rendezvous)
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port, RM_RDZV_TOKEN="%s_%s" % (port, os.getpid()), RM_RDZV_NONCE=nonce)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    for p in procs:
        rc = p.wait() or rc
    return rc


def shard_ids(config, n_per_rank, n_points, world, rank):
    """Trace indices of this rank's uuid shard of the ONE seeded workload of world x n_per_rank
    trajectories (dist.shard_by_uuid: hash(uuid) buckets balanced by point count)."""
    import numpy as np
    from reporter_amd import dist
    total = n_per_rank * world
    uuids = ["%s-veh-%07d" % (config, k) for k in range(total)]
    return dist.shard_by_uuid(uuids, np.full(total, n_points), world)[rank].astype(np.uint32)


LAUNCHES = 1   # launches of each stage per step (one per concurrent part of the batch)


def roofline(name, kernels, abytes, ms, formulation, traffic=None, valu=None):
    """abytes / ms: the step's algorithmic bytes and summed launch time of the stage; reported
    per launch (each part's launch does its share of the bytes, timed on its own stream).
    traffic: HBM bytes per launch from the PMC passes of this build (or None); dram_frac is what
    the HBM pins saw (traffic / time / peak) beside the algorithmic fraction."""
    abytes = abytes / LAUNCHES if abytes else abytes
    ms = ms / LAUNCHES if ms else ms
    if not abytes or not ms:
        return {"kernel": kernels, "formulation": formulation, "bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": None, "traffic": traffic, "dram_frac": None,
                "algorithmic_bytes_per_launch": abytes, "avg_launch_ms": ms, "launches_per_step": LAUNCHES}
    achieved = abytes / (ms * 1e-3) / 1e9
    dram = traffic / (ms * 1e-3) / 1e9 if traffic else None
    out = {"kernel": kernels, "formulation": formulation, "bound": "hbm", "achieved": achieved,
           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
           "frac_vs_measured_copy": achieved / HBM_MEASURED_GBS, "traffic": traffic,
           "dram_achieved": dram, "dram_frac": dram / HBM_PEAK_GBS if dram else None,
           "algorithmic_bytes_per_launch": abytes, "avg_launch_ms": ms, "launches_per_step": LAUNCHES}
    if valu:   # wave64 VALU instructions per launch (PMC SQ_INSTS_VALU of this build)
        out["valu_instrs"] = valu
        out["valu_frac"] = valu / (ms * 1e-3) / VALU_PEAK_WAVE_INSTR_S
        if out["valu_frac"] > out["frac"]:
            out["bound_note"] = "VALU issue is the nearer ceiling (valu_frac > frac)"
    return out


def load_traffic(path, config, traces, streams, turn_penalty=0.0):
    """Per-stage HBM bytes per launch from scripts/pmc_summary.py output, when it was measured on
    this engine.hip with the same workload; else ({}, reason)."""
    if not path or not os.path.exists(path):
        return {}, "no PMC summary at %s (engine.hip sha %s)" % (path, engine_sha())
    try:
        with open(path) as f:
            tj = json.load(f)
    except (OSError, ValueError) as e:
        return {}, "unreadable PMC summary %s: %s" % (path, e)
    if not (tj.get("config") == config and tj.get("traces") == traces and tj.get("engine_sha") == engine_sha()
            and tj.get("streams", 1) == streams and float(tj.get("turn_penalty", 0.0)) == float(turn_penalty)):
        return {}, "PMC summary %s is of another build or workload (sha %s vs %s)" % (
            os.path.relpath(path, ROOT), tj.get("engine_sha"), engine_sha())
    stages = tj.get("stages") or {"routes": {"hbm_bytes_per_launch": tj.get("hbm_bytes_per_launch"),
                                             "l2_hit_rate": tj.get("l2_hit_rate")}}
    note = ("%s: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this engine.hip (sha %s), read side x%s per "
            "MI355X_MICROARCH.md" % (os.path.relpath(path, ROOT), engine_sha(), tj.get("read_factor", 2)))
    return {k: v for k, v in stages.items() if v.get("hbm_bytes_per_launch")}, note


def timed(fn, steps, comm, sync):
    """barrier + sync, `steps` calls, sync + barrier; max over ranks."""
    sync()
    if comm is not None:
        comm.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    sync()
    if comm is not None:
        comm.barrier()
    dt = time.perf_counter() - t0
    if comm is not None:
        dt = comm.allreduce_host(dt, 1)
    return dt


def request_jsons(tr, n):
    """/report requests (reporter_service.py:184-235 contract) of the first n traces."""
    import numpy as np
    off = tr["trace_off"].tolist()
    n = min(n, len(off) - 1)
    P = off[n]
    f = '{"lat":%.6f,"lon":%.6f,"time":%d,"accuracy":%g}'
    pts = [f % q for q in zip(tr["lat"][:P].tolist(), tr["lon"][:P].tolist(), tr["time"][:P].astype(np.int64).tolist(),
                              tr["accuracy"][:P].tolist())]
    mo = '"match_options":{"mode":"auto","report_levels":[0,1],"transition_levels":[0,1]}'
    # bytes, as the reference's Python 2 service hands Match a str (= bytes) from json.dumps
    return [('{"uuid":"%d","trace":[%s],%s}' % (k, ",".join(pts[off[k]:off[k + 1]]), mo)).encode()
            for k in range(n)], P


def window_requests(tr, n_req, n_pts):
    """/report requests of n_pts consecutive points each, cut from the traces in order (the Java
    batcher posts a vehicle's points once it has >= 10 points, >= 500 m and >= 60 s,
    BatchingProcessor.java:26-29,69: ~60 points at 1 Hz)."""
    import numpy as np
    off = tr["trace_off"].astype(np.int64)
    out, P = [], 0
    f = '{"lat":%.6f,"lon":%.6f,"time":%d,"accuracy":%g}'
    mo = '"match_options":{"mode":"auto","report_levels":[0,1],"transition_levels":[0,1]}'
    for k in range(len(off) - 1):
        for a in range(int(off[k]), int(off[k + 1]) - n_pts + 1, n_pts):
            pts = ",".join(f % (tr["lat"][i], tr["lon"][i], int(tr["time"][i]), tr["accuracy"][i])
                           for i in range(a, a + n_pts))
            out.append('{"uuid":"%d-%d","trace":[%s],%s}' % (k, a, pts, mo))
            P += n_pts
            if len(out) >= n_req:
                return out, P
    return out, P


def client_service(gpath, tmpdir, reqs, clients, n, warmup, workers=None):
    """The C-ABI service client (reporter_amd/bin/rm_svc_client): `clients` threads, one
    rm_matcher each, rm_match on `n` requests with coalescing on; no Python between calls."""
    import valhalla
    from reporter_amd import build as B
    rfile = os.path.join(tmpdir, "reporter_bench_reqs_%d.txt" % os.getpid())
    with open(rfile, "w") as f:
        for r in reqs:
            f.write((r.decode() if isinstance(r, bytes) else r) + "\n")
    conf = valhalla.write_config(os.path.join(tmpdir, "reporter_bench_cli_%d.json" % os.getpid()), gpath, device=0,
                                 coalesce=True, coalesce_workers=workers)
    try:
        r = subprocess.run([B.CLIENT, conf, rfile, str(clients), str(n), str(warmup)], capture_output=True, text=True,
                           timeout=600)
    finally:
        os.remove(rfile)
    if r.returncode != 0:
        return {"error": (r.stderr or r.stdout)[-400:]}
    return json.loads(r.stdout.strip().splitlines()[-1])


def extras(gpath, tr, json_traces, tmpdir):
    """C1's defining measurement (single-trace latency through rm_match) and the JSON-boundary
    throughput of rm_match_batch (PCIe + parse + serialize inclusive), both through the drop-in
    valhalla module exactly as reporter_service.py calls it (:52, :240, :284)."""
    import numpy as np
    import valhalla
    from reporter_amd import world as W
    out = {}
    c1 = W.CONFIGS["C1"]
    c1g = os.path.join(tmpdir, "reporter_bench_C1_%d.rmg" % os.getpid())
    W.build_world(c1g, c1["rows"], c1["cols"], c1["block_m"], seed=1, cell_m=c1["cell_m"])
    c1tr = W.generate_traces(c1g, 1, c1["n_points"], c1["rate_s"], c1["noise_m"], seed=1)
    req = json.dumps(W.trace_to_request(c1tr, 0), separators=(",", ":"))
    conf = valhalla.write_config(os.path.join(tmpdir, "reporter_bench_c1_%d.json" % os.getpid()), c1g, device=0)
    valhalla.Configure(conf)
    sm = valhalla.SegmentMatcher()
    for _ in range(5):
        sm.Match(req)
    lat = []
    for _ in range(50):
        t = time.perf_counter()
        r = sm.Match(req)
        lat.append((time.perf_counter() - t) * 1e3)
    lat.sort()
    # BASELINE configs[0] itself: the CPU path on the same trace (the oracle, one core: match +
    # report(), the work reporter_service.py does per request; real meili cannot run here)
    import numpy as np
    import meili_oracle as mo
    from reporter_amd import engine as E, graphfile
    g1 = graphfile.load(c1g)
    b1 = mo.Batch(c1tr["trace_off"], c1tr["lon"], c1tr["lat"], c1tr["time"], c1tr["accuracy"], E.default_options(1),
                  np.zeros(1, np.uint32))
    cpu_ms = []
    for _ in range(5):
        hist1 = np.zeros(len(g1["seg_id"]) * 16, np.uint32)
        t = time.perf_counter()
        mo.pipeline(g1, b1, 15.0, 0x6, 0x6, hist1)
        cpu_ms.append((time.perf_counter() - t) * 1e3)
    cpu_ms.sort()
    out["c1_latency"] = {"what": "one 1,000-point 1 Hz trace (C1: 40x40 grid @100 m) through valhalla.SegmentMatcher()"
                                 ".Match -> rm_match (JSON in, JSON out; request coalescing on, one request in flight)",
                         "median_ms": lat[len(lat) // 2], "p90_ms": lat[int(len(lat) * 0.9)], "min_ms": lat[0],
                         "segments": len(json.loads(r)["segments"]), "caller_budget_ms": 10000,
                         "caller_budget_source": "HttpClient.java:80-87 (10 s socket timeout)",
                         "cpu_port_ms": {"median": cpu_ms[len(cpu_ms) // 2], "min": cpu_ms[0], "cores": 1,
                                         "what": "the oracle (C port of the matcher) + report() + histogram on the "
                                                 "same trace, one core, arrays in memory (no JSON): BASELINE "
                                                 "configs[0]'s CPU path"}}
    sm.close()
    os.remove(c1g)
    # JSON boundary: the rank's C2 traces as /report JSON through rm_match_batch
    t = time.perf_counter()
    reqs, P = request_jsons(tr, json_traces)
    build_s = time.perf_counter() - t
    conf = valhalla.write_config(os.path.join(tmpdir, "reporter_bench_c2_%d.json" % os.getpid()), gpath, device=0,
                                 coalesce=False)
    valhalla.Configure(conf)
    sm = valhalla.SegmentMatcher()
    t = time.perf_counter()
    sm.MatchMany(reqs)        # cold: route balls, workspace, pinned staging and parse buffers grow once
    cold = time.perf_counter() - t
    cold_ms = sm.last_timing()
    runs = []
    for _ in range(5):         # steady state of a long-running service: the median of five calls
        t = time.perf_counter()
        outs = sm.MatchMany(reqs)
        runs.append((time.perf_counter() - t, sm.last_timing()))
    runs.sort(key=lambda r: r[0])
    dt, steady_ms = runs[2]
    out["json_boundary"] = {"what": "%d C2 traces (%d points, %.0f MB of /report JSON) through rm_match_batch: host "
                                    "JSON parse -> H2D -> every kernel -> D2H -> segment JSON" % (
                                        len(reqs), P, sum(map(len, reqs)) / 1e6),
                            "value": P / dt, "unit": "points/s", "seconds": dt, "json_build_s_untimed": build_s,
                            "value_library": P / (steady_ms["total_ms"] * 1e-3) if steady_ms.get("total_ms") else None,
                            "value_library_what": "the same call's rm_match_batch wall time alone (no Python list "
                                                  "marshalling / reply decoding)",
                            "trace_parse": "device (k_parse_json) for compact trace arrays"
                                           if os.environ.get("RM_JSON_DEVICE", "1") != "0" else "host",
                            "reply_mb": sum(map(len, outs)) / 1e6, "host_threads": os.cpu_count() and min(16, os.cpu_count()),
                            "library_ms": steady_ms, "seconds_of_five_calls": [r[0] for r in runs],
                            "first_call": {"seconds": cold, "library_ms": cold_ms,
                                           "note": "the same call on a fresh matcher: buffers grow once"}}
    sm.close()
    # the service under concurrent load: one SegmentMatcher per client thread (as
    # reporter_service.py's threaded server, a thread per request), every Match coalesced into
    # shared batches; at 64 and 256 requests in flight (a batch takes a few ms whatever its size,
    # so the throughput follows the number of requests in flight)
    n_req = min(len(reqs), 4096)
    r60_py, _ = window_requests(tr, 8192, 60)
    # (the 60-point line, round 6: the library's default two dispatchers and one untimed pass of
    # 1,024 requests first, as the C client's lines; the 600-point lines as in earlier rounds)
    for workers, n_cli, rq in ((1, 64, reqs), (1, 256, reqs), (None, 64, [x.encode() for x in r60_py])):
        conf = valhalla.write_config(os.path.join(tmpdir, "reporter_bench_svc_%d.json" % os.getpid()), gpath, device=0,
                                     coalesce=True, coalesce_workers=workers)
        valhalla.Configure(conf)
        done = [0] * n_cli

        nq = min(len(rq), 8192 if rq is not reqs else n_req)

        def client(c, lo=0, hi=None, count=True):
            m = valhalla.SegmentMatcher()
            for q in range(lo + c, nq if hi is None else hi, n_cli):
                m.Match(rq[q])
                if count:
                    done[c] += 1
            m.close()

        import threading
        if workers is None:
            warm = [threading.Thread(target=client, args=(c, 0, 1024, False)) for c in range(n_cli)]
            for th in warm:
                th.start()
            for th in warm:
                th.join()
        ths = [threading.Thread(target=client, args=(c,)) for c in range(n_cli)]
        t = time.perf_counter()
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        dt = time.perf_counter() - t
        npt = 600 if rq is reqs else 60
        pts = sum(done) * npt
        key = "service_throughput" if (n_cli == 64 and npt == 600) else "service_throughput_%d_clients%s" % (
            n_cli, "" if npt == 600 else "_60pt")
        out[key] = {
            "what": "%d C2 /report requests (%d points each) from %d Python client threads through "
                    "valhalla.SegmentMatcher().Match with request coalescing, %s dispatcher(s)%s" % (
                        sum(done), npt, n_cli, workers or "2 (default)",
                        "; 1,024 requests untimed first" if workers is None else ""),
            "requests_per_s": sum(done) / dt, "points_per_s": pts / dt, "seconds": dt}
    # the library's own ceiling under concurrent load: the C-ABI client (no GIL), 600-point C2
    # requests and the Java batcher's ~60-point requests, 64 and 256 requests in flight
    r60, p60 = window_requests(tr, 20000, 60)
    for name, rq, nreq, cl in (("service_client_600pt_64", reqs, 8192, 64), ("service_client_600pt_256", reqs, 8192, 256),
                               ("service_client_60pt_64", r60, 20000, 64), ("service_client_60pt_256", r60, 20000, 256)):
        res = client_service(gpath, tmpdir, rq, cl, nreq, min(2048, nreq // 4))
        res["what"] = ("reporter_amd/bin/rm_svc_client: %d C threads, one rm_matcher each, rm_match (coalescing on) on "
                       "%d-point /report requests; the library's ceiling with no interpreter between calls"
                       % (cl, 600 if "600" in name else 60))
        out[name] = res
    return out


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
    from reporter_amd import _lib, dist, engine, world as W
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import meili_oracle as mo  # cpu_baseline leg only (algorithmic byte counts + CPU timing)

    cfg = dict(W.CONFIGS[a.config])
    n_per = a.traces or cfg["n_traces"]
    gdir = os.environ.get("TMPDIR", "/tmp")
    gpath = os.path.join(gdir, "reporter_bench_%s_%d_%d.rmg" % (a.config, os.getpid(), rank))
    W.build_config_graph(a.config, gpath, seed=1)
    ids = shard_ids(a.config, n_per, cfg["n_points"], world, rank)
    opts_all, trace_opt = None, None
    if a.config == "C5":
        # the C2 graph, traces split over auto / bicycle / pedestrian and
        # sigma_z in {2, 4.07, 8, 16} with GPS noise sigma = sigma_z and radius max(50, 3 sigma_z);
        # each (mode, sigma) group is a seeded set sharded by the same ids
        from reporter_amd import engine as E
        groups = [(m, sg) for m in ("auto", "bicycle", "pedestrian") for sg in (2.0, 4.07, 8.0, 16.0)]
        opts_all = E.default_options(len(groups))
        sets, tos = [], []
        for q, (m, sg) in enumerate(groups):
            opts_all[q]["mode"], opts_all[q]["sigma_z"] = W.MODES[m], sg
            opts_all[q]["search_radius"] = max(50.0, 3.0 * sg)
            gid = ids[ids % len(groups) == q]
            if len(gid):
                sets.append(W.generate_traces(gpath, 0, cfg["n_points"], cfg["rate_s"], sg, seed=5000 + q, mode=m,
                                              ids=gid))
                tos.append(np.full(len(gid), q, np.uint32))
        tr = W.concat_traces(*sets)
        trace_opt = np.concatenate(tos)
    else:
        tr = W.generate_traces(gpath, 0, cfg["n_points"], cfg["rate_s"], cfg["noise_m"], seed=1000, ids=ids)
    if a.turn_penalty > 0:   # meili's turn costs on every trace (rule 3b)
        from reporter_amd import engine as E
        if opts_all is None:
            opts_all = E.default_options(1, search_radius=cfg["search_radius"])
            trace_opt = np.zeros(len(ids), np.uint32)
        opts_all["turn_penalty_factor"] = a.turn_penalty
    P = int(tr["trace_off"][-1])
    T = len(ids)

    # CPU leg first, before this process touches the GPU (forked workers never inherit a HIP context)
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        procs = a.cpu_procs or min(16, os.cpu_count() or 1)
        cpu = cpu_baseline_leg(gpath, tr, cfg["search_radius"], procs, opts_all, trace_opt)

    comm, comm_note, tcp = None, None, None
    if a.comm == "host":
        # ranks beyond the visible GPUs share them (functional multi-rank run, not a measurement)
        cnt = C.c_int(0)
        _lib.check(_lib.lib().rm_device_count(C.byref(cnt)))
        local = local % max(1, cnt.value)
        tcp = dist.TcpAllgather(rank, world, os.environ.get("MASTER_ADDR", "127.0.0.1"),
                                int(os.environ.get("MASTER_PORT", "29500")) + 1)
        comm = dist.Comm(rank, world, local, allgather=tcp)
        comm_note = "host transport (TCP all-gather, rm_comm_init_host); %d rank(s) on %d GPU(s)" % (world, cnt.value)
    else:
        try:
            comm = dist.Comm(rank, world, local, token=os.environ.get("RM_RDZV_TOKEN"))
        except Exception as e:  # noqa: BLE001 -- one rank without RCCL still measures the matcher
            if world > 1:
                raise
            comm_note = "RCCL unavailable at N=1 (%s): histogram not all-reduced" % e
    t_up = time.perf_counter()
    eng = engine.Engine(gpath, local)
    radius = a.ball_radius if a.ball_radius is not None else cfg.get("ball_radius_m")
    if radius is not None:
        eng.set_ball_radius(radius)   # else the engine's automatic radius (balls.hpp auto_ball_radius_cm)
    global LAUNCHES
    LAUNCHES = max(1, a.streams)
    # the batch as `streams` concurrent parts (engine.MultiMatcher: one HIP stream each), or one
    bm = engine.MultiMatcher(eng, a.streams) if a.streams > 1 else engine.BatchMatcher(eng)
    nseg = eng.n_segments
    # reduce-scatter: buffers padded to world equal chunks of whole segment-id ranges (padding
    # stays 0): each rank owns cd segments, i.e. 16 * cd histogram bins (never a split segment)
    rs = a.exchange == "reduce_scatter"
    cd = -(-nseg // world) if rs else nseg
    ch = 16 * cd
    hist = dist.DeviceBuffer((ch * world if rs else nseg * 16) * 4)
    dur = dist.DeviceBuffer((cd * world if rs else nseg) * 8)   # per-segment duration sums
    opts = opts_all if opts_all is not None else engine.default_options(1, search_radius=cfg["search_radius"])
    rp = dict(hist_dev=hist.ptr, dur_dev=dur.ptr, zero_hist=True)
    bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, trace_opt, **rp)
    cold_s = time.perf_counter() - t_up

    def sync():
        _lib.check(_lib.lib().rm_device_synchronize())

    def allreduce():
        if comm is None:
            return
        if rs:
            comm.reduce_scatter(hist.ptr, ch, dist.U32, dist.SUM)
            comm.reduce_scatter(dur.ptr, cd, dist.U64, dist.SUM)
        else:
            comm.allreduce(hist.ptr, nseg * 16, dist.U32, dist.SUM)
            comm.allreduce(dur.ptr, nseg, dist.U64, dist.SUM)

    def step():
        bm.rerun(**rp)
        allreduce()

    for _ in range(a.warmup):
        step()
    # the official step (match + all-reduce), with the roofline kernel's stage (K2) timed live by
    # HIP events on each part's stream; an event record per stage would perturb the concurrent parts
    bm.set_timing_stages(("routes",))
    bm.reset_times()
    elapsed = timed(step, a.steps, comm, sync)
    kt_live = bm.kernel_times()
    bm.set_timing(False)
    t_ar = timed(allreduce, a.steps, comm, sync)             # the all-reduce alone, reported alongside
    t_match = timed(lambda: bm.rerun(**rp), a.steps, comm, sync)   # matching alone
    # the same batch as concurrent parts, one HIP stream each (rm_runners_rerun): gather-bound
    # stages of one part overlap issue-bound stages of another; reported beside the value (the
    # parts share the GPU, so their per-launch K2 roofline is not the kernel's)
    conc = None
    if a.parts_extra > 1 and a.streams == 1 and P <= 20_000_000:
        mm = engine.MultiMatcher(eng, a.parts_extra)
        mm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], opts, trace_opt, **rp)
        for _ in range(a.warmup):
            mm.rerun(**rp)
            allreduce()
        t_conc = timed(lambda: (mm.rerun(**rp), allreduce()), a.steps, comm, sync)
        conc = {"parts": len(mm.bms), "streams": len(mm.bms), "ms_per_step": t_conc / max(a.steps, 1) * 1e3,
                "value_points_per_s": (comm.allreduce_host(P, dist.SUM) if comm is not None else P) * a.steps / t_conc,
                "what": "the same step (match + all-reduce) with the batch split into contiguous trace ranges "
                        "balanced by points, run concurrently on their own HIP streams (engine.MultiMatcher / "
                        "rm_runners_rerun); bit-identical results (tests/test_gpu_multistream.py)"}
        mm.close()
    # per-stage breakdown (the other rooflines): a separate pass with every stage timed
    bm.set_timing(True)
    bm.reset_times()
    t_staged = timed(lambda: bm.rerun(**rp), a.steps, comm, sync)
    kt = bm.kernel_times()
    bm.set_timing(False)
    kt["routes"] = kt_live["routes"]
    total_points = comm.allreduce_host(P, dist.SUM) if comm is not None else P
    sizes = bm.sizes()
    step()   # one more exchanged step: the totals below are of the reduced arrays
    hist_sum = int(hist.download().sum())
    dur_sum = int(dur.download(np.uint64).sum())
    if rs and comm is not None:   # each rank holds its range: the totals are the sums of the ranges
        hv, dv = hist.download(), dur.download(np.uint64)
        hist_sum = int(comm.allreduce_host(float(hv[rank * ch:(rank + 1) * ch].sum()), dist.SUM))
        dur_sum = int(comm.allreduce_host(float(dv[rank * cd:(rank + 1) * cd].sum()), dist.SUM))
    balls = eng.ball_stats(0)
    tiers = bm.route_tiers()
    # the C2 workload with meili's stock auto turn costs (200, rule 3b), beside the value: the same
    # points re-run with the factor on every trace, K2 timed live as in the official step
    turn = None
    if a.config == "C2" and world == 1 and a.turn_penalty == 0 and a.streams == 1 and not a.no_extras:
        topts = engine.default_options(1, search_radius=cfg["search_radius"], turn_penalty_factor=200.0)
        bm.run(tr["trace_off"], tr["lon"], tr["lat"], tr["time"], tr["accuracy"], topts, None, **rp)
        for _ in range(a.warmup):
            step()
        bm.set_timing_stages(("routes",))
        bm.reset_times()
        t_turn = timed(step, a.steps, comm, sync)
        kt_turn = bm.kernel_times()
        bm.set_timing(True)
        bm.reset_times()
        timed(lambda: bm.rerun(**rp), a.steps, comm, sync)
        kt_turn_all = bm.kernel_times()
        bm.set_timing(False)
        turn = {"t": t_turn, "routes_ms": kt_turn["routes"][0] / max(a.steps, 1),
                "stages_ms": {k: v[0] / max(a.steps, 1) for k, v in kt_turn_all.items()},
                "tiers": bm.route_tiers(), "turn_rows_built": eng.turn_rows()}

    out = None
    if rank == 0:
        steps = max(a.steps, 1)
        ms = {k: v[0] / steps for k, v in kt.items()}
        counts = cpu["counts"] if cpu else {}
        ball_tier = balls["radius_m"] > 0 and balls["keys"] > 0
        # bytes of the formulation the launch runs: route-ball probes (every item answered by
        # the tables when nothing was handed over), else the bounded searches
        if counts and ball_tier and tiers["ball_to_search"] == 0 and a.turn_penalty > 0:
            abytes = mo.routes_ball_turn_algorithmic_bytes(counts)
            formulation = "route-ball table probes + turn rows (turn_penalty_factor %g)" % a.turn_penalty
        elif counts and ball_tier and tiers["ball_to_search"] == 0:
            abytes, formulation = mo.routes_ball_algorithmic_bytes(counts), "route-ball table probes"
        elif counts and "settled_to_targets" in counts:
            abytes = mo.routes_targets_algorithmic_bytes(counts)
            formulation = "bounded searches stopped at their targets (label-setting order)"
        elif counts:
            abytes, formulation = mo.routes_algorithmic_bytes(counts), "bounded searches"
        else:
            abytes, formulation = None, None
        tpath = a.traffic_json
        if not tpath:   # the newest round's PMC summary of this workload (sha-checked by load_traffic)
            for rnd in ("r06", "r05", "r04"):
                tpath = os.path.join(ROOT, "profiles", rnd, "pmc_routes_%s%s.json" % (
                    a.config.lower(), "_turn%g" % a.turn_penalty if a.turn_penalty > 0 else ""))
                if os.path.exists(tpath):
                    break
        traffic, traffic_note = load_traffic(tpath, a.config, n_per, max(1, a.streams), a.turn_penalty)
        tr_of = lambda st: (traffic.get(st) or {}).get("hbm_bytes_per_launch")
        va_of = lambda st: (traffic.get(st) or {}).get("valu_instrs")
        k2 = roofline("K2", "K2 route stage: k_src_items + k_routes_ball2 + search tiers for hand-overs", abytes,
                      ms["routes"], formulation, tr_of("routes"), va_of("routes"))
        k2["l2_hit_rate"] = (traffic.get("routes") or {}).get("l2_hit_rate")
        k2["traffic_source"] = traffic_note
        k2.update({"search_equivalent_bytes_per_launch": mo.routes_algorithmic_bytes(counts) if counts else None,
                   "counts": counts, "route_tiers": tiers, "route_balls": balls, "k1_grid_split": eng.grid_split()})
        rooflines = {
            "K1": roofline("K1", "k_candidates_lane + k_candidates_wave", mo.candidates_algorithmic_bytes(counts)
                           if counts else None, ms["candidates"], "cell-major 32 B records on the engine grid (file cells split "
                           "%dx%d; items counted by the oracle on that grid), per-road minima in registers"
                           % (eng.grid_split(), eng.grid_split()), tr_of("candidates"), va_of("candidates")),
            "K2": {k: k2.get(k) for k in ("kernel", "achieved", "frac", "algorithmic_bytes_per_launch", "avg_launch_ms",
                                      "traffic", "dram_frac", "valu_frac")},
            "K3": roofline("K3", "k_viterbi", mo.viterbi_algorithmic_bytes(counts) if counts else None, ms["viterbi"],
                           "u32 routes + f32 emissions, fp64 costs in registers", tr_of("viterbi"), va_of("viterbi")),
            "paths": roofline("paths", "path stage: k_paths_ball + search tiers for hand-overs",
                              mo.paths_algorithmic_bytes(counts) if counts and "path_rows" in counts else None,
                              ms["paths"], "route-ball labels, walk back by canonical predecessors over "
                              "self-contained in-edge records", tr_of("paths"), va_of("paths")),
            "K4": roofline("K4", "segments stage: trav_off scan + k_rec_slot + k_seg_wave",
                           mo.segments_algorithmic_bytes(counts) if counts else None, ms["segments"],
                           "wave per trace, 64 traversal records per step in registers, runs by ballot/scan",
                           tr_of("segments"), va_of("segments")),
        }
        step_ms = elapsed / steps * 1e3
        build_ms = balls["build_ms"]
        out = {
            "metric": METRIC,
            "value": total_points * a.steps / elapsed,
            "unit": "points/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": step_ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 geometry / f64 Viterbi + times / u64 (dist,time) route keys",
            "data": ("synthetic (seeded irregular city written as generic OSM PBF and ingested by rm_graph_import_osm + "
                     "generate_test_trace.py-style noisy traces)" if cfg.get("city") else
                     "synthetic (seeded perturbed-grid world + generate_test_trace.py-style noisy traces)"),
            "config": {
                "workload": "%s: %d traces x %d pts @%gs per GPU (uuid shard of one %d-trace seeded set), %dx%d %s "
                            "@%gm, radius %gm" % (a.config, n_per, cfg["n_points"], cfg["rate_s"], n_per * world,
                                                 cfg["rows"], cfg["cols"],
                                                 "junction OSM city" if cfg.get("city") else "grid", cfg["block_m"],
                                                 cfg["search_radius"]) +
                            ("; traces split over auto / bicycle / pedestrian x sigma_z {2, 4.07, 8, 16} (GPS noise "
                             "sigma = sigma_z, radius max(50, 3 sigma_z))" if a.config == "C5" else ""),
                "points_rank0": P,
                "traces_rank0": T,
                "points_all_ranks": int(total_points),
                "graph": W.graph_info(gpath),
                "parallelism": "uuid shard x%d (dist.shard_by_uuid), graph replicated, %s all-reduce of the %d x 16 "
                               "u32 speed histogram and the per-segment u64 duration sums every step; per GPU the batch runs as %d concurrent part(s), one HIP "
                               "stream each" % (world, "host-transport (TCP)" if a.comm == "host" else "RCCL", nseg,
                                                max(1, a.streams)),
            },
            "ms_allreduce": t_ar / steps * 1e3,
            "allreduce_bytes": nseg * 16 * 4 + nseg * 8,
            "exchange": a.exchange,
            "ms_matching_only": t_match / steps * 1e3,
            "value_matching_only": total_points * a.steps / t_match,
            "roofline": k2,
            "rooflines": rooflines,
            "cold_start": {"graph_upload_and_first_run_s": cold_s, "route_ball_build_ms": build_ms,
                           "ball_build_in_steps": build_ms / step_ms,
                           "value_over_first_hour_incl_ball_build": total_points / (step_ms * 1e-3) *
                           max(0.0, 3600.0 - build_ms * 1e-3) / 3600.0,
                           "note": "the route balls are built once per graph and travel mode (host, at rm_configure); "
                                   "they are outside the timed step"},
            "concurrent_parts": conc,
            "kernels_ms_per_step": ms,
            "kernels_ms_note": ("summed launch ms of each stage per step over the %d part(s); routes timed live in the "
                                "official step, the other stages in a separate pass with every stage timed (%.3f ms "
                                "per step)" % (max(1, a.streams), t_staged / steps * 1e3)),
            "sizes_rank0": sizes,
            "histogram_total": hist_sum,
            "duration_sum_total_s": dur_sum,
        }
        if turn is not None:
            ttraffic, tnote = {}, None
            for rnd in ("r06", "r05"):
                tp = os.path.join(ROOT, "profiles", rnd, "pmc_routes_c2_turn200.json")
                if os.path.exists(tp):
                    ttraffic, tnote = load_traffic(tp, a.config, n_per, 1, 200.0)
                    break
            kt2 = roofline("K2", "K2 route stage with turn costs: k_src_items + k_routes_ball2<turn> (turn rows, ties "
                           "walked through the tables) + search tiers for hand-overs",
                           mo.routes_ball_turn_algorithmic_bytes(counts) if counts and "turn_rows" in counts else None,
                           turn["routes_ms"], "route-ball table probes + turn rows",
                           (ttraffic.get("routes") or {}).get("hbm_bytes_per_launch"),
                           (ttraffic.get("routes") or {}).get("valu_instrs"))
            kt2["l2_hit_rate"] = (ttraffic.get("routes") or {}).get("l2_hit_rate")
            kt2["traffic_source"] = tnote
            out["turn_costs"] = {
                "what": "the same C2 points with meili's stock auto turn_penalty_factor 200 on every trace "
                        "(valhalla_build_config's default, reference Dockerfile:42-49; DESIGN.md rule 3b): match + "
                        "all-reduce per step, K2 timed live",
                "value": total_points * a.steps / turn["t"], "unit": "points/s", "ms_per_step": turn["t"] / steps * 1e3,
                "turn_penalty_factor": 200.0, "roofline": kt2, "kernels_ms_per_step": turn["stages_ms"],
                "route_tiers": turn["tiers"], "turn_rows": turn["turn_rows_built"]}
        if comm_note:
            out["comm_note"] = comm_note
        if cpu:
            out["cpu_baseline"] = {
                "value": cpu["value"], "unit": "points/s", "cores": cpu["cores"], "kind": "port",
                "sample": "full %s rank-0 workload (%d pts, %d traces) split into %d contiguous blocks, one "
                          "single-threaded oracle process each (match + report() + histogram); %.2fs wall, %.1f "
                          "CPU-s" % (a.config, cpu["points"], T, cpu["cores"], cpu["seconds"], cpu["cpu_seconds"]),
            }
    if comm is not None:
        comm.close()
    if tcp is not None:
        tcp.close()
    hist.close()
    dur.close()
    bm.close()
    eng.close()
    if rank == 0 and world == 1 and not a.no_extras and a.config == "C2":
        out.update(extras(gpath, tr, a.json_traces, gdir))
    if rank == 0:
        print(json.dumps(out), flush=True)
    try:
        os.remove(gpath)
    except OSError:
        pass


if __name__ == "__main__":
    main()
