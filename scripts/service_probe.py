"""Where the coalesced service's time goes (GPU box): per-batch library timings of small
uncoalesced batches (64 / 256 C2 traces through rm_match_batch), then the threaded service at
64 / 256 clients with the coalescer's batch statistics."""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import valhalla  # noqa: E402
from reporter_amd import world as W  # noqa: E402

tmp = os.environ.get("TMPDIR", "/tmp")
cfg = W.CONFIGS["C2"]
g = os.path.join(tmp, "svc_probe_c2.rmg")
W.build_world(g, cfg["rows"], cfg["cols"], cfg["block_m"], seed=1, cell_m=cfg["cell_m"])
tr = W.generate_traces(g, 4096, cfg["n_points"], cfg["rate_s"], cfg["noise_m"], seed=1)
reqs, P = bench.request_jsons(tr, 4096)
out = {}
conf = valhalla.write_config(os.path.join(tmp, "svc_probe.json"), g, device=0, coalesce=False)
valhalla.Configure(conf)
sm = valhalla.SegmentMatcher()
sm.MatchMany(reqs)
for n in (1, 16, 64, 256, 1024):
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        sm.MatchMany(reqs[:n])
        ts.append((time.perf_counter() - t) * 1e3)
    out["batch_%d" % n] = {"wall_ms": sorted(ts)[2], "library_ms": sm.last_timing()}
    print(n, out["batch_%d" % n], flush=True)
sm.close()
for workers, n_cli in ((1, 64), (1, 256), (2, 256)):
    conf = valhalla.write_config(os.path.join(tmp, "svc_probe_s.json"), g, device=0, coalesce=True, coalesce_workers=workers)
    valhalla.Configure(conf)
    s0 = valhalla.coalesce_stats()

    def client(c):
        m = valhalla.SegmentMatcher()
        for q in range(c, len(reqs), n_cli):
            m.Match(reqs[q])
        m.close()
    th = [threading.Thread(target=client, args=(c,)) for c in range(n_cli)]
    t = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t
    s1 = valhalla.coalesce_stats()
    nb, nr = s1["batches"] - s0["batches"], s1["requests"] - s0["requests"]
    r = {"clients": n_cli, "workers": workers, "seconds": dt, "points_per_s": P / dt, "batches": nb,
         "mean_batch": nr / max(nb, 1), "max_batch": s1["max_batch"], "ms_per_batch": dt * 1e3 / max(nb, 1)}
    out["service_%d_%d" % (workers, n_cli)] = r
    print(r, flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "service_probe.json"), "w"), indent=1)
