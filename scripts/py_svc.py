"""Python service clients on prepared requests (scripts/svc_prep.py output): `clients` threads,
one valhalla.SegmentMatcher each, Match on every request (coalescing on, the library's default
dispatchers), one untimed pass of 1,024 requests first; prints one JSON line.
    python scripts/py_svc.py /tmp/svcprep [clients] [requests]"""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import valhalla  # noqa: E402

d = sys.argv[1]
n_cli = int(sys.argv[2]) if len(sys.argv) > 2 else 64
n_req = int(sys.argv[3]) if len(sys.argv) > 3 else 8192
reqs = [line.rstrip("\n").encode() for line in open(os.path.join(d, "reqs.txt")) if line.strip()]
npt = sum(r.count(b'"lat"') for r in reqs[:100]) / min(100, len(reqs))
valhalla.Configure(os.path.join(d, "conf.json"))


def run(lo, hi, done):
    def client(c):
        m = valhalla.SegmentMatcher()
        for q in range(lo + c, hi, n_cli):
            m.Match(reqs[q % len(reqs)])
            done[c] += 1
        m.close()
    ths = [threading.Thread(target=client, args=(c,)) for c in range(n_cli)]
    t = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    return time.perf_counter() - t


run(0, 1024, [0] * n_cli)
done = [0] * n_cli
dt = run(1024, 1024 + n_req, done)
print(json.dumps({"clients": n_cli, "requests": sum(done), "seconds": dt, "requests_per_s": sum(done) / dt,
                  "points_per_s": sum(done) * npt / dt, "fast_match": valhalla._fast is not None}))
