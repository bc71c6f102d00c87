#!/usr/bin/env python3
"""Generate golden vectors for the reference's post-match ``report()`` step.

Runs ONLY in the build container (the reference tree does not exist on the GPU
box).  It imports ``/root/reference/py/reporter_service.py`` (Python 2 source)
under Python 3 with stdlib-name shims, feeds it seeded synthetic matcher
outputs shaped like Valhalla's ``SegmentMatcher.Match`` reply (README.md:288-301)
and records the exact reply of ``report()`` (reporter_service.py:79-179).

The produced ``report_golden.json`` is DATA (inputs + expected outputs); no
reference source is copied.  ``oracle/report_oracle.py`` and the GPU report
epilogue are both checked against it.

    python3 -B tests/golden/make_report_golden.py
"""
import copy
import json
import os
import random
import sys
import types
import urllib.parse

sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference

REF_PY = "/root/reference/py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "report_golden.json")


def _import_reference():
    import queue, http.server, socketserver, cgi
    sys.modules.setdefault("Queue", queue)
    bhs = types.ModuleType("BaseHTTPServer")
    bhs.HTTPServer = http.server.HTTPServer
    bhs.BaseHTTPRequestHandler = http.server.BaseHTTPRequestHandler
    sys.modules["BaseHTTPServer"] = bhs
    sys.modules["SocketServer"] = socketserver
    cgi.urlparse = urllib.parse
    sys.modules["valhalla"] = types.ModuleType("valhalla")  # Match is not exercised here
    sys.path.insert(0, REF_PY)
    import reporter_service  # noqa: E402
    sys.path.pop(0)
    return reporter_service


def _seg_id(rng, level):
    tile = rng.randrange(0, 1 << 22)
    idx = rng.randrange(0, 1 << 21)
    return level | (tile << 3) | (idx << 25)


def _random_case(rng):
    """A Match-shaped reply: {"segments": [...]} + trace end time + levels."""
    n = rng.choice([0, 1, 1, 2, 3, 4, 5, 6, 8, 10, 14, 20])
    t = float(rng.randrange(1483228800, 1483228800 + 86400))
    shape = 0
    segs = []
    for k in range(n):
        kind = rng.random()
        seg = {}
        internal = False
        if kind < 0.12:
            internal = True
        elif kind < 0.2:
            pass  # unassociated (no segment_id)
        else:
            seg["segment_id"] = _seg_id(rng, rng.choice([0, 1, 1, 2, 2, 2]))
        seg["way_ids"] = [rng.randrange(1, 10 ** 9)]
        length = rng.choice([rng.randrange(20, 1200), rng.randrange(20, 1200), -1])
        dur = rng.choice([rng.uniform(0.2, 90.0), rng.uniform(5, 60), rng.uniform(10, 60), rng.uniform(10, 60), 0.0, -rng.uniform(0, 3)])
        st = t if rng.random() > 0.12 else -1
        if k == 0 and rng.random() < 0.5:
            st = -1
        t_end = t + dur
        en = t_end if rng.random() > 0.12 else -1
        if st == -1 or en == -1:
            length = -1 if rng.random() < 0.85 else length
        # speed-reject bait: very short durations on long segments
        if rng.random() < 0.1 and st != -1 and en != -1:
            en = st + rng.uniform(0.5, 5.0)
            length = rng.randrange(300, 1500)
        seg["start_time"] = st
        seg["end_time"] = en
        seg["queue_length"] = rng.choice([0, 0, 0, rng.randrange(0, 300)])
        seg["length"] = length
        seg["internal"] = internal
        seg["begin_shape_index"] = shape
        shape += rng.randrange(0, 30)
        seg["end_shape_index"] = shape
        if rng.random() < 0.15:
            del seg["internal"]  # report() defaults a missing flag to False
        segs.append(seg)
        t = t_end + rng.choice([0.0, 0.0, rng.uniform(0, 5)])
    end_time = t + rng.choice([0.0, 3.0, 10.0, 14.9, 15.0, 30.0, rng.uniform(0, 60)])
    levels = [[0, 1], [0, 1], [0, 1, 2], [1], [2], [], [0]]
    return {
        "match": {"segments": segs},
        "trace_end_time": end_time,
        "threshold_sec": rng.choice([15, 15, 15, 0, 5, 60]),
        "report_levels": rng.choice(levels),
        "transition_levels": rng.choice(levels),
    }


def _edge_cases():
    """Hand-made cases for Appendix-B behaviours of SURVEY.md."""
    base = 1500000000.0
    def s(i, sid, st, en, length, internal=False, q=0, b=0, e=0):
        d = {"way_ids": [i], "start_time": st, "end_time": en, "queue_length": q,
             "length": length, "internal": internal, "begin_shape_index": b, "end_shape_index": e}
        if sid is not None:
            d["segment_id"] = sid
        return d
    L0, L1, L2 = 0 | (5 << 3) | (7 << 25), 1 | (9 << 3) | (3 << 25), 2 | (11 << 3) | (4 << 25)
    cases = []
    # internal run between two level-1 segments keeps the prior
    cases.append([s(1, L1, base, base + 30, 400, b=0, e=10), s(2, None, base + 30, base + 32, 15, True, b=10, e=11),
                  s(3, L1 + (1 << 25), base + 32, base + 60, 300, b=11, e=20), s(4, L0, base + 60, -1, -1, b=20, e=25)])
    # discontinuity: partial end followed by partial start
    cases.append([s(1, L0, base, -1, -1, b=0, e=5), s(2, L0 + (1 << 25), -1, base + 50, -1, b=6, e=9),
                  s(3, L1, base + 50, base + 80, 500, b=9, e=15), s(4, L1 + (2 << 25), base + 80, -1, -1, b=15, e=22)])
    # prior t0 == -1 is not rejected by report()
    cases.append([s(1, L1, -1, base + 20, 300, b=0, e=4), s(2, L1 + (5 << 25), base + 20, base + 40, 250, b=4, e=8),
                  s(3, L0, base + 40, -1, -1, b=8, e=12)])
    # speed reject (> 160 km/h) and dt <= 0 reject
    cases.append([s(1, L0, base, base + 2, 900, b=0, e=2), s(2, L0 + (1 << 25), base + 2, base + 2, 100, b=2, e=3),
                  s(3, L0 + (2 << 25), base + 2, base + 30, 400, b=3, e=9), s(4, L2, base + 30, -1, -1, b=9, e=12)])
    # first segment internal: replaces prior (first_seg rule)
    cases.append([s(1, None, base, base + 3, 20, True, b=0, e=1), s(2, L1, base + 3, base + 40, 400, b=1, e=7),
                  s(3, L2, base + 40, base + 70, 350, b=7, e=12), s(4, L1 + (3 << 25), base + 70, -1, -1, b=12, e=20)])
    out = []
    for segs in cases:
        for thr, rl, tl in ((15, [0, 1], [0, 1]), (0, [0, 1, 2], [0, 1, 2]), (5, [1], [0, 1, 2])):
            out.append({"match": {"segments": copy.deepcopy(segs)},
                        "trace_end_time": segs[-1]["end_time"] if segs[-1]["end_time"] != -1 else base + 200,
                        "threshold_sec": thr, "report_levels": rl, "transition_levels": tl})
    return out


def main():
    rs = _import_reference()
    rng = random.Random(20171015)
    cases = _edge_cases() + [_random_case(rng) for _ in range(400)]
    records = []
    for c in cases:
        trace = {"uuid": "g", "trace": [{"lat": 0.0, "lon": 0.0, "time": c["trace_end_time"]}]}
        match = copy.deepcopy(c["match"])
        out = rs.report(match, trace, c["threshold_sec"], set(c["report_levels"]), set(c["transition_levels"]))
        records.append({"input": c, "output": json.loads(json.dumps(out))})
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_report_golden.py",
                   "reference": "py/reporter_service.py:79-179 report()",
                   "cases": records}, f, separators=(",", ":"))
    print("wrote %d cases to %s" % (len(records), OUT))


if __name__ == "__main__":
    main()
