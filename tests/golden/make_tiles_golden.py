#!/usr/bin/env python3
"""Generate golden vectors for the reference's tile anonymiser (privacy cull + CSV).

Runs ONLY in the build container (the reference tree does not exist on the GPU
box).  It imports ``/root/reference/py/simple_reporter.py`` (Python 2 source)
under Python 3 with import shims (stdlib names, and stub ``boto3`` / ``valhalla``
modules that are absent here), writes seeded synthetic time-tile files in the
line format ``simple_reporter.match`` appends (simple_reporter.py:192-196), and
records exactly what the reference's ``report()`` phase (simple_reporter.py:211-254:
string sort, privacy cull of (id, next_id) runs, CSV header) would upload, by
capturing the body handed to the stub S3 client's ``put_object``.

Python-2 behaviour kept by the harness, not by editing the reference: the tile
file name is passed as a ``bytes`` subclass whose ``split`` accepts ``str``, so
``hashlib.sha1(file_name)`` (line 247, a ``str`` argument under Python 2) works.

The produced ``tiles_golden.json`` is DATA (inputs + expected outputs); no
reference source is copied.  ``oracle/tiles_oracle.py`` and the GPU tile stage
are both checked against it.

    python3 -B tests/golden/make_tiles_golden.py
"""
import io
import json
import os
import random
import sys
import tempfile
import types
import urllib.parse

sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference

REF_PY = "/root/reference/py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tiles_golden.json")
INVALID = 0x3FFFFFFFFFFF  # simple_reporter.py:43


class _Uploads:
    bodies = []


class _FakeClient:
    def put_object(self, Bucket=None, Body=None, Key=None):
        _Uploads.bodies.append((Key, Body))


class _FakeSession:
    def client(self, name):
        return _FakeClient()


class _Path(bytes):
    """A file name usable both as a path and as Python 2's str for hashlib (line 247)."""

    def split(self, sep=None):
        return [p.decode() for p in bytes.split(self, sep.encode() if isinstance(sep, str) else sep)]

    def __str__(self):
        return self.decode()

    def __mod__(self, other):
        return self.decode() % other


def _import_reference():
    import queue, http.server, socketserver, cgi
    sys.modules.setdefault("Queue", queue)
    bhs = types.ModuleType("BaseHTTPServer")
    bhs.HTTPServer = http.server.HTTPServer
    bhs.BaseHTTPRequestHandler = http.server.BaseHTTPRequestHandler
    sys.modules["BaseHTTPServer"] = bhs
    sys.modules["SocketServer"] = socketserver
    cgi.urlparse = urllib.parse
    sys.modules["valhalla"] = types.ModuleType("valhalla")
    boto3 = types.ModuleType("boto3")
    boto3.session = types.SimpleNamespace(Session=_FakeSession)
    boto3.client = lambda name: _FakeClient()
    sys.modules["boto3"] = boto3
    csio = types.ModuleType("cStringIO")
    csio.StringIO = io.StringIO
    sys.modules["cStringIO"] = csio
    sys.path.insert(0, REF_PY)
    import simple_reporter  # noqa: E402
    sys.path.pop(0)
    simple_reporter.logger.disabled = True
    return simple_reporter


def _seg_id(rng, level):
    return level | (rng.randrange(0, 1 << 22) << 3) | (rng.randrange(0, 1 << 21) << 25)


def _line(sid, nid, dur, length, queue, start, end, source="smpl_rprt", mode="AUTO"):
    # simple_reporter.py:192-196 row layout
    return ",".join(str(x) for x in (sid, nid, dur, 1, length, queue, start, end, source, mode)) + "\n"


def _random_tile(rng):
    """Lines of one tile file: a few (id, next_id) pairs with repeat counts that
    straddle the privacy threshold, ids of different decimal lengths (string order
    differs from numeric order), and lines in arbitrary order (the reference sorts)."""
    n_pairs = rng.choice([1, 1, 2, 3, 4, 6, 9, 14])
    lines = []
    for _ in range(n_pairs):
        level = rng.choice([0, 1, 1, 2])
        sid = rng.choice([_seg_id(rng, level), rng.randrange(1, 10 ** rng.randrange(1, 14))])
        nid = rng.choice([INVALID, _seg_id(rng, rng.choice([0, 1, 2])), rng.randrange(1, 10 ** rng.randrange(1, 8))])
        reps = rng.choice([1, 1, 1, 2, 2, 3, 4, 7])
        for _ in range(reps):
            start = 1483228800 + rng.randrange(0, 3600)
            dur = rng.randrange(1, 300)
            lines.append(_line(sid, nid, dur, rng.randrange(50, 1500), rng.choice([0, 0, rng.randrange(0, 200)]),
                               start, start + dur + rng.choice([0, 1])))
    rng.shuffle(lines)
    return lines


def _edge_tiles():
    """Hand-made tiles that pin the cull loop's boundary behaviour (lines 221-239)."""
    a, b, c, d = "1", "12", "123", "9"
    L = lambda sid, nid, k: _line(sid, nid, 10 + k, 100, 0, 1483228800 + k, 1483228810 + k)
    return [
        [L(a, INVALID, 0)],                                         # one line
        [L(a, INVALID, 0), L(a, INVALID, 1)],                      # one group of two
        [L(a, INVALID, 0), L(b, INVALID, 1)],                      # two singletons: last line merges
        [L(a, INVALID, 0), L(b, INVALID, 1), L(c, INVALID, 2)],    # three singletons
        [L(a, 5, 0), L(a, 5, 1), L(a, 5, 2), L(d, 5, 3)],          # big group, singleton last
        [L(d, 5, 0), L(a, 5, 1), L(a, 5, 2)],                      # singleton first
        [L(b, 7, 0), L(b, 7, 1), L(c, 7, 2), L(d, 7, 3), L(d, 7, 4)],
        [L(a, 1, 0), L(a, 12, 1), L(a, 12, 2), L(a, 2, 3)],        # next_id string order
        [L(c, INVALID, k) for k in range(5)] + [L(a, INVALID, 9)],
    ]


def main():
    sr = _import_reference()
    rng = random.Random(20171016)
    tiles = _edge_tiles() + [_random_tile(rng) for _ in range(300)]
    cases = []
    with tempfile.TemporaryDirectory() as d:
        for k, lines in enumerate(tiles):
            for privacy in (1, 2, 3, 5):
                name = os.path.join(d, "0_3599", "1", str(1000 + k))
                os.makedirs(os.path.dirname(name), exist_ok=True)
                with open(name, "w") as f:
                    f.write("".join(lines))
                _Uploads.bodies = []
                sr.report([_Path(name.encode())], "bucket", privacy)
                body = _Uploads.bodies[0][1] if _Uploads.bodies else None
                cases.append({"lines": lines, "privacy": privacy, "body": body})
    with open(OUT, "w") as f:
        json.dump({"generator": "tests/golden/make_tiles_golden.py",
                   "reference": "py/simple_reporter.py:211-254 report() (sort, privacy cull, CSV header)",
                   "cases": cases}, f, separators=(",", ":"))
    print("wrote %d cases to %s" % (len(cases), OUT))


if __name__ == "__main__":
    main()
