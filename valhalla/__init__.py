"""Drop-in replacement for the ``valhalla`` Python module used by Open Traffic Reporter.

The reference imports ``valhalla`` and calls exactly three things
(SURVEY.md §8b):

  valhalla.Configure(conf_path)          py/reporter_service.py:284, py/simple_reporter.py:132
  valhalla.SegmentMatcher()              py/reporter_service.py:52,  py/simple_reporter.py:133
  SegmentMatcher().Match(json) -> json   py/reporter_service.py:240, py/simple_reporter.py:166

Here they bind to libreporter_match.so (the MI355X engine) through ctypes —
no PyTorch.  Errors surface as RuntimeError so the service's 500 path
(py/reporter_service.py:244-245) and the batch skip path
(py/simple_reporter.py:169-173) behave as before.  There is no CPU fallback.
"""
import ctypes as C
import json as _json
import os as _os

from reporter_amd import _lib

__all__ = ["Configure", "SegmentMatcher", "coalesce_stats"]

# Match in one CPython call (valhalla/_match.c, built beside the library by reporter_amd.build):
# the ctypes path below costs a 60-point request ~15 us of GIL-held Python under 64 threads.  Only
# with the in-tree library: the extension links that one, and a second copy (REPORTER_MATCH_LIB)
# would not share its configuration.  RM_PY_CTYPES=1 keeps the ctypes path (A/B).
_fast = None
if not _os.environ.get("RM_PY_CTYPES") and _os.path.abspath(_lib.LIB_PATH) == _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                                                    "reporter_amd", "libreporter_match.so"):
    try:
        from valhalla import _match as _fast
    except ImportError:   # not built (a source tree): the ctypes path below
        _fast = None


def Configure(conf_path):
    """Load the matcher config + graph into HBM (process-global)."""
    err = C.create_string_buffer(1024)
    rc = _lib.lib().rm_configure(_os.fsencode(conf_path), err, len(err))
    if rc != 0:
        raise RuntimeError(err.value.decode("utf-8", "replace"))


class SegmentMatcher(object):
    """One matcher per thread (the reference keeps it in threading.local)."""

    def __init__(self):
        self._h = _lib.lib().rm_matcher_create()
        if not self._h:
            raise RuntimeError(_lib.last_error())

    def Match(self, trace_json):
        """trace JSON string in, {"segments": [...]} JSON string out."""
        if _fast is not None:
            return _fast.match(self._h or 0, trace_json)
        if isinstance(trace_json, str):
            trace_json = trace_json.encode("utf-8")
        out = C.c_void_p()
        rc = _lib.lib().rm_match(self._h, trace_json, C.byref(out))
        if rc != 0:
            raise RuntimeError(_lib.last_error())
        try:
            return C.string_at(out.value).decode("utf-8")
        finally:
            _lib.lib().rm_free(out)

    def MatchMany(self, trace_jsons):
        """Batched Match: many traces in one GPU pass.  The replies come back in one buffer
        (rm_match_batch_packed) and are decoded out of one memoryview: one allocation and one free
        for the batch instead of one string_at / decode / rm_free per reply."""
        n = len(trace_jsons)
        if n == 0:
            return []
        try:
            arr = (C.c_char_p * n)(*trace_jsons)   # bytes, as the service receives them
        except TypeError:
            arr = (C.c_char_p * n)(*[t.encode("utf-8") if isinstance(t, str) else t for t in trace_jsons])
        off = (C.c_uint64 * (n + 1))()
        buf = C.c_void_p()
        rc = _lib.lib().rm_match_batch_packed(self._h, arr, n, C.byref(buf), off)
        if rc != 0:
            raise RuntimeError(_lib.last_error())
        try:
            o = list(off)
            mv = memoryview((C.c_char * o[n]).from_address(buf.value)).cast("B")
            return [str(mv[o[i]:o[i + 1]], "utf-8") for i in range(n)]
        finally:
            _lib.lib().rm_free(buf)

    def last_timing(self):
        """Host wall ms of the last uncoalesced MatchMany: parse, stage, engine, download, format, total."""
        out = (C.c_double * 6)()
        if _lib.lib().rm_matcher_timing(self._h, out) != 0:
            raise RuntimeError(_lib.last_error())
        return dict(zip(("parse_ms", "stage_ms", "engine_ms", "download_ms", "format_ms", "total_ms"), list(out)))

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().rm_matcher_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def coalesce_stats():
    """Request coalescing counters: batches run, requests served, largest batch, queued now."""
    out = (C.c_uint64 * 4)()
    if _lib.lib().rm_coalesce_stats(out) != 0:
        raise RuntimeError(_lib.last_error())
    return dict(zip(("batches", "requests", "max_batch", "queued"), [int(x) for x in out]))


def write_config(path, graph_path, device=0, coalesce=True, coalesce_window_ms=0.0, ball_radius=None,
                 coalesce_workers=None, modes=None, **meili_default):
    """Write a Valhalla-style config naming the engine's graph file (ball_radius: route-ball radius
    in metres, 0..10000, None = engine default; modes: travel modes whose route tables Configure
    builds besides auto)."""
    conf = {"meili": {"default": dict(meili_default)},
            "reporter_amd": {"graph": _os.path.abspath(graph_path), "device": int(device), "coalesce": bool(coalesce),
                             "coalesce_window_ms": float(coalesce_window_ms)}}
    if ball_radius is not None:
        conf["reporter_amd"]["ball_radius"] = float(ball_radius)
    if coalesce_workers is not None:
        conf["reporter_amd"]["coalesce_workers"] = int(coalesce_workers)
    if modes is not None:
        conf["reporter_amd"]["modes"] = list(modes)
    with open(path, "w") as f:
        _json.dump(conf, f, indent=1)
    return path
