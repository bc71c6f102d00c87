"""Build libreporter_match.so (HIP for gfx950 + C++ host runtime) in-tree.

    python -m reporter_amd.build            # incremental
    python -m reporter_amd.build --force

The shared library lands next to this file so it travels with the repo snapshot
to the GPU box.  No PyTorch and no JIT cache are involved.
"""
import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OBJ = os.path.join(HERE, "_obj")
LIB = os.path.join(HERE, "libreporter_match.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
SOURCES = ["engine.hip", "stages.hip", "capi.cpp", "graph.cpp", "graph_osm.cpp", "osm_pbf.cpp", "osm_city.cpp", "world.cpp", "balls.cpp"]
HEADERS = ["engine.hpp", "graph.hpp", "json.hpp", "rm_common.hpp", "balls.hpp", "serve_policy.hpp", "trace_json.hpp",
           "host_pool.hpp", "osm_model.hpp"]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found; the engine needs ROCm to build")


def _flags():
    # -ffp-contract=off: bit-exact fp32/fp64 against oracle/ (no FMA contraction)
    return ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "-Wall",
            "--offload-arch=" + ARCH, "-I" + os.path.join(ROOT, "include")]


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _compile(src, force):
    s = os.path.join(CSRC, src)
    o = os.path.join(OBJ, src + ".o")
    deps = [s] + [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(ROOT, "include", "reporter_match.h")]
    if not force and not _newer(o, deps):
        return o
    if src.endswith(".hip") or src == "capi.cpp":
        cmd = [_hipcc()] + _flags() + ["-c", s, "-o", o]
    else:  # pure host C++: no device pass
        cmd = ["g++", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall", "-c", s, "-o", o]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("compile failed: %s\n%s%s" % (" ".join(cmd), r.stdout, r.stderr))
    return o


def build(force=False, verbose=False):
    os.makedirs(OBJ, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=min(4, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), SOURCES))
    if force or _newer(LIB, objs):
        cmd = [_hipcc(), "--offload-arch=" + ARCH, "-shared", "-o", LIB] + objs + ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib", "-lpthread", "-lz"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed: %s\n%s%s" % (" ".join(cmd), r.stdout, r.stderr))
        if verbose:
            print("built", LIB)
    build_tools(force)
    build_python_ext(force)
    return LIB


def build_python_ext(force=False):
    """valhalla/_match (SegmentMatcher.Match in one CPython call), linked against the in-tree
    library; skipped when the Python headers are absent (Match then stays on ctypes)."""
    import sysconfig
    inc = sysconfig.get_paths().get("include")
    if not inc or not os.path.exists(os.path.join(inc, "Python.h")):
        return None
    src = os.path.join(ROOT, "valhalla", "_match.c")
    out = os.path.join(ROOT, "valhalla", "_match" + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
    if not force and not _newer(out, [src, LIB, os.path.join(ROOT, "include", "reporter_match.h")]):
        return out
    cmd = ["gcc", "-O2", "-shared", "-fPIC", "-Wall", "-I" + inc, src, "-o", out, "-L" + HERE, "-lreporter_match",
           "-Wl,-rpath,$ORIGIN/../reporter_amd"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("valhalla._match build failed: %s\n%s%s" % (" ".join(cmd), r.stdout, r.stderr))
    return out


CLIENT = os.path.join(HERE, "bin", "rm_svc_client")


def build_tools(force=False):
    """The multi-threaded C-ABI service client bench.py measures the library with (no Python
    between the calls): reporter_amd/bin/rm_svc_client, linked against the in-tree library."""
    src = os.path.join(CSRC, "svc_client.cpp")
    os.makedirs(os.path.dirname(CLIENT), exist_ok=True)
    if not force and not _newer(CLIENT, [src, LIB, os.path.join(ROOT, "include", "reporter_match.h")]):
        return CLIENT
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", src, "-o", CLIENT, "-L" + HERE, "-lreporter_match",
           "-Wl,-rpath,$ORIGIN/..", "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("client build failed: %s\n%s%s" % (" ".join(cmd), r.stdout, r.stderr))
    return CLIENT


def build_oracle(force=False):
    """Compile oracle/ (test infrastructure) with its own Makefile."""
    d = os.path.join(ROOT, "oracle")
    args = ["make", "-C", d] + (["-B"] if force else [])
    r = subprocess.run(args, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + r.stdout + r.stderr)
    return os.path.join(d, "liboracle_meili.so")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force, verbose=True))
    print(build_oracle(force=a.force))
    sys.exit(0)
