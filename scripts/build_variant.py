"""Build an experiment variant of libreporter_match.so with extra -D flags (diagnostic).

    python scripts/build_variant.py NAME -DRM_LANE_CAP=24 ...
    python scripts/build_variant.py NAME --src path/to/engine_variant.hip [-D...]
    python scripts/build_variant.py NAME --all -DFLAG ...   (every source with the flags)

Output: variants/NAME.so (git-ignored, travels to the GPU box).  Load it with
REPORTER_MATCH_LIB=variants/NAME.so (reporter_amd/_lib.py).
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from reporter_amd import build  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
src = os.path.join(build.CSRC, "engine.hip")
if "--src" in defs:
    k = defs.index("--src")
    src = os.path.abspath(defs[k + 1])
    defs = defs[:k] + defs[k + 2:]
all_src = "--all" in defs
defs = [d for d in defs if d != "--all"]
out_dir = os.path.join(ROOT, "variants")
os.makedirs(out_dir, exist_ok=True)
build.build()  # the other objects are shared with the product build
obj = os.path.join(out_dir, name + "_engine.o")
cmd = [build._hipcc()] + build._flags() + defs + ["-I" + build.CSRC, "-c", src, "-o", obj]
subprocess.run(cmd, check=True)
objs = [obj]
for s in build.SOURCES:
    if s == "engine.hip":
        continue
    if not all_src:
        objs.append(os.path.join(build.OBJ, s + ".o"))
        continue
    o = os.path.join(out_dir, name + "_" + s + ".o")
    if s.endswith(".hip") or s == "capi.cpp":
        c = [build._hipcc()] + build._flags() + defs + ["-c", os.path.join(build.CSRC, s), "-o", o]
    else:
        c = ["g++", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall"] + defs + \
            ["-I" + os.path.join(ROOT, "include"), "-c", os.path.join(build.CSRC, s), "-o", o]
    subprocess.run(c, check=True)
    objs.append(o)
lib = os.path.join(out_dir, name + ".so")
subprocess.run([build._hipcc(), "--offload-arch=" + build.ARCH, "-shared", "-o", lib] + objs +
               ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib", "-lpthread", "-lz"], check=True)
for o in objs:
    if o.startswith(out_dir):
        os.remove(o)
print(lib)
