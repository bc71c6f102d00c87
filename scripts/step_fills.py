"""Runtime fill / copy blits (__amd_rocclr_fillBufferAligned / copyBuffer) per pipeline run from a
rocprofv3 --kernel-trace SQLite output: dispatches between consecutive k_states launches (one
k_states per run), so the cold start (graph upload, first allocations) separates from the steady
state.   python scripts/step_fills.py <dir or .db>"""
import glob, os, sqlite3, sys

p = sys.argv[1]
dbs = [p] if p.endswith(".db") else glob.glob(os.path.join(p, "**", "*.db"), recursive=True)
con = sqlite3.connect(dbs[0])
cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
name = "name" if "name" in cols else "kernel_name"
rows = con.execute("select %s, start, end from kernels order by start" % name).fetchall()
starts = [i for i, r in enumerate(rows) if "k_states" in r[0]]
print("runs (k_states launches): %d; dispatches before the first: %d" % (len(starts), starts[0] if starts else len(rows)))
pre = rows[:starts[0]] if starts else rows
print("before run 1: fills %d, copies %d" % (sum("fillBuffer" in r[0] for r in pre), sum("copyBuffer" in r[0] for r in pre)))
for k, i0 in enumerate(starts):
    i1 = starts[k + 1] if k + 1 < len(starts) else len(rows)
    seg = rows[i0:i1]
    f = [r for r in seg if "fillBuffer" in r[0]]
    c = [r for r in seg if "copyBuffer" in r[0]]
    own = [r for r in seg if "rocclr" not in r[0]]
    print("run %2d: kernels %3d  fills %3d (%.1f us)  copies %3d (%.1f us)  span %.3f ms" % (
        k + 1, len(own), len(f), sum(r[2] - r[1] for r in f) / 1e3, len(c), sum(r[2] - r[1] for r in c) / 1e3,
        (seg[-1][2] - seg[0][1]) / 1e6))
