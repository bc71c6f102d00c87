"""Per-batch timeline of a rocprofv3 kernel trace of the coalesced service (scripts/gpu_svc_prof.sh):
for each engine run (one k_states launch), the span from its first to its last kernel, the summed
kernel time, the number of launches and the idle gaps between them, averaged over the runs; and
the average duration of each kernel in a run.   python scripts/svc_timeline.py gpurun_out/svcprof"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
kf = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
rows = []
with open(kf[0]) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r.get("Queue_Id", 0) or 0)))
rows.sort()
mf = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
copies = []
if mf:
    with open(mf[0]) as f:
        for r in csv.DictReader(f):
            copies.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", "")))
copies.sort()
def short(n):
    import re
    m = re.search(r"(k_\w+(?:<[^>]*>)?|__amd\w+)", n)
    return m.group(1) if m else n[:40]
runs, cur = [], None
for s, e, n, q in rows:
    sn = short(n)
    if sn.startswith("k_states"):
        cur = []
        runs.append(cur)
    if cur is not None:
        cur.append((s, e, sn))
runs = [r for r in runs[5:] if len(r) > 5]   # skip warm-up edges
per_k = defaultdict(list)
spans, busy, nk = [], [], []
for r in runs:
    spans.append((r[-1][1] - r[0][0]) / 1e3)
    busy.append(sum(e - s for s, e, _ in r) / 1e3)
    nk.append(len(r))
    for s, e, n in r:
        per_k[n].append((e - s) / 1e3)
m = lambda v: sum(v) / max(len(v), 1)
print("runs %d  span %.1f us  kernel busy %.1f us  launches %.1f  (span - busy %.1f us)" % (
    len(runs), m(spans), m(busy), m(nk), m(spans) - m(busy)))
for n, v in sorted(per_k.items(), key=lambda kv: -sum(kv[1])):
    print("  %-40s calls/run %5.2f  avg %7.2f us  per run %7.2f us" % (n, len(v) / len(runs), m(v), sum(v) / len(runs)))
if copies:
    print("memory copies per run: %.2f, avg %.2f us" % (len(copies) / max(len(runs), 1), m([(e - s) / 1e3 for s, e, _ in copies])))
