"""Per-kernel table of the PMC passes written by scripts/pmc_probe.sh (diagnostic)."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
per = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "p*", "*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("rm::(anonymous namespace)::", "").split("(")[0]
        per[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
rows = []
for k, cs in per.items():
    e = {c: sum(v) / len(v) for c, v in cs.items()}
    rows.append((e.get("GRBM_GUI_ACTIVE", 0), k, e))
rows.sort(reverse=True)
for _, k, e in rows[:14]:
    w = max(e.get("SQ_WAVES", 1), 1)
    print("%-28s" % k[:28], " ".join("%s=%.4g" % (c, v) for c, v in sorted(e.items())))
    print("    per-wave: cycles=%.0f valu=%.1f vmem_rd=%.1f vmem_wr=%.1f lds=%.1f salu=%.1f  busy-frac(valu)=%.3f"
          " vmem-level=%.2f  tcp-lat/req=%.0f" % (
              4 * e.get("SQ_WAVE_CYCLES", 0) / w, e.get("SQ_INSTS_VALU", 0) / w, e.get("SQ_INSTS_VMEM_RD", 0) / w,
              e.get("SQ_INSTS_VMEM_WR", 0) / w, e.get("SQ_INSTS_LDS", 0) / w, e.get("SQ_INSTS_SALU", 0) / w,
              e.get("SQ_ACTIVE_INST_VALU", 0) / max(e.get("SQ_WAVE_CYCLES", 1), 1),
              e.get("SQ_INST_LEVEL_VMEM", 0) / max(e.get("SQ_WAVE_CYCLES", 1), 1),
              e.get("TCP_TCC_READ_REQ_LATENCY_sum", 0) / max(e.get("TCP_TCC_READ_REQ_sum", 1), 1)))
