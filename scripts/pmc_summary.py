"""Summarise rocprofv3 outputs (kernel stats + separate PMC passes) per kernel.

    python scripts/pmc_summary.py gpurun_out profiles/r01 --config C2 --traces 10000

Writes <out>/kernel_stats.md, <out>/pmc_summary.json and <out>/pmc_routes_<cfg>.json
(the HBM bytes per k_routes launch bench.py reads as roofline.traffic).

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reads exactly 1/2 of a wide coalesced read's bytes, so the
read side is doubled ("corrected"); the uncorrected value is kept beside it
because the route kernel's 16-B gathers are not the calibrated access shape.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def short(name):
    n = name.replace("rm::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def load_pmc(d):
    per = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("out")
    ap.add_argument("--config", default="C2")
    ap.add_argument("--traces", type=int, default=10000)
    ap.add_argument("--streams", type=int, default=2, help="concurrent parts the profiled bench ran (bench --streams)")
    ap.add_argument("--turn-penalty", type=float, default=0.0, help="turn_penalty_factor of the profiled bench")
    ap.add_argument("--tag", default=None, help="output pmc_<tag>.json instead of pmc_routes_<config>.json")
    ap.add_argument("--what", default="python bench.py --steps 10 --warmup 2 --no-cpu-baseline",
                    help="the profiled command, for the kernel-stats title")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    ks = os.path.join(a.src, "prof_kt", "run_kernel_stats.csv")
    stats = list(csv.DictReader(open(ks))) if os.path.exists(ks) else []
    lines = ["| kernel | calls | avg (us) | min (us) | max (us) | % of GPU time |", "|---|---|---|---|---|---|"]
    for r in stats:
        lines.append("| %s | %s | %.1f | %.1f | %.1f | %.2f |" % (short(r["Name"]), r["Calls"], float(r["AverageNs"]) / 1e3,
                                                              float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3,
                                                              float(r["Percentage"])))
    with open(os.path.join(a.out, "kernel_stats.md"), "w") as f:
        f.write("rocprofv3 --kernel-trace --stats of `%s` (%s, %d traces)\n\n" % (a.what, a.config, a.traces))
        f.write("\n".join(lines) + "\n")
    merged = defaultdict(dict)
    for d in sorted(glob.glob(os.path.join(a.src, "pmc_*"))):
        if not os.path.isdir(d):
            continue
        for k, cs in load_pmc(d).items():
            for c, vals in cs.items():
                merged[k][c] = sum(vals) / len(vals)
    summary = {}
    for k, cs in merged.items():
        e = dict(cs)
        if "FETCH_SIZE" in cs:
            e["hbm_read_bytes_raw"] = cs["FETCH_SIZE"] * 1024
            e["hbm_read_bytes_corrected"] = cs["FETCH_SIZE"] * 2 * 1024
        if "WRITE_SIZE" in cs:
            e["hbm_write_bytes"] = cs["WRITE_SIZE"] * 1024
        if "TCC_HIT_sum" in cs and "TCC_MISS_sum" in cs and (cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"]) > 0:
            e["l2_hit_rate"] = cs["TCC_HIT_sum"] / (cs["TCC_HIT_sum"] + cs["TCC_MISS_sum"])
        summary[k] = e
    with open(os.path.join(a.out, "pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    # bench.py's stages (the kernels each stage's HIP-event pair brackets; each runs once per step)
    stage_of = {"candidates": lambda k: k.startswith("k_candidates_"),
                "routes": lambda k: k == "k_src_items" or k.startswith("k_routes_"),
                "viterbi": lambda k: k.startswith("k_viterbi"),
                "paths": lambda k: k.startswith("k_paths_"),
                "segments": lambda k: k in ("k_rec_slot", "k_seg_wave")}

    def stage_entry(kernels):
        tot = lambda key: sum(summary[k].get(key, 0) for k in kernels)
        hits, miss = tot("TCC_HIT_sum"), tot("TCC_MISS_sum")
        return {"kernels": sorted(kernels),
                "hbm_bytes_per_launch": (tot("hbm_read_bytes_corrected") + tot("hbm_write_bytes")) or None,
                "hbm_read_bytes_raw": tot("hbm_read_bytes_raw"), "hbm_write_bytes": tot("hbm_write_bytes"),
                "l2_hit_rate": hits / (hits + miss) if hits + miss else None,
                "valu_instrs": tot("SQ_INSTS_VALU") or None, "salu_instrs": tot("SQ_INSTS_SALU") or None,
                "waves": tot("SQ_WAVES") or None}

    stages = {n: stage_entry([k for k in summary if f(k)]) for n, f in stage_of.items()}
    import hashlib
    src = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "reporter_amd", "csrc", "engine.hip")
    sha = hashlib.sha256(open(src, "rb").read()).hexdigest()[:16]
    rt = dict(stages["routes"])
    rt.update({"config": a.config, "traces": a.traces, "streams": a.streams, "engine_sha": sha, "read_factor": 2,
               "turn_penalty": a.turn_penalty,
               "stages": stages,
               "note": "per-step sums of per-dispatch averages from separate --pmc passes; read side doubled per "
                       "MI355X_MICROARCH.md HBM, which profiles/r02/calib confirms for 16-B random gathers "
                       "(one 128-B line request per miss); top-level fields = the routes (K2) stage"})
    with open(os.path.join(a.out, "pmc_%s.json" % (a.tag or "routes_" + a.config.lower())), "w") as f:
        json.dump(rt, f, indent=1)
    for k in sorted(summary, key=lambda x: -summary[x].get("FETCH_SIZE", 0))[:12]:
        e = summary[k]
        print("%-22s fetchKB=%-12.0f writeKB=%-10.0f L2hit=%-6s waves=%s" % (
            k, e.get("FETCH_SIZE", 0), e.get("WRITE_SIZE", 0),
            "%.3f" % e["l2_hit_rate"] if "l2_hit_rate" in e else "-", e.get("SQ_WAVES", "-")))


if __name__ == "__main__":
    main()
