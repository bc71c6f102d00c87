"""Print the per-kernel table from a rocprofv3 --stats CSV (scripts/kt.sh output)."""
import csv
import glob
import sys

f = glob.glob((sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/kt") + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("rm::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    print("%-48s %6s %9.1f us" % (n[:48], r["Calls"], float(r["AverageNs"]) / 1e3))
