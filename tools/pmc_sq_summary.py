"""Summarise tools/pmc_sq.sh passes: counter totals for the profiled tree kernel, per wave-sample."""
import csv
import glob
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_sq"
samples = int(sys.argv[2]) if len(sys.argv) > 2 else 882
tot = {}
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "tree_prof_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
waves = tot.get("SQ_WAVES", 1.0)
for k in sorted(tot):
    print(f"{k:28s} {tot[k]:14.6g}   per wave-sample {tot[k] / waves / samples:10.1f}")
