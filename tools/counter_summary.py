"""Summarise rocprofv3 counter CSVs of tools/counters.sh: median per-dispatch value per counter for a kernel."""
import csv, glob, os, statistics, sys
d, kern = sys.argv[1], sys.argv[2]
vals = {}
for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(p)):
        if kern in row.get("Kernel_Name", ""):
            vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
for k in sorted(vals):
    print(f"{k:28s} {statistics.median(vals[k]):16.0f}  (n={len(vals[k])})")
