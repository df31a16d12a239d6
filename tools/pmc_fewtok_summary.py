"""Summarise FETCH_SIZE / WRITE_SIZE passes per (kernel, grid): median HBM bytes per launch (gfx950: 2 x FETCH_SIZE +
WRITE_SIZE, KiB -> bytes; MI355X_MICROARCH.md §HBM).  Usage: python tools/pmc_fewtok_summary.py <fetch_dir> <write_dir>"""
import collections
import csv
import glob
import os
import statistics
import sys


def load(d, name):
    out = collections.defaultdict(list)
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if r.get("Counter_Name") == name:
                out[(r["Kernel_Name"].split("(")[0][:48], r["Grid_Size"])].append(float(r["Counter_Value"]))
    return out


f, w = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE")
print(f"{'kernel':48s} {'grid':>8s} {'n':>5s} {'HBM MB/launch':>14s} {'read MB':>8s} {'write MB':>9s}")
for key in sorted(f, key=lambda k: -len(f[k])):
    if key not in w or len(f[key]) < 10:
        continue
    fk, wk = statistics.median(f[key]), statistics.median(w[key])
    print(f"{key[0]:48s} {key[1]:>8s} {len(f[key]):5d} {(2 * fk + wk) * 1024 / 1e6:14.2f} {2 * fk * 1024 / 1e6:8.2f} "
          f"{wk * 1024 / 1e6:9.2f}")
