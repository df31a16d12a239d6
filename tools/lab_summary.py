"""Per-kernel median of every counter in a tools/lab_counters.sh output dir, plus derived ratios."""
import collections, csv, glob, os, re, statistics, sys
d = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(p)):
        name = re.sub(r"\(.*", "", row.get("Kernel_Name", ""))[:90]
        vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in vals.items():
    med = {c: statistics.median(v) for c, v in cs.items()}
    print(f"== {k}")
    for c in sorted(med):
        print(f"   {c:28s} {med[c]:16.0f}")
    g = med.get("GRBM_GUI_ACTIVE", 0) / 8
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in med:
        simds = 1024
        print(f"   -> cycles/XCD {g:.0f}; MFMA busy per SIMD {med['SQ_VALU_MFMA_BUSY_CYCLES'] / simds / g:.3f}")
    wc = med.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
            if c in med:
                print(f"   -> {c}/WAVE_CYCLES {med[c] / wc:.3f}")
