"""Parse rocprofv3 counter-collection CSVs (FETCH_SIZE / WRITE_SIZE passes) into per-launch HBM bytes.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports 1/2 of the bytes of a wide
coalesced streaming read, so hbm = (2*FETCH_SIZE + WRITE_SIZE) * 1024 bytes (both counters in KiB).
Usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <kernel_substring> <out.json> [M N K [display_name]]
"""
import csv
import glob
import json
import os
import statistics
import sys


def read_counter(d, name, kern):
    vals = []
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(p) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") == name and kern in row.get("Kernel_Name", ""):
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    fdir, wdir, kern, out = sys.argv[1:5]
    shape = [int(x) for x in sys.argv[5:8]] if len(sys.argv) >= 8 else None
    display = sys.argv[8] if len(sys.argv) >= 9 else kern
    mdir = sys.argv[9] if len(sys.argv) >= 10 else None
    tdir = sys.argv[10] if len(sys.argv) >= 11 else None   # kernel-trace pass of the same command
    fetch = read_counter(fdir, "FETCH_SIZE", kern)
    write = read_counter(wdir, "WRITE_SIZE", kern)
    if not fetch or not write:
        print(f"no samples: fetch={len(fetch)} write={len(write)}")
        sys.exit(1)
    f_kib = statistics.median(fetch)
    w_kib = statistics.median(write)
    res = {"kernel": display, "kernel_match": kern, "shape": shape, "launches": [len(fetch), len(write)],
           "FETCH_SIZE_KiB_median": f_kib, "WRITE_SIZE_KiB_median": w_kib,
           "hbm_bytes_per_launch": int((2 * f_kib + w_kib) * 1024),
           "correction": "gfx950: FETCH_SIZE x2 (MI355X_MICROARCH.md §HBM); WRITE_SIZE as reported"}
    if mdir:
        # MFMA busy per SIMD = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs); the
        # effective clock = GRBM_GUI_ACTIVE / 8 / kernel duration (duration from the separate trace pass) (MI355X_MICROARCH.md 'DVFS give-back')
        grbm = read_counter(mdir, "GRBM_GUI_ACTIVE", kern)
        busy = read_counter(mdir, "SQ_VALU_MFMA_BUSY_CYCLES", kern)
        durs = []
        for p in glob.glob(os.path.join(tdir or mdir, "**", "*kernel_trace.csv"), recursive=True):
            with open(p) as f:
                for row in csv.DictReader(f):
                    if kern in row.get("Kernel_Name", ""):
                        durs.append(float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
        if grbm and busy:
            g = statistics.median(grbm) / 8
            res["mfma_busy_per_simd"] = round(statistics.median(busy) / 1024 / g, 4)
            if durs:
                res["effective_clock_ghz"] = round(g / statistics.median(durs), 3)
                res["kernel_ns_profiled"] = statistics.median(durs)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
