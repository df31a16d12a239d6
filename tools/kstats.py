"""Per-kernel duration summary from a rocprofv3 SQLite results DB (or kernel_stats/kernel_trace CSV).
Usage: python tools/kstats.py <results.db|kernel_trace.csv> [name-substring]"""
import collections
import csv
import sqlite3
import sys


def rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, start, end, dur in c.execute("select name, start, \"end\", duration from kernels order by start"):
            yield name, int(start), int(end), int(dur)
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                yield r["Kernel_Name"], s, e, e - s


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    d = collections.defaultdict(list)
    seq = []
    for name, s, e, dur in rows(path):
        short = name.split("(")[0][:90]
        if sub in name:
            d[short].append(dur)
            seq.append((s, e))
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        v = sorted(v)
        print(f"{len(v):6d}  avg {sum(v)/len(v)/1e3:9.2f} us  med {v[len(v)//2]/1e3:9.2f} us  min {v[0]/1e3:9.2f} us  {k}")
    if len(seq) > 1:
        gaps = sorted(b[0] - a[1] for a, b in zip(seq, seq[1:]))
        print(f"gap between matching kernels: median {gaps[len(gaps)//2]/1e3:.2f} us")


if __name__ == "__main__":
    main()
