"""Summarise a rocprofv3 rocpd database (or kernel_trace CSV) per kernel:
calls, total/avg/min/max duration (us).  Usage: python tools_kstats.py <db|csv>"""
import csv
import sqlite3
import sys
from collections import defaultdict


def rows(path):
    if path.endswith(".db"):
        db = sqlite3.connect(path)
        for name, start, end in db.execute("select name, start, end from kernels order by start"):
            yield name, int(start), int(end)
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                yield r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])


def main(path):
    d = defaultdict(list)
    seq = list(rows(path))
    for name, s, e in seq:
        short = name.split("(")[0].replace("void ", "")
        d[short].append((e - s) / 1000.0)
    tot = sum(sum(v) for v in d.values())
    print(f"{'kernel':48s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} {'pct':>6s}")
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k[:48]:48s} {len(v):6d} {sum(v):10.1f} {sum(v)/len(v):9.2f} {min(v):9.2f} {max(v):9.2f} {100*sum(v)/tot:6.1f}")
    # gaps between consecutive kernels of the chunking pipeline (first 12)
    return seq


if __name__ == "__main__":
    seq = main(sys.argv[1])
    if "--seq" in sys.argv:
        base = seq[0][1]
        for name, s, e in seq[-14:]:
            print(f"{(s-base)/1000:12.1f} {(e-s)/1000:9.1f}  {name.split('(')[0][:60]}")
