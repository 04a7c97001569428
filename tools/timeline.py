"""Print the last N cdc:: kernels of a rocprofv3 kernel-trace CSV as a timeline
(start, end, duration in us, queue): python tools/timeline.py <csv> [N]"""
import csv
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = [(r["Kernel_Name"].split("(")[0].replace("cdc::", ""), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
         r.get("Queue_Id")) for r in csv.DictReader(open(path))]
rows = sorted([r for r in rows if r[0].startswith("k_")], key=lambda r: r[1])[-n:]
base = rows[0][1]
for name, s, e, q in rows:
    print(f"{(s - base) / 1000:9.1f} {(e - base) / 1000:9.1f} {(e - s) / 1000:7.1f}  {name:8s} q={q}")
