"""Device timeline of the last c4b step from a rocprofv3 kernel + memory-copy
trace (tools/r03_c4b_trace.sh): per kernel / stream totals, then every event
of at least 0.3 ms (and every digest / GCM launch)."""
import collections
import csv
import sys

d = sys.argv[1]
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 14
rows = list(csv.DictReader(open(f"{d}/c4b_kernel_trace.csv")))
cp = list(csv.DictReader(open(f"{d}/c4b_memory_copy_trace.csv")))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-24:], r["Stream_Id"])
      for r in rows]
ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"][12:], r["Stream_Id"]) for r in cp]
ev.sort()
dig = [x for x in ev if "k_chunk_digest" in x[2]]
t0 = dig[-nb][0] - 15e6
t1 = [x for x in ev if "k_gcm" in x[2]][-1][1]
win = [x for x in ev if t0 <= x[0] <= t1 + 1e6]
agg = collections.defaultdict(lambda: [0, 0.0])
for s, e, n, st in win:
    agg[(n, st)][0] += 1
    agg[(n, st)][1] += (e - s) / 1e6
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:20]:
    print(f"s{k[1]:>2} {k[0]:26s} n={v[0]:5d} ms={v[1]:8.2f}")
print(f"window {(t1 - t0) / 1e6:.2f} ms")
T = win[0][0]
for s, e, n, st in win:
    if e - s >= 0.3e6 or "digest" in n or "gcm" in n:
        print(f"{(s - T) / 1e6:8.2f} +{(e - s) / 1e6:6.2f} s{st} {n}")
