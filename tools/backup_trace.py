"""Per-batch timeline of one cdc_backup_files call from its CDC_BACKUP_TRACE
CSV: python tools/backup_trace.py <trace.csv>.  Times in ms from the call's
start; reads / hashes as first start .. last end over the batch's units."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
by = collections.defaultdict(lambda: collections.defaultdict(list))
other = []
for r in rows:
    t, e, b = float(r["t_s"]) * 1e3, r["event"], int(r["batch"])
    if b < 0:
        other.append((t, e, int(r["bytes"])))
    else:
        by[b][e].append((t, int(r["bytes"])))
cols = [("read", min), ("read_end", max), ("hash_end", max), ("enq_cuts", min), ("dev_h2d", min),
        ("dev_h2d_end", min), ("dev_cuts_end", min), ("dev_dig", min), ("dev_dig_end", min), ("dev_back_end", min),
        ("lists_back", min), ("encode", min), ("encode_end", min), ("callbacks", min), ("callbacks_end", min)]
print("batch  MiB  units " + " ".join(f"{c[0][:11]:>11s}" for c in cols))
for b in sorted(by):
    ev = by[b]
    mib = sum(x[1] for x in ev.get("read", [])) / 2**20
    cells = []
    for name, f in cols:
        v = ev.get(name)
        cells.append(f"{f(x[0] for x in v):11.2f}" if v else f"{'-':>11s}")
    print(f"{b:5d} {mib:5.0f} {len(ev.get('read', [])):6d} " + " ".join(cells))
packs = [t for t, e, _ in other if e == "packfile"]
for t, e, n in other:
    if e != "packfile":
        print(f"{e:10s} {t:9.2f} ms ({n})")
if packs:
    print(f"packfiles: {len(packs)}, first {min(packs):.2f} ms, last {max(packs):.2f} ms")
