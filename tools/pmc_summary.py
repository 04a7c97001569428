"""Average PMC counters per kernel from rocprofv3 --pmc output directories.

    python tools/pmc_summary.py <dir> [kernel] [--glob PATTERN]

Reads <dir>/<PATTERN>/**/run_counter_collection.csv (PATTERN default "p*")
and <dir>/run_counter_collection.csv; a kernel matches by its bare name
(namespace and template arguments stripped)."""
import collections
import csv
import glob
import re
import sys

args = sys.argv[1:]
pat = "p*"
if "--glob" in args:
    i = args.index("--glob")
    pat = args[i + 1]
    del args[i:i + 2]
d = args[0]
ksub = args[1] if len(args) > 1 else "k_scan"


def bare(kernel_name):
    s = kernel_name.split("(")[0]
    s = re.sub(r"<.*>", "", s).split(" ")[-1]
    return s.split("::")[-1]


files = sorted(set(glob.glob(f"{d}/{pat}/**/run_counter_collection.csv", recursive=True)
                   + glob.glob(f"{d}/run_counter_collection.csv")))
agg = collections.defaultdict(list)
for p in files:
    for r in csv.DictReader(open(p)):
        if bare(r["Kernel_Name"]) == ksub:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} n={len(v):3d} avg={sum(v)/len(v):.5g}")
if not agg:
    print(f"no rows for {ksub} in {len(files)} file(s)")
