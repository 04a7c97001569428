"""Average PMC counters per kernel from tools/pmc.sh output: python tools/pmc_summary.py <dir> [kernel-substring]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
ksub = sys.argv[2] if len(sys.argv) > 2 else "k_scan"
agg = collections.defaultdict(list)
for p in sorted(glob.glob(f"{d}/p*/run_counter_collection.csv") + glob.glob(f"{d}/run_counter_collection.csv")):
    for r in csv.DictReader(open(p)):
        name = r["Kernel_Name"].split("(")[0].split(" ")[-1]
        if name == ksub or name.endswith("::" + ksub):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} n={len(v):3d} avg={sum(v)/len(v):.5g}")
