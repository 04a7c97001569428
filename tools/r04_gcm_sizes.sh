#!/bin/bash
# k_gcm ms per GiB against the call size (a fixed tail shows as a falling ms/GiB): GCM-only, random data.
O=gpurun_out/${1:-r04gcmsz}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for mib in 256 512 1024 2048 4096; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/s$mib -o run --output-format csv -- python tools/encode_bench.py --size-mib $mib --reps 3 --kinds random --labels gcm > $O/s$mib.log 2>$O/s$mib.err || { tail -5 $O/s$mib.err; exit 1; }
  f=$(ls $O/s$mib/run_kernel_stats.csv $O/s$mib/*/run_kernel_stats.csv 2>/dev/null | head -1)
  python - "$f" "$mib" <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    if "k_gcm" in row["Name"]:
        avg = float(row["AverageNs"]) / 1e6
        print(f"{sys.argv[2]:>5s} MiB: k_gcm avg {avg:7.3f} ms = {avg * 1024 / int(sys.argv[2]):6.3f} ms/GiB")
PY
done
