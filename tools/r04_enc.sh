#!/bin/bash
# Encode leg on C1 vs C2 under a kernel trace: per-kernel time per GiB of chunk bytes.
O=gpurun_out/${1:-r04enc}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
for wl in c1 c2; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/$wl -o run --output-format csv -- python bench.py --workload $wl --steps 5 --warmup 5 --digest-reps 0 --e2e-reps 0 --no-cpu-baseline --no-parity --encode-reps 5 > $O/$wl.json 2>$O/$wl.err || { tail -5 $O/$wl.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$wl.json')); e=d['encode']; print('$wl encode', e['value'], 'GiB/s', e['ms_per_pass'], 'ms/pass', e['blobs'], 'blobs')"
  f=$(ls $O/$wl/run_kernel_stats.csv $O/$wl/*/run_kernel_stats.csv 2>/dev/null | head -1)
  python - "$f" "$wl" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"].split("(")[0].replace("void ", "")
    if "enc::" in n or "copyBuffer" in n:
        print(f"  {sys.argv[2]} {n:40s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.1f} total_ms {float(r['TotalDurationNs'])/1e6:8.2f}")
PY
done
