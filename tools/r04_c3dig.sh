#!/bin/bash
# The C3 pipelined digest leg under a kernel trace: k_chunk_digest launches per stream, start / end.
O=gpurun_out/${1:-r04c3dig}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/rp -o run -- python3 bench.py --workload c3 --steps 5 --warmup 5 --no-cpu-baseline --e2e-reps 0 --encode-reps 0 > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
k=$(ls $O/rp/run_kernel_trace.csv $O/rp/*/run_kernel_trace.csv 2>/dev/null | head -1)
python3 - "$k" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1]))]
dig = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"].split("(")[0][-28:]) for r in rows
             if "k_chunk_digest" in r["Kernel_Name"] or "k_chunk_hist" in r["Kernel_Name"] or "k_scan_f" in r["Kernel_Name"])
t0 = [d for d in dig if "digest" in d[3]][-12][0]
for s, e, st, n in dig:
    if s >= t0 - 5e6 and ("digest" in n or "hist" in n):
        print(f"{(s - t0) / 1e6:9.2f} +{(e - s) / 1e6:7.2f} s{st} {n}")
sc = [d for d in dig if "k_scan_f" in d[3] and d[0] >= t0]
print("k_scan_f in window:", len(sc), "first", (sc[0][0] - t0) / 1e6 if sc else None, "last", (sc[-1][0] - t0) / 1e6 if sc else None)
PY
