#!/bin/bash
# C3 kernel trace (single stream) + a default C1 bench line.
set -e
OUT=gpurun_out/c3p; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- \
    python3 bench.py --workload c3 --steps 100 --warmup 200 --streams 1 --no-cpu-baseline --e2e-reps 0 --digest-reps 0 > "$OUT/kt_bench.json" 2> "$OUT/kt.err"
python tools/kstats.py "$OUT/kt/run_kernel_trace.csv" > "$OUT/kernel_summary.txt"; head -10 "$OUT/kernel_summary.txt"
timeout -k 10 300 python bench.py > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err"
tail -1 "$OUT/bench_c1.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d['cpu_baseline'])"
