#!/bin/bash
# Round artifacts on the GPU box: bench lines (C1..C4), the rocprofv3 kernel
# summary of the C1 bench, and the FETCH_SIZE pass behind roofline.traffic.
#   tools/round_profile.sh <tag>      (writes gpurun_out/<tag>/...)
# Every GPU step has its own time limit; the script stops at the first failure.
set -e
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"

echo "[1/5] bench c1 (default run, cpu baseline + e2e leg)"
timeout -k 10 300 python bench.py > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err"
tail -1 "$OUT/bench_c1.json" | cut -c1-300

echo "[2/5] bench c2 / c3"
timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline --e2e-reps 0 > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
timeout -k 10 200 python bench.py --workload c3 --no-cpu-baseline --e2e-reps 0 > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err"

echo "[3/5] bench c4 (host path, PCIe-inclusive)"
timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 --cpu-seconds 10 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
tail -1 "$OUT/bench_c4.json" | cut -c1-300

echo "[4/5] rocprofv3 kernel trace + stats (c1)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ktrace" -o run -- \
    python3 bench.py --steps 100 --warmup 200 --streams 1 --no-cpu-baseline --e2e-reps 0 --digest-reps 0 > "$OUT/ktrace_bench.json" 2> "$OUT/ktrace.err"
python tools/kstats.py "$OUT/ktrace/run_kernel_trace.csv" > "$OUT/kernel_summary.txt"; head -10 "$OUT/kernel_summary.txt"

echo "[5/5] rocprofv3 PMC FETCH_SIZE (c1)"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc" -o run -- \
    python3 bench.py --steps 5 --warmup 1 --streams 1 --no-cpu-baseline --e2e-reps 0 --digest-reps 0 > "$OUT/pmc_bench.json" 2> "$OUT/pmc.err"
python tools/pmc_summary.py "$OUT/pmc" k_scan | tee "$OUT/pmc_summary.txt"
echo done
