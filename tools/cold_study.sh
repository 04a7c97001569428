#!/bin/bash
# How the pass rate evolves from a cold start (the driver runs --warmup 5):
# kernel traces of long runs from 5 warm-up passes, one and two streams,
# printed as per-bin pass rates.   tools/cold_study.sh <tag> [bench args...]
set -e
TAG=${1:-cold}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for st in 2 1; do
    echo "[streams $st]"
    timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/s$st" -o run -- \
        python3 bench.py --steps 600 --warmup 5 --streams $st --no-cpu-baseline --e2e-reps 0 --digest-reps 0 $* \
        > "$OUT/s$st.json" 2> "$OUT/s$st.err"
    python tools/timeline.py "$OUT/s$st/run_kernel_trace.csv" --warmup 0 --steps 600 --bins 25 | tee "$OUT/s$st.txt"
    python tools/timeline.py "$OUT/s$st/run_kernel_trace.csv" --warmup 5 --steps 40 > "$OUT/s${st}_first.txt"
done
echo done
