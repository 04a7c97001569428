#!/bin/bash
# The driver's exact bench command, plain and under a rocprofv3 kernel trace,
# plus the GPU test suite.  Writes gpurun_out/<tag>/.
#   tools/driver_trace.sh <tag> [bench args...]   (default: --gpus 1 --steps 20 --warmup 5)
set -e
TAG=${1:-r02}
shift || true
ARGS=${*:-"--gpus 1 --steps 20 --warmup 5"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"

echo "[1/3] pytest -m gpu"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
tail -2 "$OUT/pytest_gpu.log"

echo "[2/3] bench (driver command): python3 bench.py $ARGS"
timeout -k 10 300 python3 bench.py $ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
cut -c1-400 "$OUT/bench.json"

echo "[3/3] rocprofv3 --kernel-trace --stats of the same command"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ktrace" -o run -- \
    python3 bench.py $ARGS > "$OUT/ktrace_bench.json" 2> "$OUT/ktrace.err"
cut -c1-400 "$OUT/ktrace_bench.json"
python tools/kstats.py "$OUT/ktrace/run_kernel_trace.csv" > "$OUT/kernel_summary.txt"
head -12 "$OUT/kernel_summary.txt"
echo done
