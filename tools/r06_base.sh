#!/bin/bash
# Round-6 baseline on this box: GPU suite, driver command x3, C3 line.
TAG=${1:-r06base}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
echo "[1] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -20 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
echo "[2] driver command x3"
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver_bench_$i.json" 2> "$OUT/driver_bench_$i.err" || exit 1
  cut -c1-120 "$OUT/driver_bench_$i.json"
done
echo "[3] C3"
timeout -k 10 300 python3 bench.py --workload c3 --no-cpu-baseline > "$OUT/bench_c3.json" 2> "$OUT/bench_c3.err" || exit 1
cut -c1-200 "$OUT/bench_c3.json"
echo done
