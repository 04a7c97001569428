#!/bin/bash
# Final round-2 evidence on the final code (the scan kernels are those of
# r02h, whose SQ/FETCH passes stand): GPU suite, the driver's exact bench
# command plain and under a rocprofv3 kernel trace, and the bench lines.
#   tools/r02_final.sh <tag>
set -e
TAG=${1:-r02i}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "[1] pytest -m gpu"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
tail -2 "$OUT/pytest_gpu.log"
echo "[2] driver command"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver_bench.json" 2> "$OUT/driver_bench.err"
cut -c1-200 "$OUT/driver_bench.json"
echo "[3] rocprofv3 --kernel-trace --stats of the driver command"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/driver_ktrace" -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver_ktrace_bench.json" 2> "$OUT/driver_ktrace.err"
python tools/kstats.py "$OUT/driver_ktrace/run_kernel_trace.csv" > "$OUT/driver_kernel_summary.txt"
python tools/timeline.py "$OUT/driver_ktrace/run_kernel_trace.csv" > "$OUT/driver_timeline.txt" 2>&1 || true
echo "[4] bench lines"
timeout -k 10 400 python3 bench.py > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err"
for wl in c2 c3; do
    timeout -k 10 300 python3 bench.py --workload $wl --no-cpu-baseline > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err"
done
timeout -k 10 400 python3 bench.py --workload c4 --steps 3 --warmup 1 --cpu-seconds 10 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
timeout -k 10 400 python3 bench.py --workload c4f --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench_c4f.json" 2> "$OUT/bench_c4f.err"
echo done
