#!/bin/bash
# Round-4 evidence on the current code: GPU suite, smoke, the driver's exact bench command plain and under a
# rocprofv3 kernel trace (+ per-pass timeline), the roofline loop alone under a trace (its k_scan average is the
# line's roofline.kernel_avg_ms), bench lines C1-C4 / c4f / c4b, a FETCH_SIZE pass of the C1 scan, and the N = 2
# rank rehearsal on one GPU.
#   tools/r04_final.sh <tag>
TAG=${1:-r04z}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
echo "[1] pytest -m gpu"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -20 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
echo "[2] driver command"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver_bench.json" 2> "$OUT/driver_bench.err" || exit 1
cut -c1-200 "$OUT/driver_bench.json"
echo "[3] rocprofv3 --kernel-trace --stats of the driver command"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/driver_ktrace" -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver_ktrace_bench.json" 2> "$OUT/driver_ktrace.err" || exit 1
f=$(ls $OUT/driver_ktrace/*/run_kernel_trace.csv $OUT/driver_ktrace/run_kernel_trace.csv 2>/dev/null | head -1)
python tools/kstats.py "$f" > "$OUT/driver_kernel_summary.txt"
python tools/timeline.py "$f" --warmup 5 --steps 20 > "$OUT/driver_timeline.txt" 2>&1 || true
tail -6 "$OUT/driver_timeline.txt"
echo "[4] the roofline loop alone under a trace (20 single-stream passes, nothing before them)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/roofline_ktrace" -o run -- \
    python3 bench.py --roofline-only --steps 20 --warmup 0 > "$OUT/roofline_only_bench.json" 2> "$OUT/roofline_only.err" || exit 1
f=$(ls $OUT/roofline_ktrace/*/run_kernel_trace.csv $OUT/roofline_ktrace/run_kernel_trace.csv 2>/dev/null | head -1)
python tools/kstats.py "$f" > "$OUT/roofline_kernel_summary.txt"
head -4 "$OUT/roofline_kernel_summary.txt"
python -c "import json; d=json.load(open('$OUT/roofline_only_bench.json')); print('line kernel_avg_ms', d['roofline']['kernel_avg_ms'], 'frac', d['roofline']['frac'])"
echo "[5] bench lines"
timeout -k 10 400 python3 bench.py > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err" || exit 1
cut -c1-200 "$OUT/bench_c1.json"
for wl in c2 c3; do
    timeout -k 10 300 python3 bench.py --workload $wl --no-cpu-baseline > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" || exit 1
    cut -c1-200 "$OUT/bench_$wl.json"
done
timeout -k 10 400 python3 bench.py --workload c4 --steps 3 --warmup 1 --cpu-seconds 10 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" || exit 1
timeout -k 10 400 python3 bench.py --workload c4f --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench_c4f.json" 2> "$OUT/bench_c4f.err" || exit 1
timeout -k 10 500 python3 bench.py --workload c4b --steps 5 --warmup 2 > "$OUT/bench_c4b.json" 2> "$OUT/bench_c4b.err" || exit 1
for r in 2 3; do  # run-to-run spread of the backup leg (reads from the page cache vary)
  timeout -k 10 500 python3 bench.py --workload c4b --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_c4b_$r.json" 2> "$OUT/bench_c4b_$r.err" || exit 1
done
for wl in c4 c4f c4b c4b_2 c4b_3; do cut -c1-160 "$OUT/bench_$wl.json"; done
echo "[6] N = 2 ranks rehearsed on one GPU (gloo), parity AND + CPU baseline"
BENCH_REHEARSE_ONE_GPU=1 timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 --cpu-threads 16 > "$OUT/bench_n2_rehearsal.json" 2> "$OUT/bench_n2.err" || exit 1
cut -c1-200 "$OUT/bench_n2_rehearsal.json"
echo "[7] FETCH_SIZE pass of the C1 scan"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 bench.py --roofline-only --steps 5 --warmup 0 > "$OUT/pmc_fetch.json" 2> "$OUT/pmc_fetch.err" || echo "pmc pass failed"
python tools/pmc_summary.py "$OUT/pmc_fetch" k_scan || true
echo done
