#!/bin/bash
# Round-6 evidence on the final code: GPU suite, smoke, the driver's exact bench command (three times, plain) and
# under a rocprofv3 kernel trace (+ per-pass timeline), the roofline loop alone under a trace, bench lines
# C1-C4 (C3 also under a kernel trace) / c4f / c4b (twice) / c4bl, the N = 2 rank rehearsal and the one-rank RCCL run on one GPU, PMC passes of
# the C1 scan (FETCH_SIZE; instruction counts) and of the C3 fused scan (instruction counts).
#   tools/r06_final.sh <tag> [skip-suite]
TAG=${1:-r06final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
if [ "$2" != "skip-suite" ]; then
  echo "[1] pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -20 "$OUT/pytest_gpu.log"; exit 1; }
  tail -1 "$OUT/pytest_gpu.log"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
echo "[2] driver command x3"
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver_bench_$i.json" 2> "$OUT/driver_bench_$i.err" || exit 1
  cut -c1-150 "$OUT/driver_bench_$i.json"
done
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
echo "[5] bench lines"
timeout -k 10 400 python3 bench.py > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err" || exit 1
cut -c1-200 "$OUT/bench_c1.json"
for wl in c2 c3; do
    timeout -k 10 300 python3 bench.py --workload $wl --no-cpu-baseline > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" || exit 1
    cut -c1-200 "$OUT/bench_$wl.json"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c3_ktrace" -o run -- \
    python3 bench.py --workload c3 --steps 50 --warmup 50 --no-cpu-baseline --e2e-reps 0 --digest-reps 0 --encode-reps 0 \
    > "$OUT/c3_ktrace_bench.json" 2> "$OUT/c3_ktrace.err" || exit 1
f=$(ls $OUT/c3_ktrace/*/run_kernel_trace.csv $OUT/c3_ktrace/run_kernel_trace.csv 2>/dev/null | head -1)
python tools/kstats.py "$f" > "$OUT/c3_kernel_summary.txt"
head -6 "$OUT/c3_kernel_summary.txt"
timeout -k 10 400 python3 bench.py --workload c4 --steps 3 --warmup 1 --cpu-seconds 10 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" || exit 1
timeout -k 10 400 python3 bench.py --workload c4f --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench_c4f.json" 2> "$OUT/bench_c4f.err" || exit 1
timeout -k 10 500 python3 bench.py --workload c4b --steps 5 --warmup 2 > "$OUT/bench_c4b.json" 2> "$OUT/bench_c4b.err" || exit 1
timeout -k 10 500 python3 bench.py --workload c4b --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_c4b_2.json" 2> "$OUT/bench_c4b_2.err" || exit 1
timeout -k 10 600 python3 bench.py --workload c4bl --steps 3 --warmup 1 > "$OUT/bench_c4bl.json" 2> "$OUT/bench_c4bl.err" || exit 1
for wl in c4 c4f c4b c4b_2 c4bl; do cut -c1-160 "$OUT/bench_$wl.json"; done
echo "[6] N = 2 ranks rehearsed on one GPU (gloo); one rank over RCCL"
BENCH_REHEARSE_ONE_GPU=1 timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 5 --cpu-threads 16 > "$OUT/bench_n2_rehearsal.json" 2> "$OUT/bench_n2.err" || exit 1
cut -c1-200 "$OUT/bench_n2_rehearsal.json"
BENCH_DIST_ONE_RANK=1 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_rccl_one_rank.json" 2> "$OUT/bench_rccl.err" || exit 1
cut -c1-200 "$OUT/bench_rccl_one_rank.json"
echo "[7] PMC passes (each pass its own run)"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_c1_fetch" -o run -- \
    python3 bench.py --roofline-only --steps 5 --warmup 0 > "$OUT/pmc_c1_fetch.json" 2> "$OUT/pmc_c1_fetch.err" || echo "pmc fetch failed"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $SQ --output-format csv -d "$OUT/pmc_c1_sq" -o run -- \
    python3 bench.py --roofline-only --steps 5 --warmup 0 > "$OUT/pmc_c1_sq.json" 2> "$OUT/pmc_c1_sq.err" || echo "pmc c1 sq failed"
CDC_MASKL_INDEX=2 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $SQ --output-format csv -d "$OUT/pmc_c3_sq" -o run -- \
    python3 bench.py --workload c3 --roofline-only --steps 5 --warmup 0 > "$OUT/pmc_c3_sq.json" 2> "$OUT/pmc_c3_sq.err" || echo "pmc c3 sq failed"
python tools/pmc_summary.py "$OUT" k_scan --glob "pmc_c1_*" > "$OUT/pmc_c1_k_scan.txt" 2>&1 || true
python tools/pmc_summary.py "$OUT" k_scan_f --glob "pmc_c3_*" > "$OUT/pmc_c3_k_scan_f.txt" 2>&1 || true
cat "$OUT/pmc_c1_k_scan.txt" "$OUT/pmc_c3_k_scan_f.txt"
echo done
