#!/bin/bash
# Round-2 evidence in one GPU call: GPU suite, the driver's exact bench command
# plain and under a rocprofv3 kernel trace, SQ counter passes for the scan
# kernels (C1 k_scan + k_resolve, C3 k_scan_f), FETCH_SIZE passes, and the
# other bench lines.  Writes gpurun_out/<tag>/; stops at the first failure.
#   tools/r02_profile.sh <tag> [quick]
set -e
TAG=${1:-r02}
QUICK=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SHORT="--steps 3 --warmup 1 --streams 1 --no-cpu-baseline --e2e-reps 0 --digest-reps 0 --encode-reps 0"

if [ -z "$QUICK" ]; then
    echo "[1] pytest -m gpu"
    timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
    tail -2 "$OUT/pytest_gpu.log"
fi

echo "[2] driver command: python3 bench.py --gpus 1 --steps 20 --warmup 5"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver_bench.json" 2> "$OUT/driver_bench.err"
cut -c1-300 "$OUT/driver_bench.json"

echo "[3] rocprofv3 --kernel-trace --stats of the driver command"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/driver_ktrace" -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver_ktrace_bench.json" 2> "$OUT/driver_ktrace.err"
python tools/kstats.py "$OUT/driver_ktrace/run_kernel_trace.csv" > "$OUT/driver_kernel_summary.txt"
head -8 "$OUT/driver_kernel_summary.txt"
python tools/timeline.py "$OUT/driver_ktrace/run_kernel_trace.csv" > "$OUT/driver_timeline.txt" 2>&1 || true

SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
SQ2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM GRBM_COUNT"
SQ3="SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_INST_LEVEL_LDS SQ_LDS_CMD_FIFO_FULL SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_MISC SQ_THREAD_CYCLES_VALU SQ_INSTS_SMEM"
for wl in c1 c3; do
    mkdir -p "$OUT/pmc_$wl"
    i=0
    for set in "$SQ1" "$SQ2" "$SQ3" "FETCH_SIZE"; do
        i=$((i + 1))
        echo "[4] $wl pmc pass $i: $set"
        timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/pmc_$wl/p$i" -o run -- \
            python3 bench.py --workload $wl $SHORT > "$OUT/pmc_$wl/p$i.json" 2> "$OUT/pmc_$wl/p$i.err" || {
            rc=$?; echo "pass failed rc=$rc"; tail -3 "$OUT/pmc_$wl/p$i.err"
            case $rc in 124|134|137|139) exit $rc;; esac; }
    done
    for k in k_scan k_scan_f k_scan_l k_resolve; do
        python tools/pmc_summary.py "$OUT/pmc_$wl" $k > "$OUT/pmc_${wl}_$k.txt"
    done
done
cat "$OUT/pmc_c1_k_scan.txt"

if [ -z "$QUICK" ]; then
    echo "[5] bench c1 (default command: 200 warm-up + 200 timed passes, all legs)"
    timeout -k 10 400 python3 bench.py > "$OUT/bench_c1.json" 2> "$OUT/bench_c1.err"
    cut -c1-200 "$OUT/bench_c1.json"
    for wl in c2 c3; do
        echo "[5] bench $wl"
        timeout -k 10 200 python3 bench.py --workload $wl --no-cpu-baseline > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err"
        cut -c1-200 "$OUT/bench_$wl.json"
    done
    echo "[6] bench c4 / c4f"
    timeout -k 10 400 python3 bench.py --workload c4 --steps 3 --warmup 1 --cpu-seconds 10 > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err"
    timeout -k 10 400 python3 bench.py --workload c4f --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_c4f.json" 2> "$OUT/bench_c4f.err"
    cut -c1-200 "$OUT/bench_c4f.json"
fi
echo done
