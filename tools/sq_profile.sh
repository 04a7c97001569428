#!/bin/bash
# SQ counter passes over the C1 bench (k_scan and the resolution kernels):
# issue / wait breakdown.  tools/sq_profile.sh <tag> [bench args...]
set -e
TAG=${1:-sq}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="--steps 3 --warmup 1 --streams 1 --no-cpu-baseline --e2e-reps 0 --digest-reps 0 --encode-reps 0 $*"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM GRBM_COUNT"; do
    i=$((i + 1))
    echo "[pass $i] $set"
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/p$i" -o run -- \
        python3 bench.py $ARGS > "$OUT/p$i.json" 2> "$OUT/p$i.err"
done
python tools/pmc_summary.py "$OUT" k_scan | tee "$OUT/k_scan.txt"
