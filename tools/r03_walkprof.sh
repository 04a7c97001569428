#!/bin/bash
# k_walk diagnosis: per-segment phase timestamps and SQ counters.
set -o pipefail
O=gpurun_out/${1:-r03b}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CDC_WALK_MODE=2 CDC_DEBUG_PHASE=16 timeout -k 10 120 python tools/tsdump.py > $O/tsdump_walk.txt 2>&1 || exit 1
cat $O/tsdump_walk.txt
SHORT="--steps 3 --warmup 1 --streams 1 --no-cpu-baseline --e2e-reps 0 --digest-reps 0 --encode-reps 0"
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
SQ2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM GRBM_COUNT"
i=0
for set in "$SQ1" "$SQ2" "FETCH_SIZE"; do
  i=$((i+1))
  CDC_WALK_MODE=2 timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $O/pmc/p$i -o run -- \
     python3 bench.py $SHORT > $O/pmc_p$i.json 2> $O/pmc_p$i.err || { echo "pmc pass $i rc=$?"; exit 1; }
done
python tools/pmc_summary.py $O/pmc k_walk > $O/pmc_k_walk.txt 2>&1
cat $O/pmc_k_walk.txt
