#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 invocation per counter set).
# usage: tools/pmc.sh <outdir> [bench args...]
set -e
OUT=$1; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_LDS_CMD_FIFO_FULL SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" \
           "GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_SMEM" ; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --kernel-trace --pmc $set --output-format csv -d "$OUT/p$i" -o run -- python bench.py "$@" > "$OUT/p$i.log" 2>&1
  echo "pass $i done: $set"
done
