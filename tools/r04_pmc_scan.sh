#!/bin/bash
# SQ / LDS counters of the scan with its DMAs served from L2 (var_l2w: compute alone), cold (5 launches before).
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=$PWD/gpurun_out/${1:-r04pmc}; mkdir -p $O
export PYTHONUNBUFFERED=1 PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/${2:-var_l2w}.so
i=0
for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INST_LEVEL_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_LDS_CMD_FIFO_FULL SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES" \
         "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c -d $O/p$i -o run --output-format csv -- python tools/waitdump.py --warm 5 --timed 5 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
python tools/pmc_summary.py $O k_scan
