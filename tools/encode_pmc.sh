# PMC passes over the GCM-only encode of 1 GiB of random data (k_gcm dominates):
#   tools/encode_pmc.sh [tag]   -> gpurun_out/<tag>/p<i>, summary per Encode kernel
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-gpmc}; mkdir -p $O
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE" "SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $O/p$i -o run -- python3 tools/encode_bench.py --size-mib 1024 --reps 1 --kinds random --labels gcm > $O/p$i.log 2>&1 || echo "pass $i failed"
done
for k in k_gcm; do echo "== $k"; python tools/pmc_summary.py $O $k; done
