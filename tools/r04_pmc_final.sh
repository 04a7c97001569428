#!/bin/bash
# PMC passes (separate runs, kernel trace only) on the final code: k_gcm (GCM-only encode of 1 GiB) and
# k_chunk_digest (tools/digest_bench.py: single passes over a C1 cut list), SQ busy / VALU / LDS counters.
O=gpurun_out/${1:-r04pmcf}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $O/g$i -o run -- python3 tools/encode_bench.py --size-mib 1024 --reps 1 --kinds random --labels gcm > $O/g$i.log 2>&1 || echo "gcm pass $i failed"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $O/d$i -o run -- python3 tools/digest_bench.py 1024 > $O/d$i.log 2>&1 || echo "digest pass $i failed"
done
echo "== k_gcm"; mkdir -p $O/g; cp -r $O/g1 $O/g/p1; cp -r $O/g2 $O/g/p2; python tools/pmc_summary.py $O/g k_gcm
echo "== k_chunk_digest"; mkdir -p $O/d; cp -r $O/d1 $O/d/p1; cp -r $O/d2 $O/d/p2; python tools/pmc_summary.py $O/d "k_chunk_digest<false>"
