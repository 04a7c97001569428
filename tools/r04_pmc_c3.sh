#!/bin/bash
# PMC passes (separate runs, kernel trace only) of C3's fused scan k_scan_f on the final code:
# bench.py --workload c3 --roofline-only (10 warm-up + 10 single-stream passes), SQ busy / VALU / LDS counters.
O=gpurun_out/${1:-r04pmc3}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $O/p$i -o run -- python3 bench.py --workload c3 --roofline-only --steps 10 --warmup 10 > $O/p$i.json 2> $O/p$i.err || { echo "c3 pass $i failed"; exit 1; }
done
echo "== k_scan_f"; mkdir -p $O/s; cp -r $O/p1 $O/s/p1; cp -r $O/p2 $O/s/p2; python tools/pmc_summary.py $O/s k_scan_f
