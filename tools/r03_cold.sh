#!/bin/bash
O=gpurun_out/${1:-r03e}; mkdir -p $O
export CDC_SCAN_TASKS_PER_WAVE=0
for w in 5 30 300; do
  CDC_DEBUG_PHASE=16 timeout -k 10 120 python tools/tsdump.py --warm $w > $O/ts_warm$w.txt 2>&1 || exit 1
  grep -v Warning $O/ts_warm$w.txt | grep -v ensure_init | head -40
done
