#!/bin/bash
# k_walk A/B: round 3's skip_scan vs the pipelined one, with and without junction hints (tsdump, cold).
O=gpurun_out/${1:-r04walk2}; mkdir -p $O
export PYTHONUNBUFFERED=1 CDC_WALK_MODE=2
run() { # name lib debug
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$2 CDC_DEBUG_PHASE=$3 timeout -k 10 120 python tools/tsdump.py --warm 5 > $O/$1.txt 2>&1 || { echo "$1 failed"; tail -5 $O/$1.txt; exit 1; }
  echo "== $1"; grep -v "amdgpu.ids\|UserWarning\|ensure_init" $O/$1.txt | grep -A8 "k_walk segs"
}
run v3 var_skipv3.so 16 && run v3_nohint var_skipv3.so 144 && run v4 libplakar_cdc.so 16 && run v4_nohint libplakar_cdc.so 144
