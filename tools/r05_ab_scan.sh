#!/bin/bash
# round 5: the scan phase of k_chunk vs k_scan (scan only, warm), variant libraries
O=gpurun_out/$1; mkdir -p $O
export PYTHONUNBUFFERED=1
run() {  # name lib mode debug
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$2 CDC_RESOLVE_MODE=$3 CDC_DEBUG_PHASE=$4 timeout -k 5 90 python tools/chunk_timeline.py --warm 150 > $O/$1.txt 2>&1 || { echo "$1 failed"; tail -5 $O/$1.txt; exit 1; }
  echo "== $1"; grep -E "launches|tier|end p0|no segment|last INCL" $O/$1.txt
}
run old1 v_scanonly_old.so 0 16
run chunk libplakar_cdc.so 1 272
run linear v_linear.so 1 272
run noprio v_noprio.so 1 272
run lin_noprio v_lin_noprio.so 1 272
run old2 v_scanonly_old.so 0 16
run chunk_full libplakar_cdc.so 1 16
run twolaunch libplakar_cdc.so 0 16
