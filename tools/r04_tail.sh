#!/bin/bash
# Scan task-cycle tail: per-task cycles binned by SIMD, wave slot, XCC, start rank, recheck count.
O=gpurun_out/${1:-r04tail}; mkdir -p $O
export PYTHONUNBUFFERED=1
for v in var_waits:5 var_waits:300 var_l2w:5; do
  lib=${v%%:*}; w=${v##*:}
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$lib.so timeout -k 10 120 python tools/waitdump.py --warm $w --waits --save $O/${lib}_w$w.npy > $O/${lib}_w$w.txt 2>&1 || { echo "$v failed"; tail -5 $O/${lib}_w$w.txt; exit 1; }
  echo "== $v"; cat $O/${lib}_w$w.txt
done
