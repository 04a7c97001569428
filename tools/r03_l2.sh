#!/bin/bash
# The real scan's compute with its DMAs served from L2 (CDC_DIAG_L2) vs from HBM, cold and warm.
O=gpurun_out/r03l2; mkdir -p $O
export PYTHONUNBUFFERED=1
for w in 5; do
  for v in var_l2w var_l2w_norc; do
    PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$v.so timeout -k 10 60 python tools/waitdump.py --warm $w --waits > $O/${v}_w$w.txt 2>&1 || { echo "$v failed"; tail -3 $O/${v}_w$w.txt; exit 1; }
    echo "$v $(grep -A1 '^warm' $O/${v}_w$w.txt | tr '\n' ' ')"
  done
done
