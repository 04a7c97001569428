#!/bin/bash
# Is the recheck's cost instruction-cache misses after k_resolve?  The scan alone in a loop vs with k_resolve.
O=gpurun_out/r03ic; mkdir -p $O
export PYTHONUNBUFFERED=1
for w in 5 300; do
  for v in base var_norc var_so var_so_norc; do
    lib=""; [ $v != base ] && lib=$PWD/plakar_amd/_lib/$v.so
    PLAKAR_CDC_LIB=$lib timeout -k 10 60 python tools/waitdump.py --warm $w > $O/${v}_w$w.txt 2>&1 || { echo "$v failed"; tail -3 $O/${v}_w$w.txt; exit 1; }
    echo "$v $(grep '^warm' $O/${v}_w$w.txt)"
  done
done
