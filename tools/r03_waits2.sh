#!/bin/bash
O=gpurun_out/${1:-r03w2}; mkdir -p $O
export PYTHONUNBUFFERED=1
for w in 5 300; do
  for v in base var_norc var_norc_nodma var_norc_waits var_nodma; do
    lib=""; [ $v != base ] && lib=$PWD/plakar_amd/_lib/$v.so
    x=""; [ $v = var_norc_waits ] && x=--waits
    PLAKAR_CDC_LIB=$lib timeout -k 10 60 python tools/waitdump.py --warm $w $x > $O/${v}_w$w.txt 2>&1 || { echo "$v failed"; tail -3 $O/${v}_w$w.txt; exit 1; }
    echo "$v $(grep -A1 '^warm' $O/${v}_w$w.txt | tr '\n' ' ')"
  done
done
