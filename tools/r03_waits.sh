#!/bin/bash
# Scan diagnostics: wait share (CDC_DIAG_WAITS) and the compute-only scan (CDC_DIAG_NO_DMA), cold and warm.
O=gpurun_out/${1:-r03w}; mkdir -p $O
export PYTHONUNBUFFERED=1
for w in 5 300; do
  timeout -k 10 120 python tools/waitdump.py --warm $w > $O/base_w$w.txt 2>&1 || exit 1; grep warm $O/base_w$w.txt
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/var_waits.so timeout -k 10 120 python tools/waitdump.py --warm $w --waits > $O/waits_w$w.txt 2>&1 || exit 1; grep -A1 warm $O/waits_w$w.txt
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/var_nodma.so timeout -k 10 120 python tools/waitdump.py --warm $w > $O/nodma_w$w.txt 2>&1 || exit 1; grep warm $O/nodma_w$w.txt
done
