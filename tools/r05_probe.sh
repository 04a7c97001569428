#!/bin/bash
# round 5: k_chunk probe (scan only, then the full launch), then the parity subset and the driver's command both ways
O=gpurun_out/$1; mkdir -p $O
export PYTHONUNBUFFERED=1
CDC_DEBUG_PHASE=256 timeout -k 5 60 python tools/abort_probe.py 64 1 > $O/probe_scanonly.txt 2>&1; rc=$?
grep -v Warning $O/probe_scanonly.txt | tail -4
[ $rc -eq 0 ] || { echo "scan-only probe rc $rc"; exit 1; }
timeout -k 5 60 python tools/abort_probe.py 64 1 > $O/probe_64_m1.txt 2>&1; rc=$?
grep -v Warning $O/probe_64_m1.txt | tail -4
[ $rc -eq 0 ] || { echo "probe rc $rc"; exit 1; }
bash tools/r05_try.sh $1
