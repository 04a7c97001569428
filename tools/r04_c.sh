#!/bin/bash
# round 4: k_walk phase timestamps + counters; pinned vs pageable host path per call.
O=gpurun_out/r04c; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/pinned_probe.py > $O/pinned_probe.txt 2>&1 || { tail -5 $O/pinned_probe.txt; exit 1; }
grep MiB $O/pinned_probe.txt
bash tools/r03_walkprof.sh r04c/walk 2>&1 | tail -60
