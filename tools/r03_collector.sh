#!/bin/bash
# The collector's rate with 1 / 16 / 64 concurrent callers on the C4 share.
O=gpurun_out/${1:-r03c}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/collector_bench.py --callers 1,16,64 --reps 3 > $O/collector.jsonl 2> $O/collector.err
rc=$?; echo "collector rc=$rc"; cat $O/collector.jsonl; tail -3 $O/collector.err; exit $rc
