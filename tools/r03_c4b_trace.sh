#!/bin/bash
# c4b under rocprofv3 (kernel + memory-copy trace): per-batch device timeline.
O=gpurun_out/${1:-r03t}; mkdir -p $O
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof -o c4b --output-format csv -- python3 bench.py --workload c4b --steps 2 --warmup 1 --cpu-threads 1 > $O/c4b.json 2> $O/c4b.err
rc=$?; echo "rc=$rc"; tail -2 $O/c4b.err; find $O/prof -name "*.csv" | head; exit $rc
