#!/bin/bash
# Kernel trace of a short bench run: tools/ktrace.sh <outdir> [bench args...]
OUT=$1; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python bench.py "$@" > "$OUT/bench.log" 2>&1
rc=$?
python tools/kstats.py "$OUT/run_kernel_trace.csv" | head -8
exit $rc
