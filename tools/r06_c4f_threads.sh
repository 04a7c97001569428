#!/bin/bash
# Round 6: c4f with 8 / 16 / 24 / 32 (or $THREADS) pread threads (bench.py --file-threads), interleaved twice on one box.
#   tools/r06_c4f_threads.sh <tag>
TAG=${1:-r06c4f}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for t in ${THREADS:-8 16 24 32}; do
    f="$OUT/c4f_t${t}_$rep.json"
    timeout -k 10 300 python3 bench.py --workload c4f --steps 5 --warmup 1 --no-cpu-baseline --file-threads $t > "$f" 2> "$f.err" || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(f\"{sys.argv[2]:16s} {d['value']:7.2f} GiB/s  {d['ms_per_step']:.2f} ms/step\")" "$f" "threads=$t rep$rep"
  done
done
echo done
