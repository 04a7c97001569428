#!/bin/bash
# Round 6: c4b with 8 / 12 / 16 backup reader threads (bench.py --backup-readers), interleaved twice on one box.
#   tools/r06_c4b_readers.sh <tag>
TAG=${1:-r06c4b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for t in ${THREADS:-8 12 16}; do
    f="$OUT/c4b_r${t}_$rep.json"
    timeout -k 10 400 python3 bench.py --workload c4b --steps 5 --warmup 2 --no-cpu-baseline --backup-readers $t > "$f" 2> "$f.err" || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(f\"{sys.argv[2]:16s} {d['value']:7.2f} GiB/s  wall {r.get('wall_s')} s  set by: {r.get('wall_set_by')}\")" "$f" "readers=$t rep$rep"
  done
done
echo done
