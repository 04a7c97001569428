#!/bin/bash
# Round 6: host-thread A/B of the host-bound legs (16 = the one-GPU box's CPU
# share, 24, 32 = an 8-GPU node's cores per GPU): the C3 hybrid per-chunk
# SHA-256 (--hybrid-threads) and the c4b / c4bl backup readers (--backup-readers).
TAG=${1:-r06th}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
echo "nproc $(nproc) OMP_NUM_THREADS=$OMP_NUM_THREADS affinity $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))')"
cat /sys/fs/cgroup/cpu.max 2>/dev/null || true
Q="--no-cpu-baseline --e2e-reps 0 --encode-reps 0"
for rep in 1 2; do
  for th in 16 24 32; do
    timeout -k 10 300 python3 bench.py --workload c3 --steps 20 --warmup 20 --hybrid-threads $th $Q > "$OUT/c3_h${th}_$rep.json" 2> "$OUT/c3_h${th}_$rep.err" || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); h=d['chunk_digests']['hybrid']; print('c3 hybrid threads', sys.argv[2], 'GiB/s', h['value'], 'ms', h['ms_per_pass'], 'host chunks', h['host_chunks'])" "$OUT/c3_h${th}_$rep.json" $th
  done
done
for rep in 1 2; do
  for th in 16 24 32; do
    timeout -k 10 400 python3 bench.py --workload c4b --steps 5 --warmup 2 --backup-readers $th --no-cpu-baseline > "$OUT/c4b_r${th}_$rep.json" 2> "$OUT/c4b_r${th}_$rep.err" || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('c4b readers', sys.argv[2], 'GiB/s', d['value'], 'wall', r['wall_s'], 'set by', r['wall_set_by'], 'named/wall', r['named_over_wall'], 'fill', r['fill_s'], 'drain', r['drain_s'], 'chain', r['chain_s'])" "$OUT/c4b_r${th}_$rep.json" $th
  done
done
for th in 16 32; do
  timeout -k 10 600 python3 bench.py --workload c4bl --steps 3 --warmup 1 --backup-readers $th --no-cpu-baseline > "$OUT/c4bl_r${th}.json" 2> "$OUT/c4bl_r${th}.err" || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('c4bl readers', sys.argv[2], 'GiB/s', d['value'], 'wall', r['wall_s'], 'set by', r['wall_set_by'], 'named/wall', r['named_over_wall'], 'chain', r['chain_s'], r['chain_bytes'])" "$OUT/c4bl_r${th}.json" $th
done
echo done
