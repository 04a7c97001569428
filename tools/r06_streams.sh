#!/bin/bash
# Round 6: pipelined streams 1 / 2 / 3 / 4 (bench.py --streams), the driver's command (20 / 5) twice and the
# bench default (200 / 200) once each, interleaved on one box.
#   tools/r06_streams.sh <tag>
TAG=${1:-r06st}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
QUIET="--no-cpu-baseline --e2e-reps 0 --digest-reps 0 --encode-reps 0"
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(f\"{sys.argv[2]:16s} value {d['value']:8.1f}  ms/step {d['ms_per_step']:.4f}  scan {r['kernel_avg_ms']:.4f} ms  pass {r['pipeline_avg_ms']:.4f}\")" "$1" "$2"; }
for rep in 1 2; do
  for s in 1 2 3 4; do
    timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --streams $s $QUIET > "$OUT/cold_s${s}_$rep.json" 2> "$OUT/cold_s${s}_$rep.err" || exit 1
    summ "$OUT/cold_s${s}_$rep.json" "streams=$s cold$rep"
  done
done
for s in 1 2 3 4; do
  timeout -k 10 300 python3 bench.py --streams $s $QUIET > "$OUT/warm_s$s.json" 2> "$OUT/warm_s$s.err" || exit 1
  summ "$OUT/warm_s$s.json" "streams=$s warm"
done
echo done
