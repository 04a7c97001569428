#!/bin/bash
# A/B of an environment knob on the driver's cold command (20 / 5) and a warm
# run (200 / 200), interleaved: tools/ab_env_driver.sh <tag> VAR "v1 v2 ..." [reps]
TAG=$1; VAR=$2; VALS=$3; REPS=${4:-3}
OUT=gpurun_out/abenv_$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
QUIET="--no-cpu-baseline --e2e-reps 0 --digest-reps 0 --encode-reps 0"
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(f\"{sys.argv[2]:28s} value {d['value']:8.1f}  ms/step {d['ms_per_step']:.4f}  scan {r['kernel_avg_ms']:.4f} ms frac {r['frac']:.4f}  pass {r['pipeline_avg_ms']:.4f}\")" "$1" "$2"; }
for rep in $(seq 1 $REPS); do
  for v in $VALS; do
    f="$OUT/${VAR}_${v}_cold$rep.json"
    env $VAR=$v timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 $QUIET > "$f" 2> "$f.err" || exit 1
    summ "$f" "$VAR=$v cold$rep"
  done
done
for v in $VALS; do
  f="$OUT/${VAR}_${v}_warm.json"
  env $VAR=$v timeout -k 10 120 python3 bench.py --gpus 1 --steps 200 --warmup 200 $QUIET > "$f" 2> "$f.err" || exit 1
  summ "$f" "$VAR=$v warm"
done
