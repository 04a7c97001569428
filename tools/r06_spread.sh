#!/bin/bash
# Round 6: the driver's exact command five times in fresh processes on one box
# (the headline's run-to-run and box-to-box spread), then the bench default.
#   tools/r06_spread.sh <tag>
TAG=${1:-r06sp}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
QUIET="--no-cpu-baseline --e2e-reps 0 --digest-reps 0 --encode-reps 0"
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(f\"{sys.argv[2]:10s} value {d['value']:8.1f}  ms/step {d['ms_per_step']:.4f}  scan {r['kernel_avg_ms']:.4f} ms frac {r['frac']:.4f}  pass {r['pipeline_avg_ms']:.4f}\")" "$1" "$2"; }
for i in 1 2 3 4 5; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver_$i.json" 2> "$OUT/driver_$i.err" || exit 1
  summ "$OUT/driver_$i.json" "driver$i"
done
timeout -k 10 300 python3 bench.py $QUIET > "$OUT/default.json" 2> "$OUT/default.err" || exit 1
summ "$OUT/default.json" "default"
echo done
