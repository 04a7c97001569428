#!/bin/bash
# A/B of library variants on one box, interleaved: the driver's cold command
# (20 timed / 5 warm-up passes, fresh process) and a warm run (200 / 200).
#   tools/ab.sh <tag> <variant.so>...   ("base" = the in-tree library)
# Variants are built beforehand, e.g.
#   python -c "from plakar_amd import build as b; b.build_lib(out='plakar_amd/_lib/var_x.so', defines=['X=1'])"
set -e
TAG=$1; shift
OUT=gpurun_out/ab_$TAG; mkdir -p "$OUT"
QUIET="--no-cpu-baseline --e2e-reps 0 --digest-reps 0 --encode-reps 0"
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(f\"{sys.argv[2]:28s} value {d['value']:8.1f}  ms/step {d['ms_per_step']:.4f}  scan {r['kernel_avg_ms']:.4f} ms frac {r['frac']:.4f}  pass {r['pipeline_avg_ms']:.4f}\")" "$1" "$2"; }
for rep in 1 2; do
  for v in "$@"; do
    lib=""; [ "$v" != base ] && lib="$PWD/plakar_amd/_lib/$v"
    f="$OUT/${v%.so}_cold$rep.json"
    PLAKAR_CDC_LIB=$lib timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 $QUIET > "$f" 2> "$f.err"
    summ "$f" "${v%.so} cold$rep"
    f="$OUT/${v%.so}_warm$rep.json"
    PLAKAR_CDC_LIB=$lib timeout -k 10 120 python3 bench.py --gpus 1 --steps 200 --warmup 200 $QUIET > "$f" 2> "$f.err"
    summ "$f" "${v%.so} warm$rep"
  done
done
