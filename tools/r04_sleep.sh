#!/bin/bash
# The driver's command with the default build and with variant libraries (e.g. CDC_SPIN_SLEEP builds), interleaved, three rounds.
#   tools/r04_sleep.sh <tag> lib...
TAG=${1:-r04sleep}; shift
O=gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for lib in plakar_amd/_lib/libplakar_cdc.so "$@"; do
    n=$(basename $lib .so)
    PLAKAR_CDC_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --e2e-reps 0 --digest-reps 0 --encode-reps 0 > $O/${n}_$r.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.loads(open('$O/${n}_$r.json').read().strip().splitlines()[-1]); print('$n run $r', d['value'], d['ms_per_step'], d['roofline']['pipeline_avg_ms'], d['parity_vs_oracle'])"
  done
done
