#!/bin/bash
# round 5: k_chunk timeline (stamps) + launch times: one-launch, scan-only, two-launch; then the driver's command both ways
O=gpurun_out/$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 5 60 python tools/abort_probe.py 64 1 > $O/probe_64_m1.txt 2>&1 || { echo "probe failed"; tail -5 $O/probe_64_m1.txt; exit 1; }
grep -v Warn $O/probe_64_m1.txt | grep -v ensure_init | tail -2
for v in "16 1" "272 1" "16 0"; do set -- $v
  CDC_DEBUG_PHASE=$1 CDC_RESOLVE_MODE=$2 timeout -k 5 90 python tools/chunk_timeline.py --warm 30 > $O/tl_$1_$2.txt 2>&1 || { echo "tl $v failed"; tail $O/tl_$1_$2.txt; exit 1; }
  echo "== debug $1 mode $2"; grep -v Warn $O/tl_$1_$2.txt | grep -v ensure_init
done
for m in 1 0; do
  CDC_RESOLVE_MODE=$m timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv_m$m.json 2>>$O/err.txt || { echo "bench m$m failed"; tail $O/err.txt; exit 1; }
  python -c "import json,sys;d=json.loads(open('$O/drv_m$m.json').read().strip().splitlines()[-1]);print('driver mode $m', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_vs_oracle'))"
done
