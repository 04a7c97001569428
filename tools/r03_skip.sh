#!/bin/bash
# Round 3: skip walk (k_walk) parity + A/B against the full scan.
set -o pipefail
O=gpurun_out/r03a
mkdir -p $O
export PYTHONUNBUFFERED=1
CDC_WALK_MODE=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_skip.txt 2>&1
echo "pytest skip rc=$?" | tee -a $O/status.txt
FAST="--no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0"
for m in 2 0 2 0; do
  CDC_WALK_MODE=$m timeout -k 10 120 python bench.py --steps 20 --warmup 5 $FAST > $O/c1_drv_m$m.json 2>>$O/err.txt || exit 1
  CDC_WALK_MODE=$m timeout -k 10 120 python bench.py $FAST > $O/c1_def_m$m.json 2>>$O/err.txt || exit 1
  echo "mode $m done" | tee -a $O/status.txt
done
for w in c2 c3; do
  for m in 2 0; do
    CDC_WALK_MODE=$m timeout -k 10 120 python bench.py --workload $w $FAST > $O/${w}_m$m.json 2>>$O/err.txt || exit 1
  done
done
echo done | tee -a $O/status.txt
