#!/bin/bash
# round 5: k_chunk (one launch) on the GPU: parity subset, backup tests, then the driver's command both ways
O=gpurun_out/$1; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread \
  -k "golden or sizes or sweep or dense or unaligned or sequential or nonfinal or many_buffers or pipelined" > $O/pytest_subset.txt 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_subset.txt; exit 1; }
tail -3 $O/pytest_subset.txt
for m in 1 0 1 0; do
  CDC_RESOLVE_MODE=$m timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_m$m.json 2>>$O/err.txt || { echo "bench m$m failed"; tail $O/err.txt; exit 1; }
  python -c "import json,sys;d=json.loads(open('$O/drv_m$m.json').read().strip().splitlines()[-1]);print('mode $m', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_vs_oracle'))"
done
timeout -k 10 400 python -u -m pytest tests/test_backup.py tests/test_digest.py -x -v --timeout 200 --timeout-method thread > $O/pytest_backup.txt 2>&1 || { echo "backup tests failed"; tail -30 $O/pytest_backup.txt; exit 1; }
tail -3 $O/pytest_backup.txt
