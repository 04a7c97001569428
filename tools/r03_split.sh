#!/bin/bash
# Row read split in two (stage t + 1's half a group early): parity, cycles, A/B.
O=gpurun_out/r03split; mkdir -p $O
export PYTHONUNBUFFERED=1
PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/var_split.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest var_split rc=$rc"; tail -1 $O/pytest.txt; [ $rc -eq 0 ] || exit 1
for w in 5 300; do for v in var_l2w var_split_l2w var_waits var_split_w; do
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$v.so timeout -k 10 60 python tools/waitdump.py --warm $w --waits > $O/${v}_$w.txt 2>&1 || exit 1
  echo "$v $(grep -A1 '^warm' $O/${v}_$w.txt | tr '\n' ' ')"
done; done
bash tools/ab.sh split base var_split.so
for wl in c3 c2; do for v in base var_split; do
  lib=""; [ $v != base ] && lib=$PWD/plakar_amd/_lib/$v.so
  PLAKAR_CDC_LIB=$lib timeout -k 10 120 python bench.py --workload $wl --no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0 > $O/${wl}_$v.json 2>>$O/err.txt || exit 1
  python3 -c "import json; d=json.load(open('$O/${wl}_$v.json')); r=d['roofline']; print('$wl $v', d['value'], r['kernel_avg_ms'], r['frac'])"
done; done
