#!/bin/bash
# c4b: backup pipeline slots (batches in flight between reads and packing).
O=gpurun_out/r03slots; mkdir -p $O
export PYTHONUNBUFFERED=1
for rep in 1 2; do
  for v in base var_s6 var_s8; do
    lib=""; [ $v != base ] && lib=$PWD/plakar_amd/_lib/$v.so
    PLAKAR_CDC_LIB=$lib timeout -k 10 300 python bench.py --workload c4b --steps 5 --warmup 2 --no-cpu-baseline > $O/$v.$rep.json 2>>$O/err.txt || { echo "$v failed"; tail -5 $O/err.txt; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$v.$rep.json')); b=d['backup_stages']; print('$v', d['value'], d['ms_per_step'], b['wall_s'], b['device_s'], b['read_wait_s'])"
  done
done
