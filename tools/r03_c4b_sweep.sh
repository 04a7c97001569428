#!/bin/bash
# c4b with different reader / packer thread counts (the box's CPU share is 16).
O=gpurun_out/${1:-r03s}; mkdir -p $O
export PYTHONUNBUFFERED=1
for rp in ${RP:-16:8 12:4 24:6}; do
  set -- ${rp/:/ }
  timeout -k 10 300 python bench.py --workload c4b --steps 5 --warmup 2 --no-cpu-baseline --backup-readers $1 --backup-packers $2 > $O/c4b_$1_$2.json 2> $O/c4b_$1_$2.err || exit 1
  python3 -c "
import json; d=json.load(open('$O/c4b_$1_$2.json')); b=d['backup_stages']
print('$1 $2', d['value'], d['ms_per_step'], 'wall', b['wall_s'], 'read_wait', b['read_wait_s'], 'read', b['read_s'], 'hash', b['objhash_s'], 'pack', b['pack_s'], 'dev', b['device_s'])"
done
