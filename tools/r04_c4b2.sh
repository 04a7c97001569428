#!/bin/bash
# backup with the encoder thread: tests, c4b at 512 MiB (x2) and 256 MiB, then one c4b line with its CPU baseline.
O=gpurun_out/${1:-r04c4b2}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_backup.py > $O/pytest_backup.txt 2>&1; rc=$?
tail -2 $O/pytest_backup.txt
[ $rc -eq 0 ] || exit $rc
for mib in 512 256 512; do
  timeout -k 10 300 python bench.py --workload c4b --steps 5 --warmup 2 --backup-batch-mib $mib --no-cpu-baseline > $O/c4b_$mib.json 2>$O/c4b_$mib.err || { tail -5 $O/c4b_$mib.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4b_$mib.json')); b=d['backup_stages']; print('c4b batch $mib MiB', d['value'], 'GiB/s; device_s', b['device_s'], 'encode_s', b['encode_s'], 'd2h_s', b['d2h_s'], 'wall', b['wall_s'])"
done
timeout -k 10 400 python bench.py --workload c4b --steps 5 --warmup 2 > $O/c4b_line.json 2>$O/c4b_line.err || { tail -5 $O/c4b_line.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4b_line.json')); print('c4b line', d['value'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline']['cores'], 'roofline', d['roofline']['kernel'], d['roofline']['frac'], 'parity', d['parity_vs_oracle'])"
