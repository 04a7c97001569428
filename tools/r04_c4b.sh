#!/bin/bash
# backup pipeline: tests, then c4b at two batch sizes (largest files first), the C2 line's PCIe legs.
O=gpurun_out/${1:-r04c4b}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_backup.py > $O/pytest_backup.txt 2>&1; rc=$?
tail -2 $O/pytest_backup.txt
[ $rc -eq 0 ] || exit $rc
for mib in 256 512 1024; do
  timeout -k 10 300 python bench.py --workload c4b --steps 5 --warmup 2 --backup-batch-mib $mib --no-cpu-baseline > $O/c4b_$mib.json 2>$O/c4b_$mib.err || { tail -5 $O/c4b_$mib.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4b_$mib.json')); b=d['backup_stages']; print('c4b batch $mib MiB', d['value'], 'GiB/s; device_s', b['device_s'], 'digest_s', b['digest_s'], 'wall', b['wall_s'], 'roofline', d['roofline']['frac'])"
done
timeout -k 10 300 python bench.py --workload c2 --steps 20 --warmup 20 --digest-reps 0 --encode-reps 0 --cpu-threads 1 --cpu-seconds 2 > $O/c2.json 2>$O/c2.err || { tail -5 $O/c2.err; exit 1; }
python -c "import json; d=json.load(open('$O/c2.json')); e=d['e2e_host_path']; print('c2 e2e pageable', e['value'], e['ms_per_call'], e['ms_per_call_min_max'], 'pinned', e['pinned']['value'], e['pinned']['ms_per_call'], e['pinned']['ms_per_call_min_max'])"
