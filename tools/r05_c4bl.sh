#!/bin/bash
# Round 5: the backup's piece order (round by round) -- backup tests, c4bl with its pipeline trace, c4b.
#   tools/r05_c4bl.sh <tag>
O=gpurun_out/${1:-r05c4bl}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_backup.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_backup.txt 2>&1 || { echo "backup tests failed"; tail -30 $O/pytest_backup.txt; exit 1; }
tail -1 $O/pytest_backup.txt
CDC_BACKUP_TRACE=$O/c4bl_trace.csv timeout -k 10 600 python bench.py --workload c4bl --steps 3 --warmup 1 --no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0 > $O/c4bl.json 2>>$O/err.txt || { echo "c4bl failed"; tail $O/err.txt; exit 1; }
python -c "import json;d=json.loads(open('$O/c4bl.json').read().strip().splitlines()[-1]);s=d['backup_stages'];print('c4bl', d['value'], s['wall_s'], s['device_s'], s['read_wait_s'], d['parity_vs_oracle'])"
python tools/backup_trace.py $O/c4bl_trace.csv > $O/c4bl_trace.txt 2>&1 || true
head -16 $O/c4bl_trace.txt
for r in 1 2; do
  timeout -k 10 300 python bench.py --workload c4b --steps 5 --warmup 2 --no-cpu-baseline --digest-reps 0 --encode-reps 0 --e2e-reps 0 > $O/c4b_$r.json 2>>$O/err.txt || { echo "c4b failed"; tail $O/err.txt; exit 1; }
  python -c "import json;d=json.loads(open('$O/c4b_$r.json').read().strip().splitlines()[-1]);s=d['backup_stages'];print('c4b', d['value'], s['wall_s'], s['device_s'], s['read_wait_s'], d['parity_vs_oracle'])"
done
echo done
