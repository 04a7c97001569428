#!/bin/bash
# Backup tests, then c4b with the digest streams on half the CUs (default) vs on all of them, interleaved, with pipeline traces (first line of each: the c4b result).
O=gpurun_out/${1:-r04c4bmask}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_backup.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_backup.log 2>&1 || { tail -30 $O/pytest_backup.log; exit 1; }
tail -1 $O/pytest_backup.log
for r in 1 2; do
  bash tools/r04_c4b_trace.sh ${1:-r04c4bmask}/half_$r > $O/half_$r.txt || exit 1
  grep "^c4b" $O/half_$r.txt
  CDC_BACKUP_DIGEST_CUS=all bash tools/r04_c4b_trace.sh ${1:-r04c4bmask}/all_$r > $O/all_$r.txt || exit 1
  grep "^c4b" $O/all_$r.txt
done
python3 tools/backup_trace.py $O/half_2/trace.csv
