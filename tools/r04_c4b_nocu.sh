#!/bin/bash
# The encoded blobs' copy back as a no-CU transfer (CDC_BACKUP_D2H_NOCU=1): backup tests with it on, c4b A/B interleaved, and one device trace with it on.
O=gpurun_out/${1:-r04nocu}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
CDC_BACKUP_D2H_NOCU=1 timeout -k 10 400 python -u -m pytest tests/test_backup.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_backup.log 2>&1 || { tail -30 $O/pytest_backup.log; exit 1; }
tail -1 $O/pytest_backup.log
for r in 1 2; do
  CDC_BACKUP_D2H_NOCU=1 bash tools/r04_c4b_trace.sh ${1:-r04nocu}/nocu_$r > $O/nocu_$r.txt || exit 1
  grep "^c4b" $O/nocu_$r.txt
  bash tools/r04_c4b_trace.sh ${1:-r04nocu}/blit_$r > $O/blit_$r.txt || exit 1
  grep "^c4b" $O/blit_$r.txt
done
CDC_BACKUP_D2H_NOCU=1 bash tools/r04_c4b_devtrace.sh ${1:-r04nocu}/dev > $O/dev.txt 2>&1 || exit 1
grep -A14 "^s " $O/dev.txt | head -14
