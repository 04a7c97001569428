#!/bin/bash
# round 4 check: backup tests (per-file errors, pieces, HWQ stats) then the scan counters
O=gpurun_out/r04a; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_backup.py > $O/pytest_backup.txt 2>&1; rc=$?
tail -15 $O/pytest_backup.txt
[ $rc -eq 0 ] || exit $rc
bash tools/r04_pmc_scan.sh r04pmc_l2 var_l2w
