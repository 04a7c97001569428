#!/bin/bash
# Backup tests, then c4b with its pipeline trace for the default build and for each variant library given.
#   tools/r04_c4b_ab.sh <tag> [lib ...]
TAG=${1:-r04c4bab}; shift
O=gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_backup.py tests/test_backup_cpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_backup.log 2>&1 || { tail -30 $O/pytest_backup.log; exit 1; }
tail -1 $O/pytest_backup.log
bash tools/r04_c4b_trace.sh $TAG/default || exit 1
for lib in "$@"; do
  n=$(basename $lib .so)
  PLAKAR_CDC_LIB=$PWD/$lib bash tools/r04_c4b_trace.sh $TAG/$n || exit 1
done
