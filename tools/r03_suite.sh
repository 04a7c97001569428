#!/bin/bash
# Full GPU suite + the pass-gap measurement.
O=gpurun_out/${1:-r03g}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
bash tools/r03_gap.sh ${1:-r03g}
