#!/bin/bash
# Second-level graph successors: GPU suite, resolve phases, A/B on the driver command.
O=gpurun_out/${1:-r03g2}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.txt
[ $rc -eq 0 ] || exit $rc
CDC_DEBUG_PHASE=16 timeout -k 10 100 python tools/tsdump.py --warm 5 2>&1 | grep -A12 k_resolve
bash tools/ab.sh g2 base var_base.so
