#!/bin/bash
# Recheck variants: parity of the compact recheck, then the A/B (cold driver command + warm).
O=gpurun_out/r03rc; mkdir -p $O
export PYTHONUNBUFFERED=1
PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/var_c.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_c.txt 2>&1
echo "pytest var_c rc=$?"; tail -1 $O/pytest_c.txt
bash tools/ab.sh rc base var_c.so var_co.so var_co16.so var_norc.so
