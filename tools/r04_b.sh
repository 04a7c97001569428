#!/bin/bash
# round 4 diagnostics: backup tests; the scan's task cycles with pieces removed (L2 / no DMA / no row reads /
# no recheck; timing only); the shader clock over the driver's first 45 passes, 2 streams vs 1; scan counters.
O=gpurun_out/r04b; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_backup.py > $O/pytest_backup.txt 2>&1; rc=$?
tail -12 $O/pytest_backup.txt
[ $rc -eq 0 ] || exit $rc
for v in var_l2w var_norow var_nodma var_nodma_norow var_nodma_norow_norc var_l2w_norc; do
  PLAKAR_CDC_LIB=$PWD/plakar_amd/_lib/$v.so timeout -k 10 120 python tools/waitdump.py --warm 5 --waits --save $O/$v.npy > $O/$v.txt 2>&1 || { echo "$v failed"; tail -5 $O/$v.txt; exit 1; }
  echo "== $v"; grep -v "amdgpu.ids\|UserWarning\|ensure_init" $O/$v.txt | head -4; grep "start rank\|rechecks" $O/$v.txt
done
for s in 2 1; do
  timeout -k 10 120 python tools/clock_probe.py --passes 45 --streams $s --bins 5 > $O/clock_s$s.txt 2>&1 || { echo "clock $s failed"; tail -5 $O/clock_s$s.txt; exit 1; }
  echo "== clock streams $s"; grep -v "amdgpu.ids\|UserWarning\|ensure_init" $O/clock_s$s.txt
done
bash tools/r04_pmc_scan.sh r04pmc_l2 var_l2w
