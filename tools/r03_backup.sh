#!/bin/bash
O=gpurun_out/${1:-r03h}; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_entropy.py tests/test_backup.py tests/test_abi_c.py tests/test_encode.py -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --workload c4b --cpu-threads 1 > $O/c4b.json 2> $O/c4b.err
rc=$?; echo "c4b rc=$rc"; tail -3 $O/c4b.err; python3 -c "
import json; d=json.load(open('$O/c4b.json')); print(d['value'], d['ms_per_step']); print(json.dumps(d.get('backup_stages')))"
