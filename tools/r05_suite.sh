#!/bin/bash
# Round 5: full GPU suite + smoke + the C2 bench line (Encode leg with the parallel random draw)
#   tools/r05_suite.sh <tag>
O=gpurun_out/${1:-r05suite}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --workload c2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { tail $O/bench_c2.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]);print('c2', d['value'], 'encode', d['encode']['value'], d['encode']['ms_per_pass'])"
echo done
