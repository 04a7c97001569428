#!/bin/bash
# c4b (whole backup from files) with the pipeline's own event trace of the last step.
O=gpurun_out/${1:-r04c4bt}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
CDC_BACKUP_TRACE=$PWD/$O/trace.csv timeout -k 10 400 python3 bench.py --workload c4b --steps 3 --warmup 1 --no-cpu-baseline > $O/c4b.json 2> $O/c4b.err || { tail -5 $O/c4b.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c4b.json').read().strip().splitlines()[-1]); b=d['backup_stages']; print('c4b', d['value'], d['ms_per_step'], {k: b[k] for k in ('wall_s','run_s','device_s','digest_s','encode_s','objhash_s','read_s','pack_s','callback_s')})"
python3 tools/backup_trace.py $O/trace.csv
