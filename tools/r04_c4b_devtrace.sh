#!/bin/bash
# c4b under a rocprofv3 kernel + memory-copy trace, with the pipeline's own trace of the last step.
O=gpurun_out/${1:-r04c4bdev}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
CDC_BACKUP_TRACE=$PWD/$O/trace.csv timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/rp -o run -- python3 bench.py --workload c4b --steps 2 --warmup 1 --no-cpu-baseline > $O/c4b.json 2> $O/c4b.err || { tail -5 $O/c4b.err; exit 1; }
k=$(ls $O/rp/run_kernel_trace.csv $O/rp/*/run_kernel_trace.csv 2>/dev/null | head -1)
m=$(ls $O/rp/run_memory_copy_trace.csv $O/rp/*/run_memory_copy_trace.csv 2>/dev/null | head -1)
cp "$k" $O/c4b_kernel_trace.csv; cp "$m" $O/c4b_memory_copy_trace.csv
python3 tools/backup_trace.py $O/trace.csv | tail -12
python3 tools/c4b_timeline.py $O 7 > $O/timeline.txt 2>&1; head -40 $O/timeline.txt
