set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for so in 0 1; do
  CDC_DIAG_SCAN_ONLY=$so timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU --output-format csv -d gpurun_out/clk$so -o run -- python3 bench.py --steps 20 --warmup 3 --streams 2 --no-cpu-baseline --e2e-reps 0 --digest-reps 0 > gpurun_out/clk$so.json 2> gpurun_out/clk$so.err
  python3 - <<PY
import csv,collections
rows=[r for r in csv.DictReader(open('gpurun_out/clk$so/run_counter_collection.csv')) if 'k_scan' in r['Kernel_Name']]
tr={r['Dispatch_Id']:(int(r['End_Timestamp'])-int(r['Start_Timestamp'])) for r in csv.DictReader(open('gpurun_out/clk$so/run_kernel_trace.csv')) if 'k_scan' in r['Kernel_Name']}
agg=collections.defaultdict(list)
for r in rows: agg[r['Counter_Name']].append((r['Dispatch_Id'],float(r['Counter_Value'])))
g=agg['GRBM_GUI_ACTIVE']
for d,v in g[-6:]:
    ns=tr.get(d)
    print('scan_only=$so dispatch',d,'GRBM',v,'dur_us',ns/1000 if ns else None,'GHz(per XCD /8)', v/8/ns if ns else None)
PY
done
