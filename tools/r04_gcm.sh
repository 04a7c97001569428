#!/bin/bash
# k_gcm A/B: per-GiB k_gcm time (kernel trace) for the library variants, GCM only (no LZ4) on random data.
#   tools/r04_gcm.sh <tag> <lib> [<lib> ...]     (lib: path of a build of libplakar_cdc.so)
TAG=${1:-r04gcm}; shift
O=gpurun_out/$TAG; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_encode.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_encode.log 2>&1 || { tail -20 $O/pytest_encode.log; exit 1; }
tail -1 $O/pytest_encode.log
for r in 1 2; do
for lib in "$@"; do
  n=$(basename $lib .so)
  PLAKAR_CDC_LIB=$PWD/$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/${n}_$r -o run --output-format csv -- python tools/encode_bench.py --size-mib 1024 --reps 3 --kinds random --labels gcm > $O/${n}_$r.log 2>$O/${n}_$r.err || { tail -5 $O/${n}_$r.err; exit 1; }
  f=$(ls $O/${n}_$r/run_kernel_stats.csv $O/${n}_$r/*/run_kernel_stats.csv 2>/dev/null | head -1)
  python - "$f" "$n" "$r" <<'PY'
import csv, sys
for row in csv.DictReader(open(sys.argv[1])):
    if "k_gcm" in row["Name"]:
        avg = float(row["AverageNs"]) / 1e6
        print(f"{sys.argv[2]:22s} run {sys.argv[3]} k_gcm calls {row['Calls']:>3s} avg_ms {avg:7.3f} ms_per_GiB {avg:7.3f} min_ms {float(row['MinNs'])/1e6:7.3f}")
PY
done
done
