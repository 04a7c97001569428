#!/bin/bash
# Round 6: hybrid digests with a persistent host thread pool and a key sort (in-tree) against per-call threads and
# an index stable_sort (variant): the digest GPU tests on the in-tree library, then the bench's digest leg (C1, C2,
# C3) interleaved twice.   tools/r06_hybrid_ab.sh <tag> variant.so
TAG=${1:-r06hy}; V=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_digest.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
echo "tests: $(tail -1 $OUT/pytest.log)"
Q="--no-cpu-baseline --e2e-reps 0 --digest-reps 6 --encode-reps 0 --steps 20 --warmup 5"
for rep in 1 2; do
  for wl in c1 c2 c3; do
    for v in base "$V"; do
      lib=""; [ "$v" != base ] && lib="$PWD/plakar_amd/_lib/$v"
      f="$OUT/${wl}_${v%.so}_$rep.json"
      PLAKAR_CDC_LIB=$lib timeout -k 10 300 python3 bench.py --workload $wl $Q > "$f" 2> "$f.err" || exit 1
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); h=d['chunk_digests']['hybrid']; p=d['chunk_digests']['pipelined_with_chunking']; print(f\"{sys.argv[2]:24s} hybrid {h['value']:7.1f} GiB/s  {h['ms_per_pass']:.3f} ms  pipelined {p['value']:7.1f}\")" "$f" "$wl ${v%.so} $rep"
    done
  done
done
echo done
