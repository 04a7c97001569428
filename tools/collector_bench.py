"""Rate of the collector (cdc_collector_*) with many concurrent callers on the
C4 share: 512 Zipf-sized files in pageable host memory, T threads each
chunking its files one call at a time (plakar's per-file goroutines,
snapshot/backup.go:216-225).  Every cut list is checked against the batch
path (cdc_chunk over the same files).  Prints one JSON line per setting.

    python tools/collector_bench.py [--callers 1,16,64] [--reps 3]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from plakar_amd import chunkers  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--callers", default="1,16,64")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--max-wait-us", default="200,2000")
    ap.add_argument("--batch-mib", type=int, default=256)
    a = ap.parse_args()
    files = bench.make_host_corpus(bench.WORKLOADS["c4"], 0, 1)
    total = sum(f.size for f in files)
    opts = chunkers.ChunkerOpts(MinSize=64 * 1024, NormalSize=1 << 20, MaxSize=4 << 20)  # bench.py's
    want = chunkers.ChunkBuffers(files, opts)  # the batch path, for the check
    for mw in [int(x) for x in a.max_wait_us.split(",")]:
        for T in [int(x) for x in a.callers.split(",")]:
            col = chunkers.Collector(opts, batch_bytes=a.batch_mib << 20, max_wait_us=mw)
            got = [None] * len(files)
            errors = []
            rates = []
            for rep in range(a.reps + 1):  # the first rep warms up (pinned staging, workspaces)
                def worker(t):
                    try:
                        for i in range(t, len(files), T):
                            got[i] = col.chunk(files[i])
                    except Exception as e:  # noqa: BLE001
                        errors.append(e)
                r0, b0 = col.stats()
                th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
                t0 = time.perf_counter()
                for t in th:
                    t.start()
                for t in th:
                    t.join()
                dt = time.perf_counter() - t0
                r1, b1 = col.stats()
                assert not errors, errors
                if rep:
                    rates.append((total / dt / 2**30, (r1 - r0) / max(b1 - b0, 1)))
            for i in range(len(files)):
                assert np.array_equal(got[i], want[i]), f"file {i}"
            col.close()
            best = max(r for r, _ in rates)
            print(json.dumps({"callers": T, "max_wait_us": mw, "GiB_s": round(best, 2),
                              "GiB_s_reps": [round(r, 2) for r, _ in rates],
                              "files_per_batch": round(rates[-1][1], 1), "files": len(files),
                              "bytes": int(total), "cut_lists": "equal to cdc_chunk"}), flush=True)


if __name__ == "__main__":
    main()
