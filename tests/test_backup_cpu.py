"""The c4b CPU baseline (oracle/backup_cpu.c, bench.py only): the whole backup
leg on host cores does the reference's work per file.  Checked against the C
oracle's chunkify and hashlib on a small corpus (CPU only)."""
import hashlib
import os

import numpy as np

import bench
from oracle_ref import Oracle
from plakar_amd import _lib, chunkers

OPTS = chunkers.ChunkerOpts(MinSize=65536, NormalSize=1 << 20, MaxSize=4 << 20)


def test_backup_cpu_baseline_chunks_dedups_and_counts(tmp_path):
    sizes = [0, 1, 5000, 65535, 65536, 300_000, 3 << 20, 9 << 20]
    blobs = [np.random.PCG64(7 + i).random_raw((n + 7) // 8).view(np.uint8)[:n].copy() for i, n in enumerate(sizes)]
    blobs.append(blobs[6].copy())  # a duplicate: its chunks are not stored again
    paths = []
    for i, b in enumerate(blobs):
        p = tmp_path / f"f{i}"
        p.write_bytes(b.tobytes())
        paths.append(str(p))
    paths.append(str(tmp_path / "missing"))
    r = bench.backup_cpu_baseline(paths, OPTS, 3, os.urandom(32))
    orc, gear = Oracle(), _lib.default_gear()
    digests, nchunks = set(), 0
    for b in blobs:
        if b.size < OPTS.MinSize:  # chunkify routing: one chunk (an empty file: one empty chunk)
            cuts = [(0, b.size)]
        else:
            cuts = orc.chunk(b, gear, min_size=OPTS.MinSize, normal_size=OPTS.NormalSize, max_size=OPTS.MaxSize)
        nchunks += len(cuts)
        digests |= {hashlib.sha256(b[int(o):int(o + n)].tobytes()).digest() for o, n in cuts}
    assert r["chunks"] == nchunks and r["new_blobs"] == len(digests)
    assert r["value"] > 0 and r["cores"] == 3 and "10 files" in r["sample"]
