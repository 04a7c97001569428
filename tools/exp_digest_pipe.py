"""Pipelined chunk + digest rate vs passes in flight (bench.chunk_digest_pipeline)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import WORKLOADS, chunk_digest_pipeline, make_buffers  # noqa: E402
from plakar_amd import _lib, chunkers  # noqa: E402

_lib.ensure_init()
dev = torch.device("cuda", 0)
opts = chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20)
for wl in sys.argv[1:] or ["c1"]:
    bufs = make_buffers(torch, WORKLOADS[wl], 0, dev, WORKLOADS[wl]["size"])
    for s in (1, 2, 3, 4, 6, 8, 12):
        print(wl, s, chunk_digest_pipeline(torch, bufs, opts, dev, s, max(2 * s, 8)), flush=True)
