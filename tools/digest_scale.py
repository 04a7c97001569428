"""Per-chunk SHA-256 + histogram throughput vs. chunks per launch: one
k_chunk_digest launch group over the cut lists of k independent 1-GiB C1
buffers (k = 1, 2, 4, 8, 16).
    python tools/digest_scale.py [max_k] [only] [lanes=N,M,...]
only: just k = max_k; nohist: digests only; same: every launch's k buffers are the first one (1 GiB
footprint, the same chunk count); lanes: also time each launch with the digest kernels
told that N (M, ...) lanes are resident (cdc_debug_set_digest_lanes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch

from bench import GIB, WORKLOADS, make_buffers
from plakar_amd import _lib, chunkers, device, hashing

kmax = int(sys.argv[1]) if len(sys.argv) > 1 else 16
_lib.ensure_init()
dev = torch.device("cuda", 0)
wl = dict(WORKLOADS["c2"])
wl["nbuf"] = 1 if "same" in sys.argv else kmax
bufs = make_buffers(torch, wl, 0, dev, 1 << 30)
bufs = bufs * (kmax // len(bufs))
b = device.DeviceBatch(bufs, chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20))
b.launch()
torch.cuda.synchronize()
cuts = [b.cuts[i] for i in range(b.n)]
res = [b.res[i] for i in range(b.n)]
lane_opts = [0]
for a in sys.argv:
    if a.startswith("lanes="):
        lane_opts += [int(x) for x in a[6:].split(",")]


def timed(k, lanes):
    _lib.lib().cdc_debug_set_digest_lanes(lanes)
    run = lambda: hashing.chunk_digests_batch(bufs[:k], cuts[:k], res[:k], hist="nohist" not in sys.argv)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 3


k = kmax if "only" in sys.argv else 1
while k <= kmax:
    for lanes in lane_opts:
        ms = timed(k, lanes)
        print(f"k={k:2d} buffers ({k} GiB), lanes {lanes or 'default'}: {ms:8.2f} ms per launch group, "
              f"{k / (ms * 1e-3):7.1f} GiB/s", flush=True)
    k *= 2
