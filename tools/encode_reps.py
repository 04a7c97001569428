"""Per-call times of the Encode leg (LZ4 frame + AES-256-GCM of every chunk
of a pass), one synchronised call at a time, to find what separates fast and
slow calls.  Run it under rocprofv3 --kernel-trace --memory-copy-trace to see
each call's kernels and copies (calls are marked by the CALL lines' times):

    python tools/encode_reps.py [--workload c2] [--reps 12]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--reps", type=int, default=12)
    a = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from plakar_amd import _lib, chunkers, device, encode
    _lib.ensure_init()
    dev = torch.device("cuda", 0)
    wl = bench.WORKLOADS[a.workload]
    bufs = bench.make_buffers(torch, wl, 0, dev, wl["size"])
    opts = chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20)
    b = device.DeviceBatch(bufs, opts)
    b.launch()
    cuts, _ = b.results()
    base = min(bufs, key=lambda t: t.data_ptr())
    offs, lens = [], []
    for t, c in zip(bufs, cuts):
        c = c.cpu().numpy().astype(np.int64)
        offs.append(c[:, 0] + (t.data_ptr() - base.data_ptr()))
        lens.append(c[:, 1])
    offs, lens = np.concatenate(offs), np.concatenate(lens)
    cap = sum(encode.encode_bound(int(x)) for x in lens)
    out = torch.empty(cap, dtype=torch.uint8, device=dev)
    key = os.urandom(32)
    total = sum(t.numel() for t in bufs)
    encode.encode_device(base, offs, lens, out, key=key)
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for r in range(a.reps):
        t0 = time.perf_counter()
        encode.encode_device(base, offs, lens, out, key=key)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"CALL {r:2d} start {1e3 * (t0 - t_start):9.3f} ms  returned +{1e3 * (t1 - t0):7.3f}  "
              f"done +{1e3 * (t2 - t0):7.3f} ms  {total / (t2 - t0) / 2**30:7.1f} GiB/s", flush=True)
    print(f"{len(lens)} blobs, {total / 2**30:.2f} GiB")


if __name__ == "__main__":
    main()
