"""Device Encode throughput (LZ4 frame + AES-256-GCM stream) on chunked
buffers: python tools/encode_bench.py [--size-mib 1024] [--reps 5]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size-mib", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--kinds", default="random,low_entropy,text")
    ap.add_argument("--labels", default="lz4+gcm,lz4,gcm")
    a = ap.parse_args()
    import numpy as np
    import torch

    from datagen import low_entropy, random_bytes
    from plakar_amd import _lib, chunkers, device, encode
    _lib.ensure_init()
    n = a.size_mib << 20
    kinds = {
        "random": lambda: random_bytes(n, 1),
        "low_entropy": lambda: low_entropy(n, 3),
        "text": lambda: np.frombuffer((b"backup snapshot chunk packfile plakar " * (n // 38 + 1))[:n], np.uint8).copy(),
    }
    key = os.urandom(32)
    opts = chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20)
    kinds = {k: v for k, v in kinds.items() if k in a.kinds.split(",")}
    for kind, make in kinds.items():
        t = torch.from_numpy(make()).cuda()
        b = device.DeviceBatch([t], opts)
        b.launch()
        (cuts,), _ = b.results()
        c = cuts.cpu().numpy().astype(np.int64)
        offs, lens = c[:, 0].copy(), c[:, 1].copy()
        for label, k, comp in (("lz4+gcm", key, True), ("lz4", None, True), ("gcm", key, False)):
            if label not in a.labels.split(","):
                continue
            cap = sum(encode.encode_bound(x, comp, k is not None) for x in lens)
            out = torch.empty(cap, dtype=torch.uint8, device="cuda")
            encode.encode_device(t, offs, lens, out, key=k, compress=comp)  # warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                oo = encode.encode_device(t, offs, lens, out, key=k, compress=comp)
            torch.cuda.synchronize()
            el = (time.perf_counter() - t0) / a.reps
            print(f"{kind:12s} {label:8s} {len(lens):6d} blobs  {n / el / 2**30:8.1f} GiB/s  ratio {oo[-1] / n:.3f}",
                  flush=True)


if __name__ == "__main__":
    main()
