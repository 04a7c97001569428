"""Per-copy cost of small pageable host->device copies (hipMemcpyAsync from
pageable memory, as cdc_chunk's direct staging issues them), against packing
the same buffers into pinned memory and copying once.
    python tools/h2d_small.py"""
import ctypes
import time

import numpy as np
import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
d = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
s = torch.cuda.Stream()
torch.cuda.synchronize()
for size in (4 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20):
    n = max(8, min(256, (256 << 20) // size))
    hs = [np.random.randint(0, 255, size, dtype=np.uint8) for _ in range(n)]
    for rep in range(2):
        t0 = time.perf_counter()
        off = 0
        for h in hs:
            hip.hipMemcpyAsync(ctypes.c_void_p(d.data_ptr() + off), ctypes.c_void_p(h.ctypes.data), size, 1,
                               ctypes.c_void_p(s.cuda_stream))
            off += size
        hip.hipStreamSynchronize(ctypes.c_void_p(s.cuda_stream))
        dt = time.perf_counter() - t0
    pin = torch.empty(n * size, dtype=torch.uint8, pin_memory=True).numpy()
    for rep in range(2):
        t0 = time.perf_counter()
        for i, h in enumerate(hs):
            pin[i * size:(i + 1) * size] = h
        hip.hipMemcpyAsync(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(pin.ctypes.data), n * size, 1,
                           ctypes.c_void_p(s.cuda_stream))
        hip.hipStreamSynchronize(ctypes.c_void_p(s.cuda_stream))
        dp = time.perf_counter() - t0
    print(f"{size >> 10:6d} KiB x {n}: pageable per copy {dt / n * 1e6:7.1f} us ({n * size / dt / 1e9:5.1f} GB/s); "
          f"packed into pinned + one copy {dp / n * 1e6:7.1f} us per buffer ({n * size / dp / 1e9:5.1f} GB/s)", flush=True)

# the same pageable copies issued from 4 host threads, each on its own stream
import threading
streams = [torch.cuda.Stream() for _ in range(4)]
for size in (64 << 10, 256 << 10, 1 << 20, 4 << 20):
    n = max(8, min(256, (256 << 20) // size))
    hs = [np.random.randint(0, 255, size, dtype=np.uint8) for _ in range(n)]

    def run(t):
        for i in range(t, n, 4):
            hip.hipMemcpyAsync(ctypes.c_void_p(d.data_ptr() + i * size), ctypes.c_void_p(hs[i].ctypes.data), size, 1,
                               ctypes.c_void_p(streams[t].cuda_stream))
        hip.hipStreamSynchronize(ctypes.c_void_p(streams[t].cuda_stream))
    for rep in range(2):
        t0 = time.perf_counter()
        th = [threading.Thread(target=run, args=(t,)) for t in range(4)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        dt = time.perf_counter() - t0
    print(f"{size >> 10:6d} KiB x {n}: pageable from 4 threads {dt / n * 1e6:7.1f} us per copy ({n * size / dt / 1e9:5.1f} GB/s)",
          flush=True)
