"""Host->device copy rates on the box: pinned and pageable torch copies, 1 GiB."""
import time

import torch

n = 1 << 30
d = torch.empty(n, dtype=torch.uint8, device="cuda")
for pinned in (True, False):
    h = torch.empty(n, dtype=torch.uint8, pin_memory=pinned)
    h.fill_(1)
    for _ in range(2):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
    print(f"H2D pinned={pinned}: {n / dt / 1e9:.1f} GB/s", flush=True)
h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
t0 = time.perf_counter()
for _ in range(3):
    h.copy_(d, non_blocking=True)
torch.cuda.synchronize()
print(f"D2H pinned: {3 * n / (time.perf_counter() - t0) / 1e9:.1f} GB/s")
