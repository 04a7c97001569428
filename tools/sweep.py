"""Parameter sweep of the device path (one subprocess per configuration).

    python tools/sweep.py "VAR=a,b;VAR2=c,d" [--size-mib 1024] [--workload c1]

Each configuration runs a fresh process with the env vars set, chunks the
same synthetic buffer(s) and prints scan / pipeline time and the scan kernel's
HBM-read rate.  Results are checked against the first configuration's cut
lists (a checksum), so a variant that changes results shows up at once.
"""
import itertools
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(size_mib, workload, steps):
    sys.path.insert(0, ROOT)
    import ctypes

    import torch

    from bench import WORKLOADS, make_buffers
    from plakar_amd import _lib, chunkers, device

    wl = WORKLOADS[workload]
    dev = torch.device("cuda", 0)
    _lib.ensure_init()
    bufs = make_buffers(torch, wl, 0, dev, size_mib << 20)
    opts = chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20)
    b = device.DeviceBatch(bufs, opts)
    L = _lib.lib()
    for _ in range(2):
        b.launch()
    torch.cuda.synchronize()
    L.cdc_profile_collect(None, None, None, None)
    L.cdc_profile_enable(1)
    t0 = time.perf_counter()
    for _ in range(steps):
        b.launch()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    L.cdc_profile_enable(0)
    s, p = ctypes.c_double(), ctypes.c_double()
    n, by = ctypes.c_uint64(), ctypes.c_uint64()
    L.cdc_profile_collect(ctypes.byref(s), ctypes.byref(p), ctypes.byref(n), ctypes.byref(by))
    cuts, res = b.results()
    ck = int(sum(int(c[:, 0].sum().item()) * 31 + int(c.shape[0]) for c in cuts))
    k = max(n.value, 1)
    print(json.dumps(dict(scan_ms=s.value / k, pipe_ms=p.value / k, wall_ms=(t1 - t0) / steps * 1e3,
                          scan_gbs=by.value / k / (s.value / k * 1e-3) / 1e9,
                          gibs=sum(t.numel() for t in bufs) / ((t1 - t0) / steps) / (1 << 30),
                          checksum=ck)))


def main():
    if "--child" in sys.argv:
        i = sys.argv.index("--child")
        child(int(sys.argv[i + 1]), sys.argv[i + 2], int(sys.argv[i + 3]))
        return
    spec = sys.argv[1]
    size = int(sys.argv[sys.argv.index("--size-mib") + 1]) if "--size-mib" in sys.argv else 1024
    wl = sys.argv[sys.argv.index("--workload") + 1] if "--workload" in sys.argv else "c1"
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 10
    axes = []
    for part in spec.split(";"):
        k, vals = part.split("=")
        axes.append([(k, v) for v in vals.split(",")])
    ref = None
    for combo in itertools.product(*axes):
        env = dict(os.environ)
        env.update(dict(combo))
        r = subprocess.run([sys.executable, __file__, "--child", str(size), wl, str(steps)], env=env,
                           capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        tag = " ".join(f"{k}={v}" for k, v in combo)
        if r.returncode != 0 or not line:
            print(f"{tag}: FAILED rc={r.returncode} {r.stderr[-500:]}", flush=True)
            continue
        d = json.loads(line[-1])
        if ref is None:
            ref = d["checksum"]
        ok = "ok" if d["checksum"] == ref else "CHECKSUM MISMATCH"
        print(f"{tag:40s} scan {d['scan_ms']*1e3:8.1f} us ({d['scan_gbs']:7.1f} GB/s)  pipe {d['pipe_ms']*1e3:8.1f} us  "
              f"wall {d['wall_ms']*1e3:8.1f} us  {d['gibs']:8.1f} GiB/s  {ok}", flush=True)


if __name__ == "__main__":
    main()
