#!/usr/bin/env python
"""bench.py — device-resident content-defined chunking throughput on MI355X.

Metric (BASELINE.json): "GiB/s chunked (device-resident, cut-points out) at
1/2/4/8 MI355X".  One step = one pass of the chunker over the rank's synthetic
input, already resident in HBM, with the (offset, length) cut lists written
to device memory.  Work per rank is fixed (weak scaling): every rank chunks its
own independent buffers; there is no data-path collective (independent files
shard one-per-GPU).  torch.distributed is used only for the
barrier and the max-over-ranks timing.

    python bench.py [--gpus N --steps K --warmup W --workload c1|c2|c3]

Default workload c1 = BASELINE configs[1]: 1x 1 GiB uniform random buffer per
GPU, default chunk params (64 KiB / 1 MiB / 4 MiB).  Prints ONE JSON line on
rank 0.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GiB/s chunked (device-resident, cut-points out) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
GIB = float(1 << 30)

WORKLOADS = {
    "c1": dict(desc="C1: 1x 1 GiB uniform random buffer per GPU (BASELINE configs[1])",
               nbuf=1, size=1 << 30, kind="random"),
    "c2": dict(desc="C2: 32x 64 MiB uniform random buffers per GPU (BASELINE configs[2], one GPU's share)",
               nbuf=32, size=64 << 20, kind="random"),
    "c3": dict(desc="C3: 1x 1 GiB zeros + 1% random bytes per GPU (BASELINE configs[3], one GPU's share)",
               nbuf=1, size=1 << 30, kind="low_entropy"),
}


def make_buffers(torch, wl, rank, dev, size):
    g = torch.Generator(device=dev)
    bufs = []
    for i in range(wl["nbuf"]):
        g.manual_seed(1 + 1000 * rank + i)
        if wl["kind"] == "random":
            t = torch.randint(0, 256, (size,), dtype=torch.uint8, device=dev, generator=g)
        else:
            t = torch.zeros(size, dtype=torch.uint8, device=dev)
            k = size // 100
            pos = torch.randint(0, size, (k,), device=dev, generator=g)
            t[pos] = torch.randint(0, 256, (k,), dtype=torch.uint8, device=dev, generator=g)
        bufs.append(t)
    return bufs


def load_traffic(workload):
    """Per-launch HBM bytes of k_scan from the rocprofv3 PMC pass committed under
    profiles/ (FETCH_SIZE corrected as MI355X_MICROARCH.md prescribes), if any."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(workload, {}).get("scan_hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(bufs_host, cuts_dev, opts, seconds):
    """The CPU oracle (scalar C restatement of the reference chunker, 1 thread)
    timed on a bounded sample of the same workload; also checks that the GPU
    cut lists of that sample are bit-identical."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_ref import Oracle
    from plakar_amd import _lib

    orc = Oracle()
    gear = _lib.default_gear()
    kw = dict(min_size=opts.MinSize, normal_size=opts.NormalSize, max_size=opts.MaxSize)
    parity = True
    done_bytes, reps, t0 = 0, 0, time.perf_counter()
    while True:
        for i, a in enumerate(bufs_host):
            ref = orc.chunk(a, gear, **kw)
            if reps == 0:
                got = cuts_dev[i].cpu().numpy().astype(np.uint64)
                parity &= bool(got.shape == ref.shape and (got == ref).all())
            done_bytes += a.size
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds or reps >= 64:
            break
    return dict(value=done_bytes / el / GIB, unit="GiB/s", cores=1, kind="port",
                sample=f"{len(bufs_host)} buffer(s) x {bufs_host[0].size / GIB:.3g} GiB, {reps} rep(s), "
                       f"{el:.1f} s, scalar C oracle (oracle/fastcdc_oracle.c), 1 thread, host of the GPU box "
                       f"(nproc={os.cpu_count()})"), parity


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c1", choices=sorted(WORKLOADS))
    ap.add_argument("--size-mib", type=int, default=0, help="override the per-buffer size (debug)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)

    import torch
    import torch.distributed as dist

    from plakar_amd import _lib, chunkers, device

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    def barrier():
        if world > 1:
            dist.barrier()

    wl = WORKLOADS[args.workload]
    size = (args.size_mib << 20) if args.size_mib else wl["size"]
    opts = chunkers.ChunkerOpts(MinSize=64 * 1024, NormalSize=1 << 20, MaxSize=4 << 20)
    _lib.ensure_init(dev_mask=0)
    bufs = make_buffers(torch, wl, rank, dev, size)
    batch = device.DeviceBatch(bufs, opts, final=True, device=local)
    L = _lib.lib()

    for _ in range(args.warmup):
        batch.launch()
    torch.cuda.synchronize(dev)
    barrier()
    L.cdc_profile_collect(None, None, None, None)
    L.cdc_profile_enable(1)
    torch.cuda.synchronize(dev)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        batch.launch()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    barrier()
    L.cdc_profile_enable(0)
    scan_ms, pipe_ms = ctypes.c_double(), ctypes.c_double()
    launches, scan_bytes = ctypes.c_uint64(), ctypes.c_uint64()
    _lib.check(L.cdc_profile_collect(ctypes.byref(scan_ms), ctypes.byref(pipe_ms),
                                     ctypes.byref(launches), ctypes.byref(scan_bytes)), "profile")
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    cuts, res = batch.results()
    nchunks = int(res[:, 0].sum())
    per_rank_bytes = sum(t.numel() for t in bufs)
    value = world * per_rank_bytes * args.steps / elapsed / GIB

    n = max(int(launches.value), 1)
    scan_avg_ms = scan_ms.value / n
    pipe_avg_ms = pipe_ms.value / n
    bytes_per_launch = scan_bytes.value / n
    achieved = bytes_per_launch / (scan_avg_ms * 1e-3) / 1e9
    roofline = dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(achieved / HBM_PEAK_GBS, 4), traffic=load_traffic(args.workload),
                    kernel="k_scan", kernel_avg_ms=round(scan_avg_ms, 4),
                    algorithmic_bytes_per_launch=int(bytes_per_launch),
                    pipeline_avg_ms=round(pipe_avg_ms, 4))

    baseline, parity = None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        host = [t.cpu().numpy() for t in bufs[:1]]
        baseline, parity = cpu_baseline(host, cuts[:1], opts, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (torch Philox uniform bytes generated on the GPU; no dataset)",
            "config": {"workload": wl["desc"], "bytes_per_gpu": per_rank_bytes,
                       "global_bytes": per_rank_bytes * world, "buffers_per_gpu": len(bufs),
                       "chunk_params": "FASTCDC min 65536 / normal 1048576 / max 4194304",
                       "gear": "placeholder (v0.0.8 table unavailable; see DESIGN.md)",
                       "parallelism": f"independent buffers, 1 rank per GPU x {world}, no collective",
                       "chunks_per_step": nchunks},
            "roofline": roofline,
            "cpu_baseline": baseline,
            "parity_vs_oracle": parity,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    sys.stdout.flush()
    sys.stderr.flush()
    L.cdc_shutdown()


if __name__ == "__main__":
    main()
