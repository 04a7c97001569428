"""One rank of the multi-rank parity run (tests/test_gpu_scale.py).

Launched by torch.distributed.run with N ranks: every rank chunks its own share
of BASELINE configs[2] (bench.buffer_seeds: rank r owns buffers r*nbuf ..
r*nbuf + nbuf - 1) on its GPU -- or, with DIST_ONE_GPU=1, every rank on device
0 (a one-GPU box) -- and checks every cut list against the CPU oracle.  The
ranks exchange only a failure count (gloo all_reduce), as bench.py exchanges
only its timing: independent buffers shard with no data collective
(SURVEY.md 8e).  Rank 0 prints one JSON line.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist

    from bench import WORKLOADS, buffer_seeds, make_buffers
    from oracle_ref import Oracle
    from plakar_amd import _lib, chunkers, device

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = 0 if os.environ.get("DIST_ONE_GPU") == "1" else int(os.environ.get("LOCAL_RANK", "0"))
    size = int(os.environ.get("DIST_BUF_MIB", "64")) << 20
    nbuf = int(os.environ.get("DIST_NBUF", "32"))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    _lib.ensure_init(dev_mask=1 << local)
    wl = dict(WORKLOADS["c2"], nbuf=nbuf)
    bufs = make_buffers(torch, wl, rank, dev, size, world)
    opts = chunkers.ChunkerOpts(MinSize=65536, NormalSize=1 << 20, MaxSize=4 << 20)
    batch = device.DeviceBatch(bufs, opts, final=True, device=local)
    batch.launch()
    cuts, _ = batch.results()
    orc = Oracle()
    gear = _lib.default_gear()
    bad = 0
    nchunks = 0
    for t, c in zip(bufs, cuts):
        ref = orc.chunk(t.cpu().numpy(), gear, min_size=65536, normal_size=1 << 20, max_size=4 << 20)
        got = c.cpu().numpy().astype(np.uint64)
        nchunks += got.shape[0]
        bad += int(not (got.shape == ref.shape and (got == ref).all()))
    tot = torch.tensor([bad, nchunks, len(bufs)], dtype=torch.int64)
    dist.all_reduce(tot)
    if rank == 0:
        print(json.dumps({"ranks": world, "buffers": int(tot[2]), "chunks": int(tot[1]), "mismatched_buffers": int(tot[0]),
                          "seeds_rank0": buffer_seeds(wl, 0, world)[:3]}), flush=True)
    dist.destroy_process_group()
    _lib.lib().cdc_shutdown()
    return 0 if int(tot[0]) == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
