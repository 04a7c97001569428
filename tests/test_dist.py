"""Multi-process (gloo, world_size 2) tests of the N-GPU path's host logic:
buffer sharding across ranks (no data-path collective) and the max-over-ranks
timing that bench.py reports.  CPU only."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cpu")
        out = {}
        for name, wl in bench.WORKLOADS.items():
            out[name] = bench.buffer_seeds(wl, rank, world)
        dist.barrier()
        t = bench.reduce_max(dist, world, 1.0 + rank, dev)
        # all-gather the shard assignment to check it on every rank
        gathered = [None] * world
        dist.all_gather_object(gathered, out)
        q.put((rank, t, gathered))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharding_and_max_timing_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, t, gathered in res:
        assert t == float(world)  # max over ranks of 1 + rank
        for name, wl in bench.WORKLOADS.items():
            seeds = [s for g in gathered for s in g[name]]
            assert len(seeds) == len(set(seeds)) == world * wl["nbuf"]  # disjoint shards


def test_c2_shards_cover_baseline_config():
    """At 8 ranks, C2 is exactly the 256 x 64 MiB buffers of BASELINE configs[2]."""
    wl = bench.WORKLOADS["c2"]
    seeds = [s for r in range(8) for s in bench.buffer_seeds(wl, r, 8)]
    assert len(set(seeds)) == 256 and wl["size"] == 64 << 20
