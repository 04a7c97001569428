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


def _run_bench(args, extra_env):
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra_env)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=env, cwd=root,
                       capture_output=True, text=True, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


@pytest.mark.parametrize("n", [2, 3])
def test_bench_spawns_its_own_ranks(n):
    """`python bench.py --gpus N` with no launcher starts N rank processes
    (gloo rendezvous on 127.0.0.1) and reports n_gpus = N with one timing per
    rank; BENCH_CPU_SELFTEST runs the plumbing without a GPU."""
    rc, line, err = _run_bench(["--gpus", str(n)], {"BENCH_CPU_SELFTEST": "1"})
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == n and line["selftest"]
    assert len(line["per_rank_elapsed_s"]) == n
    # every rank checked its own cut lists (AND over ranks), rank 0 timed the CPU baseline
    assert line["parity_vs_oracle"] is True
    assert line["cpu_baseline"] is not None and line["cpu_baseline"]["value"] > 0
    # the max over ranks is the slowest rank's time (rank r sleeps (r + 1) * 10 ms)
    assert line["elapsed_max_s"] == max(line["per_rank_elapsed_s"])
    assert line["per_rank_elapsed_s"][-1] >= 0.01 * n


def test_bench_parity_is_the_and_over_ranks():
    """One rank whose cut lists differ from the oracle turns the line's
    parity_vs_oracle false, whichever rank it is."""
    rc, line, err = _run_bench(["--gpus", "2"], {"BENCH_CPU_SELFTEST": "1", "BENCH_SELFTEST_BAD_RANK": "1"})
    assert rc == 0, err[-2000:]
    assert line["parity_vs_oracle"] is False


@pytest.mark.parametrize("box", ["cpu", pytest.param("gpu-box", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("when", ["before", "after"])
def test_bench_fails_fast_when_a_rank_dies(box, when):
    """a failure surfaces as an error, never a hang.  Rank 1
    exits 3 before the rendezvous (rank 0 would wait in init_process_group) or
    after it (rank 0 would wait in the next collective): `--gpus 2` returns 3
    within 60 s, the other rank terminated.  Also run in the GPU suite (the
    plumbing is the same on the box)."""
    import time
    t0 = time.time()
    rc, line, err = _run_bench(["--gpus", "2"], {"BENCH_CPU_SELFTEST": "1", "BENCH_SELFTEST_FAIL_RANK": "1",
                                                 "BENCH_SELFTEST_FAIL_AT": when, "BENCH_DIST_TIMEOUT_S": "300"})
    el = time.time() - t0
    assert rc == 3, err[-2000:]
    assert el < 60, f"took {el:.1f} s"
    assert "rank 1 exited with status 3" in err
    assert line is None


def test_bench_refuses_a_mismatched_launcher():
    """A launcher that started a different number of ranks than --gpus asks
    for is an error, never a silent 1-rank run."""
    rc, line, err = _run_bench(["--gpus", "2"], {"BENCH_CPU_SELFTEST": "1", "WORLD_SIZE": "1", "RANK": "0"})
    assert rc != 0 and line is None
    assert "WORLD_SIZE=1" in err


def test_bench_refuses_diagnostic_settings():
    """bench.py will not measure with settings that change what the kernels do
    (CDC_DIAG_*, a non-zero CDC_DEBUG_PHASE); every CDC_* variable it accepts
    is recorded in the line's config."""
    rc, line, err = _run_bench(["--gpus", "1"], {"BENCH_CPU_SELFTEST": "1", "CDC_DEBUG_PHASE": "16"})
    assert rc == 2 and line is None and "CDC_DEBUG_PHASE" in err
    rc, line, err = _run_bench(["--gpus", "1"], {"BENCH_CPU_SELFTEST": "1", "CDC_DIAG_ANYTHING": "1"})
    assert rc == 2 and "CDC_DIAG_ANYTHING" in err
