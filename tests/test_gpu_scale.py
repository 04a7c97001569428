"""GPU parity at the shapes the benchmark and the driver use (BASELINE.json
configs), plus the multi-rank and multi-device paths and the sequential
fallback's cost.  Every check is bit-exact against the CPU oracle.
"""
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from datagen import random_bytes  # noqa: E402
from plakar_amd import _lib, chunkers, device  # noqa: E402

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEF = dict(min_size=65536, normal_size=1 << 20, max_size=4 << 20)
OPTS = chunkers.ChunkerOpts(MinSize=65536, NormalSize=1 << 20, MaxSize=4 << 20)


def assert_same(got, ref, what=""):
    got = np.asarray(got).astype(np.uint64)
    assert got.shape == ref.shape, f"{what}: {got.shape[0]} chunks vs oracle {ref.shape[0]}"
    bad = np.nonzero((got != ref).any(axis=1))[0]
    assert bad.size == 0, f"{what}: first mismatch at chunk {bad[0]}: {got[bad[0]]} vs {ref[bad[0]]}"


def test_c4_full_gpu_share_host_path(oracle):
    """BASELINE configs[4], one GPU's share exactly as bench.py builds it (the
    first 512 files of the 4096-file Zipf corpus, seeds 1..512): chunkify
    routing (snapshot/backup.go:631-644: files < MinSize are one chunk, no CDC),
    the rest through cdc_chunk; every file checked against the oracle."""
    from bench import WORKLOADS, make_host_corpus
    _lib.ensure_init()
    corpus = make_host_corpus(WORKLOADS["c4"], 0, 1)
    assert len(corpus) == 512
    big = [a for a in corpus if a.size >= DEF["min_size"]]
    small = [a for a in corpus if a.size < DEF["min_size"]]
    assert big and small
    res = chunkers.ChunkBuffers(big, OPTS)
    gear = _lib.default_gear()
    for i, a in enumerate(big):
        assert_same(res[i], oracle.chunk(a, gear, **DEF), f"file {i} ({a.size} B)")
    for a in small:  # routed: one chunk, the oracle's chunkify agrees
        ref = oracle.chunk(a, gear, chunkify=True, **DEF)
        assert ref.shape[0] == 1 and int(ref[0, 1]) == a.size


def test_cdc_chunk_all_visible_devices(oracle):
    """cdc_chunk with dev_mask = 0 (every visible device, LPT over devices)."""
    _lib.ensure_init(dev_mask=0)
    n = _lib.lib().cdc_device_count()
    assert n >= 1
    bufs = [random_bytes(s, 900 + i) for i, s in enumerate([96 << 20, 5 << 20, 33 << 20, 1 << 20, 0, 200_000])]
    res = chunkers.ChunkBuffers(bufs, OPTS)
    gear = _lib.default_gear()
    for i, a in enumerate(bufs):
        assert_same(res[i], oracle.chunk(a, gear, **DEF), f"buffer {i}")


def test_buffer_over_4GiB_host_path(oracle):
    """One 4.5 GiB buffer through cdc_chunk (offsets past 2^32, staged whole)."""
    _lib.ensure_init()
    n = (4 << 30) + (512 << 20)
    a = random_bytes(n, 4242)
    (got,) = chunkers.ChunkBuffers([a], OPTS)
    ref = oracle.chunk(a, _lib.default_gear(), **DEF)
    assert int(ref[-1, 0]) > (1 << 32)
    assert_same(got, ref, "4.5 GiB")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_ranks_c2_shares_on_one_gpu():
    """The N-rank path of bench.py on hardware: 2 ranks (torch.distributed.run,
    gloo), both on device 0 of a one-GPU box, each chunking its own share of
    BASELINE configs[2] (32 x 64 MiB, bench.buffer_seeds) and checking every
    cut list against the oracle; only a failure count crosses ranks."""
    env = dict(os.environ, DIST_ONE_GPU="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dist_c2_worker.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    import json
    d = json.loads(line)
    assert d["ranks"] == 2 and d["buffers"] == 64 and d["mismatched_buffers"] == 0, d


def test_bench_spawns_two_ranks_on_one_gpu():
    """`python bench.py --gpus 2` with no launcher (the form the driver uses
    for BENCH) starts two rank processes itself; BENCH_REHEARSE_ONE_GPU puts
    both on device 0 over gloo.  The line reports both ranks."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["BENCH_REHEARSE_ONE_GPU"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--size-mib", "64", "--cpu-seconds", "1", "--cpu-threads", "1", "--digest-reps", "0", "--encode-reps",
           "0", "--e2e-reps", "0"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    import json
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert d["n_gpus"] == 2 and len(d["config"]["per_rank_gibs"]) == 2, d
    assert d["config"]["global_bytes"] == 2 * d["config"]["bytes_per_gpu"]
    # each rank's cut lists checked against the oracle (AND over ranks); the CPU baseline at N = 2
    assert d["parity_vs_oracle"] is True, d
    assert d["cpu_baseline"] is not None and d["cpu_baseline"]["value"] > 0, d


def test_bench_rccl_path_one_rank():
    """The N-GPU run's RCCL code -- init_process_group("nccl") with the
    device id, the barriers around the timed region, the max-over-ranks
    all_reduce, the per-rank all_gather and the parity AND, all on device
    tensors -- executed on a one-GPU box by a one-rank process group
    (BENCH_DIST_ONE_RANK=1).  Two ranks cannot share one GPU under RCCL, so
    this is the closest the box gets to the 8-GPU run's collective path."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["BENCH_DIST_ONE_RANK"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "1",
           "--size-mib", "64", "--no-cpu-baseline", "--digest-reps", "0", "--encode-reps", "0", "--e2e-reps", "0"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    import json
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert d["config"]["dist_backend"] == "nccl", d["config"]
    assert d["n_gpus"] == 1 and len(d["config"]["per_rank_gibs"]) == 1 and d["value"] > 0, d
    assert d["parity_vs_oracle"] is True, d


def test_sequential_fallback_cost_1GiB(oracle):
    """The sequential fallback (debug mode 1 forces it) on a 1 GiB buffer: the
    cliff a buffer whose speculative chains never merge would hit.  Bit-exact,
    and its time is printed (DESIGN.md records it)."""
    _lib.ensure_init()
    a = random_bytes(1 << 30, 77)
    t = torch.from_numpy(a).to("cuda")
    L = _lib.lib()
    try:
        L.cdc_set_debug_mode(1)
        b = device.DeviceBatch([t], OPTS)
        b.launch()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        b.launch()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        cuts, _ = b.results()
    finally:
        L.cdc_set_debug_mode(0)
    ref = oracle.chunk(a, _lib.default_gear(), **DEF)
    assert_same(cuts[0].cpu().numpy(), ref, "sequential 1 GiB")
    print(f"\nsequential fallback: 1 GiB, {ref.shape[0]} chunks in {el * 1e3:.1f} ms "
          f"({el * 1e6 / ref.shape[0]:.2f} us per chunk)")


def test_file_batch_pinned_arena(oracle, tmp_path):
    """Files read by the library (pread, 8 threads) into its pinned arena, then
    one cdc_batch_chunk; bytes and cut lists checked against the files and the
    oracle (snapshot/importer/fs/fs.go:69-71 + snapshot/backup.go:647-665)."""
    _lib.ensure_init()
    sizes = [0, 1, 65535, 65536, 3 << 20, (17 << 20) + 5, 40 << 20, 123_457]
    paths, datas = [], []
    for i, n in enumerate(sizes):
        a = random_bytes(n, 700 + i)
        p = tmp_path / f"f{i}"
        p.write_bytes(a.tobytes())
        paths.append(str(p))
        datas.append(a)
    fb = chunkers.FileBatch(sum((n + 4095) // 4096 * 4096 for n in sizes))
    assert fb.add_files(paths, threads=8) == sizes
    assert len(fb) == len(sizes)
    for i, a in enumerate(datas):
        assert np.array_equal(fb.buffer(i), a)
    res = fb.chunk(OPTS)
    gear = _lib.default_gear()
    for i, a in enumerate(datas):
        assert_same(res[i], oracle.chunk(a, gear, **DEF), f"file {i}")
    fb.reset()
    assert len(fb) == 0
    fb.close()


def test_file_batch_more_files_than_fd_limit(oracle, tmp_path):
    """A batch of more files than RLIMIT_NOFILE allows: the library holds at
    most one descriptor per reader thread (stat for sizes, then open / read /
    close per file), so both file-arena calls succeed with the soft limit
    lowered to 64 descriptors."""
    import resource
    _lib.ensure_init()
    nfiles = 300
    sizes = [(i * 7919) % 200_000 + (70_000 if i % 3 == 0 else 0) for i in range(nfiles)]
    paths, datas = [], []
    for i, n in enumerate(sizes):
        a = random_bytes(n, 900 + i)
        p = tmp_path / f"h{i}"
        p.write_bytes(a.tobytes())
        paths.append(str(p))
        datas.append(a)
    cap = sum((n + 4095) // 4096 * 4096 for n in sizes)
    fb = chunkers.FileBatch(cap)
    soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
    resource.setrlimit(resource.RLIMIT_NOFILE, (min(64, hard), hard))
    try:
        got_sizes = fb.add_files(paths, threads=8)
        res1 = fb.chunk(OPTS)
        fb.reset()
        res2 = fb.add_and_chunk(paths, OPTS, threads=8)
    finally:
        resource.setrlimit(resource.RLIMIT_NOFILE, (soft, hard))
    assert got_sizes == sizes
    gear = _lib.default_gear()
    for i, a in enumerate(datas):
        ref = oracle.chunk(a, gear, **DEF)
        assert_same(res1[i], ref, f"add_files file {i}")
        assert_same(res2[i], ref, f"chunk_files file {i}")
    fb.close()


def test_file_batch_chunk_files_overlapped(oracle, tmp_path):
    """cdc_batch_chunk_files: the files read into the arena by reader threads
    while the device chunks each >= 256-MiB sub-batch (here two) as soon as
    it is read; cut lists vs the oracle, bytes kept in the arena, and
    CDC_E_NOSPACE with the needed count when the cut array is short."""
    import ctypes
    _lib.ensure_init()
    sizes = [0, 1, 65535, 150 << 20, 3 << 20, 130 << 20, 77_000, 40 << 20]
    paths, datas = [], []
    for i, n in enumerate(sizes):
        a = random_bytes(n, 800 + i)
        p = tmp_path / f"g{i}"
        p.write_bytes(a.tobytes())
        paths.append(str(p))
        datas.append(a)
    cap = sum((n + 4095) // 4096 * 4096 for n in sizes)
    fb = chunkers.FileBatch(cap)
    res = fb.add_and_chunk(paths, OPTS, threads=8)
    assert len(fb) == len(sizes)
    gear = _lib.default_gear()
    for i, a in enumerate(datas):
        assert np.array_equal(fb.buffer(i), a)
        assert_same(res[i], oracle.chunk(a, gear, **DEF), f"file {i}")
    total = sum(r.shape[0] for r in res)
    fb.reset()
    L = _lib.lib()
    n = len(paths)
    arr = (ctypes.c_char_p * n)(*[p.encode() for p in paths])
    out = (_lib.cdc_cut * 3)()
    counts = (ctypes.c_uint64 * n)()
    needed = ctypes.c_uint64()
    st = L.cdc_batch_chunk_files(fb._h, arr, n, 4, ctypes.byref(OPTS._c()), out, 3, counts, ctypes.byref(needed), None)
    assert st == _lib.CDC_E_NOSPACE and needed.value == total
    assert [counts[i] for i in range(n)] == [r.shape[0] for r in res]
    fb.close()


def test_backup_batch_packfiles(oracle):
    """chunkify on the device -> PutBlob of every new chunk -> packfiles (the
    re-plumbed snapshot/backup.go:594-629 + snapshot/packer.go): each packfile
    parses as packfile.go's format (tests/packfile_ref.py), every new chunk is
    stored once, already-known ones are skipped, and every blob is Encode(the
    file's bytes at the device cut) with that chunk's SHA-256 as its key."""
    import hashlib
    import zlib

    import packfile_ref as ref
    from plakar_amd import snapshot
    _lib.ensure_init()
    files = [random_bytes(n, 60 + i) for i, n in enumerate([0, 1000, 70_000, 5 << 20, 9 << 20, 33 << 20])]
    files.append(files[3].copy())  # duplicate content: deduplicated
    gear = _lib.default_gear()
    want = {}
    for f in files:
        rows = oracle.chunk(f, gear, chunkify=True, **DEF) if f.size else np.array([[0, 0]], np.uint64)
        for o, n in rows:
            data = f[int(o):int(o + n)].tobytes()
            want[hashlib.sha256(data).digest()] = data
    first = next(iter(want))
    for encode in (None, lambda b: zlib.compress(b, 1)):
        known = {first}
        objs, packs = snapshot.backup_batch(files, known=set(known), max_size=8 << 20, encode=encode, timestamp=5)
        assert len(objs) == len(files)
        got = {}
        for pk in packs:
            pf = ref.parse(pk)
            assert pf.timestamp == 5
            for t, c, o, n in pf.index:
                assert t == ref.TYPE_CHUNK and c not in got
                got[c] = bytes(pf.blobs[o:o + n])
        assert set(got) == set(want) - {first}
        for c, blob in got.items():
            assert blob == (want[c] if encode is None else zlib.compress(want[c], 1))


def test_collector_concurrent_callers(oracle):
    """Per-file calls from 16 threads at once through one collector (the
    scanner goroutines of snapshot/backup.go:216-225, each chunking its own
    file): every cut list matches the oracle, and the calls were batched."""
    import threading
    _lib.ensure_init()
    gear = _lib.default_gear()
    rng = np.random.default_rng(5)
    sizes = [int(x) for x in rng.choice([0, 1, 4096, 65536, 70000, 1 << 20, 3 << 20, 9 << 20, 17 << 20], size=96)]
    files = [random_bytes(n, 1200 + i) for i, n in enumerate(sizes)]
    col = chunkers.Collector(OPTS, batch_bytes=64 << 20, max_wait_us=2000)
    got = [None] * len(files)
    errors = []

    def worker(t):
        try:
            for i in range(t, len(files), 16):
                got[i] = col.chunk(files[i])
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for i, a in enumerate(files):
        assert_same(got[i], oracle.chunk(a, gear, **DEF) if a.size else np.zeros((0, 2), np.uint64), f"file {i}")
    req, batches = col.stats()
    col.close()
    assert req == len(files) and batches < req, (req, batches)


def test_stream_read_peak_is_measured():
    """cdc_debug_stream_read (the measured HBM stream-read rate the bench line
    reports beside the spec peak): for 1 GiB every form's best launch is
    positive, no slower than its median, and its rate lies between 1 and
    8 TB/s; invalid arguments are refused."""
    import ctypes
    import torch
    _lib.ensure_init()
    L = _lib.lib()
    n = 1 << 30
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    best, med = (ctypes.c_double * 3)(), (ctypes.c_double * 3)()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert L.cdc_debug_stream_read(0, ctypes.c_void_p(t.data_ptr()), n, 5, best, med, s) == 0
    for b, m in zip(best, med):
        assert 0 < b <= m
        assert 1e12 < n / (b * 1e-6) < 8.0e12, (b, m)
    assert L.cdc_debug_stream_read(0, ctypes.c_void_p(t.data_ptr() + 1), n - 16, 1, best, med, s) == _lib.CDC_E_INVALID
    assert L.cdc_debug_stream_read(0, ctypes.c_void_p(t.data_ptr()), 8, 1, best, med, s) == _lib.CDC_E_INVALID
