"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle, bit-exact.

Every test here runs the product library on an MI355X and compares its cut
lists with oracle/fastcdc_oracle.c on the same bytes.  PARITY UNPINNED w.r.t.
the Go module: the oracle is a restatement, pinned by the
committed golden vectors in tests/golden/.
"""
import io
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from datagen import gear_table, low_entropy, random_bytes, zipf_sizes  # noqa: E402
from oracle_ref import DEFAULT_MASK_L, DEFAULT_MASK_S  # noqa: E402
from plakar_amd import _lib, chunkers, device, repository  # noqa: E402
from plakar_amd.chunking import Configuration, DefaultConfiguration  # noqa: E402

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DEF = dict(min_size=65536, normal_size=1 << 20, max_size=4 << 20)


def _placeholder():
    return _lib.default_gear()


def _opts(p):
    return chunkers.ChunkerOpts(MinSize=p["min_size"], NormalSize=p["normal_size"], MaxSize=p["max_size"])


def gpu_chunk(arrays, p, gear=None, cut_adj=0, final=True, offsets=None):
    """Chunk host numpy arrays on the GPU via the device path; returns a list of
    uint64 (n, 2) arrays."""
    _lib.ensure_init(gear=gear, cut_convention=cut_adj)
    ts = []
    for i, a in enumerate(arrays):
        off = 0 if offsets is None else offsets[i]
        t = torch.empty(a.size + off + 16, dtype=torch.uint8, device="cuda")
        t[off:off + a.size].copy_(torch.from_numpy(np.ascontiguousarray(a)))
        ts.append(t[off:off + a.size])
    b = device.DeviceBatch(ts, _opts(p), final=final)
    b.launch()
    cuts, res = b.results()
    return [c.cpu().numpy().astype(np.uint64) for c in cuts], res


def assert_same(got, ref, what=""):
    assert got.shape == ref.shape, f"{what}: {got.shape[0]} chunks vs oracle {ref.shape[0]}"
    bad = np.nonzero((got != ref).any(axis=1))[0]
    assert bad.size == 0, f"{what}: first mismatch at chunk {bad[0]}: {got[bad[0]]} vs {ref[bad[0]]}"


# the suite's MaskL index mode (CDC_MASKL_INDEX, as the library reads it), restored after each test
_MASKL_ENV = os.environ.get("CDC_MASKL_INDEX", "1")[:1]
_MASKL_MODE = int(_MASKL_ENV) if _MASKL_ENV in ("0", "1", "2", "3") else 1


@pytest.fixture(autouse=True)
def _reset_debug():
    device.set_debug_mode(0)
    yield
    device.set_debug_mode(0)
    device.set_maskl_index_mode(_MASKL_MODE)
    _lib.ensure_init(gear=_lib.default_gear())


# ---------------------------------------------------------------- golden vectors
def _golden_cases():
    with open(os.path.join(GOLDEN, "golden_vectors.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("case", _golden_cases(), ids=lambda c: c["name"])
def test_device_matches_golden(oracle, case):
    import sys
    sys.path.insert(0, GOLDEN)
    import make_golden as mg
    data = mg.make_input(case["input"])
    gear = mg.gear_for(case["gear"])
    (got,), _ = gpu_chunk([data], case["params"], gear=gear, cut_adj=case["cut_adj"])
    assert [int(x) for x in got[:, 1]] == case["lengths"]
    assert int(got[:, 1].sum()) == data.size


# ---------------------------------------------------------------- parameter sweep
PARAMS = [
    dict(min_size=64, normal_size=256, max_size=1024),
    dict(min_size=64, normal_size=100, max_size=130),
    dict(min_size=2048, normal_size=8192, max_size=65536),
    dict(min_size=4096, normal_size=16384, max_size=20000),
    DEF,
]


@pytest.mark.parametrize("p", PARAMS, ids=lambda p: f"{p['min_size']}-{p['normal_size']}-{p['max_size']}")
@pytest.mark.parametrize("kind", ["random", "low_entropy", "zeros", "mixed"])
@pytest.mark.parametrize("cut_adj", [0, 1])
def test_device_param_sweep(oracle, p, kind, cut_adj):
    n = 3 << 20
    if kind == "random":
        data = random_bytes(n, 21)
    elif kind == "low_entropy":
        data = low_entropy(n, 22, 0.01)
    elif kind == "zeros":
        data = np.zeros(n, np.uint8)
    else:
        data = np.concatenate([random_bytes(n // 3, 23), np.zeros(n // 3, np.uint8), low_entropy(n // 3, 24, 0.002)])
    gear = gear_table(31)
    (got,), _ = gpu_chunk([data], p, gear=gear, cut_adj=cut_adj)
    assert_same(got, oracle.chunk(data, gear, cut_adj=cut_adj, **p), f"{kind}")


@pytest.mark.parametrize("size", [0, 1, 63, 64, 65, 1000, 65535, 65536, 65537, 65536 + 49, 1 << 20, (4 << 20) + 1, 9_999_999])
def test_device_sizes(oracle, size):
    data = random_bytes(size, size)
    gear = _placeholder()
    (got,), res = gpu_chunk([data], DEF, gear=gear)
    ref = oracle.chunk(data, gear, **DEF)
    assert_same(got, ref, f"size {size}")
    assert int(res[0, 1]) == size  # consumed


@pytest.mark.parametrize("off", [1, 3, 7, 8, 13, 15])
def test_device_unaligned(oracle, off):
    p = dict(min_size=2048, normal_size=8192, max_size=65536)
    data = random_bytes((1 << 20) + off * 7, off)
    gear = gear_table(off)
    (got,), _ = gpu_chunk([data], p, gear=gear, offsets=[off])
    assert_same(got, oracle.chunk(data, gear, **p), f"offset {off}")


def test_device_dense_candidates(oracle):
    """G[0] = 0: every all-zero window hits MaskS, so every index block
    overflows and the chains never merge (offset-preserving): exercises the
    dense raw rescans and the sequential fallback resolver."""
    gear = gear_table(40)
    gear[0] = 0
    data = np.concatenate([np.zeros(24 << 20, np.uint8), random_bytes(8 << 20, 41)])
    (got,), _ = gpu_chunk([data], DEF, gear=gear)
    assert_same(got, oracle.chunk(data, gear, **DEF), "dense")


def test_device_alternative_masks(oracle):
    """Masks are runtime parameters (v0.0.8 values unverified)."""
    ms, ml = 0x0000000000001FFF, 0x00000000000001FF   # low bits: W = 13
    _lib.ensure_init(gear=gear_table(50), mask_s=ms, mask_l=ml)
    data = random_bytes(2 << 20, 50)
    t = torch.from_numpy(data).cuda()
    p = dict(min_size=1024, normal_size=8192, max_size=32768)
    b = device.DeviceBatch([t], _opts(p))
    b.launch()
    (c,), _ = b.results()
    got = c.cpu().numpy().astype(np.uint64)
    assert_same(got, oracle.chunk(data, gear_table(50), mask_s=ms, mask_l=ml, **p), "masks")


# ---------------------------------------------------------------- MaskL index modes
@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_maskl_index_modes(oracle, mode):
    """C3-like data (zeros + 1 % random bytes): a quarter of the chunks pass
    Normal and end on MaskL candidates. Never / adaptive / always building the
    MaskL index (2: in the fused pass k_scan_f, 3: by k_scan_l) gives the same
    cuts; several launches so adaptive mode runs with and without the index."""
    data = low_entropy(48 << 20, 71)
    gear = _placeholder()
    ref = oracle.chunk(data, gear, **DEF)
    assert (ref[:, 1] > DEF["normal_size"]).any(), "no chunk reaches the MaskL region"
    device.set_maskl_index_mode(mode)
    for rep in range(3):
        (got,), _ = gpu_chunk([data], DEF, gear=gear)
        assert_same(got, ref, f"maskl mode {mode} rep {rep}")


def test_maskl_adaptive_follows_the_data(oracle):
    """Adaptive mode: random data never raises the MaskL hint; on C3-like
    data a probing group (every 16th) raises it and the next groups build the
    MaskL index. Cuts are identical in every group."""
    gear = _placeholder()
    _lib.ensure_init(gear=gear)
    device.set_maskl_index_mode(1)  # clears the adaptive state
    assert device.maskl_state()[0] == 0
    rnd = random_bytes(8 << 20, 73)
    ref = oracle.chunk(rnd, gear, **DEF)
    for rep in range(17):  # at least one probing group
        (got,), _ = gpu_chunk([rnd], DEF, gear=gear)
        assert_same(got, ref, f"random rep {rep}")
    assert device.maskl_state()[0] == 0, "random data raised the MaskL hint"
    low = low_entropy(24 << 20, 74)
    ref = oracle.chunk(low, gear, **DEF)
    assert (ref[:, 1] > DEF["normal_size"]).any()
    built = 0
    for rep in range(20):
        (got,), _ = gpu_chunk([low], DEF, gear=gear)
        assert_same(got, ref, f"low-entropy rep {rep}")
        built += device.maskl_state()[0]
    assert built >= 3, "the probe never raised the MaskL hint"


@pytest.mark.parametrize("masks", [
    (0x0000000000001FFF, 0x00000000000001FF),  # MaskL inside MaskS's span: fused (loop frame 32)
    (0x0000000000001FF7, 0x00000000000003FF),  # 9 shared bits, MaskL bit 3 outside MaskS: fused
    (0x0000000000001FFF, 0x0000000000001C01),  # 4 shared bits: too weak a filter, two passes
    (0x0000000000001FFF, 0x00000000000301FF),  # MaskL's top bit above MaskS's: two passes
    (0x0003590703530000, 0x0000800000000001),  # MaskL spans 48 bits, no shared bit: two passes
    (0x0003590703530000, 0x0000D90003530000),  # the FastCDC masks (10 shared bits, loop frame 16)
], ids=["fusable", "fusable-lonly", "shared-weak", "maskl-above", "maskl-wide", "fastcdc"])
@pytest.mark.parametrize("mode", [1, 2, 3])
def test_maskl_index_alternative_masks(oracle, masks, mode):
    """k_scan_f's loop frame and key are derived from the masks; where the
    masks do not allow one (MaskL above MaskS, fewer than 8 shared bits), mode
    2 falls back to k_scan + k_scan_l. At these sizes many chunks pass Normal
    and end on MaskL candidates."""
    ms, ml = masks
    gear = gear_table(52)
    _lib.ensure_init(gear=gear, mask_s=ms, mask_l=ml)
    device.set_maskl_index_mode(mode)
    p = dict(min_size=1024, normal_size=8192, max_size=32768)
    data = random_bytes(4 << 20, 52)
    ref = oracle.chunk(data, gear, mask_s=ms, mask_l=ml, **p)
    assert (ref[:, 1] > p["normal_size"]).any(), "no chunk reaches the MaskL region"
    t = torch.from_numpy(data).cuda()
    for rep in range(3):
        b = device.DeviceBatch([t], _opts(p))
        b.launch()
        (c,), _ = b.results()
        assert_same(c.cpu().numpy().astype(np.uint64), ref, f"masks {ms:#x}/{ml:#x} mode {mode} rep {rep}")


# ---------------------------------------------------------------- debug resolver
@pytest.mark.parametrize("kind", ["random", "low_entropy"])
def test_sequential_resolver_matches(oracle, kind):
    data = random_bytes(16 << 20, 60) if kind == "random" else low_entropy(16 << 20, 61)
    gear = _placeholder()
    device.set_debug_mode(1)
    (got,), _ = gpu_chunk([data], DEF, gear=gear)
    device.set_debug_mode(0)
    assert_same(got, oracle.chunk(data, gear, **DEF), "sequential")


# ---------------------------------------------------------------- streaming windows
@pytest.mark.parametrize("window", [(4 << 20) + 4096, 9 << 20, 33 << 20])
def test_nonfinal_windows_compose(oracle, window):
    """final = 0 windows + resume at `consumed` == the whole stream (the
    Peek(MaxSize) carry of ext chunker.go)."""
    data = np.concatenate([random_bytes(40 << 20, 70), low_entropy(20 << 20, 71)])
    gear = _placeholder()
    ref = oracle.chunk(data, gear, **DEF)
    got, off = [], 0
    while off < data.size:
        w = min(window, data.size - off)
        fin = off + w == data.size
        (c,), res = gpu_chunk([data[off:off + w]], DEF, gear=gear, final=fin)
        c = c.copy()
        c[:, 0] += np.uint64(off)
        got.append(c)
        consumed = int(res[0, 1])
        assert fin or consumed > 0
        off = off + w if fin else off + consumed
    assert_same(np.concatenate(got), ref, f"window {window}")


# ---------------------------------------------------------------- batched buffers
def test_batch_many_buffers(oracle):
    """Independent buffers in one launch group (and more than one group)."""
    p = dict(min_size=2048, normal_size=8192, max_size=65536)
    sizes = [0, 5, 2047, 2048, 70000, 1 << 20, 3 << 20] * 6
    arrays = [random_bytes(s, 80 + i) if i % 3 else low_entropy(s, 80 + i) for i, s in enumerate(sizes)]
    gear = gear_table(81)
    got, res = gpu_chunk(arrays, p, gear=gear)
    for i, a in enumerate(arrays):
        assert_same(got[i], oracle.chunk(a, gear, **p), f"buffer {i} ({a.size} B)")


def test_pipelined_streams(oracle):
    """Two batches over the same buffers alternate over two streams (bench.py's
    pipelined steps): one batch's resolution kernels run beside the next
    batch's scan; every pass must still produce the oracle's cut lists."""
    arrays = [random_bytes(24 << 20, 71), random_bytes((5 << 20) + 123, 72), low_entropy(9 << 20, 73)]
    gear = _placeholder()
    _lib.ensure_init(gear=gear)
    ts = [torch.from_numpy(a).cuda() for a in arrays]
    batches = [device.DeviceBatch(ts, _opts(DEF)) for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    for i in range(6):
        batches[i % 2].launch(streams[i % 2])
    refs = [oracle.chunk(a, gear, **DEF) for a in arrays]
    for k, b in enumerate(batches):
        cuts, _ = b.results()
        for i, (c, r) in enumerate(zip(cuts, refs)):
            assert_same(c.cpu().numpy().astype(np.uint64), r, f"stream {k} buffer {i}")


def test_c2_shape_32x64MiB(oracle):
    """BASELINE configs[2], one GPU's share: 32 x 64 MiB random buffers."""
    arrays = [random_bytes(64 << 20, 100 + i) for i in range(32)]
    gear = _placeholder()
    got, _ = gpu_chunk(arrays, DEF, gear=gear)
    for i, a in enumerate(arrays):
        assert_same(got[i], oracle.chunk(a, gear, **DEF), f"buffer {i}")


def test_c1_full_1GiB(oracle):
    """BASELINE configs[1]: 1 GiB random, default params, bit-exact."""
    data = random_bytes(1 << 30, 1)
    gear = _placeholder()
    (got,), _ = gpu_chunk([data], DEF, gear=gear)
    assert_same(got, oracle.chunk(data, gear, **DEF), "C1")


def test_c3_low_entropy_1GiB(oracle):
    """BASELINE configs[3], one GPU's share: 1 GiB zeros + 1 % random bytes."""
    data = low_entropy(1 << 30, 200)
    gear = _placeholder()
    (got,), _ = gpu_chunk([data], DEF, gear=gear)
    assert_same(got, oracle.chunk(data, gear, **DEF), "C3")


# ---------------------------------------------------------------- host paths / Go API mirror
@pytest.mark.parametrize("group_mb,maxbuf_mb", [(None, None), (16, 16), (16, 64)])
def test_chunk_buffers_host_path(oracle, monkeypatch, group_mb, maxbuf_mb):
    """cdc_chunk: host buffers in, host lists out, through the two-slot staging
    pipeline.  (16, 16): the 40 MiB buffer is chunked as a stream of windows;
    (16, 64): it is a launch group of its own; several groups alternate slots."""
    if group_mb:
        monkeypatch.setenv("CDC_HOST_GROUP_MB", str(group_mb))
        monkeypatch.setenv("CDC_HOST_MAXBUF_MB", str(maxbuf_mb))
    _lib.ensure_init()
    arrays = [random_bytes(s, 90 + i) for i, s in enumerate([0, 100, 65536, 70000, 5 << 20, 40 << 20, 1 << 20])]
    gear = _placeholder()
    res = chunkers.ChunkBuffers(arrays, _opts(DEF))
    for i, a in enumerate(arrays):
        assert_same(res[i], oracle.chunk(a, gear, **DEF), f"host buffer {i}")


def test_chunk_buffers_many_groups(oracle, monkeypatch):
    """More buffers than one launch group holds (32) and more bytes than the
    group budget: groups alternate between the two pipeline slots."""
    monkeypatch.setenv("CDC_HOST_GROUP_MB", "16")
    _lib.ensure_init()
    rng = np.random.default_rng(7)
    sizes = [int(x) for x in rng.integers(0, 3 << 20, size=80)]
    arrays = [random_bytes(sz, 500 + i) for i, sz in enumerate(sizes)]
    gear = _placeholder()
    res = chunkers.ChunkBuffers(arrays, _opts(DEF))
    for i, a in enumerate(arrays):
        assert_same(res[i], oracle.chunk(a, gear, **DEF), f"host buffer {i}")


def test_chunker_next_mirror(oracle):
    """chunkers.NewChunker("fastcdc", rd, opts) + Next() until EOF."""
    _lib.ensure_init()
    data = np.concatenate([random_bytes(150 << 20, 95), low_entropy(30 << 20, 96)])
    chk = chunkers.NewChunker("fastcdc", io.BytesIO(data.tobytes()), _opts(DEF))
    lens = []
    while True:
        chunk, err = chk.Next()
        if err is chunkers.EOF:
            assert chunk is None
            break
        lens.append(len(chunk))
    ref = oracle.chunk(data, _placeholder(), **DEF)
    assert lens == [int(x) for x in ref[:, 1]]
    # empty stream: (nil, io.EOF) at once
    chk = chunkers.NewChunker("fastcdc", io.BytesIO(b""), _opts(DEF))
    assert chk.Next() == (None, chunkers.EOF)


@pytest.mark.parametrize("window_mib,size_mib", [(200, 93), (200, 199)])
def test_chunker_large_window_final_fill(oracle, window_mib, size_mib):
    """A stream through an explicit 200-MiB window whose final fill is shorter
    than the window: the plan of the shorter fill can need more workspace than
    the window's (the scan lane rounds up), and the stream regrows it."""
    _lib.ensure_init()
    data = random_bytes((size_mib << 20) + 12345, 97 + size_mib)
    chk = chunkers.NewChunker("fastcdc", io.BytesIO(data.tobytes()), _opts(DEF), window_bytes=window_mib << 20)
    lens = []
    while True:
        chunk, err = chk.Next()
        if err is chunkers.EOF:
            break
        lens.append(len(chunk))
    ref = oracle.chunk(data, _placeholder(), **DEF)
    assert lens == [int(x) for x in ref[:, 1]]


def test_chunker_rejects_like_go():
    _lib.ensure_init()
    with pytest.raises(_lib.CdcError):
        chunkers.NewChunker("ultracdc", io.BytesIO(b"x"), _opts(DEF))
    with pytest.raises(_lib.CdcError):
        chunkers.NewChunker("fastcdc", io.BytesIO(b"x"), chunkers.ChunkerOpts(65536, 65536, 1 << 20))


def test_repository_chunkify_mirror(oracle):
    """snapshot/backup.go:631-666 routing through Repository.Chunker."""
    _lib.ensure_init()
    repo = repository.Repository(DefaultConfiguration())
    gear = _placeholder()
    for size in [0, 1, 65535, 65536, 65537, 3 << 20]:
        data = random_bytes(size, 300 + size % 97)
        lens = repository.chunkify_lengths(repo, size, io.BytesIO(data.tobytes()))
        ref = oracle.chunk(data, gear, chunkify=True, **DEF)
        assert lens == [int(x) for x in ref[:, 1]], size
    # lower-cased algorithm name, like repository.go:288
    repo2 = repository.Repository(Configuration("FastCDC", 2048, 8192, 65536))
    data = random_bytes(1 << 20, 301)
    lens = repository.chunkify_lengths(repo2, data.size, io.BytesIO(data.tobytes()))
    assert lens == [int(x) for x in oracle.chunk(data, gear, min_size=2048, normal_size=8192, max_size=65536)[:, 1]]


def test_c4_mixed_corpus_host_path(oracle):
    """BASELINE configs[4] shape (subsampled): Zipf-sized files, chunkify routing:
    < MinSize files are one chunk, the rest go through ChunkBuffers."""
    _lib.ensure_init()
    sizes = zipf_sizes(300, 300)
    files = [random_bytes(int(s), 400 + i) for i, s in enumerate(sizes)]
    big = [f for f in files if f.size >= DEF["min_size"]]
    res = chunkers.ChunkBuffers(big, _opts(DEF))
    gear = _placeholder()
    for i, f in enumerate(big):
        assert_same(res[i], oracle.chunk(f, gear, **DEF), f"file {i} ({f.size} B)")


def test_wave_primitives_selftest():
    """DPP weighted prefix scan and wave minimum used by next() vs serial sums."""
    import ctypes
    L = _lib.lib()
    L.cdc_selftest_wave.argtypes = [ctypes.POINTER(ctypes.c_uint32)]
    out = (ctypes.c_uint32 * 6)()
    assert L.cdc_selftest_wave(out) == 0
    assert list(out)[:3] == [0, 0, 0], list(out)
