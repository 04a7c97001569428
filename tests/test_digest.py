"""Per-chunk digests: SHA-256 and byte histogram of
every chunk on the device vs hashlib / numpy, the reference's hashing config
mirror, and the entropy formula of snapshot/backup.go:548-569.

SHA-256 parity is pinned by the FIPS 180-4 known answers (and hashlib, the
CPython restatement of the same standard); the histogram is exact integer
counting.  GPU tests are marked `gpu`.
"""
import hashlib
import math

import numpy as np
import pytest

from datagen import random_bytes

# FIPS 180-4 / NIST CSRC SHA-256 examples
KATS = [
    (b"", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
    (b"abc", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
    (b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq",
     "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
    (b"abcdefghbcdefghicdefghijdefghijkefghijklfghijklmghijklmnhijklmnoijklmnopjklmnopqklmnopqrlmnopqrsmnopqrstnopqrstu",
     "cf5b16a778af8380036ce59e7b0492370b249b11e8f07a51afac45037afee9d1"),
    (b"a" * 1000000, "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0"),
]


def test_kats_pin_hashlib():
    """The oracle (hashlib) agrees with the FIPS 180-4 known answers."""
    for msg, hexd in KATS:
        assert hashlib.sha256(msg).hexdigest() == hexd


def test_hashing_configuration_mirror():
    from plakar_amd import hashing
    c = hashing.DefaultConfiguration()
    assert (c.Algorithm, c.Bits) == ("SHA256", 256)
    c2, err = hashing.LookupDefaultConfiguration("BLAKE3")
    assert c2 is None and str(err) == "unknown hashing algorithm: BLAKE3"


def _entropy_direct(data):
    """snapshot/backup.go:548-569 restated over the bytes (Go's Log2)."""
    from plakar_amd.hashing import go_log2
    if len(data) == 0:
        return 0.0, [0.0] * 256
    freq = [0.0] * 256
    for b in data:
        freq[b] += 1
    e = 0.0
    size = float(len(data))
    for f in freq:
        if f > 0:
            p = f / size
            e -= p * go_log2(p)
    return e, freq


def test_entropy_from_histogram_matches_reference_formula():
    from plakar_amd import hashing
    for n, seed in [(0, 0), (1, 1), (255, 2), (4096, 3)]:
        data = random_bytes(n, seed)
        e, freq = _entropy_direct(data.tobytes())
        hist = np.bincount(data, minlength=256) if n else np.zeros(256, np.int64)
        assert hashing.entropy_from_freq(hist.tolist(), n) == e  # same terms, same order: bit-identical
        assert [float(x) for x in hist] == freq


def test_go_log2_restatement():
    """Go's math.Log2 = frexp split + fdlibm log (math/log2.go, math/log.go):
    exact at powers of two, within 1 ulp of log2 elsewhere, and the numpy
    form is bit-identical to the scalar form."""
    from plakar_amd import hashing
    for k in range(-40, 41):
        assert hashing.go_log2(2.0 ** k) == float(k)
    xs = np.random.default_rng(5).random(50000) + 1e-300
    v = hashing.go_log2_array(xs)
    assert np.array_equal(v[:5000], np.array([hashing.go_log2(float(x)) for x in xs[:5000]]))
    ref = np.log2(xs)
    assert (np.abs(v - ref) <= np.spacing(np.abs(ref))).all()
    # fdlibm log itself: within 1 ulp of math.log on the reduced range
    for x in np.linspace(0.5, 1.0, 1001)[:-1]:
        f1, ki = math.frexp(float(x))
        assert abs(hashing._go_log_reduced(f1, ki) - math.log(float(x))) <= 2 * np.spacing(abs(math.log(float(x))) + 1e-300)


def test_entropy_rows_matches_scalar():
    """The vectorised entropy (bins summed left to right with cumsum) is
    bit-identical to the scalar reference loop, including empty rows,
    single-valued rows and rows with empty bins."""
    from plakar_amd import hashing
    rng = np.random.default_rng(9)
    rows = [np.zeros(256, np.int64), np.eye(256, dtype=np.int64)[7] * 1000]
    for n in (1, 2, 3, 100, 4096, 70000):
        rows.append(np.bincount(rng.integers(0, rng.integers(1, 257), n), minlength=256))
    hist = np.stack(rows)
    lens = hist.sum(axis=1)
    got = hashing.entropy_rows(hist, lens)
    for i in range(len(rows)):
        assert got[i] == hashing.entropy_from_freq(hist[i].tolist(), int(lens[i]))


def test_chunkify_routing():
    from plakar_amd import snapshot
    assert snapshot.route(0, 65536) == "empty"
    assert snapshot.route(1, 65536) == "whole"
    assert snapshot.route(65535, 65536) == "whole"
    assert snapshot.route(65536, 65536) == "cdc"


# ------------------------------------------------------------------ GPU parity
def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _run(buf, cuts):
    torch = _gpu()
    from plakar_amd import _lib, hashing
    _lib.ensure_init()
    t = torch.from_numpy(np.ascontiguousarray(buf)).cuda()
    c = torch.tensor(np.asarray(cuts, dtype=np.int64).reshape(-1, 2), device="cuda")
    d, h = hashing.chunk_digests(t, c)
    torch.cuda.synchronize()
    return d.cpu().numpy(), h.cpu().numpy()


def _check(buf, cuts, d, h):
    for i, (o, n) in enumerate(cuts):
        part = buf[o:o + n].tobytes()
        assert bytes(d[i]) == hashlib.sha256(part).digest(), f"chunk {i} ({o}, {n})"
        assert (h[i] == np.bincount(np.frombuffer(part, np.uint8), minlength=256)).all(), f"histogram {i}"


@pytest.mark.gpu
def test_gpu_digest_kats():
    msgs = [m for m, _ in KATS]
    buf = np.frombuffer(b"".join(msgs), np.uint8).copy()
    cuts, o = [], 0
    for m in msgs:
        cuts.append((o, len(m)))
        o += len(m)
    d, h = _run(buf, cuts)
    for i, (_, hexd) in enumerate(KATS):
        assert bytes(d[i]).hex() == hexd
    _check(buf, cuts, d, h)


@pytest.mark.gpu
def test_gpu_digest_padding_boundaries_and_alignment():
    """Lengths around the one/two final-block boundary (55/56, 63/64, ...) at
    every byte alignment of the chunk start."""
    buf = random_bytes(1 << 20, 11)
    lens = [0, 1, 3, 4, 5, 54, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 129, 1000, 4095, 4096, 65537]
    cuts, o = [], 0
    for k, n in enumerate(lens * 4):
        o += k % 7  # gaps: every alignment
        cuts.append((o, n))
        o += n
    assert o < buf.size
    d, h = _run(buf, cuts)
    _check(buf, cuts, d, h)


@pytest.mark.gpu
def test_gpu_digest_of_device_cut_list():
    """The device path's own cut list of 48 MiB of random bytes, digests and
    histograms straight from device memory (count bounded by the result row),
    checked chunk by chunk; and the processChunk records."""
    torch = _gpu()
    from plakar_amd import _lib, chunkers, device, hashing
    _lib.ensure_init()
    data = random_bytes(48 << 20, 12)
    t = torch.from_numpy(data).cuda()
    b = device.DeviceBatch([t], chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20))
    b.launch()
    d, h = hashing.chunk_digests(t, b.cuts[0], result=b.res[0])
    torch.cuda.synchronize()
    (cuts,), res = b.results()
    n = cuts.shape[0]
    cl = cuts.cpu().numpy()
    dd, hh = d[:n].cpu().numpy(), h[:n].cpu().numpy()
    _check(data, [(int(o), int(m)) for o, m in cl], dd, hh)
    recs = hashing.chunk_records(t, cuts)
    o, m = int(cl[0][0]), int(cl[0][1])
    e, freq = _entropy_direct(data[o:o + m].tobytes())
    assert recs[0].Checksum == hashlib.sha256(data[o:o + m].tobytes()).digest()
    assert recs[0].Length == m and recs[0].Entropy == e
    assert recs[0].Distribution == [f / m for f in freq]


@pytest.mark.gpu
def test_gpu_digest_batch_many_buffers():
    """One launch group over several buffers (the batched entry point), with
    per-buffer counts bounded on the device."""
    torch = _gpu()
    from plakar_amd import _lib, hashing
    _lib.ensure_init()
    bufs, cut_lists, res, refs = [], [], [], []
    for k in range(5):
        data = random_bytes(200000 + 7919 * k, 40 + k)
        cuts, o = [], k
        while o + 3000 < data.size:
            n = int((o * 2654435761) % 9000)
            n = min(n, data.size - o)
            cuts.append((o, n))
            o += n + 1
        cuts.append((0, 0))
        keep = len(cuts) - 3 if k % 2 else len(cuts)  # the result row bounds the count on odd buffers
        bufs.append(torch.from_numpy(data).cuda())
        cut_lists.append(torch.tensor(np.asarray(cuts, np.int64), device="cuda"))
        res.append(torch.tensor([keep, 0, 0, 0], dtype=torch.int64, device="cuda"))
        refs.append((data, cuts[:keep]))
    outs = hashing.chunk_digests_batch(bufs, cut_lists, res)
    torch.cuda.synchronize()
    for (data, cuts), (d, h) in zip(refs, outs):
        _check(data, cuts, d[:len(cuts)].cpu().numpy(), h[:len(cuts)].cpu().numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("host_min_len", [0, 1, 30000, 1 << 40])
def test_gpu_digest_hybrid_matches_hashlib(host_min_len):
    """cdc_chunk_digests_hybrid: the longest chunks' SHA-256 on host cores,
    the rest and every histogram on the device; every row equals hashlib /
    bincount whatever the split (0: the library's balance, 1: every non-empty
    chunk on the host, 1 << 40: none), over several buffers with unaligned
    chunks, empty ones, gaps and result rows that bound the counts."""
    torch = _gpu()
    from plakar_amd import _lib, hashing
    _lib.ensure_init()
    bufs, cut_lists, res, refs = [], [], [], []
    for k in range(4):
        data = random_bytes(3_000_000 + 104729 * k, 60 + k)
        cuts, o = [], k
        while o + 70000 < data.size:
            n = int((o * 2654435761) % 60000) + (40000 if (o // 7) % 5 == 0 else 0)
            n = min(n, data.size - o)
            cuts.append((o, n))
            o += n + (o % 3)
        cuts.append((0, 0))
        keep = len(cuts) - 2 if k % 2 else len(cuts)
        bufs.append(torch.from_numpy(data).cuda())
        cut_lists.append(torch.tensor(np.asarray(cuts, np.int64), device="cuda"))
        res.append(torch.tensor([keep, 0, 0, 0], dtype=torch.int64, device="cuda"))
        refs.append((data, cuts[:keep]))
    outs, hc, hb = hashing.chunk_digests_hybrid(bufs, cut_lists, res, host_threads=8, host_min_len=host_min_len)
    torch.cuda.synchronize()
    for (data, cuts), (d, h) in zip(refs, outs):
        _check(data, cuts, d[:len(cuts)].cpu().numpy(), h[:len(cuts)].cpu().numpy())
    nonempty = sum(1 for _, cuts in refs for _, n in cuts if n)
    if host_min_len == 1:
        assert hc == nonempty and hb == sum(n for _, cuts in refs for _, n in cuts)
    elif host_min_len == 1 << 40:
        assert hc == 0 and hb == 0
    else:
        assert 0 <= hc <= nonempty


@pytest.mark.gpu
def test_gpu_digest_hybrid_c1_pass():
    """The hybrid split on a C1 pass (1 GiB random, the device's own cut
    lists): digests equal the device-only path's, and some chunks went to
    the host."""
    torch = _gpu()
    from plakar_amd import _lib, chunkers, device, hashing
    _lib.ensure_init()
    t = torch.from_numpy(random_bytes(1 << 30, 1)).cuda()
    b = device.DeviceBatch([t], chunkers.ChunkerOpts(65536, 1 << 20, 4 << 20))
    b.launch()
    (d0, h0), = hashing.chunk_digests_batch([t], [b.cuts[0]], [b.res[0]])
    (d1, h1), = hashing.chunk_digests_hybrid([t], [b.cuts[0]], [b.res[0]], host_threads=16)[0]
    torch.cuda.synchronize()
    n = int(b.results()[1][0, 0])
    assert torch.equal(d0[:n], d1[:n]) and torch.equal(h0[:n], h1[:n])


@pytest.mark.gpu
@pytest.mark.parametrize("lanes", [1, 3, 64, 100])
def test_gpu_digest_multi_chunk_lanes(lanes):
    """A launch with more chunks than resident lanes gives each lane a run of
    consecutive chunks (k = ceil(chunks / lanes)): forced here with small lane
    counts over the padding-boundary lengths at every alignment, empty chunks,
    gaps and overlaps, chunks past 1023 blocks (histogram halves flushed
    mid-chunk and accumulated), and several buffers in one launch group."""
    torch = _gpu()
    from plakar_amd import _lib, hashing
    _lib.ensure_init()
    L = _lib.lib()
    buf = random_bytes(3 << 20, 13)
    lens = [0, 1, 55, 56, 63, 64, 65, 119, 120, 4095, 65537, 0, 70000, 200000, 3, 127]
    cuts, o = [], 0
    for k, n in enumerate(lens * 3):
        o += k % 5
        cuts.append((o, n))
        o += n
    cuts.append((100, 5000))  # overlaps an earlier chunk
    assert o < buf.size
    refs = [(buf, cuts)]
    for k in range(3):  # more buffers in the same launch group, counts bounded by result rows
        b2 = random_bytes(300000 + 977 * k, 50 + k)
        c2 = [(i * 997 % 1000, 1000 + (i * 7919) % 30000) for i in range(40)]
        refs.append((b2, c2))
    try:
        assert L.cdc_debug_set_digest_lanes(lanes) == 0
        bufs = [torch.from_numpy(np.ascontiguousarray(b)).cuda() for b, _ in refs]
        cls = [torch.tensor(np.asarray(c, np.int64).reshape(-1, 2), device="cuda") for _, c in refs]
        res = [torch.tensor([len(c) - (i % 2), 0, 0, 0], dtype=torch.int64, device="cuda")
               for i, (_, c) in enumerate(refs)]
        outs = hashing.chunk_digests_batch(bufs, cls, res)
        torch.cuda.synchronize()
    finally:
        L.cdc_debug_set_digest_lanes(0)
    for i, ((b, c), (d, h)) in enumerate(zip(refs, outs)):
        keep = len(c) - (i % 2)
        _check(b, c[:keep], d[:keep].cpu().numpy(), h[:keep].cpu().numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("nbufs,lanes", [(33, 0), (300, 0), (70, 64)])
def test_gpu_digest_many_buffers_one_launch_group(nbufs, lanes):
    """More than 32 buffers in one call: one launch group whose descriptors
    live in device memory (launch_digests_many), empty buffers and empty cut
    lists among them, counts bounded by result rows on every third; repeated
    calls cycle the descriptor ring past its 16 slots."""
    torch = _gpu()
    from plakar_amd import _lib, hashing
    _lib.ensure_init()
    L = _lib.lib()
    refs = []
    for k in range(nbufs):
        n = 0 if k % 17 == 5 else 1000 + (k * 7919) % 90000
        b = random_bytes(n, 900 + k)
        cuts, o = [], 0
        while o < n:
            m = min(n - o, 100 + (o * 2654435761 + k) % 9000)
            cuts.append((o, m))
            o += m
        if k % 11 == 3:
            cuts.append((0, 0))
        refs.append((b, cuts))
    try:
        if lanes:
            assert L.cdc_debug_set_digest_lanes(lanes) == 0
        bufs = [torch.from_numpy(np.ascontiguousarray(b)).cuda() if b.size else torch.zeros(1, dtype=torch.uint8,
                                                                                            device="cuda")
                for b, _ in refs]
        cls = [torch.tensor(np.asarray(c, np.int64).reshape(-1, 2), device="cuda") for _, c in refs]
        keeps = [len(c) - 1 if (i % 3 == 0 and c) else len(c) for i, (_, c) in enumerate(refs)]
        res = [torch.tensor([kp, 0, 0, 0], dtype=torch.int64, device="cuda") for kp in keeps]
        for _ in range(3 if nbufs < 100 else 1):
            outs = hashing.chunk_digests_batch(bufs, cls, res)
        torch.cuda.synchronize()
    finally:
        L.cdc_debug_set_digest_lanes(0)
    for (b, c), kp, (d, h) in zip(refs, keeps, outs):
        _check(b, c[:kp], d[:kp].cpu().numpy(), h[:kp].cpu().numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("lanes", [1, 128, 700])
def test_gpu_digest_queue_order(lanes):
    """Workgroups with more chunks than lanes: up to 1,024 of them handed out
    longest first (a bitonic sort in LDS), more in cut-list order; lengths
    spread from 0 to 40 KiB so that the order matters."""
    torch = _gpu()
    from plakar_amd import _lib, hashing
    _lib.ensure_init()
    L = _lib.lib()
    buf = random_bytes(24 << 20, 17)
    rng = np.random.default_rng(5)
    cuts, o = [], 0
    while True:
        n = int(rng.integers(0, 40000)) if rng.random() < 0.9 else 0
        if o + n > buf.size or len(cuts) >= 1500:
            break
        cuts.append((o, n))
        o += n
    try:
        assert L.cdc_debug_set_digest_lanes(lanes) == 0
        t = torch.from_numpy(buf).cuda()
        c = torch.tensor(np.asarray(cuts, np.int64), device="cuda")
        d, h = hashing.chunk_digests(t, c)
        torch.cuda.synchronize()
    finally:
        L.cdc_debug_set_digest_lanes(0)
    _check(buf, cuts, d.cpu().numpy(), h.cpu().numpy())


@pytest.mark.gpu
def test_gpu_chunkify_batch_objects(oracle):
    """snapshot.chunkify_batch against the reference's per-file work restated
    on the CPU: routing (backup.go:631-645), oracle cuts, hashlib chunk and
    object checksums, exact counts, Go-Log2 entropies, the object entropy as
    the length-weighted sum in chunk order."""
    torch = _gpu()
    from datagen import low_entropy
    from plakar_amd import _lib, snapshot
    from plakar_amd.hashing import go_log2
    _lib.ensure_init(gear=_lib.default_gear())
    gear = _lib.default_gear()
    files = [b"", b"x", random_bytes(1000, 50).tobytes(), random_bytes(65535, 51).tobytes(),
             random_bytes(65536, 52).tobytes(), random_bytes(3 << 20, 53).tobytes(),
             low_entropy(9 << 20, 54).tobytes(), random_bytes((2 << 20) + 12345, 55).tobytes()]
    objs = snapshot.chunkify_batch(files, device_object_max=4 << 20)
    assert len(objs) == len(files)
    for f, o in zip(files, objs):
        a = np.frombuffer(f, np.uint8)
        if a.size == 0:
            cuts = [(0, 0)]
        elif a.size < 65536:
            cuts = [(0, a.size)]
        else:
            cuts = [(int(x), int(y)) for x, y in oracle.chunk(a, gear)]
        assert [c.Length for c in o.Chunks] == [n for _, n in cuts]
        assert o.Checksum == hashlib.sha256(f).digest()
        tot_e, tot = 0.0, 0
        for (off, n), c in zip(cuts, o.Chunks):
            part = f[off:off + n]
            assert c.Checksum == hashlib.sha256(part).digest()
            freq = [float(x) for x in np.bincount(np.frombuffer(part, np.uint8), minlength=256)]
            e = 0.0
            for x in freq:  # backup.go:560-566, bins in order
                if x > 0:
                    q = x / float(n)
                    e -= q * go_log2(q)
            assert c.Entropy == e
            assert list(c.Distribution) == ([x / n for x in freq] if n else [0.0] * 256)
            tot_e += c.Entropy * float(n)
            tot += n
        assert o.Entropy == (tot_e / float(tot) if tot else 0.0)
        assert list(o.Distribution) == [0.0] * 256


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(12))
def test_gpu_digest_random_cut_lists(seed):
    """Random buffers and cut lists (chunks of 0 B-600 KiB at any alignment,
    gaps and overlaps allowed, result rows that bound the counts) through the
    device-only batch path and the hybrid path at a random split and thread
    count: every digest equals hashlib, every histogram numpy.bincount."""
    torch = _gpu()
    from plakar_amd import _lib, hashing
    _lib.ensure_init()
    rng = np.random.default_rng(np.random.PCG64(7700 + seed))
    bufs, cut_lists, res, refs = [], [], [], []
    for k in range(int(rng.integers(1, 9))):
        data = random_bytes(int(rng.integers(1, 6 << 20)), 7800 + 16 * seed + k)
        cuts = []
        for _ in range(int(rng.integers(0, 200))):
            o = int(rng.integers(0, data.size))
            n = int(min(data.size - o, np.exp(rng.uniform(0, np.log(600 << 10))) if rng.random() > 0.05 else 0))
            cuts.append((o, n))
        keep = len(cuts) if rng.random() < 0.7 else int(rng.integers(0, len(cuts) + 1))
        bufs.append(torch.from_numpy(data).cuda())
        cut_lists.append(torch.tensor(np.asarray(cuts or [(0, 0)], np.int64).reshape(-1, 2), device="cuda"))
        res.append(torch.tensor([keep if cuts else 0, 0, 0, 0], dtype=torch.int64, device="cuda"))
        refs.append((data, cuts[:keep]))
    outs = hashing.chunk_digests_batch(bufs, cut_lists, res)
    torch.cuda.synchronize()
    for (data, cuts), (d, h) in zip(refs, outs):
        _check(data, cuts, d[:len(cuts)].cpu().numpy(), h[:len(cuts)].cpu().numpy())
    host_min_len = int(rng.choice([0, 1, 100_000]))
    outs, _, _ = hashing.chunk_digests_hybrid(bufs, cut_lists, res, host_threads=int(rng.integers(1, 25)),
                                              host_min_len=host_min_len)
    torch.cuda.synchronize()
    for (data, cuts), (d, h) in zip(refs, outs):
        _check(data, cuts, d[:len(cuts)].cpu().numpy(), h[:len(cuts)].cpu().numpy())
