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
SHA_LANES = 256 * 2 * 128  # k_chunk_digest: resident SHA-256 lanes (2 workgroups of 2 x 64 round lanes per CU)
SHA_BLOCK_S = 2.05e-6      # one 64-B block per lane: the round wave's ~905 VALU at one wave per SIMD
GIB = float(1 << 30)

WORKLOADS = {
    "c1": dict(desc="C1: 1x 1 GiB uniform random buffer per GPU (BASELINE configs[1])",
               nbuf=1, size=1 << 30, kind="random"),
    "c2": dict(desc="C2: 32x 64 MiB uniform random buffers per GPU (BASELINE configs[2], one GPU's share)",
               nbuf=32, size=64 << 20, kind="random"),
    "c3": dict(desc="C3: 1x 1 GiB zeros + 1% random bytes per GPU (BASELINE configs[3], one GPU's share)",
               nbuf=1, size=1 << 30, kind="low_entropy"),
    "c4": dict(desc="C4: Zipf(1.1) corpus of 4 KiB-128 MiB files, 512 per GPU (BASELINE configs[4], one GPU's "
                    "share), host buffers in -> cut lists in host memory (PCIe-inclusive)",
               nbuf=512, size=0, kind="zipf", host=True),
    "c4f": dict(desc="C4 from files: the same 512-file share written to disk once (untimed), then per step read by the "
                     "library (pread, --file-threads: half the CPU share) into its pinned arena and chunked (pinned H2D, cut lists to host), "
                     "the reads running ahead of the device by 256-MiB sub-batches; warm page cache",
                nbuf=512, size=0, kind="zipf", host=True, files=True),
    "c4b": dict(desc="C4 end-to-end backup: the same 512-file share written to disk once (untimed), then per step "
                     "the whole backup through the native pipeline (cdc_backup_run): reads + object SHA-256, cut "
                     "points, chunk SHA-256 + histograms, BlobExists, Encode (LZ4 + AES-256-GCM, random key), 8 "
                     "concurrent packers -> packfiles (20 MiB); every file, small ones included; warm page cache",
                nbuf=512, size=0, kind="zipf", host=True, files=True, backup=True),
    "c4bl": dict(desc="c4b over large files: 4 files of 1536 / 1280 / 768 / 520 MiB (each several device batches, "
                      "so every file is backed up in pieces) and 60 Zipf files of the C4 distribution; same pipeline",
                 nbuf=64, size=0, kind="zipf", host=True, files=True, backup=True,
                 large_mib=(1536, 1280, 768, 520)),
}


def buffer_seeds(wl, rank, world):
    """Seeds of the buffers rank `rank` chunks.  Work per GPU is fixed (weak
    scaling): rank r owns buffers r*nbuf .. r*nbuf + nbuf - 1 of the global
    workload, so at N GPUs the job covers N*nbuf independent buffers (C2 at
    N = 8: the 256 x 64 MiB of BASELINE configs[2]).  No buffer is shared:
    independent files shard one-per-GPU with no collective."""
    assert 0 <= rank < world
    return [1 + rank * wl["nbuf"] + i for i in range(wl["nbuf"])]


def _dist_on(dist):
    return dist is not None and dist.is_available() and dist.is_initialized()


def reduce_max(dist, world, value, dev):
    """Max over ranks of a host float (the slowest rank sets the job time)."""
    if not _dist_on(dist):
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64,
                     device=dev if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def make_buffers(torch, wl, rank, dev, size, world=1):
    g = torch.Generator(device=dev)
    bufs = []
    for seed in buffer_seeds(wl, rank, world):
        g.manual_seed(seed)
        if wl["kind"] == "random":
            t = torch.randint(0, 256, (size,), dtype=torch.uint8, device=dev, generator=g)
        else:
            t = torch.zeros(size, dtype=torch.uint8, device=dev)
            k = size // 100
            pos = torch.randint(0, size, (k,), device=dev, generator=g)
            t[pos] = torch.randint(0, 256, (k,), dtype=torch.uint8, device=dev, generator=g)
        bufs.append(t)
    return bufs


def zipf_sizes(count, seed, s=1.1, unit=4096, kmax=32768):
    """C4 file sizes: bounded Zipf(s) over {unit * k, k = 1..kmax}."""
    import numpy as np
    k = np.arange(1, kmax + 1, dtype=np.float64)
    p = k ** -s
    cdf = np.cumsum(p) / p.sum()
    u = (np.random.PCG64(seed).random_raw(count) >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    return ((np.searchsorted(cdf, u) + 1) * unit).astype(np.int64)


def make_host_corpus(wl, rank, world):
    """C4: the rank's share of the corpus as pageable host buffers (uniform bytes)."""
    import numpy as np
    sizes = zipf_sizes(wl["nbuf"] * world, 300)[rank * wl["nbuf"]:(rank + 1) * wl["nbuf"]]
    large = [m << 20 for m in wl.get("large_mib", ())]
    if large:  # c4bl: the large files first, then Zipf files to nbuf
        sizes = list(large) + list(sizes[:wl["nbuf"] - len(large)])
    out = []
    for seed, n in zip(buffer_seeds(wl, rank, world), sizes):
        n = int(n)
        out.append(np.random.PCG64(seed).random_raw((n + 7) // 8).view(np.uint8)[:n].copy())
    return out


def e2e_host_rate(chunkers, opts, host_bufs, reps):
    """PCIe-inclusive rate of the host-buffer path (cdc_chunk: host bytes ->
    HBM -> kernels -> cut lists in host memory), from the MEDIAN call of
    `reps` timed calls after a warm-up call (one call in ~10 was seen to take
    5x the others from pinned memory on a 64-MiB buffer, which a 3-call mean
    turned into "pinned slower than pageable"; tools/pinned_probe.py).
    Returns (GiB/s of the median call, its seconds, the cut lists, per-call
    seconds)."""
    import statistics
    chunkers.ChunkBuffers(host_bufs, opts)  # warm-up: arenas, pinned staging
    total = sum(a.size for a in host_bufs)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        res = chunkers.ChunkBuffers(host_bufs, opts)
        ts.append(time.perf_counter() - t0)
    med = statistics.median(ts)
    return total / med / GIB, med, res, ts


def load_traffic(workload):
    """Per-launch HBM bytes of k_scan from the rocprofv3 PMC pass committed under
    profiles/ (FETCH_SIZE corrected as MI355X_MICROARCH.md prescribes), if any."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            return json.load(f).get(workload, {}).get("scan_hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def stream_read_peak(torch, L, bufs, dev, local, reps=20):
    """The device's measured HBM stream-read rate (report it
    beside the 8 TB/s spec), in the same clock state as the roofline loop it
    follows: three read-only kernels over 1 GiB (the first buffer when it is
    that large, else a scratch tensor, so the Infinity Cache does not serve
    it), `reps` launches each, interleaved; best and median per form, and the
    fastest form's best as `best_GBps`."""
    import ctypes
    n = 1 << 30
    src = bufs[0] if bufs[0].numel() >= n else torch.empty(n, dtype=torch.uint8, device=dev)
    best, med = (ctypes.c_double * 3)(), (ctypes.c_double * 3)()
    st = L.cdc_debug_stream_read(local, ctypes.c_void_p(src.data_ptr()), n, reps, best, med,
                                 ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    if st != 0 or min(best) <= 0:
        return dict(error=int(st))
    names = ("k_stream_read (grid-stride, four plain 16-B loads in flight per lane)",
             "k_stream_read_nt (8-KiB pieces per wave, eight nontemporal 16-B loads per lane)",
             "k_stream_read_lds (the scan's LDS-DMA with its nt policy: 4-KiB steps per wave into a two-slot ring, nothing computed)")
    forms = {nm.split()[0]: dict(best_GBps=round(n / (b * 1e-6) / 1e9, 1), median_GBps=round(n / (m * 1e-6) / 1e9, 1),
                                 form=nm) for nm, b, m in zip(names, best, med)}
    top = max(forms.values(), key=lambda f: f["best_GBps"])
    return dict(best_GBps=top["best_GBps"], median_GBps=top["median_GBps"], bytes=n, reps=reps, forms=forms,
                kernel="cdc_debug_stream_read, the fastest of three read-only forms",
                note="measured after the roofline loop; frac_of_measured_peak = achieved / best_GBps")


# The host's CPU share per GPU: OMP_NUM_THREADS where the launcher sets it
# (16 on the one-GPU box), else 16.
def _cpu_share():
    v = os.environ.get("OMP_NUM_THREADS", "")
    return int(v) if v.isdigit() and int(v) > 0 else 16


CPU_SHARE = _cpu_share()


def digest_leg(torch, batch, bufs, reps, check, host_threads=16):
    """Per-chunk SHA-256 + byte histogram (processChunk, snapshot/backup.go:594-629)
    over the device cut lists of the pass: device-resident, events around the
    digest kernels.  Not part of `value`.  On rank 0 of a 1-GPU run the first
    buffer's digests are checked against hashlib on a bounded sample, and hashlib
    (1 core) is timed on the same sample as its CPU baseline."""
    import hashlib
    import numpy as np
    from plakar_amd import hashing
    cut_lists = [batch.cuts[i] for i in range(batch.n)]
    res_rows = [batch.res[i] for i in range(batch.n)]

    def run():  # every buffer's chunks in one launch group
        return hashing.chunk_digests_batch(bufs, cut_lists, res_rows)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        out = run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    total = sum(t.numel() for t in bufs)
    cuts, _ = batch.results()
    longest = max(int(c[:, 1].max().item()) for c in cuts if c.shape[0])
    nchunks = sum(int(c.shape[0]) for c in cuts)
    d = dict(value=round(total / (ms * 1e-3) / GIB, 2), unit="GiB/s", ms_per_pass=round(ms, 3), chunks=nchunks,
             longest_chunk=longest, kernel="k_chunk_digest (SHA-256: per chunk a producer lane and a round lane) + k_chunk_hist (a wave per chunk)",
             bound="one launch lasts as long as its longest chunk's SHA-256 chain: 64-B blocks x ~905 VALU of one "
                   "round wave per block")
    # the hybrid single pass (cdc_chunk_digests_hybrid): the longest chunks'
    # SHA-256 on host_threads host cores (--hybrid-threads: default the box's
    # CPU share per GPU), the rest on the device
    if len(bufs) <= 32:
        hout, hc, hb = hashing.chunk_digests_hybrid(bufs, cut_lists, res_rows, host_threads=host_threads)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            hout, hc, hb = hashing.chunk_digests_hybrid(bufs, cut_lists, res_rows, host_threads=host_threads)
        torch.cuda.synchronize()
        hms = (time.perf_counter() - t0) / reps * 1e3
        same = all(torch.equal(a[0][:c.shape[0]], b[0][:c.shape[0]]) and torch.equal(a[1][:c.shape[0]], b[1][:c.shape[0]])
                   for a, b, c in zip(out, hout, cuts))
        d["hybrid"] = dict(value=round(total / (hms * 1e-3) / GIB, 2), unit="GiB/s", ms_per_pass=round(hms, 3),
                           host_threads=host_threads, host_chunks=hc, host_bytes=hb, equal_to_device_only=bool(same),
                           note="cdc_chunk_digests_hybrid, wall time incl. the cut lists back to the host: the "
                                "longest chunks' SHA-256 on host cores (x86 SHA extensions, ~35 ns per 64-B block "
                                "against a device chain's ~2 us), the rest and every histogram on the device")
    if check:
        host = bufs[0][:min(bufs[0].numel(), 256 << 20)].cpu().numpy()
        c0 = cuts[0].cpu().numpy()
        dg = out[0][0][:c0.shape[0]].cpu().numpy()
        hs = out[0][1][:c0.shape[0]].cpu().numpy()
        ok, nbytes, t0 = True, 0, time.perf_counter()
        for i, (o, n) in enumerate(c0):
            if o + n > host.size:
                break
            part = host[o:o + n]
            ok &= hashlib.sha256(part.tobytes()).digest() == bytes(dg[i])
            ok &= bool((np.bincount(part, minlength=256) == hs[i]).all())
            nbytes += int(n)
        el = time.perf_counter() - t0
        t0 = time.perf_counter()
        for i, (o, n) in enumerate(c0):
            if o + n > host.size:
                break
            hashlib.sha256(host[o:o + n].tobytes()).digest()
        el = time.perf_counter() - t0
        d["parity_vs_hashlib"] = ok
        d["cpu_baseline"] = dict(value=round(nbytes / el / GIB, 3), unit="GiB/s", cores=1, kind="hashlib",
                                 sample=f"SHA-256 of the first {nbytes >> 20} MiB of chunks of buffer 0, 1 thread")
    return d


def _cpu_encode_rate(host, cuts, seconds=3.0):
    """CPU baseline of Encode on one host core: LZ4 frames (the system's
    liblz4, LZ4F_compressFrame) then AES-256-GCM over 64-KiB pieces (OpenSSL
    libcrypto), chunk by chunk over a bounded sample; None without the libraries."""
    import ctypes
    import ctypes.util
    try:
        lz = ctypes.CDLL(ctypes.util.find_library("lz4") or "liblz4.so.1")
        cr = ctypes.CDLL(ctypes.util.find_library("crypto") or "libcrypto.so.3")
    except OSError:
        return None
    lz.LZ4F_compressFrameBound.restype = ctypes.c_size_t
    lz.LZ4F_compressFrameBound.argtypes = [ctypes.c_size_t, ctypes.c_void_p]
    lz.LZ4F_compressFrame.restype = ctypes.c_size_t
    lz.LZ4F_compressFrame.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    cr.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
    cr.EVP_aes_256_gcm.restype = ctypes.c_void_p
    cr.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p]
    cr.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.c_void_p,
                                     ctypes.c_int]
    cr.EVP_EncryptFinal_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    cr.EVP_CIPHER_CTX_ctrl.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    cr.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
    key, nonce = os.urandom(32), os.urandom(12)
    dst = ctypes.create_string_buffer(int(lz.LZ4F_compressFrameBound(4 << 20, None)) + 64)
    enc = ctypes.create_string_buffer((4 << 20) + 4096)
    tag = ctypes.create_string_buffer(16)
    ol = ctypes.c_int()
    nbytes, t0 = 0, time.perf_counter()
    for o, n in cuts:
        src = host[int(o):int(o + n)]
        m = lz.LZ4F_compressFrame(dst, len(dst), src.ctypes.data, int(n), None)
        for p0 in range(0, int(m), 65536):
            ctx = cr.EVP_CIPHER_CTX_new()
            cr.EVP_EncryptInit_ex(ctx, cr.EVP_aes_256_gcm(), None, key, nonce)
            cr.EVP_EncryptUpdate(ctx, enc, ctypes.byref(ol), ctypes.addressof(dst) + p0, min(65536, int(m) - p0))
            cr.EVP_EncryptFinal_ex(ctx, enc, ctypes.byref(ol))
            cr.EVP_CIPHER_CTX_ctrl(ctx, 0x10, 16, tag)
            cr.EVP_CIPHER_CTX_free(ctx)
        nbytes += int(n)
        if time.perf_counter() - t0 > seconds:
            break
    el = time.perf_counter() - t0
    return dict(value=round(nbytes / el / GIB, 3), unit="GiB/s", cores=1, kind="liblz4 + OpenSSL AES-256-GCM",
                sample=f"{nbytes >> 20} MiB of chunks of buffer 0, LZ4F_compressFrame then GCM per 64-KiB piece, 1 thread")


def encode_leg(torch, batch, bufs, reps, baseline):
    """Encode (LZ4 frame + AES-256-GCM stream, repository/repository.go:212-236)
    of every chunk of the pass, device-resident, with a random key; GiB/s of
    chunk bytes, the encoded/raw ratio, and a 1-core CPU baseline.  Not part
    of `value`."""
    import numpy as np
    from plakar_amd import encode
    key = os.urandom(32)
    cuts, _ = batch.results()
    # one call for the whole pass: every chunk of every buffer addressed from
    # the lowest buffer's address (offsets are plain 64-bit device addresses
    # relative to the base)
    base = min(bufs, key=lambda t: t.data_ptr())
    offs, lens = [], []
    for t, c in zip(bufs, cuts):
        c = c.cpu().numpy().astype(np.int64)
        offs.append(c[:, 0] + (t.data_ptr() - base.data_ptr()))
        lens.append(c[:, 1])
    offs, lens = np.concatenate(offs), np.concatenate(lens)
    cap = sum(encode.encode_bound(int(x)) for x in lens)
    plans = [(base, offs, lens, torch.empty(max(cap, 1), dtype=torch.uint8, device=base.device))]
    encoded = 0
    for t, offs, lens, out in plans:  # warm
        encoded += int(encode.encode_device(t, offs, lens, out, key=key)[-1])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for t, offs, lens, out in plans:
            encode.encode_device(t, offs, lens, out, key=key)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / reps
    total = sum(t.numel() for t in bufs)
    d = dict(value=round(total / el / GIB, 2), unit="GiB/s", ms_per_pass=round(el * 1e3, 3),
             ratio=round(encoded / max(total, 1), 4), blobs=sum(len(p[2]) for p in plans),
             kernels="k_xxh32 (side stream), k_lz4_seq, k_lz4_size, k_enc_plan, k_blob_keys, k_blob_pows, k_lz4_emit, k_frame_fin, k_gcm",
             note="one call per pass (every chunk of every buffer); wall time incl. the host plan (segment/block tables) and its upload")
    if baseline:
        host = bufs[0][:min(bufs[0].numel(), 256 << 20)].cpu().numpy()
        c0 = [(o, n) for o, n in zip(plans[0][1], plans[0][2]) if o + n <= host.size]
        d["cpu_baseline"] = _cpu_encode_rate(host, c0)
    return d


def chunk_digest_pipeline(torch, bufs, opts, dev, window, rounds):
    """Chunking + per-chunk SHA-256 and histograms (processChunk's device work,
    snapshot/backup.go:594-629) as a backup streams batches: passes chunk the
    rank's buffers on two alternating streams, and every `window` passes one
    digest launch group, on the next of four digest streams, hashes the
    chunks of those passes (a window's cut lists stay in HBM until their
    digests are done; three windows rotate, so chunking runs ahead while the
    previous windows hash, and a window's longest chains overlap the next
    windows' launches).  Hashing a window at once is what fills the device: a SHA-256
    chain is serial per chunk, so a launch needs many chunks in flight (one
    C1 pass has ~11 K, the device keeps ~65 K lanes resident).  Combined GiB/s
    of input bytes; not part of `value`."""
    from plakar_amd import device as devmod
    from plakar_amd import hashing
    cstreams = [torch.cuda.Stream(dev) for _ in range(2)]
    dstreams = [torch.cuda.Stream(dev) for _ in range(4)]
    nsets = 3  # windows in flight: a window's longest chains overlap the next two windows' launches
    sets = [[devmod.DeviceBatch(bufs, opts, final=True, device=dev.index) for _ in range(window)]
            for _ in range(nsets)]
    chunked = [[torch.cuda.Event() for _ in range(window)] for _ in range(nsets)]
    hashed = [[] for _ in range(nsets)]
    wbufs = [t for _ in range(window) for t in bufs]
    per = len(wbufs)  # one launch group per window (descriptors in device memory past 32 buffers)

    def one_round(r):
        w = r % nsets
        for i in range(window):
            s = cstreams[i % 2]
            if i < 2:  # the set's previous digests are done with its cut lists
                for e in hashed[w]:
                    s.wait_event(e)
            sets[w][i].launch(s)
            chunked[w][i].record(s)
        cuts = [b.cuts[k] for b in sets[w] for k in range(b.n)]
        res = [b.res[k] for b in sets[w] for k in range(b.n)]
        hashed[w] = []
        for g in range(0, len(wbufs), per):  # launch groups (and rounds) alternate over the digest streams,
            ds = dstreams[(r + g // per) % len(dstreams)]  # so one window's long chains overlap the next's
            for e in chunked[w]:
                ds.wait_event(e)
            with torch.cuda.stream(ds):
                hashing.chunk_digests_batch(wbufs[g:g + per], cuts[g:g + per], res[g:g + per], stream=ds)
            ev = torch.cuda.Event()
            ev.record(ds)
            hashed[w].append(ev)
    for r in range(nsets):  # warm-up
        one_round(r)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for r in range(rounds):
        one_round(r)
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    passes = rounds * window
    total = sum(t.numel() for t in bufs) * passes
    return dict(value=round(total / el / GIB, 2), unit="GiB/s", window=window, passes=passes,
                ms_per_pass=round(el / passes * 1e3, 3),
                bound="SHA-256 lanes resident (two 128-lane workgroups per CU) x the per-64-B-block time of a "
                      "chain; the window's longest chunk run sets its launch's tail")


def cpu_baseline(bufs_host, cuts_dev, opts, seconds, threads=1):
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
                got = cuts_dev[i]
                got = np.asarray(got.cpu().numpy() if hasattr(got, "cpu") else got).astype(np.uint64)
                parity &= bool(got.shape == ref.shape and (got == ref).all())
            done_bytes += a.size
        reps += 1
        el = time.perf_counter() - t0
        if el >= seconds or reps >= 1024:  # the time bound governs
            break
    one = dict(value=done_bytes / el / GIB, unit="GiB/s", cores=1, kind="port",
               sample=f"{len(bufs_host)} buffer(s) x {bufs_host[0].size / GIB:.3g} GiB, {reps} rep(s), "
                      f"{el:.1f} s, scalar C oracle (oracle/fastcdc_oracle.c), 1 thread, host of the GPU box "
                      f"(nproc={os.cpu_count()})")
    if threads > 1:
        one["multi_thread"] = cpu_threads_leg(orc, gear, kw, bufs_host, threads, seconds / 2)
    return one, parity


def cpu_threads_leg(orc, gear, kw, bufs_host, threads, seconds):
    """the same oracle on N host threads, one independent
    64-MiB piece of the sample per call (plakar chunks files concurrently, one
    goroutine per file). ctypes drops the GIL for the C call."""
    from concurrent.futures import ThreadPoolExecutor
    piece = 64 << 20
    parts = [a[o:o + piece] for a in bufs_host for o in range(0, a.size, piece)]
    done_bytes, t0 = 0, time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        while True:
            done_bytes += sum(ex.map(lambda x: (orc.chunk(x, gear, **kw), x.size)[1], parts))
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    return dict(value=round(done_bytes / el / GIB, 2), unit="GiB/s", cores=threads, kind="port",
                sample=f"{len(parts)} independent 64-MiB pieces of the sample per round, {done_bytes / GIB:.0f} GiB "
                       f"in {el:.1f} s, {threads} threads")


def parity_check(bufs_host, cuts, opts, budget_bytes=1 << 30):
    """This rank's cut lists against the CPU oracle on a bounded sample (the
    first buffers, up to ~1 GiB): True iff every sampled list is bit-identical.
    Runs after the timed region on every rank; the line reports the AND over
    ranks."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_ref import Oracle
    from plakar_amd import _lib
    orc, gear = Oracle(), _lib.default_gear()
    kw = dict(min_size=opts.MinSize, normal_size=opts.NormalSize, max_size=opts.MaxSize)
    ok, done = True, 0
    for a, c in zip(bufs_host, cuts):
        if done >= budget_bytes:
            break
        ref = orc.chunk(a, gear, **kw)
        got = np.asarray(c.cpu().numpy() if hasattr(c, "cpu") else c).astype(np.uint64)
        ok &= bool(got.shape == ref.shape and (got == ref).all())
        done += a.size
    return ok, done


def reduce_and(dist, world, flag, dev):
    """AND over ranks of a host bool (None counts as False)."""
    if not _dist_on(dist):
        return bool(flag)
    import torch
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def backup_cpu_baseline(paths, opts, threads, key, compress=True):
    """c4b's CPU baseline: the same backup of the same files on host cores
    (oracle/backup_cpu.c: pread, object SHA-256, the C oracle's chunkify,
    per-chunk SHA-256 + histogram + entropy, BlobExists, LZ4 frame +
    AES-256-GCM stream, packfile serialisation; OpenSSL + liblz4), `threads`
    worker threads taking files in turn (the reference's goroutine per file).
    Warm page cache, as the GPU leg."""
    import numpy as np
    from plakar_amd import _lib

    class Params(ctypes.Structure):
        _fields_ = [("gear", ctypes.c_void_p), ("mask_s", ctypes.c_uint64), ("mask_l", ctypes.c_uint64),
                    ("min_size", ctypes.c_uint64), ("normal_size", ctypes.c_uint64), ("max_size", ctypes.c_uint64),
                    ("cut_adj", ctypes.c_uint32)]

    class Stats(ctypes.Structure):
        _fields_ = [(n, ctypes.c_uint64) for n in ("files", "bytes", "chunks", "new_blobs", "encoded_bytes",
                                                   "packfiles", "packed_bytes", "failed_files")] + \
                   [("wall_s", ctypes.c_double)]
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libbackup_cpu.so"))
    lib.backup_cpu_run.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(Params),
                                   ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.POINTER(Stats)]
    gear = np.ascontiguousarray(_lib.default_gear(), dtype=np.uint64)
    P = Params(gear.ctypes.data, 0x0003590703530000, 0x0000d90003530000, opts.MinSize, opts.NormalSize,
               opts.MaxSize, 0)
    arr = (ctypes.c_char_p * len(paths))(*[p.encode() for p in paths])
    kb = ctypes.create_string_buffer(bytes(key), 32) if key else None
    st = Stats()
    assert lib.backup_cpu_run(arr, len(paths), threads, ctypes.byref(P), kb, 1 if compress else 0, 20 << 20,
                              ctypes.byref(st)) == 0
    return dict(value=round(st.bytes / st.wall_s / GIB, 3), unit="GiB/s", cores=threads, kind="port",
                chunks=st.chunks, new_blobs=st.new_blobs,
                sample=f"the same {st.files} files ({st.bytes / GIB:.2f} GiB), one whole backup in {st.wall_s:.2f} s, "
                       f"{threads} threads (oracle/backup_cpu.c: pread, object SHA-256, the C oracle's chunkify, "
                       f"chunk SHA-256 + histogram + entropy, dedup, LZ4 frame + AES-256-GCM stream, packfiles; "
                       f"OpenSSL libcrypto + liblz4), warm page cache, nproc={os.cpu_count()}")


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def dist_timeout():
    """Bound on a rank's rendezvous and on each collective (BENCH_DIST_TIMEOUT_S,
    default 120 s): a rank whose peer died fails instead of waiting forever
    (a device failure surfaces as an error, never a hang)."""
    import datetime
    return datetime.timedelta(seconds=float(os.environ.get("BENCH_DIST_TIMEOUT_S", "120")))


def host_sha256_rate(L, mib=128, reps=3):
    """One host core's SHA-256 rate (GB/s) through the library's cdc_sha256
    (the reader threads' object hash), best of `reps` over `mib` MiB."""
    import ctypes
    import numpy as np
    buf = np.random.default_rng(7).integers(0, 256, mib << 20, dtype=np.uint8)
    out = (ctypes.c_uint8 * 32)()
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        if L.cdc_sha256(buf.ctypes.data, buf.size, 0, out) != 0:
            return float("nan")
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    return buf.size / best / 1e9


def spawn_ranks(argv, n):
    """`python bench.py --gpus N` with no launcher: start N rank processes of
    this script (one per GPU, RANK = LOCAL_RANK = i, WORLD_SIZE = N, rendezvous
    on 127.0.0.1) and poll them.  The first rank that exits non-zero ends the
    run: the others are terminated (SIGTERM, then SIGKILL after 10 s) and its
    exit status is returned, so one dead rank never leaves the rest blocked in
    a rendezvous or a collective.  0 when every rank exits 0.  The parent never
    initialises HIP (device_count() does not, on this image); it refuses to
    run when fewer than N devices are visible (unless every rank is told to
    share device 0: BENCH_REHEARSE_ONE_GPU=1, or BENCH_CPU_SELFTEST=1)."""
    import subprocess
    shared = os.environ.get("BENCH_REHEARSE_ONE_GPU") == "1" or os.environ.get("BENCH_CPU_SELFTEST") == "1"
    if not shared:
        import torch
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py: --gpus {n} but only {have} device(s) visible", file=sys.stderr)
            return 2
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), WORLD_SIZE=str(n),
                LOCAL_WORLD_SIZE=str(n))
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                              env=dict(base, RANK=str(i), LOCAL_RANK=str(i))) for i in range(n)]
    first_bad = 0
    while True:
        running = [p for p in procs if p.poll() is None]
        bad = [p for p in procs if p.returncode not in (None, 0)]
        if bad:
            first_bad = bad[0].returncode
            r = procs.index(bad[0])
            print(f"bench.py: rank {r} exited with status {first_bad}; stopping the other ranks", file=sys.stderr)
            break
        if not running:
            return 0
        time.sleep(0.05)
    for p in procs:
        if p.poll() is None:
            p.terminate()
    deadline = time.time() + 10
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    # a negative status (killed by a signal) maps to a shell-style exit code
    return first_bad if first_bad > 0 else 128 + (-first_bad)


def gather_per_rank(dist, world, value, dev):
    """Every rank's host float, in rank order (rank 0 reports each rank's rate)."""
    if not _dist_on(dist):
        return [value]
    import torch
    on = dev if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=on)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]


def cpu_selftest(args, world, rank):
    """BENCH_CPU_SELFTEST=1: the multi-rank plumbing alone (rendezvous, barrier,
    max-over-ranks time, per-rank gather, the JSON line) over gloo, no GPU.
    Each rank "chunks" by sleeping; tests/test_dist.py runs it without a
    launcher to check that --gpus N starts N ranks."""
    import torch.distributed as dist
    fail_rank = os.environ.get("BENCH_SELFTEST_FAIL_RANK")
    fail_at = os.environ.get("BENCH_SELFTEST_FAIL_AT", "before")
    if fail_rank == str(rank) and fail_at == "before":
        sys.exit(3)  # a rank that dies before the rendezvous
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=dist_timeout())
        dist.barrier()
    if fail_rank == str(rank) and fail_at == "after":
        sys.exit(3)  # a rank that dies after the rendezvous, while the others are in a collective
    t0 = time.perf_counter()
    time.sleep(0.01 * (1 + rank))
    el = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    elapsed = reduce_max(dist, world, el, None)
    per = gather_per_rank(dist, world, el, None)
    # the post-timed legs of a real run, on host bytes: every rank checks its
    # own (CPU-oracle) cut lists of a small sample, the line carries the AND;
    # rank 0 times the CPU baseline at any N
    import numpy as np
    from plakar_amd import chunkers
    opts = chunkers.ChunkerOpts(MinSize=64 * 1024, NormalSize=1 << 20, MaxSize=4 << 20)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_ref import Oracle
    from plakar_amd import _lib
    host = [np.random.PCG64(1 + rank).random_raw(1 << 20).view(np.uint8)]
    cuts = [Oracle().chunk(host[0], _lib.default_gear(), min_size=opts.MinSize, normal_size=opts.NormalSize,
                           max_size=opts.MaxSize)]
    if os.environ.get("BENCH_SELFTEST_BAD_RANK") == str(rank):
        cuts = [cuts[0][:-1]]  # a wrong list on one rank must turn the AND false
    ok, _ = parity_check(host, cuts, opts)
    parity = reduce_and(dist, world, ok, None)
    baseline = None
    if rank == 0:
        baseline, _ = cpu_baseline(host, cuts, opts, 0.2, threads=1)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "n_gpus": world, "selftest": True,
                          "elapsed_max_s": elapsed, "per_rank_elapsed_s": per,
                          "parity_vs_oracle": parity, "cpu_baseline": baseline}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", type=int, default=1)
    # ~50 ms of passes each: the GPU's clocks take tens of ms of load to settle
    # (20 passes after 3 warm-up ones measured 3.78 TB/s-equivalent, 200 after
    # 200 4.57)
    ap.add_argument("--steps", type=int, default=None, help="default 200 (device workloads), 5 (host workload c4)")
    ap.add_argument("--warmup", type=int, default=None, help="default 200 (device workloads), 2 (host workload c4)")
    ap.add_argument("--workload", default="c1", choices=sorted(WORKLOADS))
    ap.add_argument("--size-mib", type=int, default=0, help="override the per-buffer size (debug)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="threads of the multi-threaded CPU oracle leg (16 = the GPU box's CPU share; 1 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the per-rank oracle check after the timed region")
    ap.add_argument("--roofline-only", action="store_true",
                    help="only the roofline loop (--steps single-stream passes after --warmup ones; no timed "
                         "pipelined region, no side legs): under rocprofv3 --kernel-trace --stats the k_scan "
                         "average of the summary is the line's roofline.kernel_avg_ms")
    ap.add_argument("--backup-readers", type=int, default=CPU_SHARE,
                    help="c4b: reader threads (reads + object SHA-256); default the CPU share per GPU")
    ap.add_argument("--hybrid-threads", type=int, default=CPU_SHARE * 3 // 2,
                    help="host threads of the hybrid per-chunk SHA-256 leg; default 1.5 x the CPU share per GPU "
                         "(threads wait on the copy-back parts: 24 on 16 CPUs beat 16 by 10 %, 32 no better; "
                         "profiles/r06_host_threads_ab.txt)")
    ap.add_argument("--file-threads", type=int, default=max(1, CPU_SHARE // 2),
                    help="c4f: pread threads filling the pinned arena; default half the CPU share per GPU "
                         "(4-8 threads read 37-41 GiB/s on 16 CPUs, 16 threads 33-37: profiles/r06_c4f_threads_ab.txt)")
    ap.add_argument("--backup-packers", type=int, default=8, help="c4b: packer threads")
    ap.add_argument("--backup-batch-mib", type=int, default=512,
                    help="c4b: bytes per device batch (MiB; 512 measured best of 256 / 512 / 1024, profiles/r04_c4b_batch.txt)")
    ap.add_argument("--streams", type=int, default=2,
                    help="device workloads: consecutive steps alternate over this many streams, each with its "
                         "own workspace, so one batch's resolution kernels overlap the next batch's scan")
    ap.add_argument("--encode-reps", type=int, default=3,
                    help="Encode leg (LZ4 frame + AES-256-GCM of every chunk, not part of value); 0 disables")
    ap.add_argument("--digest-reps", type=int, default=3,
                    help="reps of the per-chunk SHA-256 + histogram leg (SURVEY.md 8f; 0 = skip)")
    ap.add_argument("--digest-window", type=int, default=8,
                    help="passes per digest launch in the pipelined chunk + digest leg")
    ap.add_argument("--e2e-reps", type=int, default=9,
                    help="timed calls of the PCIe-inclusive host-buffer leg, median reported (0 = skip)")
    args = ap.parse_args()
    if args.roofline_only:
        args.digest_reps = args.encode_reps = args.e2e_reps = 0
        args.no_cpu_baseline = True
    host_default = WORKLOADS[args.workload].get("host", False)
    if args.steps is None:
        args.steps = 5 if host_default else 200
    if args.warmup is None:
        args.warmup = 2 if host_default else 200

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(sys.argv[1:], args.gpus))  # before anything touches the GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks", file=sys.stderr)
        sys.exit(2)
    cdc_env = {k: v for k, v in sorted(os.environ.items()) if k.startswith("CDC_")}
    diag = [k for k, v in cdc_env.items() if k.startswith("CDC_DIAG") or (k == "CDC_DEBUG_PHASE" and v not in ("", "0"))]
    if diag:
        print(f"bench.py: refusing to measure with diagnostic settings {diag} (they change what the kernels do)",
              file=sys.stderr)
        sys.exit(2)
    if os.environ.get("BENCH_CPU_SELFTEST") == "1":
        return cpu_selftest(args, world, rank)
    if WORKLOADS[args.workload].get("backup"):
        # the backup pipeline's streams (H2D + cuts, digests x 2, Encode + its
        # aux) run independently only with one hardware queue each; HIP's
        # default of 4 queues per process shares them.  Set
        # before the HIP runtime starts.
        # The GPU box exports HIP's default of 4; the line records the value
        # found and the one applied (BENCH_KEEP_HW_QUEUES=1 measures with the
        # value found, as a host that does not set it would run; BENCH_HW_QUEUES
        # picks another count: 16 measured the same as 8, profiles/r04_c4b_hwq_ab.txt).
        os.environ["BENCH_GPU_MAX_HW_QUEUES_GIVEN"] = os.environ.get("GPU_MAX_HW_QUEUES", "")
        if os.environ.get("BENCH_KEEP_HW_QUEUES") != "1":
            os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("BENCH_HW_QUEUES", "8")

    import torch
    import torch.distributed as dist

    from plakar_amd import _lib, chunkers, device

    # BENCH_REHEARSE_ONE_GPU=1: every rank on device 0 over gloo, to rehearse
    # the N-rank launch, barrier and max-over-ranks timing on a one-GPU box.
    # The numbers of such a run are not a scaling measurement.
    rehearse = os.environ.get("BENCH_REHEARSE_ONE_GPU") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # BENCH_DIST_ONE_RANK=1: a one-rank nccl (RCCL) process group even at
    # N = 1, so the launch, barrier, max-over-ranks and gather code of the
    # N-GPU run executes over RCCL on a one-GPU box (tests/test_gpu_scale.py)
    one_rank_dist = world == 1 and os.environ.get("BENCH_DIST_ONE_RANK") == "1"
    if one_rank_dist:
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("MASTER_PORT", str(free_port()))
    if world > 1 or one_rank_dist:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if rehearse:
            dist.init_process_group("gloo", rank=rank, world_size=world, timeout=dist_timeout())
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev, timeout=dist_timeout())

    def barrier():
        if _dist_on(dist):
            dist.barrier()

    wl = WORKLOADS[args.workload]
    host_mode = wl.get("host", False)
    opts = chunkers.ChunkerOpts(MinSize=64 * 1024, NormalSize=1 << 20, MaxSize=4 << 20)
    _lib.ensure_init(dev_mask=1 << local)  # this rank's GPU only
    L = _lib.lib()

    routed_bytes = 0
    post_step = None  # turns the last step's output into cut rows, after the timed region
    if host_mode:
        corpus = make_host_corpus(wl, rank, world)
        # plakar chunkify routing (snapshot/backup.go:631-644): files < MinSize are one chunk, no CDC
        host_bufs = [a for a in corpus if a.size >= opts.MinSize]
        routed_bytes = sum(a.size for a in corpus if a.size < opts.MinSize)
        per_rank_bytes = sum(a.size for a in host_bufs)
        nbufs = len(host_bufs)

        def step():
            return chunkers.ChunkBuffers(host_bufs, opts)

        backup_stats = [None]
        if wl.get("backup"):  # every file of the share, small ones included: the pipeline routes them
            host_bufs = corpus
            routed_bytes = 0
            per_rank_bytes = sum(a.size for a in host_bufs)
            nbufs = len(host_bufs)
        if wl.get("files"):
            import tempfile
            tmpdir = tempfile.mkdtemp(prefix="cdc_c4f_")
            paths = []
            for i, a in enumerate(host_bufs):
                pth = os.path.join(tmpdir, f"f{i:04d}")
                with open(pth, "wb") as f:
                    f.write(a.tobytes())
                paths.append(pth)
            # the share is on disk before the first pass: its dirty pages written
            # back now, not by the kernel's flusher during the timed reads
            os.sync()
            del corpus
            fbatch = chunkers.FileBatch(sum((a.size + 4095) // 4096 * 4096 for a in host_bufs))

            def step():
                fbatch.reset()
                return fbatch.add_and_chunk(paths, opts, threads=args.file_threads)

            if wl.get("backup"):
                from plakar_amd import snapshot
                session_key = os.urandom(32)
                session = snapshot.BackupSession(key=session_key, compression="LZ4", packers=args.backup_packers,
                                                 readers=args.backup_readers,
                                                 batch_bytes=args.backup_batch_mib << 20,
                                                 dev=local)

                def step():  # one whole backup of the share per step (an empty repository each time)
                    t = time.perf_counter()
                    objs, _, st = session.run(paths, keep_packfiles=False)
                    st["run_s"] = time.perf_counter() - t  # the Python call: wall_s + its Python side
                    backup_stats[0] = st
                    return objs

                def post_step(objs):  # after the timed region: the (offset, length) rows, as the chunker reports them
                    import numpy as np
                    out = []  # (none for an empty file)
                    for o in objs:
                        lens = np.array([c.Length for c in o.Chunks if c.Length], dtype=np.uint64)
                        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64) if lens.size else lens
                        out.append(np.stack([offs, lens], axis=1) if lens.size else np.zeros((0, 2), np.uint64))
                    return out
    else:
        size = (args.size_mib << 20) if args.size_mib else wl["size"]
        bufs = make_buffers(torch, wl, rank, dev, size, world)
        nstreams = max(1, args.streams)
        batches = [device.DeviceBatch(bufs, opts, final=True, device=local) for _ in range(nstreams)]
        streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
        batch = batches[0]
        per_rank_bytes = sum(t.numel() for t in bufs)
        nbufs = len(bufs)
        step_no = [0]

        def step():
            i = step_no[0] % nstreams
            step_no[0] += 1
            batches[i].launch(streams[i])

    timed_steps = 0 if args.roofline_only else args.steps
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    barrier()
    t0 = time.perf_counter()
    out = None
    for _ in range(timed_steps):
        out = step()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    barrier()
    if out is None and host_mode:
        out = step()
    if post_step is not None:
        out = post_step(out)
    elapsed = reduce_max(dist, world, t1 - t0, dev)
    per_rank = gather_per_rank(dist, world, t1 - t0, dev)
    value = world * per_rank_bytes * timed_steps / elapsed / GIB if timed_steps else None

    # Roofline pass (after the timed region, not part of `value`): the scan
    # kernel's duration from hipEvents on its own launch stream, one pass at a
    # time (no other pass overlapping it), so it is the kernel's own time.
    L.cdc_profile_collect(None, None, None, None)
    L.cdc_profile_enable(1)
    rsteps = args.steps if args.roofline_only else max(5, min(args.steps, 50))
    for _ in range(rsteps):
        if host_mode:
            chunkers.ChunkBuffers(host_bufs, opts)
        else:
            batch.launch(streams[0])
    torch.cuda.synchronize(dev)
    L.cdc_profile_enable(0)
    scan_ms, pipe_ms = ctypes.c_double(), ctypes.c_double()
    launches, scan_bytes = ctypes.c_uint64(), ctypes.c_uint64()
    _lib.check(L.cdc_profile_collect(ctypes.byref(scan_ms), ctypes.byref(pipe_ms),
                                     ctypes.byref(launches), ctypes.byref(scan_bytes)), "profile")

    if host_mode:
        host_cuts = out
        nchunks = sum(len(c) for c in host_cuts)
    else:
        cuts, res = batch.results()
        nchunks = int(res[:, 0].sum())
        for i, other in enumerate(batches[1:], 1):  # every stream's batch produced the same cut lists
            if step_no[0] <= i:  # never launched (--roofline-only without warmup: only batch 0 runs)
                continue
            oc, _ = other.results()
            assert all(a.shape == b.shape and bool((a == b).all()) for a, b in zip(cuts, oc)), \
                "pipelined batches disagree"

    n = max(int(launches.value), 1)
    scan_avg_ms = scan_ms.value / n
    pipe_avg_ms = pipe_ms.value / n
    bytes_per_launch = scan_bytes.value / n
    achieved = bytes_per_launch / (scan_avg_ms * 1e-3) / 1e9 if scan_avg_ms > 0 else 0.0
    roofline = dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(achieved / HBM_PEAK_GBS, 4), traffic=load_traffic(args.workload),
                    kernel="k_scan (k_scan_f while the MaskL index is fused into it)", kernel_avg_ms=round(scan_avg_ms, 4),
                    algorithmic_bytes_per_launch=int(bytes_per_launch),
                    timed_passes=n,
                    pipeline_avg_ms=round(pipe_avg_ms, 4))
    if not host_mode:
        roofline["measured_stream_read"] = stream_read_peak(torch, L, bufs, dev, local)
        best = roofline["measured_stream_read"].get("best_GBps")
        if best:
            roofline["frac_of_measured_peak"] = round(achieved / best, 4)

    digest = None
    if not host_mode and args.digest_reps > 0:
        digest = digest_leg(torch, batch, bufs, args.digest_reps, rank == 0, args.hybrid_threads)
        digest["pipelined_with_chunking"] = chunk_digest_pipeline(torch, bufs, opts, dev, args.digest_window, 8)

    encode_res = None
    if not host_mode and args.encode_reps > 0:
        encode_res = encode_leg(torch, batch, bufs, args.encode_reps, rank == 0)

    # Every rank checks its own cut lists (a bounded sample, ~1 GiB) against
    # the CPU oracle; the line carries the AND over ranks.  Rank 0 also times
    # the CPU baseline, at any N (not part of `value`).
    import numpy as np
    if args.no_parity:
        parity = None
    elif host_mode:
        parity, _ = parity_check(host_bufs, host_cuts, opts)
    else:
        parity, _ = parity_check([t.cpu().numpy() for t in bufs[:max(1, (1 << 30) // max(1, bufs[0].numel()))]],
                                 cuts, opts)
    if parity is not None:
        parity = reduce_and(dist, world, parity, dev)
    baseline, e2e = None, None
    if rank == 0:
        if host_mode:
            sample, tot = [], 0
            for a in host_bufs:  # bounded sample: the first ~1 GiB of the corpus
                if tot >= (1 << 30):
                    break
                sample.append(a)
                tot += a.size
            sample_cuts = [np.asarray(c) for c in host_cuts[:len(sample)]]
        elif args.e2e_reps > 0 or not args.no_cpu_baseline:
            host = [t.cpu().numpy() for t in bufs[:1]]
            if args.e2e_reps > 0:
                rate, sec, e2e_cuts, ts = e2e_host_rate(chunkers, opts, host, args.e2e_reps)
                dev_cuts = [c.cpu().numpy().astype(np.uint64) for c in cuts[:len(e2e_cuts)]]
                same = all(a.shape == d.shape and bool((a == d).all()) for a, d in zip(e2e_cuts, dev_cuts))
                e2e = dict(value=round(rate, 2), unit="GiB/s", ms_per_call=round(sec * 1e3, 2),
                           ms_per_call_min_max=[round(min(ts) * 1e3, 2), round(max(ts) * 1e3, 2)],
                           path="cdc_chunk: pageable host -> H2D (runtime-staged) -> kernels -> D2H cut lists",
                           sample=f"{len(host)} x {host[0].size / GIB:.3g} GiB, median of {args.e2e_reps} calls",
                           same_cuts_as_device_path=same)
                # the same bytes from pinned host memory (north_star's "pinned hipMemcpyAsync" form)
                pinned = [torch.empty(t.numel(), dtype=torch.uint8, pin_memory=True) for t in bufs[:1]]
                for p, t in zip(pinned, bufs[:1]):
                    p.copy_(t)
                hostp = [p.numpy() for p in pinned]
                rate_p, sec_p, cuts_p, ts_p = e2e_host_rate(chunkers, opts, hostp, args.e2e_reps)
                same_p = all(a.shape == d.shape and bool((a == d).all()) for a, d in zip(cuts_p, dev_cuts))
                e2e["pinned"] = dict(value=round(rate_p, 2), unit="GiB/s", ms_per_call=round(sec_p * 1e3, 2),
                                     ms_per_call_min_max=[round(min(ts_p) * 1e3, 2), round(max(ts_p) * 1e3, 2)],
                                     path="cdc_chunk: pinned host -> H2D (direct DMA) -> kernels -> D2H cut lists",
                                     same_cuts_as_device_path=same_p)
                del hostp, pinned
            sample = host
            sample_cuts = cuts[:1]
        if not args.no_cpu_baseline and wl.get("backup"):
            baseline = backup_cpu_baseline(paths, opts, max(1, args.cpu_threads), session_key)
            # the chunker alone on 1 core over the same sample, as the other workloads report it
            baseline["chunker_only_1_core"], _ = cpu_baseline(sample, sample_cuts, opts, args.cpu_seconds / 2, 1)
        elif not args.no_cpu_baseline:
            baseline, sample_ok = cpu_baseline(sample, sample_cuts, opts, args.cpu_seconds, args.cpu_threads)
            baseline["sample_parity"] = sample_ok

    if rank == 0:
        config = {"workload": wl["desc"], "bytes_per_gpu": per_rank_bytes,
                  "global_bytes": per_rank_bytes * world, "buffers_per_gpu": nbufs,
                  "chunk_params": "FASTCDC min 65536 / normal 1048576 / max 4194304",
                  "gear": "placeholder (v0.0.8 table unavailable; see DESIGN.md)",
                  "parallelism": f"independent buffers, 1 rank per GPU x {world}, no collective",
                  "dist_backend": dist.get_backend() if _dist_on(dist) else None,
                  "per_rank_gibs": [round(per_rank_bytes * timed_steps / e / GIB, 2) if timed_steps else None
                                    for e in per_rank],
                  "chunks_per_step": nchunks,
                  "cdc_env": cdc_env}
        if host_mode:
            config["routed_bytes_per_gpu"] = routed_bytes
            config["timing"] = ("end-to-end incl. file reads into pinned memory, host->device copies and cut lists back "
                            "to host" if wl.get("files") else
                            "end-to-end incl. host->device copies and cut lists back to host")
        else:
            config["streams"] = nstreams
            config["timing"] = ("K independent passes over the input, each a full chunking of every buffer into "
                                "its own cut lists; consecutive passes alternate over the streams, so one pass's "
                                "resolution kernels overlap the next pass's scan; roofline.pipeline_avg_ms is the "
                                "single-pass latency (first kernel to cut lists final)")
        line = {
            "metric": METRIC, "value": round(value, 2) if value is not None else None, "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / timed_steps * 1e3, 4) if timed_steps else None, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": ("synthetic (numpy PCG64 uniform bytes in host memory; no dataset)" if host_mode else
                     "synthetic (torch Philox uniform bytes generated on the GPU; no dataset)"),
            "config": config,
            "roofline": roofline,
            "cpu_baseline": baseline,
            "parity_vs_oracle": parity,
            "e2e_host_path": e2e,
            "chunk_digests": digest,
            "encode": encode_res,
        }
        if host_mode and wl.get("backup") and backup_stats[0]:
            bs = backup_stats[0]
            # What bounds the leg is read from its own stage split.  The host's
            # object SHA-256 (objectHasher, snapshot/backup.go:583, 604: one
            # serial chain per file) runs on the reader threads; its stage
            # time is their summed hashing time / readers.  Its ceiling is the
            # readers x one core's SHA-NI rate (measured here, after the timed
            # region).  The device's side (the per-chunk SHA-256, k_chunk_digest)
            # is reported beside it with the device-busy fraction.
            device_kernel = None
            if bs.get("batches") and bs.get("digest_s"):
                # SHA-256 issue ceiling: every resident SHA lane (256 CUs x 2
                # workgroups x 128) finishing a 64-B block per 2.05 us
                peak_d = SHA_LANES * 64 / SHA_BLOCK_S / 1e9
                per = bs["digest_s"] / bs["batches"]
                ach_d = bs["bytes"] / bs["batches"] / per / 1e9
                device_kernel = dict(bound="issue", kernel="k_chunk_digest (per-chunk SHA-256 + histograms)",
                                     achieved=round(ach_d, 1), peak=round(peak_d, 1), unit="GB/s",
                                     frac=round(ach_d / peak_d, 4), kernel_avg_ms=round(per * 1e3, 3),
                                     algorithmic_bytes_per_launch=int(bs["bytes"] / bs["batches"]),
                                     chunks_per_batch=int(bs.get("chunks", 0) / bs["batches"]),
                                     note="a launch lasts as long as its longest chunk's serial SHA-256 chain; a "
                                          f"{args.backup_batch_mib}-MiB batch holds ~{int(bs.get('chunks', 0) / bs['batches'])} "
                                          f"chunks against {SHA_LANES} resident lanes")
            readers = max(1, args.backup_readers)
            core = host_sha256_rate(L)
            wall = bs["wall_s"]
            # Per-thread time of each overlapped stage; the longest one names
            # the steady state.  What sets the wall is that stage between the
            # pipeline's fill (until batch 0's reads land) and drain (after the
            # last batch's device stages), or -- for multi-GiB files -- the
            # longest serial object hash (one file's pieces hash in sequence).
            stages = {"object SHA-256 (readers)": bs["objhash_s"] / readers, "reads (readers)": bs["read_s"] / readers,
                      "device (calling thread)": bs["device_s"], "packers": bs["pack_s"] / max(1, args.backup_packers)}
            bound_stage = max(stages, key=stages.get)
            stage_s = stages[bound_stage]
            fill, drain, chain = bs.get("fill_s", 0.0), bs.get("drain_s", 0.0), bs.get("chain_s", 0.0)
            pipeline_s = fill + stage_s + drain
            if chain >= pipeline_s:
                bound, named_s = "host-sha256 serial chain (the largest file's object hash)", chain
            else:
                bound, named_s = f"{bound_stage} between fill and drain", pipeline_s
            sha_s = bs["objhash_s"] / readers
            ach = bs["bytes"] / sha_s / 1e9 if sha_s > 0 else None
            kinds = {"object SHA-256 (readers)": "host-sha256", "reads (readers)": "host-reads",
                     "device (calling thread)": "device", "packers": "host-packers"}
            line["roofline"] = dict(
                bound=kinds[bound_stage] if chain < pipeline_s else "host-sha256-chain",
                wall_set_by=bound, named_s=round(named_s, 4), named_over_wall=round(named_s / wall, 3) if wall else None,
                wall_s=round(wall, 4), fill_s=round(fill, 4), drain_s=round(drain, 4),
                longest_stage=bound_stage, longest_stage_s=round(stage_s, 4),
                stage_over_wall=round(stage_s / wall, 3) if wall else None,
                chain_s=round(chain, 4), chain_bytes=bs.get("chain_bytes", 0),
                chain_over_wall=round(chain / wall, 3) if wall else None,
                chain_GBps=round(bs.get("chain_bytes", 0) / chain / 1e9, 3) if chain > 0 else None,
                kernel="object SHA-256 on the reader threads (cdc_sha256, x86 SHA extensions; "
                       "objectHasher, snapshot/backup.go:583, 604)",
                achieved=round(ach, 2) if ach else None, peak=round(readers * core, 2), unit="GB/s",
                frac=round(ach / (readers * core), 4) if ach else None, traffic=None,
                per_core_GBps=round(core, 3), readers=readers,
                device_busy_frac=round(bs["device_s"] / wall, 3) if wall else None,
                stage_split_s={k: round(v, 4) for k, v in stages.items()},
                note="named_s = what sets the wall: fill + the longest per-thread stage + drain, or the longest "
                     "serial object SHA-256 chain when that is longer; achieved / peak = the readers' object "
                     "hashing (bytes / (summed hash time / readers)) against readers x one core's SHA-NI rate; "
                     "device_busy_frac = the calling thread's device time / wall",
                device_kernel=device_kernel, scan=roofline)
            line["backup_stages"] = dict(
                {k: (round(v, 4) if isinstance(v, float) else v) for k, v in bs.items()},
                readers=args.backup_readers, packers=args.backup_packers, batch_mib=args.backup_batch_mib,
                GPU_MAX_HW_QUEUES=os.environ.get("GPU_MAX_HW_QUEUES"),
                GPU_MAX_HW_QUEUES_given=os.environ.get("BENCH_GPU_MAX_HW_QUEUES_GIVEN") or None,
                note="per step (the last one): seconds per stage; read_s / objhash_s / pack_s are thread times "
                     "summed over threads, device_s / read_wait_s the calling thread's (read_wait_s: the device "
                     "waiting for a batch's reads), callback_s the callback thread's; the stages overlap")
        print(json.dumps(line), flush=True)
    if host_mode and wl.get("files"):
        import shutil
        fbatch.close()
        shutil.rmtree(tmpdir, ignore_errors=True)
    if _dist_on(dist):
        dist.destroy_process_group()
    sys.stdout.flush()
    sys.stderr.flush()
    L.cdc_shutdown()


if __name__ == "__main__":
    main()
