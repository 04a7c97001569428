"""Batched chunkify: plakar's per-file chunking work for a batch of whole
in-memory files, on the device.

    snapshot/backup.go:631-666   routing: empty file -> one empty chunk; smaller
                                 than Chunking.MinSize -> the whole file, no CDC;
                                 otherwise the chunker's cuts
    snapshot/backup.go:594-629   processChunk: chunk SHA-256, entropy() and the
                                 normalised byte distribution -> objects.Chunk
    snapshot/backup.go:668-681   the object's Entropy (length-weighted mean of
                                 the chunk entropies) and Checksum (SHA-256 of
                                 the whole file, objectHasher)
    objects/objects.go:26-36, 73-79   Object / Chunk

This is the batch form that SURVEY.md section 8b proposes for the re-plumbed
backup: one call per batch of files instead of one chunker per file.  The
cut points come from the device chunker (libplakar_cdc.so), the chunk
checksums and byte counts from one batched k_chunk_digest launch group, and
only the float64 arithmetic runs on the host.

The float64 arithmetic keeps the reference's order (hashing.entropy_rows: bins
0..255 in sequence, Go's math.Log2 restated; the object entropy summed over
the chunks in sequence).  Nothing here could be run against Go in this
container, so the bit-identity of the floats to Go is unpinned; the integer
parts (cuts, checksums, counts) are exact.

Chunk.Distribution and Object.Distribution are float64 numpy rows of 256
(the Go [256]float64 arrays).

backup_batch adds the consumer side: every
chunk not stored yet (BlobExists, backup.go:625) goes through PutBlob
(blobs.go:11-26: Encode, then the packer channel) into packfiles built by the
native packer (packer.py over cdc_packer_*, snapshot/packer.go and
packfile/packfile.go), flushed at Size() > MaxSize as packerJob does
(snapshot/snapshot.go:51-92).

Out of scope, as in SURVEY.md: the content type (mime detection), the
classifier, the repository state and storage backends, and the object's
Distribution (the reference never assigns it from its running total:
backup.go:668-677 leaves it zero).

The per-object SHA-256 is one serial chain per file.  On the device it is one
lane per file, ~32 MB/s per lane: it pays for many small files hashed
together and loses to a host core (~2 GB/s with SHA extensions) on a large
file.  object_hash="auto" hashes files up to `device_object_max` bytes on the
device (batched) and the rest with hashlib on host threads, overlapped with
the device work.
"""
import collections.abc
import concurrent.futures
import gc
import hashlib
import warnings
from dataclasses import dataclass, field
from typing import List

import numpy as np
import torch

from . import chunkers, device, hashing
from .repository import Repository

# ------------------------------------------------------------------- records
class ChunkRecords(collections.abc.Sequence):
    """The chunks of one object as the native backup pipeline reports them
    (objects.Chunk's fields, objects/objects.go:73-79): digests, lengths,
    entropies and byte histograms held as arrays, each hashing.Chunk made
    when it is read (Distribution = histogram / length, as chunkify_batch
    computes it).  A backup reports tens of thousands of chunks per run; as
    arrays they cost the callbacks a few copies instead of an object each
    (and the cyclic collector nothing).  Read-only: indexing makes a new
    Chunk each time, so edits to it are not kept (to_list() gives a list of
    Chunks to edit); == compares chunk by chunk with any sequence of Chunks."""
    __slots__ = ("_dg", "_lens", "_ent", "_hist")

    def __init__(self, dg=b"", lens=None, ent=None, hist=None):
        self._dg = dg
        self._lens = np.zeros(0, np.int64) if lens is None else lens
        self._ent = np.zeros(0, np.float64) if ent is None else ent
        self._hist = np.zeros((0, 256), np.uint32) if hist is None else hist

    @classmethod
    def concat(cls, parts):
        parts = [p for p in parts if len(p)]
        if len(parts) == 1:
            return parts[0]
        if not parts:
            return cls()
        return cls(b"".join(p._dg for p in parts), np.concatenate([p._lens for p in parts]),
                   np.concatenate([p._ent for p in parts]), np.concatenate([p._hist for p in parts]))

    def __len__(self):
        return len(self._lens)

    def __getitem__(self, k):
        if isinstance(k, slice):
            return [self[i] for i in range(*k.indices(len(self)))]
        n = len(self)
        if k < 0:
            k += n
        if not 0 <= k < n:
            raise IndexError(k)
        length = int(self._lens[k])
        return hashing.Chunk(self._dg[32 * k:32 * k + 32], length, float(self._ent[k]),
                             self._hist[k] / float(max(length, 1)))

    def to_list(self):
        """The chunks as a list of hashing.Chunk (copies)."""
        return [self[i] for i in range(len(self))]

    def __eq__(self, other):
        if not isinstance(other, collections.abc.Sequence) or isinstance(other, (str, bytes)):
            return NotImplemented
        if len(other) != len(self):
            return False
        return all(a.Checksum == b.Checksum and a.Length == b.Length and a.Entropy == b.Entropy and
                   np.array_equal(a.Distribution, b.Distribution) for a, b in zip(self, other))

    __hash__ = None

    def __repr__(self):
        return f"ChunkRecords({len(self)} chunks)"


@dataclass
class Object:
    """objects.Object (objects/objects.go:26-36), the fields chunkify fills."""
    Checksum: bytes
    Chunks: List[hashing.Chunk] = field(default_factory=list)
    ContentType: str = ""
    Entropy: float = 0.0
    Distribution: np.ndarray = field(default_factory=lambda: np.zeros(256))


def route(size, min_size):
    """snapshot/backup.go:631-645: 'empty', 'whole' (one chunk, no CDC) or 'cdc'."""
    if size == 0:
        return "empty"
    if size < min_size:
        return "whole"
    return "cdc"


def _object_entropy(chunk_entropies, lengths):
    """backup.go:612-627 + 668-670: totalEntropy += e * len (chunk order);
    Entropy = totalEntropy / totalDataSize."""
    total = int(np.sum(lengths, dtype=np.uint64))
    if total == 0:
        return 0.0
    acc = np.cumsum(np.asarray(chunk_entropies, np.float64) * np.asarray(lengths, np.float64))[-1]
    return float(acc) / float(total)


def chunkify_batch(files, repo: Repository = None, dev=0, object_hash="auto", device_object_max=1 << 20,
                   host_threads=8):
    """chunkify() for a batch of whole files held in host memory (bytes,
    bytearray or uint8 arrays).  Returns one Object per file, in order."""
    repo = repo or Repository()
    cfg = repo.Chunking
    opts = chunkers.ChunkerOpts(MinSize=int(cfg.MinSize), NormalSize=int(cfg.NormalSize),
                                MaxSize=int(cfg.MaxSize))
    chunkers.Validate(cfg.Algorithm.lower(), opts)
    arrs = [np.frombuffer(f, dtype=np.uint8) if not isinstance(f, np.ndarray) else np.ascontiguousarray(f, np.uint8)
            for f in files]
    n = len(arrs)
    if n == 0:
        return []
    routes = [route(a.size, opts.MinSize) for a in arrs]
    d = torch.device("cuda", dev)

    # per-object SHA-256 of the large files on host threads, overlapped
    host_obj = [i for i in range(n) if object_hash == "host" or (object_hash == "auto" and arrs[i].size > device_object_max)]
    pool = concurrent.futures.ThreadPoolExecutor(max_workers=max(1, host_threads)) if host_obj else None
    futs = {i: pool.submit(lambda a: hashlib.sha256(memoryview(a)).digest(), arrs[i]) for i in host_obj}

    with warnings.catch_warnings():  # read-only views of bytes objects: only read here
        warnings.simplefilter("ignore", UserWarning)
        tens = [torch.from_numpy(a).to(d) if a.size else torch.empty(0, dtype=torch.uint8, device=d) for a in arrs]
    # cut lists: device chunker for 'cdc' files, one whole-file cut otherwise
    cdc_idx = [i for i in range(n) if routes[i] == "cdc"]
    cuts = [None] * n
    if cdc_idx:
        b = device.DeviceBatch([tens[i] for i in cdc_idx], opts)
        b.launch()
        got, _ = b.results()
        for i, c in zip(cdc_idx, got):
            cuts[i] = c.contiguous()
    whole_idx = [i for i in range(n) if cuts[i] is None]
    if whole_idx:  # one host-to-device copy for every whole-file cut
        rows = torch.tensor([[0, arrs[i].size] for i in whole_idx], dtype=torch.int64).to(d)
        for k, i in enumerate(whole_idx):
            cuts[i] = rows[k:k + 1]
    # every chunk's SHA-256 + byte counts: one batched launch group
    nonempty = [i for i in range(n) if tens[i].numel() > 0]
    outs = hashing.chunk_digests_batch([tens[i] for i in nonempty], [cuts[i] for i in nonempty]) if nonempty else []
    dev_obj = [i for i in nonempty if i not in futs]
    obj_outs = []
    if dev_obj:
        whole = torch.tensor([[0, arrs[i].size] for i in dev_obj], dtype=torch.int64).to(d)
        obj_outs = hashing.chunk_digests_batch([tens[i] for i in dev_obj], [whole[k:k + 1] for k in range(len(dev_obj))],
                                               hist=False)
    # one device-to-host copy of each kind for the whole batch
    if nonempty:
        lens_all = torch.cat([cuts[i][:, 1] for i in nonempty]).cpu().numpy().astype(np.int64)
        dg_all = torch.cat([o[0] for o in outs]).cpu().numpy()
        hist_all = torch.cat([o[1] for o in outs]).cpu().numpy()
    obj_all = torch.cat([o[0] for o in obj_outs]).cpu().numpy() if obj_outs else None
    obj_row = {i: k for k, i in enumerate(dev_obj)}
    if nonempty:
        ent_all = hashing.entropy_rows(hist_all, lens_all)
        dist_all = hist_all.astype(np.float64) / np.maximum(lens_all, 1)[:, None].astype(np.float64)

    empty_sha = hashlib.sha256(b"").digest()
    objects = []
    k0 = 0
    for i in range(n):
        if arrs[i].size == 0:  # backup.go:631-635: one empty chunk, entropy 0, zero distribution
            objects.append(Object(Checksum=empty_sha, Chunks=[hashing.Chunk(empty_sha, 0, 0.0, np.zeros(256))]))
            continue
        m = cuts[i].shape[0]
        sl = slice(k0, k0 + m)
        k0 += m
        lens, ent = lens_all[sl], ent_all[sl]
        chunks = [hashing.Chunk(dg_all[k].tobytes(), int(lens_all[k]), float(ent_all[k]), dist_all[k])
                  for k in range(sl.start, sl.stop)]
        checksum = futs[i].result() if i in futs else obj_all[obj_row[i]].tobytes()
        objects.append(Object(Checksum=checksum, Chunks=chunks, Entropy=_object_entropy(ent, lens)))
    if pool:
        pool.shutdown()
    return objects


def backup_batch(files, repo: Repository = None, known=None, max_size=None, encode=None, timestamp=None, **kw):
    """chunkify_batch, then PutBlob of every new chunk into packfiles.

    known: set of chunk checksums already stored (BlobExists); updated.
    encode: Repository.Encode (compression, then encryption:
    repository/repository.go:212-236) applied to each blob before it is
    packed, as PutBlob does: a callable per blob, or an
    encode.DeviceEncoder (all new blobs of the batch in one device call);
    None = no compression / no encryption.
    Returns (objects, packfiles): the Object records and the serialised
    packfiles (packfile.go Serialize form)."""
    from . import packer as packer_mod
    max_size = packer_mod.DEFAULT_MAX_SIZE if max_size is None else int(max_size)
    known = set() if known is None else known
    objects = chunkify_batch(files, repo, **kw)
    arrs = [np.frombuffer(f, dtype=np.uint8) if not isinstance(f, np.ndarray) else np.ascontiguousarray(f, np.uint8)
            for f in files]
    if encode is None:  # the native path: cut rows and digests straight into the packer
        cut_lists, digest_lists, keep = [], [], []
        for a, obj in zip(arrs, objects):
            lens = np.array([c.Length for c in obj.Chunks], dtype=np.uint64)
            offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64) if lens.size else lens
            cut_lists.append(np.stack([offs, lens], axis=1) if lens.size else np.zeros((0, 2), np.uint64))
            digest_lists.append(np.frombuffer(b"".join(c.Checksum for c in obj.Chunks), dtype=np.uint8))
            keep.append(a)
        packs = packer_mod.pack_chunks(keep, cut_lists, digest_lists, max_size=max_size, known=known,
                                       timestamp=timestamp)
        return objects, packs
    packs = []
    pk = packer_mod.Packer(max_size, timestamp)
    if hasattr(encode, "encode_many"):  # encode.DeviceEncoder: every new blob of the batch in one device call
        todo = []
        for a, obj in zip(arrs, objects):
            off = 0
            for c in obj.Chunks:
                data = a[off:off + c.Length]
                off += c.Length
                if c.Checksum in known:
                    continue
                known.add(c.Checksum)
                todo.append((c.Checksum, data))
        for (csum, _), enc in zip(todo, encode.encode_many([d for _, d in todo])):
            if pk.AddBlob(packer_mod.TYPE_CHUNK, csum, enc):
                packs.append(pk.Serialize())
                pk.Reset()
        if pk.Count():
            packs.append(pk.Serialize())
        pk.close()
        return objects, packs
    for a, obj in zip(arrs, objects):
        off = 0
        for c in obj.Chunks:
            data = a[off:off + c.Length]
            off += c.Length
            if c.Checksum in known:
                continue
            known.add(c.Checksum)
            if pk.AddBlob(packer_mod.TYPE_CHUNK, c.Checksum, encode(data.tobytes())):
                packs.append(pk.Serialize())
                pk.Reset()
    if pk.Count():
        packs.append(pk.Serialize())
    pk.close()
    return objects, packs


class BackupSession:
    """A native backup context (cdc_backup_new): the repository's chunking
    parameters, Encode configuration (compression "LZ4" or None, the 32-byte
    key or None), the digests already stored (BlobExists), packfile MaxSize
    and the worker counts, with its device buffers kept across runs.  Each
    run() is one backup of a list of files through the pipeline of
    cdc_backup_files (reads + object SHA-256, cut points, chunk SHA-256 +
    histograms, dedup, Encode, `packers` concurrent packerJob workers,
    snapshot/snapshot.go:51-92)."""

    def __init__(self, repo: Repository = None, key=None, compression="LZ4", known=None, max_size=None,
                 packers=8, readers=8, batch_bytes=256 << 20, timestamp=0, dev=0):
        import ctypes
        from . import _lib, packer as packer_mod
        repo = repo or Repository()
        cfg = repo.Chunking
        opts = chunkers.ChunkerOpts(MinSize=int(cfg.MinSize), NormalSize=int(cfg.NormalSize),
                                    MaxSize=int(cfg.MaxSize))
        chunkers.Validate(cfg.Algorithm.lower(), opts)
        if compression not in (None, "LZ4"):
            raise ValueError(f"unsupported compression {compression!r}")
        _lib.ensure_init()
        o = _lib.cdc_backup_opts()
        o.chunking = _lib.cdc_opts(opts.MinSize, opts.NormalSize, opts.MaxSize, 0)
        o.packfile_max = int(packer_mod.DEFAULT_MAX_SIZE if max_size is None else max_size)
        o.compress = 1 if compression == "LZ4" else 0
        keybuf = knownbuf = None
        if key is not None:
            key = bytes(key)
            if len(key) != 32:
                raise ValueError("the repository key is 32 bytes (AES-256)")
            keybuf = ctypes.create_string_buffer(key, 32)
            o.key = ctypes.cast(keybuf, ctypes.c_void_p)
        o.packers, o.readers, o.batch_bytes, o.timestamp = int(packers), int(readers), int(batch_bytes), int(timestamp)
        if known:
            ks = sorted(bytes(k) for k in known)
            knownbuf = ctypes.create_string_buffer(b"".join(ks), 32 * len(ks))
            o.known, o.nknown = ctypes.cast(knownbuf, ctypes.c_void_p), len(ks)
        self._h = ctypes.c_void_p()
        _lib.check(_lib.lib().cdc_backup_new(int(dev), ctypes.byref(o), ctypes.byref(self._h)), "cdc_backup_new")

    def run(self, paths, keep_packfiles=True, content_type=None):
        """Back up the files: (objects, packfiles, stats), as backup_files.
        A file that cannot be read has no object (None) and its status in
        self.failed; the others are backed up.  content_type(path, first_chunk)
        -> str, when given, fills Object.ContentType from the path and the
        bytes of the file's first chunk, as chunkify does with
        mime.TypeByExtension and mimetype.Detect (snapshot/backup.go:580,
        598-601); the bytes come from the pipeline's own read (no re-read)."""
        import ctypes
        from . import _lib
        if not self._h:
            raise ValueError("session closed")
        n = len(paths)
        arr = (ctypes.c_char_p * max(n, 1))(*[str(p).encode() for p in paths])
        objects = [None] * n
        pending = {}  # file index -> ChunkRecords of its pieces so far (files larger than batch_bytes)
        ctypes_of = {}  # file index -> ContentType (from its first piece)
        self.failed = {}  # file index -> status of the files that could not be read (recordError)
        self.callback_order = []  # (file index, piece) in the order the pipeline delivered them
        packs = []
        errors = []

        def on_file(_ctx, fp):
            try:
                f = fp.contents
                i = int(f.index)
                self.callback_order.append((i, int(f.piece)))
                if f.status != 0:  # backupCtx.recordError (snapshot/backup.go:264-267): no object, the run goes on
                    self.failed[i] = int(f.status)
                    pending.pop(i, None)
                    return
                m = int(f.nchunks)
                parts = pending.pop(i, [])
                if m:  # copies: the pipeline reuses these buffers once the callback returns
                    cuts = np.ctypeslib.as_array(ctypes.cast(f.cuts, ctypes.POINTER(ctypes.c_uint8)),
                                                 (16 * m,)).view(np.dtype(_lib.CUT_DTYPE_FIELDS))
                    if content_type is not None and int(f.piece) == 0 and f.data:
                        first = ctypes.string_at(f.data, min(int(cuts["length"][0]), int(f.data_len)))
                        ctypes_of[i] = content_type(paths[i], first)
                    parts.append(ChunkRecords(
                        np.ctypeslib.as_array(f.digests, (32 * m,)).tobytes(),
                        cuts["length"].astype(np.int64),
                        np.ctypeslib.as_array(f.entropy, (m,)).copy(),  # the device's entropy() per chunk
                        np.ctypeslib.as_array(f.hists, (256 * m,)).reshape(m, 256).copy()))
                if int(f.piece) + 1 < int(f.pieces):
                    pending[i] = parts
                    return
                objects[i] = Object(Checksum=bytes(f.checksum), Chunks=ChunkRecords.concat(parts),
                                    ContentType=ctypes_of.pop(i, ""), Entropy=float(f.object_entropy))
            except Exception as e:  # noqa: BLE001 - re-raised after the call
                errors.append(e)

        def on_pack(_ctx, data, length):
            packs.append(ctypes.string_at(data, length) if keep_packfiles else None)
            return 0

        fcb, pcb = _lib.BACKUP_FILE_FN(on_file), _lib.BACKUP_PACK_FN(on_pack)
        st = _lib.cdc_backup_stats()
        # The callbacks create a few objects per file, none of them in a
        # cycle.  The cyclic collector is off for the whole call (gc.disable
        # is process-wide): a collection triggered by those allocations would
        # walk the whole heap between callbacks.
        gc_was = gc.isenabled()
        gc.disable()
        try:
            rc = _lib.lib().cdc_backup_files(self._h, arr, n, fcb, pcb, None, ctypes.byref(st))
        finally:
            if gc_was:
                gc.enable()
        _lib.check(rc, "cdc_backup_files")
        if errors:
            raise errors[0]
        stats = {name: getattr(st, name) for name, _ in _lib.cdc_backup_stats._fields_}
        return objects, [p for p in packs if p is not None], stats

    def close(self):
        from . import _lib
        if self._h:
            _lib.lib().cdc_backup_free(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def backup_files(paths, repo: Repository = None, key=None, compression="LZ4", known=None, max_size=None,
                 packers=8, readers=8, batch_bytes=256 << 20, timestamp=0, dev=0, keep_packfiles=True):
    """One backup of a list of files through the native pipeline (a
    BackupSession for this call only).  known: iterable of 32-byte digests
    already in the repository (not stored again).  Returns (objects,
    packfiles, stats): one Object per path in order (entropy and
    Distribution computed here from the device histograms, as chunkify_batch
    does), the serialised packfiles in the order the packers flushed them,
    and the per-stage stats of cdc_backup_stats."""
    with BackupSession(repo, key, compression, known, max_size, packers, readers, batch_bytes, timestamp,
                       dev) as s:
        return s.run(paths, keep_packfiles)


__all__ = ["Object", "ChunkRecords", "route", "chunkify_batch", "backup_batch", "BackupSession", "backup_files"]
