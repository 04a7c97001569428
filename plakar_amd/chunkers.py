"""Mirror of the chunker API plakar consumes from ext go-cdc-chunkers v0.0.8.

    chunkers.ChunkerOpts{MinSize, NormalSize, MaxSize}   (chunking/chunking_test.go:19-23)
    chunkers.NewChunker(name, rd, opts)                  (repository/repository.go:288-292)
    (*Chunker).Next() ([]byte, error)                    (snapshot/backup.go:651-665)

Names, argument meaning and error behaviour follow the Go API: Next() returns
(chunk, err) where err is None or EOF; the empty stream yields (None, EOF) at
once.  Every chunk is cut on the GPU by libplakar_cdc.so (there is no CPU
path): the stream is staged through a pinned window the library owns and
chunked by the device kernels; ChunkBuffers is the batch form used by the
re-plumbed backup (one call for many files).
"""
import ctypes
import os

from . import _lib
from ._lib import CDC_EOF, CDC_NEED_DATA, CDC_OK, CdcError, check, ensure_init, lib


class _EOFType(Exception):
    """io.EOF."""

    def __repr__(self):
        return "EOF"


EOF = _EOFType("EOF")


class ChunkerOpts:
    """chunkers.ChunkerOpts."""

    __slots__ = ("MinSize", "NormalSize", "MaxSize")

    def __init__(self, MinSize=0, NormalSize=0, MaxSize=0):
        self.MinSize = int(MinSize)
        self.NormalSize = int(NormalSize)
        self.MaxSize = int(MaxSize)

    def __eq__(self, other):
        return (isinstance(other, ChunkerOpts) and self.MinSize == other.MinSize
                and self.NormalSize == other.NormalSize and self.MaxSize == other.MaxSize)

    def __repr__(self):
        return (f"ChunkerOpts(MinSize={self.MinSize}, NormalSize={self.NormalSize}, "
                f"MaxSize={self.MaxSize})")

    def _c(self):
        return _lib.cdc_opts(self.MinSize, self.NormalSize, self.MaxSize, 0)


def FastCDCDefaultOptions():
    """(*FastCDC).DefaultOptions(): used when NewChunker gets nil options."""
    return ChunkerOpts(MinSize=2 * 1024, NormalSize=8 * 1024, MaxSize=64 * 1024)


def Validate(algorithm, opts):
    """chunkers.NewChunker's registry lookup + (*FastCDC).Validate; raises CdcError."""
    o = opts._c()
    check(lib().cdc_validate(algorithm.encode(), ctypes.byref(o)), "NewChunker")


class Chunker:
    """*chunkers.Chunker over an io.Reader-like object (read(n) / readinto)."""

    def __init__(self, algorithm, reader, opts, window_bytes=0, device=0):
        ensure_init()
        self._rd = reader
        self._opts = opts
        self._h = ctypes.c_void_p()
        o = opts._c()
        check(lib().cdc_stream_new(algorithm.encode(), ctypes.byref(o), window_bytes, device,
                                   ctypes.byref(self._h)), "NewChunker")
        self._eof = False

    def _fill(self):
        L = lib()
        ptr = ctypes.POINTER(ctypes.c_uint8)()
        space = ctypes.c_uint64()
        check(L.cdc_stream_buffer(self._h, ctypes.byref(ptr), ctypes.byref(space)))
        n = space.value
        if n == 0:
            return
        dst = (ctypes.c_uint8 * n).from_address(ctypes.addressof(ptr.contents))
        view = memoryview(dst).cast("B")
        got = 0
        readinto = getattr(self._rd, "readinto", None)
        while got < n:
            if readinto is not None:
                k = readinto(view[got:])
            else:
                data = self._rd.read(n - got)
                k = len(data)
                view[got:got + k] = data
            if not k:
                self._eof = True
                break
            got += k
        check(L.cdc_stream_commit(self._h, got, 1 if self._eof else 0))

    def Next(self):
        """Return (chunk bytes, None), or (None, EOF) once the stream is drained."""
        L = lib()
        ptr = ctypes.POINTER(ctypes.c_uint8)()
        ln = ctypes.c_uint64()
        while True:
            st = L.cdc_stream_next(self._h, ctypes.byref(ptr), ctypes.byref(ln))
            if st == CDC_OK:
                return ctypes.string_at(ptr, ln.value), None
            if st == CDC_EOF:
                return None, EOF
            if st == CDC_NEED_DATA:
                self._fill()
                continue
            raise CdcError(st, "Next")

    def __iter__(self):
        while True:
            chunk, err = self.Next()
            if err is EOF:
                return
            yield chunk

    def close(self):
        if self._h:
            lib().cdc_stream_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def NewChunker(algorithm, reader, opts=None, window_bytes=0):
    """chunkers.NewChunker(algorithm, rd, opts); raises CdcError for an unknown
    algorithm or invalid sizes (the Go call returns them as its error)."""
    if opts is None:
        opts = FastCDCDefaultOptions()
    Validate(algorithm, opts)
    return Chunker(algorithm, reader, opts, window_bytes=window_bytes)


def ChunkBuffers(bufs, opts):
    """Batch API of the re-plumbed backup: chunk whole in-memory files on the
    GPU(s) in one call.  Returns, per buffer, a uint64 array of shape (n, 2)
    holding (offset, length) rows."""
    import numpy as np

    ensure_init()
    o = opts._c()
    check(lib().cdc_validate(b"fastcdc", ctypes.byref(o)), "ChunkBuffers")
    n = len(bufs)
    keep = []
    cbufs = (_lib.cdc_buf * max(n, 1))()
    total_cap = 0
    for i, b in enumerate(bufs):
        a = np.frombuffer(b, dtype=np.uint8) if not isinstance(b, np.ndarray) else b
        a = np.ascontiguousarray(a, dtype=np.uint8)
        keep.append(a)
        cbufs[i].data = a.ctypes.data if a.size else None
        cbufs[i].len = a.size
        total_cap += a.size // max(opts.MinSize, 1) + 2
    out = np.zeros((max(total_cap, 1), 2), dtype=np.uint64)
    counts = (ctypes.c_uint64 * max(n, 1))()
    needed = ctypes.c_uint64()
    check(lib().cdc_chunk(cbufs, n, ctypes.byref(o),
                          ctypes.cast(out.ctypes.data, ctypes.POINTER(_lib.cdc_cut)),
                          out.shape[0], counts, ctypes.byref(needed)), "ChunkBuffers")
    res, k = [], 0
    for i in range(n):
        c = counts[i]
        part = out[k:k + c].copy()
        part[:, 1] &= np.uint64(0xFFFFFFFF)
        res.append(part)
        k += c
    return res


class FileBatch:
    """A batch of whole files read straight into library-owned pinned host
    memory (cdc_batch_*), chunked in one call with pinned host-to-device
    copies.  This is the importer side of the re-plumbed backup: plakar opens
    and reads each file (snapshot/importer/fs/fs.go:69-71) and chunks it
    (snapshot/backup.go:647-665); here a whole batch of files is read by
    `threads` threads into the arena and chunked at once.  The bytes stay
    readable (`buffer(i)`) until `reset()`, for the per-chunk work."""

    def __init__(self, capacity):
        ensure_init()
        self._h = ctypes.c_void_p()
        check(lib().cdc_batch_new(int(capacity), ctypes.byref(self._h)), "cdc_batch_new")

    def add_files(self, paths, threads=8):
        """Append whole files (all or none); returns their sizes."""
        n = len(paths)
        arr = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(p) for p in paths])
        sizes = (ctypes.c_uint64 * max(n, 1))()
        check(lib().cdc_batch_add_files(self._h, arr, n, int(threads), sizes), "cdc_batch_add_files")
        return [int(sizes[i]) for i in range(n)]

    def add_and_chunk(self, paths, opts, threads=8):
        """add_files(paths) and the chunking of those files, overlapped
        (cdc_batch_chunk_files: reader threads run ahead of the device, which
        chunks each >= 256-MiB sub-batch of whole files once it is read).
        Returns per file a uint64 (n, 2) array of (offset, length) rows."""
        import numpy as np
        o = opts._c()
        check(lib().cdc_validate(b"fastcdc", ctypes.byref(o)), "FileBatch.add_and_chunk")
        n = len(paths)
        arr = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(p) for p in paths])
        sizes = (ctypes.c_uint64 * max(n, 1))()
        cap = sum(os.path.getsize(p) // max(opts.MinSize, 1) + 2 for p in paths)
        out = np.zeros((max(cap, 1), 2), dtype=np.uint64)
        counts = (ctypes.c_uint64 * max(n, 1))()
        needed = ctypes.c_uint64()
        check(lib().cdc_batch_chunk_files(self._h, arr, n, int(threads), ctypes.byref(o),
                                          ctypes.cast(out.ctypes.data, ctypes.POINTER(_lib.cdc_cut)), out.shape[0],
                                          counts, ctypes.byref(needed), sizes), "FileBatch.add_and_chunk")
        res, k = [], 0
        for i in range(n):
            c = counts[i]
            part = out[k:k + c].copy()
            part[:, 1] &= np.uint64(0xFFFFFFFF)
            res.append(part)
            k += c
        return res

    def add_fd(self, fd, length):
        check(lib().cdc_batch_add_fd(self._h, int(fd), int(length)), "cdc_batch_add_fd")

    def __len__(self):
        return lib().cdc_batch_count(self._h)

    def buffer(self, i):
        """The bytes of buffer i (a numpy view of the pinned arena; valid until reset())."""
        import numpy as np
        ptr = ctypes.POINTER(ctypes.c_uint8)()
        ln = ctypes.c_uint64()
        check(lib().cdc_batch_get(self._h, int(i), ctypes.byref(ptr), ctypes.byref(ln)), "cdc_batch_get")
        if ln.value == 0:
            return np.zeros(0, dtype=np.uint8)
        return np.ctypeslib.as_array(ptr, shape=(ln.value,))

    def chunk(self, opts):
        """cdc_chunk over every buffer: per buffer a uint64 (n, 2) array of (offset, length) rows."""
        import numpy as np
        o = opts._c()
        check(lib().cdc_validate(b"fastcdc", ctypes.byref(o)), "FileBatch.chunk")
        n = len(self)
        total = 0
        for i in range(n):
            ptr = ctypes.POINTER(ctypes.c_uint8)()
            ln = ctypes.c_uint64()
            check(lib().cdc_batch_get(self._h, i, ctypes.byref(ptr), ctypes.byref(ln)))
            total += ln.value // max(opts.MinSize, 1) + 2
        out = np.zeros((max(total, 1), 2), dtype=np.uint64)
        counts = (ctypes.c_uint64 * max(n, 1))()
        needed = ctypes.c_uint64()
        check(lib().cdc_batch_chunk(self._h, ctypes.byref(o), ctypes.cast(out.ctypes.data, ctypes.POINTER(_lib.cdc_cut)),
                                    out.shape[0], counts, ctypes.byref(needed)), "FileBatch.chunk")
        res, k = [], 0
        for i in range(n):
            c = counts[i]
            part = out[k:k + c].copy()
            part[:, 1] &= np.uint64(0xFFFFFFFF)
            res.append(part)
            k += c
        return res

    def reset(self):
        lib().cdc_batch_reset(self._h)

    def close(self):
        if self._h:
            lib().cdc_batch_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Collector:
    """Concurrent per-file chunking, batched for the device (cdc_collector_*).

    plakar chunks each file in its own goroutine (snapshot/backup.go:216-225,
    each running the Next() loop of backup.go:647-665).  Threads call
    `chunk(buf)` concurrently; the library queues the calls and submits them
    to the devices as batches (up to `batch_bytes`, 64 files, or `max_wait_us`
    after the first file of a batch arrived).  Each call blocks until its own
    cut list is back: a uint64 (n, 2) array of (offset, length) rows."""

    def __init__(self, opts, batch_bytes=256 << 20, max_wait_us=200):
        ensure_init()
        self._opts = opts
        o = opts._c()
        self._h = ctypes.c_void_p()
        check(lib().cdc_collector_new(ctypes.byref(o), int(batch_bytes), int(max_wait_us), ctypes.byref(self._h)),
              "cdc_collector_new")

    def chunk(self, buf):
        import numpy as np
        a = np.ascontiguousarray(np.asarray(buf, dtype=np.uint8).reshape(-1))
        cap = a.size // max(self._opts.MinSize, 1) + 2
        out = np.zeros((cap, 2), dtype=np.uint64)
        n = ctypes.c_uint64()
        check(lib().cdc_collector_chunk(self._h, ctypes.c_void_p(a.ctypes.data if a.size else 0), a.size,
                                        ctypes.cast(out.ctypes.data, ctypes.POINTER(_lib.cdc_cut)), cap,
                                        ctypes.byref(n)), "Collector.chunk")
        res = out[:n.value].copy()
        res[:, 1] &= np.uint64(0xFFFFFFFF)
        return res

    def stats(self):
        """(requests, batches) so far."""
        r, b = ctypes.c_uint64(), ctypes.c_uint64()
        check(lib().cdc_collector_stats(self._h, ctypes.byref(r), ctypes.byref(b)))
        return r.value, b.value

    def close(self):
        if self._h:
            lib().cdc_collector_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
