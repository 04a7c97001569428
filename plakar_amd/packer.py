"""Mirror of plakar's snapshot/packer.go over libplakar_cdc.so's native packfile
builder (cdc_packer_*): Packer.AddBlob / Size, packfile.Serialize and the
PutPackfile layout (snapshot/snapshot.go:232-267), plus the batched form that
consumes a cut list and its per-chunk digests directly (PutBlob of every new
chunk of processChunk, snapshot/backup.go:625-626)."""
import ctypes
import struct
import time

import numpy as np

from . import _lib
from ._lib import CdcError, check, lib

TYPE_CHUNK = 1
DEFAULT_MAX_SIZE = 20 << 20  # packfile.DefaultConfiguration().MaxSize


class Packer:
    def __init__(self, max_size=DEFAULT_MAX_SIZE, timestamp=None):
        self._h = ctypes.c_void_p()
        check(lib().cdc_packer_new(int(max_size), ctypes.byref(self._h)), "cdc_packer_new")
        self._fixed = timestamp is not None  # a fixed Footer.Timestamp (tests); else packfile.New's time.Now()
        self.timestamp = time.time_ns() if timestamp is None else int(timestamp)

    def AddBlob(self, typ, checksum, data):
        """Packer.AddBlob; returns True once Size() > MaxSize (packerJob then flushes)."""
        buf = (ctypes.c_uint8 * 32).from_buffer_copy(bytes(checksum))
        a = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
        a = np.ascontiguousarray(a, dtype=np.uint8)
        st = lib().cdc_packer_add_blob(self._h, int(typ), buf, a.ctypes.data if a.size else None, a.size)
        check(st, "AddBlob")
        return st == 1

    def add_chunks(self, base, cuts, digests, skip=None):
        """TYPE_CHUNK blobs base[off:off+len] for the (n, 2) cut rows with digests (n, 32); rows with
        skip[i] set are left out (BlobExists).  Stops once the packfile is full; returns rows consumed."""
        base = np.ascontiguousarray(base, dtype=np.uint8)
        n = int(cuts.shape[0])
        rows = np.zeros((n, 2), dtype=np.uint64)
        rows[:, 0] = cuts[:, 0]
        rows[:, 1] = cuts[:, 1] & np.uint64(0xFFFFFFFF)
        dg = np.ascontiguousarray(digests, dtype=np.uint8).reshape(n, 32)
        sk = None if skip is None else np.ascontiguousarray(skip, dtype=np.uint8)
        r = lib().cdc_packer_add_chunks(self._h, base.ctypes.data, ctypes.cast(rows.ctypes.data, ctypes.POINTER(_lib.cdc_cut)),
                                        n, dg.ctypes.data, None if sk is None else sk.ctypes.data)
        if r < 0:
            raise CdcError(int(r), "add_chunks")
        return int(r)

    def Size(self):
        return int(lib().cdc_packer_size(self._h))

    def Count(self):
        return int(lib().cdc_packer_count(self._h))

    def _bytes(self, fn, *args):
        ln = ctypes.c_uint64()
        st = fn(self._h, *args, None, 0, ctypes.byref(ln))  # the size (CDC_E_NOSPACE unless empty)
        if st not in (_lib.CDC_OK, _lib.CDC_E_NOSPACE):
            raise CdcError(st, "serialize")
        out = (ctypes.c_uint8 * max(ln.value, 1))()
        check(fn(self._h, *args, out, ln.value, ctypes.byref(ln)), "serialize")
        return bytes(out[:ln.value])

    def Serialize(self):
        """(*PackFile).Serialize (packfile/packfile.go:241-294)."""
        return self._bytes(lib().cdc_packer_serialize, ctypes.c_int64(self.timestamp))

    def SerializePart(self, part):
        """0 SerializeData, 1 SerializeIndex, 2 SerializeFooter."""
        return self._bytes(lib().cdc_packer_serialize_part, int(part), ctypes.c_int64(self.timestamp))

    def PutPackfileBytes(self, encode=lambda b: b):
        """The bytes PutPackfile stores (snapshot/snapshot.go:236-267): data, Encode(index),
        Encode(footer), version u32 little-endian, u8 length of Encode(footer)."""
        data, idx, foot = self.SerializePart(0), self.SerializePart(1), self.SerializePart(2)
        ef = encode(foot)
        return data + encode(idx) + ef + struct.pack("<I", 100) + bytes([len(ef) & 0xFF])

    def Reset(self):
        lib().cdc_packer_reset(self._h)
        if not self._fixed:
            self.timestamp = time.time_ns()

    def close(self):
        if self._h:
            lib().cdc_packer_free(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pack_chunks(files, cut_lists, digest_lists, max_size=DEFAULT_MAX_SIZE, known=None, timestamp=None):
    """packerJob for one producer (snapshot/snapshot.go:51-92): every chunk not
    yet stored (known: a set of checksums, BlobExists; updated in place) is
    added once; a packfile is flushed when Size() > MaxSize, and the last
    partial one at the end.  Returns the serialised packfiles (Serialize form)."""
    known = set() if known is None else known
    out = []
    pk = Packer(max_size, timestamp)
    for f, cuts, dg in zip(files, cut_lists, digest_lists):
        n = int(cuts.shape[0])
        dg = np.asarray(dg, dtype=np.uint8).reshape(n, 32)
        skip = np.zeros(n, dtype=np.uint8)
        for i in range(n):
            d = dg[i].tobytes()
            if d in known:
                skip[i] = 1
            else:
                known.add(d)
        i = 0
        while i < n:
            used = pk.add_chunks(f, cuts[i:], dg[i:], skip[i:])
            i += used
            if pk.Size() > max_size:
                out.append(pk.Serialize())
                pk.Reset()
    if pk.Count():
        out.append(pk.Serialize())
    pk.close()
    return out
