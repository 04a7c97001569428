"""The packfile builder (cdc_packer_*, host code) against the CPU restatement
of packfile.go (tests/packfile_ref.py): byte-identical packfiles, the
NewFromBytes round trip, the PutPackfile layout and packerJob's flush rule.
Runs without a GPU (the packer is host code of libplakar_cdc.so)."""
import hashlib
import struct

import numpy as np

import packfile_ref as ref
from datagen import random_bytes
from plakar_amd import packer


def _blobs(seed, n):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        ln = int(rng.integers(0, 200_000)) if i % 7 else 0
        data = random_bytes(ln, seed * 1000 + i).tobytes()
        out.append((int(rng.integers(0, 9)), hashlib.sha256(data).digest(), data))
    return out


def test_serialize_matches_packfile_go():
    ts = 1_734_912_000_123_456_789
    p = packer.Packer(timestamp=ts)
    r = ref.PackFile(ts)
    for typ, csum, data in _blobs(1, 40):
        p.AddBlob(typ, csum, data)
        r.add_blob(typ, csum, data)
    assert p.Size() == r.size() and p.Count() == r.count
    got = p.Serialize()
    assert got == r.serialize()
    assert p.SerializePart(0) == bytes(r.blobs)
    assert p.SerializePart(1) == r.serialize_index()
    assert p.SerializePart(2) == r.serialize_footer()
    back = ref.parse(got)  # NewFromBytes, index checksum included
    assert back.timestamp == ts and back.count == 40 and back.index == r.index
    for t, c, o, n in back.index:
        assert hashlib.sha256(bytes(back.blobs[o:o + n])).digest() == c


def test_put_packfile_layout_and_empty():
    p = packer.Packer(timestamp=7)
    r = ref.PackFile(7)
    assert p.Serialize() == r.serialize()  # an empty packfile: index empty, footer only
    for typ, csum, data in _blobs(2, 5):
        p.AddBlob(typ, csum, data)
        r.add_blob(typ, csum, data)
    enc = lambda b: b[::-1] + b"x"  # any Encode: the layout frames whatever it returns
    got = p.PutPackfileBytes(enc)
    assert got == ref.put_packfile_layout(r, enc)
    assert struct.unpack("<I", got[-5:-1])[0] == 100 and got[-1] == len(enc(r.serialize_footer()))


def test_flush_rule_and_add_chunks():
    """packerJob flushes once Size() > MaxSize; add_chunks consumes cut rows with digests and skips known ones."""
    base = random_bytes(3 << 20, 5)
    offs = np.arange(0, base.size, 100_000, dtype=np.uint64)
    lens = np.minimum(np.uint64(100_000), np.uint64(base.size) - offs)
    cuts = np.stack([offs, lens], axis=1)
    dg = np.stack([np.frombuffer(hashlib.sha256(base[int(o):int(o + n)].tobytes()).digest(), np.uint8)
                   for o, n in cuts])
    skip = np.zeros(len(cuts), np.uint8)
    skip[3] = 1
    p = packer.Packer(max_size=1 << 20, timestamp=11)
    used = p.add_chunks(base, cuts, dg, skip)
    assert p.Size() > (1 << 20) and used < len(cuts)
    r = ref.PackFile(11)
    for i in range(used):
        if not skip[i]:
            o, n = int(cuts[i, 0]), int(cuts[i, 1])
            r.add_blob(ref.TYPE_CHUNK, dg[i].tobytes(), base[o:o + n].tobytes())
    assert r.size() > (1 << 20) and r.size() - int(cuts[used - 1, 1]) <= (1 << 20)
    assert p.Serialize() == r.serialize()


def test_pack_chunks_dedup_and_roundtrip():
    files = [random_bytes(1 << 20, 8), random_bytes(2 << 20, 9)]
    files.append(files[0].copy())  # a duplicate file: its chunks are stored once
    cut_lists, digests = [], []
    for f in files:
        offs = np.arange(0, f.size, 65_536, dtype=np.uint64)
        lens = np.minimum(np.uint64(65_536), np.uint64(f.size) - offs)
        c = np.stack([offs, lens], axis=1)
        cut_lists.append(c)
        digests.append(np.stack([np.frombuffer(hashlib.sha256(f[int(o):int(o + n)].tobytes()).digest(), np.uint8)
                                 for o, n in c]))
    packs = packer.pack_chunks(files, cut_lists, digests, max_size=1 << 20, timestamp=3)
    seen = {}
    for pk in packs:
        pf = ref.parse(pk)
        assert pf.size() <= (1 << 20) + 65_536
        for t, c, o, n in pf.index:
            assert t == ref.TYPE_CHUNK and c not in seen
            seen[c] = bytes(pf.blobs[o:o + n])
    want = {d.tobytes() for ds in digests for d in ds}
    assert set(seen) == want
    for c, data in seen.items():
        assert hashlib.sha256(data).digest() == c
