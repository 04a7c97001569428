"""Device Encode: plakar's (*Repository).Encode --
the LZ4 frame of compression.DeflateLZ4Stream, then the AES-256-GCM stream of
encryption.EncryptStream -- checked with independent decoders (the system's
liblz4 and OpenSSL libcrypto, tests/crypto_ref.py) and the NIST SP 800-38D
AES-256 test vectors.  Nonces and subkeys are random in the reference, so the
encrypted bytes are checked by round trip and by structure; the AES-GCM
arithmetic itself is pinned by the vectors."""
import os
import struct

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import crypto_ref as ref  # noqa: E402
from datagen import low_entropy, random_bytes  # noqa: E402
from plakar_amd import _lib, encode  # noqa: E402

pytestmark = pytest.mark.gpu

KEY = bytes(range(32))

# NIST GCM test vectors, AES-256 (test cases 13-15 of the GCM specification).
NIST = [
    (bytes(32), bytes(12), b"", "", "530f8afbc74536b9a963b4f1c4cb738b"),
    (bytes(32), bytes(12), bytes(16), "cea7403d4d606b6e074ec5d3baf39d18", "d0d1c8a799996bf0265b98b5d48ab919"),
    (bytes.fromhex("feffe9928665731c6d6a8f9467308308feffe9928665731c6d6a8f9467308308"),
     bytes.fromhex("cafebabefacedbaddecaf888"),
     bytes.fromhex("d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a72"
                   "1c3c0c95956809532fcf0e2449a6b525b16aedf5aa0de657ba637b391aafd255"),
     "522dc1f099567d07f47f37a32a84427d643a8cdcbfe5c0c97598a2bd2555d1aa"
     "8cb08e48590dbb3da7b08b1056828838c5f61e6393ba7a0abcc9f662898015ad",
     "b094dac5d93471bdec1a502270e3cc6c"),
]


@pytest.fixture(scope="module", autouse=True)
def _init():
    _lib.ensure_init()


@pytest.mark.parametrize("case", range(len(NIST)))
def test_gcm_nist_vectors(case):
    """Encode without compression, the blob sealed under subkey = the vector's
    key with data nonce = its IV: the first piece is exactly IV || C || T; the
    header opens under the repository key to that subkey."""
    k, iv, p, c, t = NIST[case]
    rnd = k + bytes(range(100, 112)) + iv  # subkey, subkey nonce, data nonce
    (out,) = encode.encode_blobs([p], key=KEY, compress=False, random=rnd)
    assert out[:12] == bytes(range(100, 112))
    assert ref.gcm_open(KEY, out[:12], out[12:60]) == k
    if p:
        assert out[60:72] == iv
        assert out[72:].hex() == c + t
    else:
        assert len(out) == 60  # EncryptStream writes no piece for an empty stream
        assert ref.gcm_seal(k, iv, b"").hex() == t  # the checker itself, on the empty vector


def test_gcm_against_libcrypto_pieces():
    """Multi-piece streams (64-KiB pieces, a short last one) against
    libcrypto, piece by piece, with the per-piece nonce rule."""
    blob = random_bytes(3 * 65536 + 1000, 31).tobytes()
    rnd = os.urandom(56)
    (out,) = encode.encode_blobs([blob], key=KEY, compress=False, random=rnd)
    sub, dn = rnd[:32], rnd[44:56]
    pos, k = 60, 0
    while pos < len(out):
        nonce = dn[:8] + (int.from_bytes(dn[8:], "big") ^ k).to_bytes(4, "big")
        piece = blob[k * 65536:(k + 1) * 65536]
        assert out[pos:pos + 12] == nonce
        assert out[pos + 12:pos + 12 + len(piece) + 16] == ref.gcm_seal(sub, nonce, piece)
        pos += 12 + len(piece) + 16
        k += 1
    assert k == 4 and pos == len(out)


SIZES = [0, 1, 15, 16, 17, 4095, 16384, 16385, 65535, 65536, 65537, (1 << 20) + 13, 4 << 20, (4 << 20) + 1,
         (9 << 20) + 77]


def _blobs(kind):
    out = []
    for i, n in enumerate(SIZES):
        if kind == "random":
            out.append(random_bytes(n, 500 + i).tobytes())
        elif kind == "low":
            out.append(low_entropy(n, 600 + i).tobytes())
        else:  # text-like: repeated words with variation
            words = [b"backup ", b"snapshot ", b"chunk ", b"packfile ", b"plakar ", b"%d " % i]
            r = np.random.default_rng(i)
            s = b"".join(words[j] for j in r.integers(0, len(words), size=n // 4 + 1))
            out.append(s[:n])
    return out


@pytest.mark.parametrize("kind", ["random", "low", "text"])
def test_lz4_frames_decode_with_liblz4(kind):
    """Compression only: every frame decodes with liblz4 (block sizes,
    content checksum) to the blob; the header is pierrec/lz4 v4's default
    (FLG 0x64: version 1, independent blocks, content checksum; BD 0x70:
    4-MiB blocks); compressible data shrinks."""
    import xxhash
    blobs = _blobs(kind)
    outs = encode.encode_blobs(blobs, key=None, compress=True)
    for b, o in zip(blobs, outs):
        if not b:  # an empty blob compresses to an empty stream, not a frame (compression/compression.go:58-62)
            assert o == b""
            continue
        assert o[:4] == struct.pack("<I", 0x184D2204) and o[4] == 0x64 and o[5] == 0x70
        assert o[6] == (xxhash.xxh32(o[4:6]).intdigest() >> 8) & 0xFF
        assert o[-4:] == struct.pack("<I", xxhash.xxh32(b).intdigest())
        assert ref.lz4f_decompress(o) == b, f"{len(b)} bytes"
    total_in = sum(len(b) for b in blobs)
    total_out = sum(len(o) for o in outs)
    if kind == "random":
        assert total_out <= total_in + 19 * len(blobs) + 4 * 5  # stored blocks
    else:
        assert total_out < 0.5 * total_in, (total_out, total_in)


def test_encode_empty_blob_like_the_reference():
    """plakar PutBlobs an empty chunk for every empty file
    (snapshot/backup.go:631-635).  Encode of it: DeflateStream returns an
    empty stream for empty input (compression/compression.go:58-62), and
    EncryptStream of an empty stream writes only its 60-byte header -- the
    subkey nonce and the sealed subkey -- and no piece
    (encryption/symmetric.go:116-157: ReadFull returns n = 0 at once)."""
    rnd = os.urandom(56)
    for compress in (True, False):
        (enc,) = encode.encode_blobs([b""], key=KEY, compress=compress, random=rnd)
        assert len(enc) == 60
        assert enc[:12] == rnd[32:44]
        assert ref.gcm_open(KEY, enc[:12], enc[12:60]) == rnd[:32]  # the sealed subkey
        assert ref.decode(enc, key=KEY, compressed=compress) == b""
        (plain,) = encode.encode_blobs([b""], key=None, compress=compress)
        assert plain == b""
    # empty blobs between non-empty ones keep every offset right
    blobs = [b"", random_bytes(70_000, 3).tobytes(), b"", b"x", b""]
    outs = encode.encode_blobs(blobs, key=KEY)
    assert [len(o) for o in outs][0::2] == [60, 60, 60]
    for b, o in zip(blobs, outs):
        assert ref.decode(o, key=KEY) == b


@pytest.mark.parametrize("compress", [True, False])
def test_encode_roundtrip(compress):
    """The whole Encode: DecryptStream (restated over libcrypto) then the LZ4
    frame reader (liblz4) give back every blob; random material from the
    OS CSPRNG, as the reference's crypto/rand."""
    blobs = _blobs("text")[:10] + _blobs("random")[8:12]
    outs = encode.encode_blobs(blobs, key=KEY, compress=compress)
    for b, o in zip(blobs, outs):
        assert ref.decode(o, key=KEY, compressed=compress) == b
        with pytest.raises(ValueError):  # a flipped ciphertext bit fails its tag
            bad = bytearray(o)
            bad[-1] ^= 1
            ref.decode(bytes(bad), key=KEY, compressed=compress)


def test_encode_device_resident_batch():
    """The device entry point over blobs at arbitrary offsets of one buffer
    (a chunked file's cut list), output offsets as documented."""
    data = low_entropy(12 << 20, 77)
    t = torch.from_numpy(data).cuda()
    cuts = [(0, 70_000), (70_000, 1 << 20), ((1 << 20) + 70_000, 3 << 20), ((4 << 20) + 70_000, 5_000_000),
            (12 << 20, 0)]
    offs, lens = [c[0] for c in cuts], [c[1] for c in cuts]
    cap = sum(encode.encode_bound(n) for n in lens)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    oo = encode.encode_device(t, offs, lens, out, key=KEY)
    host = out.cpu().numpy()
    for i, (o, n) in enumerate(cuts):
        enc = host[oo[i]:oo[i + 1]].tobytes()
        assert ref.decode(enc, key=KEY) == data[o:o + n].tobytes()
    small = torch.empty(int(oo[-1]) - 1, dtype=torch.uint8, device="cuda")
    with pytest.raises(_lib.CdcError):
        encode.encode_device(t, offs, lens, small, key=KEY)


def test_gcm_device_plaintext_at_every_alignment():
    """GCM only (no LZ4): pieces read straight from the caller's buffer, at
    every byte offset mod 16 and with ragged last blocks, whole pieces and
    short ones, decrypt to their bytes."""
    data = random_bytes(6 << 20, 91)
    t = torch.from_numpy(data).cuda()
    cuts, pos = [], 0
    for i, n in enumerate([65536, 2 * 65536 + 5, 1000, 17, 3 * 65536 + 3, 65535, 16, 1, 4 * 65536, 70_001,
                           31, 65536 + 16, 200_000, 48, 65537, 12345]):
        pos += i % 16 + 1  # start at offset i mod 16 (+1) past the previous blob
        cuts.append((pos, n))
        pos += n
    assert pos <= data.size
    offs, lens = [c[0] for c in cuts], [c[1] for c in cuts]
    cap = sum(encode.encode_bound(n, False, True) for n in lens)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    oo = encode.encode_device(t, offs, lens, out, key=KEY, compress=False)
    host = out.cpu().numpy()
    for i, (o, n) in enumerate(cuts):
        enc = host[oo[i]:oo[i + 1]].tobytes()
        assert ref.decode(enc, key=KEY, compressed=False) == data[o:o + n].tobytes(), (o, n)


def test_backup_batch_device_encoder():
    """backup_batch with the device Encode: every blob in the packfiles opens
    under the repository key and inflates to its chunk (Decode, then the
    chunk's SHA-256 is its index checksum)."""
    import hashlib

    import packfile_ref as pf
    from plakar_amd import snapshot
    files = [low_entropy(n, 80 + i) for i, n in enumerate([0, 5000, 70_000, 6 << 20, 13 << 20])]
    files.append(random_bytes(3 << 20, 90))
    enc = encode.DeviceEncoder(key=KEY)
    objs, packs = snapshot.backup_batch(files, known=set(), max_size=4 << 20, encode=enc, timestamp=7)
    seen = 0
    for pk in packs:
        p = pf.parse(pk)
        for t, c, o, n in p.index:
            plain = ref.decode(bytes(p.blobs[o:o + n]), key=KEY)
            assert hashlib.sha256(plain).digest() == c
            seen += 1
    assert seen == len({c.Checksum for ob in objs for c in ob.Chunks})


def test_encode_device_offsets_across_tensors():
    """Offsets are plain device-address displacements from d_base, so one call
    can cover the chunks of several device buffers (bench.py's encode leg)."""
    parts = [low_entropy(3 << 20, 41), random_bytes((2 << 20) + 333, 42)]
    ts = [torch.from_numpy(p).cuda() for p in parts]
    base = min(ts, key=lambda t: t.data_ptr())
    offs, lens, src = [], [], []
    for p, t in zip(parts, ts):
        for a, n in ((0, 70_000), (70_000, 1_000_001), (1_070_001, p.size - 1_070_001)):
            offs.append(t.data_ptr() - base.data_ptr() + a)
            lens.append(n)
            src.append(p[a:a + n].tobytes())
    cap = sum(encode.encode_bound(n) for n in lens)
    out = torch.empty(cap, dtype=torch.uint8, device="cuda")
    oo = encode.encode_device(base, offs, lens, out, key=KEY)
    host = out.cpu().numpy()
    for i, s in enumerate(src):
        assert ref.decode(host[oo[i]:oo[i + 1]].tobytes(), key=KEY) == s


@pytest.mark.parametrize("seed", range(12))
def test_encode_random_batches(seed):
    """Random batches: 1-300 blobs of 0 B-9 MiB (across the 64-KiB GCM pieces,
    the 8-KiB match segments and the 4-MiB LZ4 blocks), random, low-entropy,
    repetitive and text-like contents, each encoding; every blob comes back
    through DecryptStream + the LZ4 frame reader."""
    rng = np.random.default_rng(np.random.PCG64(4200 + seed))
    blobs = []
    for i in range(int(rng.integers(1, 301))):
        r = rng.random()
        n = 0 if r < 0.05 else int(rng.choice([65536, 4 << 20, 8192])) + int(rng.integers(-2, 3)) if r < 0.2 \
            else int(np.exp(rng.uniform(0, np.log(9 << 20))))
        n = max(0, n)
        k = int(rng.integers(0, 4))
        if k == 0:
            b = random_bytes(n, 4300 + 512 * seed + i).tobytes()
        elif k == 1:
            b = low_entropy(n, 4300 + 512 * seed + i, 0.02).tobytes()
        elif k == 2:
            b = (random_bytes(int(rng.integers(1, 300)), i).tobytes() * (n // 7 + 1))[:n]
        else:
            b = (b"backup snapshot chunk packfile plakar %d " % i * (n // 30 + 1))[:n]
        blobs.append(b)
    key = KEY if seed % 3 != 2 else None
    compress = seed % 2 == 0
    outs = encode.encode_blobs(blobs, key=key, compress=compress)
    for i, (b, o) in enumerate(zip(blobs, outs)):
        assert ref.decode(o, key=key, compressed=compress) == b, f"seed {seed} blob {i} ({len(b)} B)"
