"""The native end-to-end backup pipeline (cdc_backup_run, snapshot.backup_files):
files -> reads + object SHA-256 -> cut points -> chunk SHA-256 + histograms ->
BlobExists -> Encode -> concurrent packers -> packfiles (SURVEY.md §8f rank 3;
snapshot/backup.go:571-687, snapshot/blobs.go:9-24, snapshot/snapshot.go:51-92).

Checked against the already-validated batch path (snapshot.chunkify_batch:
cut points vs the oracle, digests vs hashlib) and by opening every packfile
with the packfile.go restatement (tests/packfile_ref.py) and every blob with
DecryptStream + the LZ4 reader (tests/crypto_ref.py)."""
import hashlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import crypto_ref as ref  # noqa: E402
import packfile_ref as pf  # noqa: E402
from datagen import low_entropy, random_bytes  # noqa: E402
from plakar_amd import _lib, snapshot  # noqa: E402

pytestmark = pytest.mark.gpu

KEY = bytes(range(32, 64))


@pytest.fixture(scope="module")
def corpus(tmp_path_factory):
    d = tmp_path_factory.mktemp("backup")
    files = [b"", random_bytes(1, 1).tobytes(), random_bytes(1000, 2).tobytes(),
             random_bytes(65535, 3).tobytes(), random_bytes(65536, 4).tobytes(), random_bytes(70_000, 5).tobytes(),
             random_bytes(3 << 20, 6).tobytes(), low_entropy(6 << 20, 7).tobytes(), random_bytes(13 << 20, 8).tobytes()]
    files.append(files[6])        # a duplicate file: its chunks are not stored again
    files.append(b"")             # a second empty file: the empty chunk is stored once
    files.append(files[8][:5 << 20] + random_bytes(1 << 20, 9).tobytes())  # shares a prefix
    paths = []
    for i, b in enumerate(files):
        p = d / f"f{i:02d}"
        p.write_bytes(b)
        paths.append(str(p))
    return paths, files


def _blobs_of(packs, key, compressed):
    out = {}
    for pk in packs:
        p = pf.parse(pk)
        for t, c, o, n in p.index:
            assert t == 1  # TYPE_CHUNK
            assert c not in out, "a chunk was stored twice"
            raw = bytes(p.blobs[o:o + n])
            out[c] = ref.decode(raw, key=key, compressed=compressed) if (key or compressed) else raw
    return out


@pytest.mark.parametrize("key,compression", [(KEY, "LZ4"), (None, None), (None, "LZ4")])
def test_backup_files_matches_chunkify_and_packs_every_chunk_once(corpus, key, compression):
    paths, files = corpus
    objs, packs, st = snapshot.backup_files(paths, key=key, compression=compression, max_size=2 << 20,
                                            packers=3, readers=4, batch_bytes=8 << 20, timestamp=11)
    ref_objs = snapshot.chunkify_batch(files)
    assert len(objs) == len(files)
    for i, (o, r) in enumerate(zip(objs, ref_objs)):
        assert o.Checksum == r.Checksum == hashlib.sha256(files[i]).digest(), f"file {i}"
        assert [c.Length for c in o.Chunks] == [c.Length for c in r.Chunks], f"file {i}"
        assert [c.Checksum for c in o.Chunks] == [c.Checksum for c in r.Chunks], f"file {i}"
        assert [c.Entropy for c in o.Chunks] == [c.Entropy for c in r.Chunks], f"file {i}"
        for a, b in zip(o.Chunks, r.Chunks):
            assert np.array_equal(a.Distribution, b.Distribution)
        assert o.Entropy == r.Entropy
    blobs = _blobs_of(packs, key, compression == "LZ4")
    want = {}
    for f, o in zip(files, objs):
        off = 0
        for c in o.Chunks:
            want[c.Checksum] = f[off:off + c.Length]
            off += c.Length
    assert set(blobs) == set(want)
    for c, plain in blobs.items():
        assert plain == want[c] and hashlib.sha256(plain).digest() == c
    assert st["files"] == len(files) and st["new_blobs"] == len(want) and st["batches"] >= 3
    assert st["packfiles"] == len(packs) and st["bytes"] == sum(len(f) for f in files)
    for pk in packs:  # flushed at Size() > MaxSize: no packfile holds much more than one blob past it
        assert pf.parse(pk).timestamp == 11


def test_backup_files_known_digests_are_skipped(corpus):
    """BlobExists: digests the repository already holds are not stored."""
    paths, files = corpus
    objs, _, _ = snapshot.backup_files(paths, key=KEY)
    every = {c.Checksum for o in objs for c in o.Chunks}
    objs2, packs2, st2 = snapshot.backup_files(paths, key=KEY, known=every)
    assert packs2 == [] and st2["new_blobs"] == 0
    assert [o.Checksum for o in objs2] == [o.Checksum for o in objs]
    some = set(list(sorted(every))[: len(every) // 2])
    _, packs3, st3 = snapshot.backup_files(paths, key=KEY, known=some)
    assert set(_blobs_of(packs3, KEY, True)) == every - some and st3["new_blobs"] == len(every - some)


def test_backup_files_unreadable_files_are_recorded_and_the_rest_backed_up(tmp_path):
    """A missing path, a directory and a file that ends before its stat()
    size each fail on their own (status CDC_E_IO, no object), as
    backupCtx.recordError does (snapshot/backup.go:264-267); every other file
    is backed up and packed."""
    good = [random_bytes(200_000, 31).tobytes(), b"x" * 100, random_bytes(3 << 20, 32).tobytes()]
    paths = []
    for i, b in enumerate(good):
        p = tmp_path / f"ok{i}"
        p.write_bytes(b)
        paths.append(str(p))
    (tmp_path / "adir").mkdir()
    bad = [str(tmp_path / "missing"), str(tmp_path / "adir")]
    # a sysfs attribute: stat() says 4096 bytes, a read returns fewer (a file that shrank)
    short = next((q for q in ("/sys/kernel/mm/transparent_hugepage/enabled", "/sys/kernel/profiling")
                  if __import__("os").path.exists(q)), None)
    if short:
        bad.append(short)
    order = [paths[0], bad[0], paths[1], bad[1], paths[2]] + bad[2:]
    with snapshot.BackupSession(key=KEY, batch_bytes=8 << 20, packers=2) as s:
        objs, packs, st = s.run(order)
        failed = dict(s.failed)
    idx_bad = [order.index(b) for b in bad]
    assert sorted(failed) == idx_bad and all(v == _lib.CDC_E_IO for v in failed.values())
    assert all(objs[i] is None for i in idx_bad)
    ref_objs = snapshot.chunkify_batch(good)
    for p, r in zip(paths, ref_objs):
        o = objs[order.index(p)]
        assert o.Checksum == r.Checksum and [c.Checksum for c in o.Chunks] == [c.Checksum for c in r.Chunks]
    assert st["failed_files"] == len(bad) and st["files"] == len(order)
    assert st["bytes"] == sum(len(b) for b in good)
    assert set(_blobs_of(packs, KEY, True)) == {c.Checksum for o in objs if o for c in o.Chunks}


def test_backup_files_larger_than_the_batch_go_in_pieces(tmp_path):
    """Files many times batch_bytes are processed piece by piece, each piece
    chunked from the previous one's carried chunk start: the same cut points,
    digests, entropies and object checksum as the whole-file path, while the
    per-slot arena stays within batch_bytes + Max (not the largest file)."""
    files = [random_bytes(70 << 20, 41).tobytes(), random_bytes(1 << 20, 42).tobytes(),
             low_entropy(40 << 20, 43).tobytes(), random_bytes(33 << 20, 44).tobytes()]
    paths = []
    for i, b in enumerate(files):
        p = tmp_path / f"big{i}"
        p.write_bytes(b)
        paths.append(str(p))
    objs, packs, st = snapshot.backup_files(paths, key=KEY, batch_bytes=8 << 20, packers=3)
    ref_objs = snapshot.chunkify_batch(files)
    for i, (o, r) in enumerate(zip(objs, ref_objs)):
        assert o.Checksum == r.Checksum == hashlib.sha256(files[i]).digest(), f"file {i}"
        assert [c.Length for c in o.Chunks] == [c.Length for c in r.Chunks], f"file {i}"
        assert [c.Checksum for c in o.Chunks] == [c.Checksum for c in r.Chunks], f"file {i}"
        assert [c.Entropy for c in o.Chunks] == [c.Entropy for c in r.Chunks], f"file {i}"
        assert o.Entropy == r.Entropy, f"file {i}"
    piece = max(8 << 20, 4 * (4 << 20))  # cdc_backup: pieces of max(batch_bytes, 4 Max)
    assert st["pieces"] == sum(max(1, -(-len(b) // piece)) if len(b) > piece else 1 for b in files)
    assert st["slot_arena_bytes"] <= piece + (4 << 20)
    assert st["bytes"] == sum(len(b) for b in files) and st["failed_files"] == 0
    assert set(_blobs_of(packs, KEY, True)) == {c.Checksum for o in objs for c in o.Chunks}


def test_backup_pieces_of_large_files_go_round_by_round(tmp_path):
    """Every file's first piece comes first (largest file first), then the
    later pieces round by round, so the object hashes of several large files
    (one serial chain each) run side by side; a file's pieces still arrive in
    order and the objects equal the whole-file path's."""
    sizes = [50 << 20, 40 << 20, 3 << 20, 35 << 20]
    files = [random_bytes(n, 61 + i).tobytes() for i, n in enumerate(sizes)]
    paths = []
    for i, b in enumerate(files):
        p = tmp_path / f"r{i}"
        p.write_bytes(b)
        paths.append(str(p))
    with snapshot.BackupSession(key=KEY, batch_bytes=8 << 20, packers=2) as s:
        objs, _, st = s.run(paths)
        order = list(s.callback_order)
    piece = 4 * (4 << 20)  # max(batch_bytes, 4 Max)
    npieces = [-(-n // piece) if n > piece else 1 for n in sizes]
    assert sorted(order) == sorted((i, j) for i, k in enumerate(npieces) for j in range(k))
    assert [i for i, j in order if j == 0] == [0, 1, 3, 2]  # round 0, largest first
    rounds = [j for _, j in order]
    assert rounds == sorted(rounds)  # round by round
    for i in range(len(files)):
        assert [j for f, j in order if f == i] == list(range(npieces[i]))
    ref = snapshot.chunkify_batch(files)
    for o, r, b in zip(objs, ref, files):
        assert o.Checksum == r.Checksum == hashlib.sha256(b).digest()
        assert [c.Checksum for c in o.Chunks] == [c.Checksum for c in r.Chunks]
    assert st["failed_files"] == 0


def test_backup_large_file_failing_in_a_middle_piece(tmp_path, monkeypatch):
    """A file in pieces whose third piece cannot be read (the library's test
    hook CDC_BACKUP_FAIL_PIECE=file:piece, as a file that shrank mid-run):
    that file fails (status CDC_E_IO, no object), failed_files is 1, and the
    other files -- a large one read in pieces beside it included -- are backed
    up intact.  The failing file's later pieces are read ahead of its device
    work (piece reads no longer wait for the previous piece's cut list)."""
    files = [random_bytes(70 << 20, 51).tobytes(), random_bytes(1 << 20, 52).tobytes(),
             random_bytes(40 << 20, 53).tobytes()]
    paths = []
    for i, b in enumerate(files):
        p = tmp_path / f"m{i}"
        p.write_bytes(b)
        paths.append(str(p))
    monkeypatch.setenv("CDC_BACKUP_FAIL_PIECE", "0:2")
    with snapshot.BackupSession(key=KEY, batch_bytes=8 << 20, packers=2) as s:
        objs, packs, st = s.run(paths)
        failed = dict(s.failed)
    assert failed == {0: _lib.CDC_E_IO} and objs[0] is None
    assert st["failed_files"] == 1 and st["files"] == len(files)
    ref_objs = snapshot.chunkify_batch(files[1:])
    for o, r, b in zip(objs[1:], ref_objs, files[1:]):
        assert o.Checksum == r.Checksum == hashlib.sha256(b).digest()
        assert [c.Checksum for c in o.Chunks] == [c.Checksum for c in r.Chunks]
    stored = set(_blobs_of(packs, KEY, True))
    assert {c.Checksum for o in objs[1:] for c in o.Chunks} <= stored


def test_backup_device_failure_in_a_middle_piece(tmp_path, monkeypatch):
    """A large file whose third piece's launch group aborts on the device (the
    hook CDC_BACKUP_FAIL_DEVICE=file:piece runs that launch in debug mode 2:
    a bounded wait gives up, every result row reports CDC_E_DEVICE).  The
    backup returns CDC_E_DEVICE -- the reference aborts a backup on a chunker
    error (snapshot/backup.go:98-101) -- instead of publishing a stale carry
    to the next piece's reader; the same session then backs up the same files
    intact."""
    files = [random_bytes(70 << 20, 54).tobytes(), random_bytes(1 << 20, 55).tobytes(),
             random_bytes(40 << 20, 56).tobytes()]
    paths = []
    for i, b in enumerate(files):
        p = tmp_path / f"d{i}"
        p.write_bytes(b)
        paths.append(str(p))
    with snapshot.BackupSession(key=KEY, batch_bytes=8 << 20, packers=2) as s:
        monkeypatch.setenv("CDC_BACKUP_FAIL_DEVICE", "0:2")
        with pytest.raises(_lib.CdcError) as e:
            s.run(paths)
        assert e.value.status == _lib.CDC_E_DEVICE
        monkeypatch.delenv("CDC_BACKUP_FAIL_DEVICE")
        objs, packs, st = s.run(paths)
    assert st["failed_files"] == 0
    ref_objs = snapshot.chunkify_batch(files)
    for o, r, b in zip(objs, ref_objs, files):
        assert o.Checksum == r.Checksum == hashlib.sha256(b).digest()
        assert [c.Checksum for c in o.Chunks] == [c.Checksum for c in r.Chunks]


def test_backup_stats_report_the_hardware_queues():
    """cdc_backup_new records GPU_MAX_HW_QUEUES (0: unset, HIP's default of 4)
    and whether the pipeline's streams share hardware queues."""
    import os
    _, _, st = snapshot.backup_files([])
    q = int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)
    assert st["hw_queues"] == q and st["streams_serialised"] == (1 if q < 8 else 0)


def test_backup_session_reused_across_runs(corpus, tmp_path):
    """One context, several backups: each run is a fresh backup (its own
    dedup set), buffers grow when a later run needs more."""
    paths, files = corpus
    big = tmp_path / "big"
    big.write_bytes(random_bytes(40 << 20, 123).tobytes())
    with snapshot.BackupSession(key=KEY, batch_bytes=8 << 20, packers=2) as s:
        o1, p1, s1 = s.run(paths[:6])
        o2, p2, s2 = s.run(paths + [str(big)])
        o3, p3, s3 = s.run(paths[:6])
    assert [o.Checksum for o in o1] == [o.Checksum for o in o3]
    assert s1["new_blobs"] == s3["new_blobs"] > 0
    assert o2[-1].Checksum == hashlib.sha256(big.read_bytes()).digest()
    assert set(_blobs_of(p3, KEY, True)) == {c.Checksum for o in o3 for c in o.Chunks}


def test_backup_content_type_sees_each_files_first_chunk(corpus, tmp_path):
    """Object.ContentType: chunkify takes mime.TypeByExtension, else
    mimetype.Detect of the first chunk (snapshot/backup.go:580, 598-601).
    cdc_backup_file carries the piece's bytes for that; the callback gets
    exactly the file's first chunk, also for a file that goes in pieces."""
    paths, files = corpus
    big = tmp_path / "big.bin"
    big.write_bytes(random_bytes(20 << 20, 321).tobytes())
    allp, allf = paths + [str(big)], files + [big.read_bytes()]
    seen = {}

    def sniff(path, first):
        seen[path] = first
        return "application/x-test-%d" % len(first)

    with snapshot.BackupSession(key=KEY, batch_bytes=8 << 20, packers=2) as s:
        objs, _, _ = s.run(allp, content_type=sniff)
    for p, b, o in zip(allp, allf, objs):
        n = o.Chunks[0].Length
        assert seen[p] == b[:n], p
        assert o.ContentType == "application/x-test-%d" % n


def test_backup_many_small_files_rotate_every_slot(tmp_path):
    """Thousands of files over many more batches than the pipeline has slots
    (each slot is claimed, released and claimed again many times; reads run
    ahead of the object hashes): every object and chunk as chunkify gives
    them, every blob packed once."""
    rng = np.random.default_rng(77)
    sizes = rng.integers(0, 48 << 10, size=2500)
    files, paths = [], []
    for i, n in enumerate(sizes):
        b = random_bytes(int(n), 5000 + i).tobytes() if i % 7 else b"dup-%d" % (i % 3)
        p = tmp_path / f"s{i:05d}"
        p.write_bytes(b)
        files.append(b)
        paths.append(str(p))
    objs, packs, st = snapshot.backup_files(paths, key=KEY, compression="LZ4", packers=4, readers=8,
                                            batch_bytes=1 << 20)
    assert st["batches"] > 20 and st["files"] == len(files)
    for i, (o, b) in enumerate(zip(objs, files)):
        assert o.Checksum == hashlib.sha256(b).digest(), i
        assert sum(c.Length for c in o.Chunks) == len(b), i
    want = {c.Checksum for o in objs for c in o.Chunks}
    assert set(_blobs_of(packs, KEY, True)) == want and st["new_blobs"] == len(want)


@pytest.mark.parametrize("seed", range(int(__import__("os").environ.get("BACKUP_FUZZ_CASES", "8"))))
def test_backup_random_corpora(tmp_path, seed):
    """Random corpora through the whole pipeline: 1-40 files of 0 B-24 MiB
    (duplicates and shared prefixes among them), random chunking sizes, batch
    sizes that cut large files into pieces, reader / packer counts, packfile
    sizes and encodings.  Objects equal the batch path's (chunkify_batch: cut
    points vs the oracle, digests vs hashlib); every stored blob decodes to its
    chunk's bytes, once."""
    from plakar_amd.chunking import Configuration
    from plakar_amd.repository import Repository
    rng = np.random.default_rng(np.random.PCG64(9500 + seed))
    mn = 4096 << int(rng.integers(0, 5))
    cfg = Configuration("FASTCDC", mn, mn << int(rng.integers(1, 4)), 0)
    cfg.MaxSize = cfg.NormalSize << int(rng.integers(1, 3))
    repo = Repository(cfg)
    files = []
    for i in range(int(rng.integers(1, 41))):
        r = rng.random()
        if files and r < 0.1:
            files.append(files[int(rng.integers(0, len(files)))])  # a duplicate
        elif files and r < 0.2:
            f = files[int(rng.integers(0, len(files)))]
            files.append(f[:len(f) // 2] + random_bytes(int(rng.integers(1, 1 << 20)), 9600 + 64 * seed + i).tobytes())
        else:
            n = 0 if r < 0.25 else int(np.exp(rng.uniform(0, np.log(24 << 20))))
            gen = random_bytes if rng.random() < 0.7 else (lambda k, s: low_entropy(k, s, 0.01))
            files.append(gen(n, 9700 + 64 * seed + i).tobytes())
    paths = []
    for i, b in enumerate(files):
        p = tmp_path / f"f{i:02d}"
        p.write_bytes(b)
        paths.append(str(p))
    key, compression = [(KEY, "LZ4"), (None, None), (None, "LZ4"), (KEY, None)][seed % 4]
    batch = int(rng.choice([4 << 20, 8 << 20, 32 << 20]))
    objs, packs, st = snapshot.backup_files(paths, repo=repo, key=key, compression=compression,
                                            max_size=int(rng.choice([1 << 20, 4 << 20, 20 << 20])),
                                            packers=int(rng.integers(1, 5)), readers=int(rng.integers(1, 9)),
                                            batch_bytes=batch, timestamp=seed)
    what = f"seed {seed}: {cfg} batch {batch} sizes {[len(f) for f in files]}"
    ref_objs = snapshot.chunkify_batch(files, repo=repo)
    assert len(objs) == len(files), what
    want = {}
    for i, (o, r) in enumerate(zip(objs, ref_objs)):
        assert o.Checksum == r.Checksum == hashlib.sha256(files[i]).digest(), f"{what}: file {i}"
        assert [c.Length for c in o.Chunks] == [c.Length for c in r.Chunks], f"{what}: file {i}"
        assert [c.Checksum for c in o.Chunks] == [c.Checksum for c in r.Chunks], f"{what}: file {i}"
        off = 0
        for c in o.Chunks:
            want[c.Checksum] = files[i][off:off + c.Length]
            off += c.Length
    blobs = _blobs_of(packs, key, compression == "LZ4")
    assert set(blobs) == set(want), what
    for c, plain in blobs.items():
        assert plain == want[c], what
    assert st["bytes"] == sum(len(f) for f in files) and st["new_blobs"] == len(want), what
