"""Mirror of the plakar call sites around the chunker.

    (*Repository).Chunker(rd)   repository/repository.go:283-294
    chunkify routing            snapshot/backup.go:631-666

Only the parts on the chunking path: the repository's Chunking configuration
drives the chunker exactly as the Go code does (algorithm name lower-cased,
sizes widened to int).
"""
from . import chunkers
from .chunking import Configuration, DefaultConfiguration


class Repository:
    def __init__(self, chunking: Configuration = None):
        self._chunking = chunking or DefaultConfiguration()

    def Configuration(self):
        return self

    @property
    def Chunking(self):
        return self._chunking

    def Chunker(self, rd):
        """repository/repository.go:283-294."""
        c = self._chunking
        return chunkers.NewChunker(c.Algorithm.lower(), rd, chunkers.ChunkerOpts(
            MinSize=int(c.MinSize), NormalSize=int(c.NormalSize), MaxSize=int(c.MaxSize)))


def chunkify_lengths(repo: Repository, size: int, rd):
    """snapshot/backup.go:631-666: the chunk lengths plakar records for a file of
    `size` bytes read from `rd` (empty file -> one empty chunk; smaller than
    MinSize -> the whole file as one chunk, no CDC; otherwise the chunker)."""
    if size == 0:
        return [0]
    if size < repo.Chunking.MinSize:
        return [len(rd.read())]
    lens = []
    chk = repo.Chunker(rd)
    try:
        while True:
            chunk, err = chk.Next()
            if chunk is None:
                break
            lens.append(len(chunk))
            if err is chunkers.EOF:
                break
    finally:
        chk.close()
    return lens
