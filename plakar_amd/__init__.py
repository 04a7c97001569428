"""plakar_amd: MI355X-native content-defined chunker for plakar.

Drop-in for plakar's chunking path (chunking/ + the go-cdc-chunkers FastCDC
chunker it configures): HIP kernels for gfx950 behind the C ABI in
include/plakar_cdc.h (libplakar_cdc.so), with Python mirrors of the Go API:

    plakar_amd.chunking    Configuration / DefaultConfiguration
    plakar_amd.chunkers    ChunkerOpts / NewChunker / Chunker.Next / ChunkBuffers
    plakar_amd.repository  Repository.Chunker / chunkify routing
    plakar_amd.device      device-resident batches (torch tensors in HBM)
"""
from . import chunking  # noqa: F401

__all__ = ["chunking", "chunkers", "repository", "device", "build"]
