"""Mirror of plakar's chunking/ package (chunking/chunking.go:3-17).

The configuration contract of the drop-in: plakar persists it in the
repository CONFIG (storage/storage.go:48, 61) and feeds it to the chunker
factory (repository/repository.go:283-294).
"""
from dataclasses import dataclass


@dataclass
class Configuration:
    """chunking.Configuration (chunking/chunking.go:3-8)."""
    Algorithm: str   # content-defined chunking algorithm ("FASTCDC")
    MinSize: int     # uint32, minimum chunk size
    NormalSize: int  # uint32, expected (average) chunk size
    MaxSize: int     # uint32, maximum chunk size


def DefaultConfiguration() -> Configuration:
    """chunking.DefaultConfiguration() (chunking/chunking.go:10-17)."""
    return Configuration(Algorithm="FASTCDC", MinSize=64 * 1024, NormalSize=1 * 1024 * 1024,
                         MaxSize=4 * 1024 * 1024)
