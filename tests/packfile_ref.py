"""CPU restatement of plakar's packfile format and packer (TEST INFRASTRUCTURE:
the checker for libplakar_cdc.so's cdc_packer_*).  Pure Python over struct and
hashlib, following the reference line by line:

  packfile/packfile.go:140-150  New (Version 100, Timestamp, Count 0)
  packfile/packfile.go:389-394  AddBlob (Offset = len(Blobs), Count++, IndexOffset)
  packfile/packfile.go:241-294  Serialize (Blobs, index entries, footer)
  packfile/packfile.go:152-239  NewFromBytes (footer at -52, index checksum check)
  snapshot/packer.go:21-31      Packer.AddBlob / Size
  snapshot/snapshot.go:232-267  PutPackfile layout
"""
import hashlib
import struct

VERSION = 100
TYPE_CHUNK = 1


class PackFile:
    def __init__(self, timestamp=0):
        self.blobs = bytearray()
        self.index = []  # (type, checksum, offset, length)
        self.version, self.timestamp, self.count, self.index_offset = VERSION, timestamp, 0, 0
        self.index_checksum = b"\0" * 32

    def add_blob(self, typ, checksum, data):
        self.index.append((typ, bytes(checksum), len(self.blobs), len(data)))
        self.blobs += bytes(data)
        self.count += 1
        self.index_offset = len(self.blobs)

    def size(self):
        return len(self.blobs)

    def serialize_index(self):
        return b"".join(struct.pack("<B32sII", t, c, o, n) for t, c, o, n in self.index)

    def serialize_footer(self):
        idx = self.serialize_index()
        self.index_checksum = hashlib.sha256(idx).digest()
        return struct.pack("<IqII32s", self.version, self.timestamp, self.count, self.index_offset,
                           self.index_checksum)

    def serialize(self):
        idx = self.serialize_index()
        return bytes(self.blobs) + idx + self.serialize_footer()


def parse(serialized):
    """NewFromBytes: footer from the last 52 bytes, data up to IndexOffset, index entries after it,
    their SHA-256 checked against the footer."""
    version, ts, count, index_offset, csum = struct.unpack("<IqII32s", serialized[-52:])
    p = PackFile(ts)
    p.version, p.count, p.index_offset, p.index_checksum = version, count, index_offset, csum
    p.blobs = bytearray(serialized[:index_offset])
    raw = serialized[index_offset:-52]
    assert len(raw) % 41 == 0, "index entries are 41 bytes"
    for k in range(0, len(raw), 41):
        t, c, o, n = struct.unpack("<B32sII", raw[k:k + 41])
        if o + n > index_offset:
            raise ValueError("chunk offset + chunk length exceeds total length of packfile")
        p.index.append((t, c, o, n))
    if hashlib.sha256(raw).digest() != csum:
        raise ValueError("index checksum mismatch")
    return p


def put_packfile_layout(p, encode=lambda b: b):
    """snapshot/snapshot.go:259-267: data, Encode(index), Encode(footer), version u32, u8 len(Encode(footer))."""
    data = bytes(p.blobs)
    ei = encode(p.serialize_index())
    ef = encode(p.serialize_footer())
    return data + ei + ef + struct.pack("<I", p.version) + bytes([len(ef) & 0xFF])
