"""Test infrastructure: independent checkers for the device Encode, from the
system's libraries (OpenSSL libcrypto for AES-256-GCM, liblz4 for LZ4 frames)
through ctypes, plus the reference's decode logic restated in Python:
encryption.DecryptStream (encryption/symmetric.go:165-240) and the LZ4 frame
reader behind compression.InflateStream (compression/compression.go)."""
import ctypes
import ctypes.util

_crypto = None
_lz4 = None


def crypto():
    global _crypto
    if _crypto is None:
        name = ctypes.util.find_library("crypto") or "libcrypto.so.3"
        L = ctypes.CDLL(name)
        L.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
        L.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
        L.EVP_aes_256_gcm.restype = ctypes.c_void_p
        for f in ("EVP_EncryptInit_ex", "EVP_DecryptInit_ex"):
            getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p,
                                      ctypes.c_char_p]
        for f in ("EVP_EncryptUpdate", "EVP_DecryptUpdate"):
            getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                      ctypes.c_char_p, ctypes.c_int]
        for f in ("EVP_EncryptFinal_ex", "EVP_DecryptFinal_ex"):
            getattr(L, f).argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.EVP_CIPHER_CTX_ctrl.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        _crypto = L
    return _crypto


EVP_CTRL_GCM_SET_IVLEN, EVP_CTRL_GCM_GET_TAG, EVP_CTRL_GCM_SET_TAG = 0x9, 0x10, 0x11


def gcm_seal(key, nonce, pt):
    """AES-256-GCM Seal (Go's cipher.AEAD.Seal: ciphertext || 16-byte tag)."""
    L = crypto()
    ctx = L.EVP_CIPHER_CTX_new()
    try:
        assert L.EVP_EncryptInit_ex(ctx, L.EVP_aes_256_gcm(), None, None, None) == 1
        assert L.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_GCM_SET_IVLEN, len(nonce), None) == 1
        assert L.EVP_EncryptInit_ex(ctx, None, None, bytes(key), bytes(nonce)) == 1
        out = ctypes.create_string_buffer(len(pt) + 16)
        n = ctypes.c_int()
        if pt:
            assert L.EVP_EncryptUpdate(ctx, ctypes.addressof(out), ctypes.byref(n), bytes(pt), len(pt)) == 1
        m = ctypes.c_int()
        assert L.EVP_EncryptFinal_ex(ctx, ctypes.addressof(out) + n.value, ctypes.byref(m)) == 1
        tag = ctypes.create_string_buffer(16)
        assert L.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_GCM_GET_TAG, 16, tag) == 1
        return out.raw[:len(pt)] + tag.raw
    finally:
        L.EVP_CIPHER_CTX_free(ctx)


def gcm_open(key, nonce, ct_tag):
    """AES-256-GCM Open; raises ValueError when the tag does not verify."""
    L = crypto()
    ct, tag = bytes(ct_tag[:-16]), bytes(ct_tag[-16:])
    ctx = L.EVP_CIPHER_CTX_new()
    try:
        assert L.EVP_DecryptInit_ex(ctx, L.EVP_aes_256_gcm(), None, None, None) == 1
        assert L.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_GCM_SET_IVLEN, len(nonce), None) == 1
        assert L.EVP_DecryptInit_ex(ctx, None, None, bytes(key), bytes(nonce)) == 1
        out = ctypes.create_string_buffer(max(len(ct), 1))
        n = ctypes.c_int()
        if ct:
            assert L.EVP_DecryptUpdate(ctx, ctypes.addressof(out), ctypes.byref(n), ct, len(ct)) == 1
        tb = ctypes.create_string_buffer(tag, 16)
        assert L.EVP_CIPHER_CTX_ctrl(ctx, EVP_CTRL_GCM_SET_TAG, 16, tb) == 1
        m = ctypes.c_int()
        if L.EVP_DecryptFinal_ex(ctx, ctypes.addressof(out) + n.value, ctypes.byref(m)) != 1:
            raise ValueError("GCM tag mismatch")
        return out.raw[:len(ct)]
    finally:
        L.EVP_CIPHER_CTX_free(ctx)


def lz4():
    global _lz4
    if _lz4 is None:
        name = ctypes.util.find_library("lz4") or "liblz4.so.1"
        L = ctypes.CDLL(name)
        L.LZ4F_createDecompressionContext.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
        L.LZ4F_freeDecompressionContext.argtypes = [ctypes.c_void_p]
        L.LZ4F_decompress.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                                      ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p]
        L.LZ4F_decompress.restype = ctypes.c_size_t
        L.LZ4F_isError.argtypes = [ctypes.c_size_t]
        L.LZ4F_getErrorName.argtypes = [ctypes.c_size_t]
        L.LZ4F_getErrorName.restype = ctypes.c_char_p
        _lz4 = L
    return _lz4


def lz4f_decompress(frame, limit=1 << 31):
    """Decode one LZ4 frame with liblz4 (checks block sizes and the content
    checksum); returns the content."""
    L = lz4()
    ctx = ctypes.c_void_p()
    assert L.LZ4F_createDecompressionContext(ctypes.byref(ctx), 100) == 0
    try:
        src = ctypes.create_string_buffer(bytes(frame), len(frame))
        pos, out = 0, bytearray()
        buf = ctypes.create_string_buffer(1 << 22)
        while True:
            dst_n = ctypes.c_size_t(len(buf))
            src_n = ctypes.c_size_t(len(frame) - pos)
            r = L.LZ4F_decompress(ctx, ctypes.addressof(buf), ctypes.byref(dst_n), ctypes.addressof(src) + pos,
                                  ctypes.byref(src_n), None)
            if L.LZ4F_isError(r):
                raise ValueError("LZ4F: " + L.LZ4F_getErrorName(r).decode())
            out += buf.raw[:dst_n.value]
            pos += src_n.value
            if r == 0:
                break
            if src_n.value == 0 and dst_n.value == 0:
                raise ValueError("LZ4F: truncated frame")
            if len(out) > limit:
                raise ValueError("LZ4F: output too large")
        if pos != len(frame):
            raise ValueError(f"LZ4F: {len(frame) - pos} trailing bytes")
        return bytes(out)
    finally:
        L.LZ4F_freeDecompressionContext(ctx)


def decrypt_stream(key, data):
    """encryption.DecryptStream: the subkey header, then nonce || sealed piece
    records of at most 64 KiB + 16 bytes each."""
    nonce, enc_sub = data[:12], data[12:60]
    sub = gcm_open(key, nonce, enc_sub)
    pos, out = 60, bytearray()
    while pos < len(data):
        dn = data[pos:pos + 12]
        rec = data[pos + 12:pos + 12 + 65536 + 16]
        out += gcm_open(sub, dn, rec)
        pos += 12 + len(rec)
    return bytes(out), sub, nonce


def decode(data, key=None, compressed=True):
    """(*Repository).Decode of one blob: decrypt, then inflate."""
    if key is not None:
        data, _, _ = decrypt_stream(key, data)
    if compressed and len(data) == 0:  # InflateStream of empty input (compression/compression.go InflateStream)
        return b""
    return lz4f_decompress(data) if compressed else data
