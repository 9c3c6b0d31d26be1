"""Seeded mutation corpora shared by the CPU acceptance test (tests/test_oracle_vs_stock.py:
the oracle's decoders against zlib / liblz4 / libzstd) and the GPU mutation tests
(tests/test_gpu_mutations.py: the GPU decoders against the oracle).  Test infrastructure
only; no GPU and no torch here."""
import ctypes
import zlib

import numpy as np

import oracle_lib as O

SEG = 65536


def mutations(frame, rng, count, hot=None):
    """count seeded mutations of frame: bit flips, byte sets, truncations, and bit flips in
    `hot` = (lo, hi), the byte range that holds the structure under test (block / table
    headers, the sequence bitstream)."""
    out = []
    for _ in range(count):
        b = bytearray(frame)
        kind = int(rng.integers(0, 5))
        if kind == 0:  # bit flip anywhere
            i = int(rng.integers(0, len(b)))
            b[i] ^= 1 << int(rng.integers(0, 8))
        elif kind == 1:  # byte set
            i = int(rng.integers(0, len(b)))
            b[i] = int(rng.integers(0, 256))
        elif kind == 2:  # truncation
            b = b[:int(rng.integers(0, len(b)))]
        else:  # one or two bit flips in the hot range
            lo, hi = hot if hot else (0, len(b))
            hi = max(lo + 1, min(hi, len(b)))
            for _ in range(1 + (kind == 4)):
                i = int(rng.integers(lo, hi))
                b[i] ^= 1 << int(rng.integers(0, 8))
        out.append(bytes(b) if b else b"\x00")
    return out


def libzstd():
    try:
        L = ctypes.CDLL("/opt/conda/lib/libzstd.so.1.4.9")
    except OSError:
        return None
    L.ZSTD_compress.restype = ctypes.c_size_t
    L.ZSTD_compress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                ctypes.c_size_t, ctypes.c_int]
    L.ZSTD_decompress.restype = ctypes.c_size_t
    L.ZSTD_decompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                  ctypes.c_size_t]
    L.ZSTD_isError.restype = ctypes.c_uint
    L.ZSTD_isError.argtypes = [ctypes.c_size_t]
    return L


def liblz4():
    for name in ("liblz4.so.1", "/opt/conda/lib/liblz4.so.1"):
        try:
            L = ctypes.CDLL(name)
        except OSError:
            continue
        L.LZ4_compress_default.restype = ctypes.c_int
        L.LZ4_compress_default.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                           ctypes.c_int]
        L.LZ4_decompress_safe.restype = ctypes.c_int
        L.LZ4_decompress_safe.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                          ctypes.c_int]
        return L
    return None


def dynamic_sources():
    """(stream, plain): our dynamic-Huffman DEFLATE encoder's and zlib level 1's"""
    srcs = []
    for kind, n, seed in ((1, 59460, 11), (2, 59460, 12), (6, 40000, 13), (5, 30000, 14),
                          (1, 20000, 15)):
        plain = O.fill(kind, seed, n).tobytes()
        r, ours = O.deflate_dynamic(plain)  # == deflate_dyn_*_kernel's stream (bit-exact)
        assert r == 0 and O.deflate_dynamic_mode(plain) == 2  # a dynamic block
        z = zlib.compressobj(1, zlib.DEFLATED, -15, 8, zlib.Z_DEFAULT_STRATEGY)
        stock = z.compress(plain) + z.flush()  # zlib level 1: the reference's frame
        srcs += [(ours, plain), (stock, plain)]
    return srcs


def fixed_sources():
    """fixed-Huffman / stored streams: ours and zlib's Z_FIXED"""
    srcs = []
    for kind, n, seed in ((1, 59460, 21), (6, 30000, 22), (0, 20000, 23)):
        plain = O.fill(kind, seed, n).tobytes()
        r, fixed = O.deflate_fixed(plain)
        assert r == 0
        z = zlib.compressobj(1, zlib.DEFLATED, -15, 8, zlib.Z_FIXED)
        srcs += [(fixed, plain), (z.compress(plain) + z.flush(), plain)]
    return srcs


def zstd_sources():
    """(frame, plain): our level-1-class frames and libzstd level 1's (no checksum)"""
    srcs = []
    Z = libzstd()
    for kind, n, seed in ((2, 65536, 31), (1, 65536, 32), (5, 65536, 33), (6, 50000, 34),
                          (2, 30000, 35)):
        plain = O.fill(kind, seed, n).tobytes()
        r, ours = O.zstd_compress(plain)  # == the GPU encoder's frame (bit-exact)
        assert r == 0
        srcs.append((ours, plain))
        if Z is not None:
            buf = ctypes.create_string_buffer(n + 1024)
            r = Z.ZSTD_compress(buf, n + 1024, plain, n, 1)
            assert not Z.ZSTD_isError(r)
            srcs.append((buf.raw[:r], plain))
    # a literal-heavy record-batch column: our 8-block frame (>= 32 KiB of literals)
    plain = O.fill(2, 1000, 17 * 65536)[16 * 65536:].tobytes()
    r, ours = O.zstd_compress(plain)
    assert r == 0
    srcs.append((ours, plain))
    return srcs


def lz4_far_sources():
    """LZ4 blocks whose matches reach past the GPU decoder's ring: the wide parse's and
    liblz4's"""
    bases = []
    for kind, n, seed in ((1, 65536, 41), (2, 65536, 42), (5, 65536, 43), (6, 40000, 44)):
        plain = O.fill(kind, seed, n).tobytes()
        r, wide = O.lz4_wide_compress(plain)
        assert r == 0
        bases.append((wide, plain))
    L = liblz4()
    if L is not None:
        for kind, n, seed in ((1, 65536, 45), (5, 65536, 46)):
            plain = O.fill(kind, seed, n).tobytes()
            buf = ctypes.create_string_buffer(n + n // 255 + 16)
            r = L.LZ4_compress_default(plain, buf, n, len(buf))
            assert r > 0
            bases.append((buf.raw[:r], plain))
    return bases


def fcs_flip(frame):
    """frame with the low bit of its Frame_Content_Size flipped (RFC 8878 3.1.1.1)"""
    fhd = frame[4]
    single, did = (fhd >> 5) & 1, fhd & 3
    at = 5 + (0 if single else 1) + (0, 1, 2, 4)[did]
    assert single or fhd >> 6, "frame without a content size"
    b = bytearray(frame)
    b[at] ^= 1
    return bytes(b)


# the corpora of the GPU mutation tests (same seeds, same order)
def inflate_dynamic_cases():
    rng = np.random.default_rng(1951)
    cases = []
    for stream, _ in dynamic_sources():
        cases += mutations(stream, rng, 48, hot=(0, 80))
    return cases


def inflate_fixed_cases():
    rng = np.random.default_rng(1952)
    cases = []
    srcs = fixed_sources()
    for k in range(0, len(srcs), 2):
        cases += mutations(srcs[k][0], rng, 32, hot=(0, 64))
        cases += mutations(srcs[k + 1][0], rng, 32, hot=(0, 64))
    return cases


def zstd_cases():
    rng = np.random.default_rng(8878)
    srcs = zstd_sources()
    cases = []
    for frame, _ in srcs:
        cases += mutations(frame, rng, 48, hot=(2 * len(frame) // 3, len(frame)))
    cases += [fcs_flip(frame) for frame, _ in srcs]
    return cases


def lz4_far_cases():
    rng = np.random.default_rng(1977)
    cases = []
    for b, _ in lz4_far_sources():
        cases += mutations(b, rng, 40, hot=(len(b) // 2, len(b)))
    return cases


def lz4_near_sources():
    """our fast parse's LZ4 blocks (every match inside the decoder's LDS ring)"""
    out = []
    for kind, n, seed in ((1, 65536, 51), (2, 65536, 52), (5, 65536, 53), (6, 40000, 54)):
        plain = O.fill(kind, seed, n).tobytes()
        r, blk = O.lz4_compress(plain)
        assert r == 0
        out.append((blk, plain))
    return out


def lz4_near_cases():
    """mutations of our own LZ4 blocks aimed at their last 64 bytes (end-of-block conditions,
    the batch -> general path hand-over) and anywhere"""
    rng = np.random.default_rng(1978)
    cases = []
    for b, _ in lz4_near_sources():
        cases += mutations(b, rng, 40, hot=(len(b) - 64, len(b)))
        cases += mutations(b, rng, 20)
    return cases


def lz4_block(seqs, final):
    """an LZ4 block from (literals, offset, match length) sequences and the final literals"""
    out = bytearray()

    def ext(v):
        while v >= 255:
            out.append(255)
            v -= 255
        out.append(v)
    for lits, off, ml in list(seqs) + [(final, 0, 0)]:
        ll, m = len(lits), ml - 4 if ml else 0
        out.append((min(ll, 15) << 4) | (min(m, 15) if ml else 0))
        if ll >= 15:
            ext(ll - 15)
        out += lits
        if not ml:
            break
        out += bytes([off & 255, off >> 8])
        if m >= 15:
            ext(m - 15)
    return bytes(out)


def lz4_end_rule_cases():
    """blocks around the end-of-block conditions: k short batchable sequences (3 literals +
    a 4..8-byte match at offset 7), then the last match of length `ml` and `fl` final
    literals; the last match of some of them is decoded inside a batch on the GPU"""
    rng = np.random.default_rng(1979)
    cases = []
    for k in (0, 1, 5, 30, 31, 32, 33, 60, 61, 62, 63, 64, 65, 100, 200, 333):
        for ml in (4, 5, 6, 7, 8, 12, 19, 40):
            for fl in (0, 1, 4, 5, 6, 7, 8, 11, 12, 20):
                seqs = [(bytes(rng.integers(0, 256, 3).astype(np.uint8)), 7,
                         4 + int(rng.integers(0, 5))) for _ in range(k)]
                seqs.insert(0, (bytes(rng.integers(0, 256, 16).astype(np.uint8)), 0, 0))
                first = seqs.pop(0)[0]
                seqs = [(first + seqs[0][0], seqs[0][1], seqs[0][2])] + seqs[1:] if seqs else []
                lits = bytes(rng.integers(0, 256, 9).astype(np.uint8))
                if not seqs:
                    lits = first + lits
                seqs.append((lits, 5, ml))
                cases.append(lz4_block(seqs, bytes(rng.integers(0, 256, fl).astype(np.uint8))))
    return cases
