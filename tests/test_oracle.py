"""CPU tests: pin the oracle against the golden vectors and the reference's rules.

These run without a GPU (-m "not gpu").  The oracle is the checker for the HIP path, so it
is pinned first: its decoders must reproduce every third-party golden vector, its encoders
must produce streams the third-party decoders accept, and its segment-level rules must
match the reference's device.cc / config.cc behaviour.
"""
import ctypes
import hashlib
import zlib

import numpy as np
import pytest

import golden_lib
import oracle_lib as O


# --- Configuration::UpdateCompressedSegSize (reference src/config.cc:59-73) ------------
# Expected values worked by hand from the reference's integer loop (highest set bit of
# 2*seg; above 32 KiB the slot is (uint16)(seg*1.1)); 59460 -> 65406 is the demo's slot
# (apps/app_common.h:39).
@pytest.mark.parametrize("seg,slot", [(8, 16), (2048, 4096), (4096, 8192), (16384, 32768),
                                      (17000, 32768), (20000, 32768), (32768, 36044),
                                      (59460, 65406), (1000, 1024), (1025, 2048)])
def test_slot_size_rule(seg, slot):
    assert O.compressed_seg_size(seg) == slot


def test_generator_is_pinned():
    m = golden_lib.manifest()
    for key, inp in m["inputs"].items():
        data = O.fill(inp["kind"], inp["seed"], inp["n"]).tobytes()
        assert hashlib.sha256(data).hexdigest() == inp["sha256"], key


def test_oracle_lz4_decodes_all_golden():
    n = 0
    for e, blob, plain in golden_lib.vectors("lz4"):
        r, out = O.lz4_decompress(blob, max(len(plain), 1))
        assert r == 0, (e["producer"], e["input"])
        assert out == plain, (e["producer"], e["input"])
        n += 1
    assert n >= 100


def test_oracle_inflate_decodes_all_golden():
    n = 0
    for e, blob, plain in golden_lib.vectors("deflate"):
        r, out = O.inflate(blob, max(len(plain), 1))
        assert r == 0, (e["producer"], e["input"])
        assert out == plain, (e["producer"], e["input"])
        n += 1
    assert n >= 300


def _liblz4():
    try:
        L = ctypes.CDLL("/opt/conda/lib/liblz4.so.1.9.3")
    except OSError:
        return None
    L.LZ4_decompress_safe.restype = ctypes.c_int
    L.LZ4_decompress_safe.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                      ctypes.c_int]
    return L


SIZES = [0, 1, 12, 13, 14, 100, 2047, 4096, 59460, 65536]


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("n", SIZES)
def test_oracle_lz4_roundtrip_and_liblz4_accepts(kind, n):
    data = O.fill(kind, 7, n).tobytes()
    r, comp = O.lz4_compress(data)
    assert r == 0 and len(comp) <= O.lz4_bound(n)
    r, back = O.lz4_decompress(comp, max(n, 1))
    assert r == 0 and back == data
    L = _liblz4()
    if L is not None:  # third-party decoder, exact capacity (enforces MFLIMIT/LASTLITERALS)
        dst = ctypes.create_string_buffer(max(n, 1))
        got = L.LZ4_decompress_safe(comp, dst, len(comp), n)
        assert got == n and dst.raw[:n] == data


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("n", SIZES)
def test_oracle_deflate_fixed_roundtrip_and_zlib_accepts(kind, n):
    data = O.fill(kind, 9, n).tobytes()
    r, comp = O.deflate_fixed(data)
    assert r == 0 and len(comp) <= O.deflate_bound(n)
    assert zlib.decompress(comp, -15) == data
    r, back = O.inflate(comp, max(n, 1))
    assert r == 0 and back == data


def test_lz4_compresses_compressible_data():
    data = O.fill(O.KIND_MIXED, 1, 3 << 20).tobytes()
    tot = 0
    for off in range(0, len(data), 65536):
        r, comp = O.lz4_compress(data[off:off + 65536])
        tot += len(comp)
    assert len(data) / tot > 1.5


# --- malformed input: decoders must fail with IOError, never read/write out of bounds ---
def test_lz4_malformed():
    data = O.fill(O.KIND_MIXED, 3, 5000).tobytes()
    _, comp = O.lz4_compress(data)
    assert O.lz4_decompress(b"", 10)[0] == O.BO_ERR_IO
    for cut in (1, 2, len(comp) // 2, len(comp) - 1):
        r, out = O.lz4_decompress(comp[:cut], 5000)
        # a cut that lands right after a literal run is itself a valid (shorter) block
        assert r == O.BO_ERR_IO or (r == 0 and out == data[:len(out)] and len(out) < 5000)
    # output larger than capacity -> OUT_OF_SPACE -> IOError (device.cc:512-520)
    assert O.lz4_decompress(comp, 4999)[0] == O.BO_ERR_IO
    # offset 0 and offset before the segment start
    assert O.lz4_decompress(bytes([0x10, 0x41, 0x00, 0x00, 0x00]), 100)[0] == O.BO_ERR_IO
    assert O.lz4_decompress(bytes([0x10, 0x41, 0x02, 0x00, 0x00]), 100)[0] == O.BO_ERR_IO


def test_inflate_malformed():
    comp = zlib.compress(O.fill(O.KIND_MIXED, 3, 5000).tobytes(), 6)[2:-4]
    for cut in (0, 1, len(comp) // 2, len(comp) - 1):
        assert O.inflate(comp[:cut], 5000)[0] == O.BO_ERR_IO
    assert O.inflate(comp, 4999)[0] == O.BO_ERR_IO
    assert O.inflate(bytes([0x07]), 10)[0] == O.BO_ERR_IO  # BTYPE=11 reserved
    assert O.inflate(bytes([0x01, 0x01, 0x00, 0x00, 0x00, 0x41]), 10)[0] == O.BO_ERR_IO


# --- segment-level rules of CompressDevice (device.cc:156-318) --------------------------
@pytest.mark.parametrize("codec", [O.CODEC_LZ4, O.CODEC_DEFLATE])
def test_segment_roundtrip(codec):
    seg = 59460
    data = O.fill(O.KIND_ARROW, 5, 3 * seg + 17)
    stride = 65536 + 512
    r, slab, sizes = O.compress_segments(codec, data, seg, stride, threads=4)
    assert r == 0 and sizes.size == 4
    blobs = [slab[i * stride:i * stride + int(sizes[i])] for i in range(sizes.size)]
    r, out, produced = O.decompress_segments(codec, blobs, seg, 4 * seg, threads=3)
    assert r == 0
    assert list(produced) == [seg, seg, seg, 17]
    assert np.array_equal(out, data)


def test_segment_empty_and_capacity():
    r, slab, sizes = O.compress_segments(O.CODEC_LZ4, np.zeros(0, np.uint8), 2048, 4096)
    assert r == 0 and sizes.size == 0  # empty input -> empty BufferVector (161-164)
    r, out, _ = O.decompress_segments(O.CODEC_LZ4, [], 2048, 0)
    assert r == 0 and out.size == 0  # empty vector -> OK (244-246)
    data = O.fill(0, 1, 5000)
    r, slab, sizes = O.compress_segments(O.CODEC_LZ4, data, 2048, 4096)
    blobs = [slab[i * 4096:i * 4096 + int(sizes[i])] for i in range(sizes.size)]
    r, _, _ = O.decompress_segments(O.CODEC_LZ4, blobs, 2048, 3 * 2048 - 1)
    assert r == O.BO_ERR_CAPACITY  # capacity < n*seg (248-254)


# ---- Zstandard (oracle/bitar_zstd.c) -----------------------------------------------------
def _libzstd():
    try:
        L = ctypes.CDLL("/opt/conda/lib/libzstd.so.1.4.9")
    except OSError:
        pytest.skip("libzstd not present")
    L.ZSTD_decompress.restype = ctypes.c_size_t
    L.ZSTD_decompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                  ctypes.c_size_t]
    L.ZSTD_isError.restype = ctypes.c_uint
    L.ZSTD_isError.argtypes = [ctypes.c_size_t]
    return L


def test_oracle_zstd_decodes_all_golden():
    n = 0
    for e, blob, plain in golden_lib.vectors("zstd"):
        r, out = O.zstd_decompress(blob, max(len(plain), 1))
        assert r == 0, (e["producer"], e["input"])
        assert out == plain, (e["producer"], e["input"])
        n += 1
    assert n >= 300


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4, 5, 6])
def test_libzstd_decodes_oracle_frames(kind):
    Z = _libzstd()
    for n in (0, 1, 12, 13, 100, 255, 256, 257, 4096, 59460, 65536):
        data = O.fill(kind, 9, n).tobytes()
        r, frame = O.zstd_compress(data)
        assert r == 0 and len(frame) <= O.zstd_bound(n)
        out = ctypes.create_string_buffer(max(n, 1))
        rr = Z.ZSTD_decompress(out, max(n, 1), frame, len(frame))
        assert not Z.ZSTD_isError(rr) and out.raw[:rr] == data, (kind, n)
        r2, back = O.zstd_decompress(frame, max(n, 1))
        assert r2 == 0 and back == data


def test_oracle_zstd_rejects_malformed():
    data = O.fill(O.KIND_MIXED, 3, 20000).tobytes()
    r, frame = O.zstd_compress(data)
    assert r == 0
    bad = [frame[:3], frame[:len(frame) // 2], frame[:-1], frame + b"\x00",
           b"\x28\xb5\x2f\xfe" + frame[4:],               # magic
           frame[:4] + bytes([frame[4] | 8]) + frame[5:]]  # reserved header bit
    for b in bad:
        r, _ = O.zstd_decompress(b, 20000)
        assert r != 0
    # capacity: a frame larger than the segment slot is an error, not a truncation
    r, _ = O.zstd_decompress(frame, 19999)
    assert r != 0
    # content checksum: flip one checksum bit in a libzstd +checksum vector
    for e, blob, plain in golden_lib.vectors("zstd"):
        if "checksum" in e["producer"] and len(plain) > 100:
            r, _ = O.zstd_decompress(blob[:-1] + bytes([blob[-1] ^ 1]), len(plain))
            assert r != 0
            break


def _zstd_blocks(frame):
    """Structure of a single-segment frame the oracle wrote, one dict per block: block type,
    and for a compressed block the literal section (type, streams, sizes, Huffman description
    header byte) and the sequence section (count, table modes)."""
    fh = 6 if frame[4] == 0x20 else 7
    p = fh
    out = []
    while True:
        h = frame[p] | (frame[p + 1] << 8) | (frame[p + 2] << 16)
        last, btype, bsize = h & 1, (h >> 1) & 3, h >> 3
        info = {"block": btype, "bsize": bsize}
        out.append(info)
        end = p + 3 + (bsize if btype != 1 else 1)
        if btype == 2:
            q0 = p + 3
            b0 = frame[q0]
            lt, sf = b0 & 3, (b0 >> 2) & 3
            if lt < 2:
                if sf in (0, 2):
                    reg, hs = b0 >> 3, 1
                elif sf == 1:
                    reg, hs = (b0 >> 4) + (frame[q0 + 1] << 4), 2
                else:
                    reg, hs = (b0 >> 4) + (frame[q0 + 1] << 4) + (frame[q0 + 2] << 12), 3
                lsz, streams, desc = hs + (reg if lt == 0 else 1), 0, None
            else:
                hs = 3 if sf <= 1 else 4 if sf == 2 else 5
                c = int.from_bytes(frame[q0:q0 + hs], "little")
                bits = 10 if hs == 3 else 14 if hs == 4 else 18
                reg, cs = (c >> 4) & ((1 << bits) - 1), c >> (4 + bits)
                lsz, streams = hs + cs, 1 if sf == 0 else 4
                desc = frame[q0 + hs] if lt == 2 else None
            q = q0 + lsz
            nseq = frame[q]
            if nseq >= 128:
                nseq, q = ((nseq - 128) << 8) + frame[q + 1], q + 2
            else:
                q += 1
            modes = None
            if nseq:
                m = frame[q]
                modes = (m >> 6, (m >> 4) & 3, (m >> 2) & 3)
            info.update(lit_type=lt, nlit=reg, lit_bytes=lsz, streams=streams, huf_desc=desc,
                        nseq=nseq, modes=modes)
        p = end
        if last:
            break
    assert p == len(frame)
    return out


def _zstd_info(frame):
    """The first block's structure, with the frame's block count and total sequences."""
    bl = _zstd_blocks(frame)
    i = dict(bl[0])
    i["nblocks"] = len(bl)
    i["nseq_total"] = sum(b.get("nseq", 0) for b in bl)
    return i


def test_oracle_zstd_frame_structure():
    """One block per segment below 64 sequences, else 4 blocks of equal sequence counts, 8
    with >= 32 KiB of literals (raw when the frame does not shrink); literals raw / RLE / Huffman with 1 stream below 256
    literals, else 4 (per block); the first Huffman block carries the tree and later ones are
    Treeless; FSE-compressed Huffman weights when more than 128 would be sent directly;
    table descriptions in the first block, Repeat_Mode in the others."""
    rnd = O.fill(0, 1, 65536).tobytes()
    r, f = O.zstd_compress(rnd)
    assert r == 0 and _zstd_info(f)["block"] == 0 and len(f) == 7 + 3 + 65536
    # one distinct literal byte: RLE literals
    i = _zstd_info(O.zstd_compress(b"\x07" * 5000)[1])
    assert i["block"] == 2 and i["lit_type"] == 1
    # text: Huffman, 1 stream below 256 literals, else 4
    text = O.fill(6, 3, 8000).tobytes()
    i = _zstd_info(O.zstd_compress(text[:600])[1])
    assert i["block"] == 2 and i["lit_type"] == 2 and i["streams"] == 1 and i["nlit"] < 256
    assert i["nblocks"] == 1
    i = _zstd_info(O.zstd_compress(text)[1])
    assert i["lit_type"] == 2 and i["streams"] == 4 and i["nlit"] >= 256
    rng = np.random.default_rng(5)
    # 16 equiprobable byte values: every weight equal -> not FSE-codable -> direct weights
    small = bytes(rng.integers(0, 16, 30000).astype(np.uint8))
    i = _zstd_info(O.zstd_compress(small)[1])
    assert i["lit_type"] == 2 and i["huf_desc"] == 127 + 15
    # skewed bytes across the whole range: > 128 weights -> FSE-compressed (byte < 128)
    p = 0.5 ** (1 + np.arange(256) % 9)
    skew = bytes(rng.choice(256, size=30000, p=p / p.sum()).astype(np.uint8))
    i = _zstd_info(O.zstd_compress(skew)[1])
    assert i["lit_type"] == 2 and i["huf_desc"] < 128
    col = O.fill(5, 1, 65536).tobytes()  # int64 column: sequences on FSE tables
    bl = _zstd_blocks(O.zstd_compress(col)[1])
    assert len(bl) == 4 and all(b["block"] == 2 for b in bl)
    assert sum(b["nseq"] for b in bl) > 1000 and 2 in bl[0]["modes"]
    counts = [b["nseq"] for b in bl]
    assert max(counts) - min(counts) <= 1                     # equal sequence counts
    assert all(b["modes"] == (3, 3, 3) for b in bl[1:])       # Repeat_Mode
    huff = [b for b in bl if b["lit_type"] in (2, 3)]
    assert huff and huff[0]["lit_type"] == 2 and all(b["lit_type"] == 3 for b in huff[1:])
    # literal-heavy frames (a near-incompressible record-batch column): 8 blocks
    rb = O.fill(2, 1000, 17 * 65536)[16 * 65536:].tobytes()
    bl = _zstd_blocks(O.zstd_compress(rb)[1])
    assert len(bl) == 8 and all(b["block"] == 2 for b in bl)
    assert sum(b["nlit"] for b in bl) >= 32768 and sum(b["nseq"] for b in bl) >= 64
    counts = [b["nseq"] for b in bl]
    assert max(counts) - min(counts) <= 1
    assert all(b["modes"] == (3, 3, 3) for b in bl[1:])
    assert bl[0]["lit_type"] == 2 and all(b["lit_type"] == 3 for b in bl[1:])
    # one block again with the single-block setting (rounds 1-4's frames)
    L = O.lib()
    L.bo_set_zstd_blocks.restype = ctypes.c_uint32
    L.bo_set_zstd_blocks.argtypes = [ctypes.c_uint32]
    old = L.bo_set_zstd_blocks(1)
    try:
        assert len(_zstd_blocks(O.zstd_compress(col)[1])) == 1
    finally:
        L.bo_set_zstd_blocks(old)


def test_oracle_zstd_ratio_vs_libzstd1():
    """The level-1-class encoder: on the Arrow-like kind-2 input (all four 1 MiB columns) and
    the Silesia-style kind 1, at least 95 % of libzstd level 1's ratio on the same segments."""
    Z = _libzstd()
    Z.ZSTD_compress.restype = ctypes.c_size_t
    Z.ZSTD_compressBound.restype = ctypes.c_size_t
    seg = 65536
    for kind, n in ((2, 4 << 20), (1, 3 << 20)):
        data = O.fill(kind, 1000, n).tobytes()
        ours = theirs = 0
        out = ctypes.create_string_buffer(int(Z.ZSTD_compressBound(seg)))
        for i in range(0, n, seg):
            s = data[i:i + seg]
            r, f = O.zstd_compress(s)
            assert r == 0
            ours += len(f)
            c = Z.ZSTD_compress(out, len(out), s, len(s), 1)
            assert not Z.ZSTD_isError(c)
            theirs += c
        assert n / ours >= 0.95 * (n / theirs), (kind, n / ours, n / theirs)


# ---- dynamic-Huffman DEFLATE (oracle/bitar_deflate_dyn.c) ----------------------------------
def test_deflate_dynamic_zlib_decodes_every_kind():
    import zlib
    for kind in range(7):
        for n in (1, 2, 12, 13, 64, 100, 4096, 59460, 65536):
            d = O.fill(kind, 3, n).tobytes()
            r, c = O.deflate_dynamic(d)
            assert r == 0 and zlib.decompress(c, -15) == d, (kind, n)
            r2, p = O.inflate(c, n)
            assert r2 == 0 and p == d
            assert len(c) <= O.deflate_bound(n)


def test_deflate_dynamic_beats_fixed_on_compressible_data():
    for kind in (1, 2, 5, 6):
        d = O.fill(kind, 4, 59460).tobytes()
        assert len(O.deflate_dynamic(d)[1]) < len(O.deflate_fixed(d)[1])
    assert O.deflate_dynamic_mode(O.fill(0, 1, 59460).tobytes()) == 0   # random -> stored
    assert O.deflate_dynamic_mode(O.fill(6, 1, 59460).tobytes()) == 2   # text -> dynamic
    assert O.deflate_dynamic_mode(b"abc") == 1                          # tiny -> fixed


def _kraft(lens, maxlen):
    return sum(1 << (maxlen - int(x)) for x in lens if x)


def test_huff_lengths_are_complete_and_limited():
    """Length limiting (zlib's gen_bitlen scheme) on skewed (Fibonacci) and random
    frequencies: every code complete (Kraft sum exactly 1), no length above the limit."""
    rng = np.random.default_rng(1)
    fib = [1, 1]
    while len(fib) < 40:
        fib.append(fib[-1] + fib[-2])
    cases = [(np.array(fib[:30], np.uint32), 15), (np.array(fib[:19], np.uint32), 7)]
    f = np.zeros(286, np.uint32)
    f[:30] = fib[:30]
    cases.append((f, 15))
    for t in range(200):
        nsym = int(rng.choice([19, 30, 286]))
        ml = 7 if nsym == 19 else 15
        f = np.zeros(nsym, np.uint32)
        k = int(rng.integers(1, nsym + 1))
        idx = rng.choice(nsym, k, replace=False)
        f[idx] = (rng.pareto(0.5, k) * 3 + 1).astype(np.uint32) if t % 2 else rng.integers(1, 1000, k)
        cases.append((f, ml))
    for f, ml in cases:
        lens = O.huff_lengths(f, ml)
        assert lens.max() <= ml
        assert _kraft(lens, ml) == 1 << ml
        if (f > 0).sum() >= 2:
            assert np.array_equal(lens > 0, f > 0)


def test_lz4_skip_parse_ratio_cost():
    """The LZ4 parse's window skipping (BO_PARSE_SKIP: probes of stride 2 / 4 after missed
    windows, no work inside a match) costs at most 1 % of ratio against the plain window-scan
    parse on every synthetic kind, and liblz4 decodes its streams."""
    import ctypes
    L = O.lib()
    L.bo_set_lz4_parse_flags.restype = ctypes.c_uint32
    L.bo_set_lz4_parse_flags.argtypes = [ctypes.c_uint32]
    n, seg = 2 << 20, 65536
    stride = (O.lz4_bound(seg) + 255) & ~255
    old = L.bo_set_lz4_parse_flags(0)
    try:
        for kind in (0, 1, 2, 3, 4, 5, 6):
            d = O.fill(kind, 5, n)
            ratios = []
            for flags in (0, 2):
                L.bo_set_lz4_parse_flags(flags)
                r, slab, sizes = O.compress_segments(O.CODEC_LZ4, d, seg, stride, 4)
                assert r == 0
                ratios.append(n / float(sizes.astype(np.int64).sum()))
            assert ratios[1] >= 0.99 * ratios[0], (kind, ratios)
            for i in (0, sizes.size - 1):  # the skip parse's streams are ordinary LZ4 blocks
                blob = slab[i * stride:i * stride + sizes[i]]
                r, out = O.lz4_decompress(blob.tobytes(), seg)
                assert r == 0 and out == d[i * seg:(i + 1) * seg].tobytes()
    finally:
        L.bo_set_lz4_parse_flags(old)


def test_lz4_wide_parse_ratio_and_streams():
    """BITAR_HIP_CODEC_LZ4_WIDE (16 KiB history, 4096-entry table) gains ratio on every
    compressible kind against the fast parse and writes ordinary LZ4 blocks (liblz4 and the
    oracle decode them; distances reach past the fast parse's 2560)."""
    n, seg = 2 << 20, 65536
    stride = (O.lz4_bound(seg) + 255) & ~255
    for kind in (1, 2, 5, 6):
        d = O.fill(kind, 9, n)
        r, slab, sizes = O.compress_segments(O.CODEC_LZ4, d, seg, stride, 4)
        rw, slabw, sizesw = O.compress_segments(O.CODEC_LZ4_WIDE, d, seg, stride, 4)
        assert r == 0 and rw == 0
        assert sizesw.astype(np.int64).sum() < sizes.astype(np.int64).sum(), kind
        blobs = [slabw[i * stride:i * stride + sizesw[i]] for i in range(sizesw.size)]
        r, out, prod = O.decompress_segments(O.CODEC_LZ4_WIDE, blobs, seg, n, 4)
        assert r == 0 and np.array_equal(out, d)


def _set_zstd_flags(flags):
    L = O.lib()
    L.bo_set_zstd_parse_flags.restype = ctypes.c_uint32
    L.bo_set_zstd_parse_flags.argtypes = [ctypes.c_uint32]
    return L.bo_set_zstd_parse_flags(flags)


REP, SKIP, DROP = 1, 2, 1 << 17


def test_zstd_skip_parse_frames_and_ratio():
    """The Zstd parse is the repeat-offset form with window skipping (REP | SKIP, the shipped
    zstd_parse_kernel): libzstd decodes every frame it writes on every kind, and skipping costs
    at most 0.5 % of ratio against the plain repeat-offset scan."""
    Z = _libzstd()
    seg, n = 65536, 2 << 20
    old = _set_zstd_flags(REP | SKIP)
    try:
        assert old == REP | SKIP  # the default
        for kind in range(7):
            data = O.fill(kind, 21, n).tobytes()
            sizes = {}
            for flags in (REP, REP | SKIP):
                _set_zstd_flags(flags)
                tot = 0
                for i in range(0, n, seg):
                    s = data[i:i + seg]
                    r, f = O.zstd_compress(s)
                    assert r == 0
                    tot += len(f)
                    if flags & SKIP:
                        out = ctypes.create_string_buffer(seg)
                        rr = Z.ZSTD_decompress(out, seg, f, len(f))
                        assert not Z.ZSTD_isError(rr) and out.raw[:rr] == s, (kind, i)
                sizes[flags] = tot
            assert sizes[REP | SKIP] <= 1.005 * sizes[REP], (kind, sizes)
    finally:
        _set_zstd_flags(old)


def test_zstd_dropped_gap_literals_are_rejected():
    """Root cause of round 3's REP + SKIP corruption: the GPU literal collector left out the
    literal bytes of skipped probe windows, so a frame's sequences declared more literals than
    its literal section held.  Restated by BO_ZSTD_DROP_GAP_LITERALS, such frames are rejected
    by libzstd ("corruption detected") AND by the oracle's decoder -- the oracle's RFC 8878
    acceptance is not looser than libzstd's on this class."""
    Z = _libzstd()
    seg = 65536
    L = O.lib()
    L.bo_set_zstd_blocks.restype = ctypes.c_uint32
    L.bo_set_zstd_blocks.argtypes = [ctypes.c_uint32]
    old_blocks = L.bo_set_zstd_blocks(1)  # (the round-3 frames: one block; DROP implies it)
    old = _set_zstd_flags(REP | SKIP | DROP)
    bad = 0
    try:
        for kind in (2,):  # (its float64 column: probes that miss, then a hit)
            data = O.fill(kind, 3, 64 * seg).tobytes()
            for i in range(0, len(data), seg):
                s = data[i:i + seg]
                _set_zstd_flags(REP | SKIP | DROP)
                r, f = O.zstd_compress(s)
                _set_zstd_flags(REP | SKIP)
                r0, good = O.zstd_compress(s)
                assert r == 0 and r0 == 0
                if f == good:
                    continue  # no gap before a scanned window in this segment
                bad += 1
                out = ctypes.create_string_buffer(seg)
                rr = Z.ZSTD_decompress(out, seg, f, len(f))
                assert Z.ZSTD_isError(rr) or out.raw[:rr] != s, (kind, i)
                r2, back = O.zstd_decompress(f, seg)
                assert (r2 != 0) == bool(Z.ZSTD_isError(rr)), (kind, i, r2)
                if r2 == 0:
                    assert back == out.raw[:rr]
    finally:
        L.bo_set_zstd_blocks(old_blocks)
        _set_zstd_flags(old)
    assert bad >= 4
