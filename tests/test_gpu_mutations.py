"""Adversarial parity for the branch-free decoder paths (seeded mutations), through the C ABI.

Targets the two decode paths whose hot loops run without exec-mask branches and write
through per-lane trash slots, where an out-of-bounds write or a wrong verdict would hide:
  * the inflate_kernel batch walk (inflate.hip huff_batch: speculative symbol records,
    v_writelane walk, prefix max) on dynamic-Huffman streams long enough to run many batches
    -- our own encoder's and stock zlib level 1's (the reference's frame, config.cc:83-105);
  * the Zstd hand-off -> zstd_seqdec_kernel -> zstd_exec_kernel path (frames whose last block
    holds >= 16 sequences and no checksum): our level-1-class frames and libzstd level 1's.
Every mutated stream (bit flips, byte sets, truncations, corrupted block / table headers)
must decode exactly as the oracle decides (oracle/bitar_oracle.c bo_inflate_raw,
oracle/bitar_zstd.c bo_zstd_decompress): the same accept / reject verdict per segment, and
byte-equal output when accepted -- the reference's per-op rule (src/device.cc:512-520: a
failed op fails the call, never yields wrong bytes).  The context's path counters
(bitar_hip_path_counters) show that the mutations reached the targeted kernels.
"""
import ctypes
import zlib

import numpy as np
import pytest

import oracle_lib as O
from test_gpu_lz4 import _decode_blobs, eng  # noqa: F401  (fixture reuse)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

SEG = 65536


def _mutations(frame, rng, count, hot=None):
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


def _check_like_oracle(eng, codec, cases, oracle):
    ok, out, prod = _decode_blobs(eng, codec, cases, SEG)
    n_ok = 0
    for k, c in enumerate(cases):
        r, ref = oracle(c, SEG)
        if r == 0:
            n_ok += 1
            assert prod[k] == len(ref), (k, int(prod[k]), len(ref))
            assert out[k * SEG:k * SEG + len(ref)].tobytes() == ref, k
        else:
            assert prod[k] == 0xFFFFFFFF, (k, r, int(prod[k]))
    return n_ok


# ---- DEFLATE: the wave inflater's batch walk ----------------------------------------------
@pytest.fixture(params=[4, 0], ids=["lanes4", "wave"])
def counting_inflate(request, eng):
    old = eng.set_decoder_options(inflate_lanes=request.param, count_paths=1)
    eng.path_counters()  # reset
    yield request.param
    eng.set_decoder_options(**old)


def _dynamic_sources():
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


def test_inflate_batch_mutations_like_oracle(eng, counting_inflate):
    srcs = _dynamic_sources()
    # the unmutated streams decode and run the batch path
    _check_like_oracle(eng, O.CODEC_DEFLATE, [s for s, _ in srcs], O.inflate)
    c0 = eng.path_counters()
    assert c0["inflate_wave"] == len(srcs) and c0["inflate_wave_reject"] == 0
    assert c0["inflate_batch_segs"] == len(srcs), c0
    rng = np.random.default_rng(1951)
    cases = []
    for stream, _ in srcs:
        # hot range: the block header and the code-length / literal-length tables
        cases += _mutations(stream, rng, 48, hot=(0, 80))
    n_ok = _check_like_oracle(eng, O.CODEC_DEFLATE, cases, O.inflate)
    c = eng.path_counters()
    # every mutated stream went to inflate_kernel (dynamic blocks: the lane inflater defers
    # them all), most of them ran batches, and the oracle both accepted and rejected some
    assert c["inflate_wave"] == len(cases), c
    assert c["inflate_batch_segs"] >= len(cases) // 3, c
    assert 0 < c["inflate_wave_reject"] < len(cases), c
    assert c["inflate_wave_reject"] == len(cases) - n_ok
    print(f"inflate mutations: {len(cases)} cases, {n_ok} accepted, counters {c}")


def test_inflate_fixed_and_stored_mutations_like_oracle(eng, counting_inflate):
    """Fixed-Huffman (the lane inflater's own path) and stored streams, mutated."""
    rng = np.random.default_rng(1952)
    cases = []
    for kind, n, seed in ((1, 59460, 21), (6, 30000, 22), (0, 20000, 23)):
        plain = O.fill(kind, seed, n).tobytes()
        r, fixed = O.deflate_fixed(plain)
        assert r == 0
        z = zlib.compressobj(1, zlib.DEFLATED, -15, 8, zlib.Z_FIXED)
        cases += _mutations(fixed, rng, 32, hot=(0, 64))
        cases += _mutations(z.compress(plain) + z.flush(), rng, 32, hot=(0, 64))
    _check_like_oracle(eng, O.CODEC_DEFLATE, cases, O.inflate)


# ---- Zstd: hand-off -> phase A (seqdec) -> phase B (exec) ---------------------------------
@pytest.fixture(params=[16, 0], ids=["lanes16-seq", "wave-seq"])
def counting_zstd(request, eng):
    old = eng.set_decoder_options(zstd_lanes=request.param, zstd_seq=1, count_paths=1)
    eng.path_counters()
    yield request.param
    eng.set_decoder_options(**old)


def _libzstd():
    try:
        L = ctypes.CDLL("/opt/conda/lib/libzstd.so.1.4.9")
    except OSError:
        return None
    L.ZSTD_compress.restype = ctypes.c_size_t
    L.ZSTD_compress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                ctypes.c_size_t, ctypes.c_int]
    L.ZSTD_isError.restype = ctypes.c_uint
    L.ZSTD_isError.argtypes = [ctypes.c_size_t]
    return L


def _zstd_sources():
    srcs = []
    Z = _libzstd()
    for kind, n, seed in ((2, 65536, 31), (1, 65536, 32), (5, 65536, 33), (6, 50000, 34),
                          (2, 30000, 35)):
        plain = O.fill(kind, seed, n).tobytes()
        r, ours = O.zstd_compress(plain)  # == the GPU encoder's frame (bit-exact), no checksum
        assert r == 0
        srcs.append((ours, plain))
        if Z is not None:  # libzstd level 1, ZSTD_compress: no checksum by default
            buf = ctypes.create_string_buffer(n + 1024)
            r = Z.ZSTD_compress(buf, n + 1024, plain, n, 1)
            assert not Z.ZSTD_isError(r)
            srcs.append((buf.raw[:r], plain))
    return srcs


def _fcs_flip(frame):
    """frame with the low bit of its Frame_Content_Size flipped (RFC 8878 3.1.1.1)"""
    fhd = frame[4]
    single, fcs_flag, did = (fhd >> 5) & 1, fhd >> 6, fhd & 3
    at = 5 + (0 if single else 1) + (0, 1, 2, 4)[did]
    assert single or fcs_flag, "frame without a content size"
    b = bytearray(frame)
    b[at] ^= 1
    return bytes(b)


def test_zstd_sequence_path_mutations_like_oracle(eng, counting_zstd):
    srcs = _zstd_sources()
    _check_like_oracle(eng, O.CODEC_ZSTD, [s for s, _ in srcs], O.zstd_decompress)
    c0 = eng.path_counters()
    # every source frame takes the hand-off -> seqdec -> exec path (with the lane decoder in
    # front, those it does not defer excepted)
    assert c0["zstd_handed"] == c0["zstd_exec"] == c0["zstd_wave"], c0
    if counting_zstd == 0:
        assert c0["zstd_handed"] == len(srcs), c0
    rng = np.random.default_rng(8878)
    cases = []
    for frame, _ in srcs:
        # hot range: the last third of the frame -- the sequence section's headers and the
        # backward FSE bitstream (its first bytes are read first)
        cases += _mutations(frame, rng, 48, hot=(2 * len(frame) // 3, len(frame)))
    # the frame content size off by one: the sequences decode, phase B's final check rejects
    cases += [_fcs_flip(frame) for frame, _ in srcs]
    n_ok = _check_like_oracle(eng, O.CODEC_ZSTD, cases, O.zstd_decompress)
    c = eng.path_counters()
    assert c["zstd_handed"] >= len(cases) // 3, c
    assert 0 < c["zstd_seqdec"] <= c["zstd_handed"], c
    assert c["zstd_exec"] > 0 and c["zstd_seqdec_reject"] > 0, c
    assert c["zstd_exec_reject"] > 0, c  # (the content-size flips of the < 64 KiB frames)
    assert n_ok < len(cases)
    print(f"zstd mutations: {len(cases)} cases, {n_ok} accepted, counters {c}")


def test_two_engines_with_different_decoders_concurrently(eng):
    """Decoder options are per context: two engines, one with the lane decoders and one with
    the wave decoders alone, decode the same batch at the same time on their own streams;
    each context's counters show its own path."""
    import bitar_amd
    a = bitar_amd.Engine(0, num_streams=1, flags=bitar_amd.FLAG_COUNT_PATHS)
    b = bitar_amd.Engine(0, num_streams=1, flags=bitar_amd.FLAG_COUNT_PATHS
                         | bitar_amd.FLAG_INFLATE_WAVE_ONLY | bitar_amd.FLAG_ZSTD_WAVE_ONLY)
    try:
        assert a.decoder_options()["inflate_lanes"] == 0  # the default since round 3
        a.set_decoder_options(inflate_lanes=4)
        assert a.decoder_options()["inflate_lanes"] == 4
        assert b.decoder_options()["inflate_lanes"] == 0 and b.decoder_options()["zstd_lanes"] == 0
        n, seg = 64 * 59460, 59460
        data = a.empty(n)
        a.fill(1, 3, data)
        torch.cuda.synchronize()
        slab, stride, sizes = a.compress(bitar_amd.CODEC_DEFLATE, data, seg)  # fixed Huffman
        a.sync()
        nseg = sizes.numel()
        outs = []
        for e in (a, b):
            out = e.empty(nseg * seg)
            prod = e.empty(nseg, dtype=torch.int32)
            outs.append((e, out, prod))
        for e, out, prod in outs:  # queued back to back on two different streams
            e.decompress_slab_into(bitar_amd.CODEC_DEFLATE, slab, stride, sizes, nseg, seg, out,
                                   prod, stream=e.queue_pair_stream(0))
        for e, out, prod in outs:
            e.sync(e.queue_pair_stream(0))
            assert torch.equal(out[:n], data)
        ca, cb = a.path_counters(), b.path_counters()
        assert ca["inflate_wave"] == 0, ca  # the lane inflater took every fixed stream
        assert cb["inflate_wave"] == nseg, cb  # the wave inflater alone
    finally:
        a.close()
        b.close()


# ---- LZ4: the far-history kernel (lz4_decompress_kernel<true>) ------------------------------
def test_lz4_far_path_mutations_like_oracle(eng):
    """Streams whose matches reach past the decoder's LDS ring -- the wide parse's (<= 14848
    back) and liblz4's (<= 65535) -- are deferred to lz4_decompress_kernel<true>, whose FAR
    batches read history back from HBM after a wave fence.  Mutated, they must decode as the
    oracle's bo_lz4_decompress_block decides; the counters show the far kernel ran."""
    old = eng.set_decoder_options(count_paths=1)
    try:
        eng.path_counters()
        rng = np.random.default_rng(1977)
        bases = []
        for kind, n, seed in ((1, 65536, 41), (2, 65536, 42), (5, 65536, 43), (6, 40000, 44)):
            plain = O.fill(kind, seed, n).tobytes()
            r, wide = O.lz4_wide_compress(plain)
            assert r == 0
            bases.append(wide)
        try:
            L = ctypes.CDLL("liblz4.so.1")
            L.LZ4_compress_default.restype = ctypes.c_int
            for kind, n, seed in ((1, 65536, 45), (5, 65536, 46)):
                plain = O.fill(kind, seed, n).tobytes()
                buf = ctypes.create_string_buffer(n + n // 255 + 16)
                r = L.LZ4_compress_default(plain, buf, n, len(buf))
                assert r > 0
                bases.append(buf.raw[:r])
        except OSError:
            pass
        _check_like_oracle(eng, O.CODEC_LZ4, bases, O.lz4_decompress)
        c0 = eng.path_counters()
        assert c0["lz4_far"] > 0, c0
        cases = []
        for b in bases:
            cases += _mutations(b, rng, 40, hot=(len(b) // 2, len(b)))
        n_ok = _check_like_oracle(eng, O.CODEC_LZ4, cases, O.lz4_decompress)
        c = eng.path_counters()
        assert c["lz4_far"] > len(cases) // 4, c
        assert n_ok < len(cases)
        print(f"lz4 far mutations: {len(cases)} cases, {n_ok} accepted, counters {c}")
    finally:
        eng.set_decoder_options(**old)
