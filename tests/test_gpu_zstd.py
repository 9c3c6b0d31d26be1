"""GPU parity tests for the Zstandard path (BASELINE configs[5]), through the C ABI.

Pinning: the HIP frame decoder must reproduce every libzstd 1.4.9 golden vector (levels
1/3/9/19, with and without content checksum / content size, small windows), decode frames
libzstd produces at run time (the same library the golden vectors came from, when the box
has it), decode the oracle's frames, and accept / reject exactly the streams the oracle
(oracle/bitar_zstd.c) accepts / rejects -- including a few hundred seeded mutations.
"""
import ctypes

import numpy as np
import pytest

import golden_lib
import oracle_lib as O
from test_gpu_lz4 import _decode_blobs, down, eng, up  # noqa: F401  (fixture reuse)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(autouse=True, params=[(16, 1), (64, 0), (0, 1)],
                ids=["lanes16-seq", "lanes64-handoff", "wave-seq"])
def zstd_decoder(request, eng):
    """Every test runs with the lane-per-segment decoder in front (zstd_lanes.hip, 16 or 64
    segments per wave; it defers what it does not take to the wave kernel) and with the
    wave-per-segment decoder alone; the sequence sections the wave kernel hands over run
    through the two-phase record path (zstd_seq.hip, "seq") or the lane executor
    (zstd_handoff_kernel, "handoff")."""
    lanes, seq = request.param
    old = eng.set_decoder_options(zstd_lanes=lanes, zstd_seq=seq)
    yield request.param
    eng.set_decoder_options(**old)


def _libzstd():
    try:
        L = ctypes.CDLL("/opt/conda/lib/libzstd.so.1.4.9")
    except OSError:
        pytest.skip("libzstd not present")
    L.ZSTD_compress.restype = ctypes.c_size_t
    L.ZSTD_compress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                ctypes.c_size_t, ctypes.c_int]
    L.ZSTD_compressBound.restype = ctypes.c_size_t
    L.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
    L.ZSTD_isError.restype = ctypes.c_uint
    L.ZSTD_isError.argtypes = [ctypes.c_size_t]
    return L


def _check_batch(eng, blobs, plains, seg):
    ok, out, prod = _decode_blobs(eng, O.CODEC_ZSTD, blobs, seg)
    assert ok
    for k, plain in enumerate(plains):
        assert prod[k] == len(plain), (k, int(prod[k]), len(plain))
        assert out[k * seg:k * seg + len(plain)].tobytes() == plain, k


def test_zstd_decode_all_golden(eng):
    vecs = [(e, blob, plain) for e, blob, plain in golden_lib.vectors("zstd")
            if len(plain) <= 65536]
    assert len(vecs) >= 200
    seg = 65536
    ok, out, prod = _decode_blobs(eng, O.CODEC_ZSTD, [b for _, b, _ in vecs], seg)
    assert ok
    for k, (e, blob, plain) in enumerate(vecs):
        assert prod[k] == len(plain), (e["producer"], e["input"], int(prod[k]))
        assert out[k * seg:k * seg + len(plain)].tobytes() == plain, (e["producer"], e["input"])


@pytest.mark.parametrize("level", [1, 3, 6, 12, 19])
def test_zstd_decode_libzstd_frames(eng, level):
    Z = _libzstd()
    blobs, plains = [], []
    for kind in range(7):
        for n in (0, 1, 100, 4096, 59460, 65536):
            data = O.fill(kind, 1000 + level, n).tobytes()
            cap = Z.ZSTD_compressBound(n)
            buf = ctypes.create_string_buffer(cap)
            r = Z.ZSTD_compress(buf, cap, data, n, level)
            assert not Z.ZSTD_isError(r)
            blobs.append(buf.raw[:r])
            plains.append(data)
    _check_batch(eng, blobs, plains, 65536)


@pytest.mark.parametrize("seg", [65536, 59460, 4096, 13])
def test_zstd_decode_oracle_frames(eng, seg):
    import bitar_amd
    n = 4 * seg + seg // 3 + 1 if seg > 100 else 700
    for kind in range(7):
        data = O.fill(kind, 31, n)
        stride = bitar_amd.slot_size(bitar_amd.CODEC_ZSTD, seg)
        r, slab, sizes = O.compress_segments(O.CODEC_ZSTD, data, seg, stride)
        assert r == 0
        blobs = [slab[i * stride:i * stride + sizes[i]].tobytes() for i in range(sizes.size)]
        plains = [data[i * seg:(i + 1) * seg].tobytes() for i in range(sizes.size)]
        _check_batch(eng, blobs, plains, seg)


def _mutations(frame, rng, count):
    out = []
    for _ in range(count):
        b = bytearray(frame)
        kind = rng.integers(0, 3)
        if kind == 0:  # bit flip
            i = int(rng.integers(0, len(b)))
            b[i] ^= 1 << int(rng.integers(0, 8))
        elif kind == 1:  # byte set
            i = int(rng.integers(0, len(b)))
            b[i] = int(rng.integers(0, 256))
        else:  # truncation
            b = b[:int(rng.integers(0, len(b)))]
        out.append(bytes(b) if b else b"\x00")
    return out


def test_zstd_accepts_and_rejects_like_oracle(eng):
    seg = 8192
    vecs = [(blob, plain) for e, blob, plain in golden_lib.vectors("zstd")
            if 200 <= len(plain) <= seg]
    assert vecs
    rng = np.random.default_rng(7)
    cases = []
    for blob, _ in vecs[:24]:
        cases += _mutations(blob, rng, 12)
    data = O.fill(O.KIND_MIXED, 3, 5000).tobytes()
    r, frame = O.zstd_compress(data)
    assert r == 0
    cases += [frame[:3], frame[:-1], frame + b"\x00", b"\x28\xb5\x2f\xfe" + frame[4:],
              frame[:4] + bytes([frame[4] | 8]) + frame[5:]]
    ok, out, prod = _decode_blobs(eng, O.CODEC_ZSTD, cases, seg)
    n_ok = 0
    for k, c in enumerate(cases):
        r, ref = O.zstd_decompress(c, seg)
        if r == 0:
            n_ok += 1
            assert prod[k] == len(ref), (k, c[:16])
            assert out[k * seg:k * seg + len(ref)].tobytes() == ref, k
        else:
            assert prod[k] == 0xFFFFFFFF, (k, r, int(prod[k]))
    assert not ok  # at least the malformed tail cases fail
    assert 0 < n_ok < len(cases)


def test_zstd_checksum_and_capacity(eng):
    vec = next((blob, plain) for e, blob, plain in golden_lib.vectors("zstd")
               if "checksum" in e["producer"] and 100 < len(plain) <= 65536)
    blob, plain = vec
    bad = blob[:-1] + bytes([blob[-1] ^ 1])
    ok, out, prod = _decode_blobs(eng, O.CODEC_ZSTD, [blob, bad], 65536)
    assert prod[0] == len(plain) and out[:len(plain)].tobytes() == plain
    assert prod[1] == 0xFFFFFFFF and not ok
    # a frame larger than the segment is an error, not a truncation
    seg = len(plain) - 1
    ok, out, prod = _decode_blobs(eng, O.CODEC_ZSTD, [blob], seg)
    assert prod[0] == 0xFFFFFFFF and not ok


# ---- the HIP Zstandard compressor (zstd_compress.hip) ------------------------------------
@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("seg", [65536, 59460, 2048, 255, 13, 8])
def test_zstd_compress_bit_exact_vs_oracle(eng, kind, seg):
    """GPU frames equal the oracle's byte for byte and decode back (GPU and libzstd)."""
    import bitar_amd
    n = 5 * seg + seg // 3 + 1 if seg > 100 else 1000
    data = O.fill(kind, 77, n)
    slab, stride, sizes = eng.compress(bitar_amd.CODEC_ZSTD, up(data)[:n], seg)
    eng.sync()
    r, oslab, osizes = O.compress_segments(O.CODEC_ZSTD, data, seg, stride)
    assert r == 0
    gsizes = down(sizes).astype(np.uint32)
    assert np.array_equal(gsizes, osizes)
    gslab = down(slab)
    for i in range(gsizes.size):
        a = gslab[i * stride:i * stride + gsizes[i]]
        b = oslab[i * stride:i * stride + osizes[i]]
        assert np.array_equal(a, b), f"segment {i}"
    out, prod = eng.decompress(bitar_amd.CODEC_ZSTD, slab, stride, sizes, seg)
    eng.sync()
    assert np.array_equal(down(out)[:n], data)
    assert int(down(prod).astype(np.int64).sum()) == n


def test_libzstd_decodes_gpu_frames(eng):
    import bitar_amd
    Z = _libzstd()
    Z.ZSTD_decompress.restype = ctypes.c_size_t
    Z.ZSTD_decompress.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                  ctypes.c_size_t]
    seg = 65536
    for kind in range(7):
        n = 3 * seg + 999
        data = O.fill(kind, 5, n)
        slab, stride, sizes = eng.compress(bitar_amd.CODEC_ZSTD, up(data)[:n], seg)
        eng.sync()
        gs, g = down(sizes).astype(np.uint32), down(slab)
        for i in range(gs.size):
            frame = g[i * stride:i * stride + gs[i]].tobytes()
            plain = data[i * seg:(i + 1) * seg].tobytes()
            buf = ctypes.create_string_buffer(seg)
            r = Z.ZSTD_decompress(buf, seg, frame, len(frame))
            assert not Z.ZSTD_isError(r) and buf.raw[:r] == plain, (kind, i)


def _zstd_blocks(frame):
    """number of blocks in one RFC 8878 frame (header fields per RFC 8878 3.1.1.1)"""
    frame = bytes(frame)  # (python ints: numpy uint8 shifts would wrap)
    fhd = frame[4]
    single = (fhd >> 5) & 1
    p = 5 + (0 if single else 1) + (0, 1, 2, 4)[fhd & 3]
    p += (1 if single else 0, 2, 4, 8)[fhd >> 6]
    nb = 0
    while True:
        h = frame[p] | frame[p + 1] << 8 | frame[p + 2] << 16
        nb += 1
        p += 3 + (1 if (h >> 1) & 3 == 1 else h >> 3)
        if h & 1:
            return nb


def test_zstd_multiblock_units_in_different_waves(eng):
    """4-block and 8-block frames mixed in one call of >= 2048 units: the cost-ordered
    dispatch of zstd_seqdec_kernel<4, 4> puts the two 4-block units of an 8-block frame in
    different workgroups, and one of them may start after the other finished and moved the
    segment to kRecs (it must still take its blocks).  Every byte checked, and
    phase A must have run on every multi-block frame."""
    import bitar_amd
    seg, nseg = 65536, 6144
    n = seg * nseg
    data = eng.empty(n)
    eng.fill(2, 11, data)  # the Arrow record batch: literal-heavy columns get 8 blocks
    slab, stride, sizes = eng.compress(bitar_amd.CODEC_ZSTD, data, seg)
    eng.sync()
    gs, g = down(sizes).astype(np.uint32), down(slab)
    nb = np.array([_zstd_blocks(g[i * stride:i * stride + gs[i]]) for i in range(nseg)])
    assert (nb == 8).sum() >= 64 and (nb == 4).sum() >= 64, np.bincount(nb)
    old = eng.set_decoder_options(count_paths=1)
    try:
        for rep in range(2):
            out, prod = eng.decompress(bitar_amd.CODEC_ZSTD, slab, stride, sizes, seg)
            eng.sync()
            assert torch.equal(out[:n], data), rep
            assert int(prod.to(torch.int64).sum().item()) == n
        pc = eng.path_counters()
    finally:
        eng.set_decoder_options(**old)
    if eng.decoder_options()["zstd_seq"]:
        assert pc["zstd_seqdec"] >= 2 * int((nb >= 2).sum()), pc
    del data, slab, out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("kind", [1, 2])
def test_zstd_full_size_roundtrip_1gib(eng, kind):
    """BASELINE configs[5] per GPU: 1 GiB, 64 KiB segments, round trip + oracle samples."""
    import bitar_amd
    n, seg = 1 << 30, 65536
    data = eng.empty(n)
    eng.fill(kind, 0, data)
    slab, stride, sizes = eng.compress(bitar_amd.CODEC_ZSTD, data, seg)
    eng.sync()
    out, prod = eng.decompress(bitar_amd.CODEC_ZSTD, slab, stride, sizes, seg)
    eng.sync()
    assert torch.equal(out[:n], data)
    assert int(prod.to(torch.int64).sum().item()) == n
    gs = down(sizes).astype(np.uint32)
    assert gs.sum() < n  # it compresses
    for i in (0, 1, 4097, 16383):
        plain = down(data[i * seg:(i + 1) * seg])
        r, comp = O.zstd_compress(plain.tobytes())
        assert r == 0 and len(comp) == gs[i]
        assert down(slab[i * stride:i * stride + int(gs[i])]).tobytes() == comp, f"segment {i}"
    del data, slab, out
    torch.cuda.empty_cache()
