"""GPU parity tests for the raw-DEFLATE path (the reference's frame), through the C ABI.

Pinning: the HIP inflater must reproduce every zlib 1.2.11 / libdeflate 1.8 golden vector
(stored, fixed and dynamic Huffman blocks); the HIP fixed-Huffman compressor must emit the
oracle's exact bitstream, which zlib must decode byte-exactly (the reference's frames are
one raw-DEFLATE stream per <= 59460-B segment: config.cc:83-105, app_common.h:39).
"""
import zlib

import numpy as np
import pytest

import golden_lib
import oracle_lib as O
from test_gpu_lz4 import _decode_blobs, down, eng, up  # noqa: F401  (fixture reuse)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(autouse=True, params=[16, 32, 0], ids=["lanes16", "lanes32", "wave"])
def inflate_decoder(request):
    """Every test runs with the lane-per-segment inflater in front (inflate_lanes.hip; it
    defers dynamic-Huffman and failing streams to the wave kernel) and with the
    wave-per-segment inflater alone."""
    import bitar_amd
    L = bitar_amd.lib()
    old = L.bitar_hip_debug_set_inflate_lanes(request.param)
    yield request.param
    L.bitar_hip_debug_set_inflate_lanes(old)


def test_inflate_all_golden(eng):
    vecs = [(e, blob, plain) for e, blob, plain in golden_lib.vectors("deflate")
            if len(plain) <= 65536]  # one segment each (larger inputs: oracle tests)
    seg = 65536
    blobs = [blob for _, blob, _ in vecs]
    ok, out, prod = _decode_blobs(eng, O.CODEC_DEFLATE, blobs, seg)
    assert ok
    for k, (e, blob, plain) in enumerate(vecs):
        assert prod[k] == len(plain), (e["producer"], e["input"], int(prod[k]))
        assert out[k * seg:k * seg + len(plain)].tobytes() == plain, (e["producer"], e["input"])


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("seg", [59460, 65536, 2048, 13])
def test_deflate_fixed_bit_exact_vs_oracle(eng, kind, seg):
    import bitar_amd
    n = 4 * seg + seg // 3 + 1 if seg > 100 else 700
    data = O.fill(kind, 91, n)
    slab, stride, sizes = eng.compress(bitar_amd.CODEC_DEFLATE, up(data)[:n], seg)
    eng.sync()
    r, oslab, osizes = O.compress_segments(O.CODEC_DEFLATE, data, seg, stride)
    assert r == 0
    gsizes = down(sizes).astype(np.uint32)
    assert np.array_equal(gsizes, osizes)
    gslab = down(slab)
    for i in range(gsizes.size):
        a = gslab[i * stride:i * stride + gsizes[i]]
        b = oslab[i * stride:i * stride + osizes[i]]
        assert np.array_equal(a, b), f"segment {i}"
        plain = data[i * seg:(i + 1) * seg].tobytes()
        assert zlib.decompress(a.tobytes(), -15) == plain  # third-party decoder
    out, prod = eng.decompress(bitar_amd.CODEC_DEFLATE, slab, stride, sizes, seg)
    eng.sync()
    assert np.array_equal(down(out)[:n], data)


def test_inflate_malformed_like_oracle(eng):
    plain = O.fill(O.KIND_MIXED, 3, 5000).tobytes()
    good = zlib.compress(plain, 6)[2:-4]
    fixed = zlib.compressobj(6, zlib.DEFLATED, -15, 8, zlib.Z_FIXED)
    fixed = fixed.compress(plain) + fixed.flush()
    cases = [good[:0], good[:1], good[:len(good) // 2], good[:-1], good, fixed[:-2],
             bytes([0x07]), bytes([0x01, 0x01, 0x00, 0x00, 0x00, 0x41]),
             bytes([0x01, 0x05, 0x00, 0xFA, 0xFF]) + b"hello", bytes([0x01, 0x00, 0x00, 0xFF, 0xFF]),
             bytes([0xFD] * 40), bytes([0x05] + [0xFF] * 30), bytes(range(256))]
    seg = 5000
    for c in cases:
        ok, out, prod = _decode_blobs(eng, O.CODEC_DEFLATE, [c if c else b"\x00", good], seg)
        c = c if c else b"\x00"
        r, ref = O.inflate(c, seg)
        if r == 0:
            assert prod[0] == len(ref) and out[:len(ref)].tobytes() == ref, c[:8]
        else:
            assert prod[0] == 0xFFFFFFFF and not ok, c[:8]
        assert prod[1] == 5000 and out[seg:2 * seg].tobytes() == plain


@pytest.mark.parametrize("kind", [1, 2])
def test_full_size_deflate_roundtrip(eng, kind):
    """1 GiB at the reference's 59460-B segments (18059 streams): round trip + zlib samples."""
    import bitar_amd
    n = 1 << 30
    seg = 59460
    data = eng.empty(n)
    eng.fill(kind, 5, data)
    slab, stride, sizes = eng.compress(bitar_amd.CODEC_DEFLATE, data, seg)
    eng.sync()
    out, prod = eng.decompress(bitar_amd.CODEC_DEFLATE, slab, stride, sizes, seg)
    eng.sync()
    assert torch.equal(out[:n], data)
    gs = down(sizes).astype(np.uint32)
    for i in (0, 7, 9000, gs.size - 1):
        blob = down(slab[i * stride:i * stride + int(gs[i])]).tobytes()
        plain = down(data[i * seg:min(n, (i + 1) * seg)]).tobytes()
        assert zlib.decompress(blob, -15) == plain
    del data, slab, out
    torch.cuda.empty_cache()
