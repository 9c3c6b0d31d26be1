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


@pytest.fixture(autouse=True, params=[4, 16, 0], ids=["lanes4", "lanes16", "wave"])
def inflate_decoder(request, eng):
    """Every test runs with the lane-per-segment inflater in front (inflate_lanes.hip; it
    defers dynamic-Huffman and failing streams to the wave kernel) and with the
    wave-per-segment inflater alone (decoder options of the test's context)."""
    old = eng.set_decoder_options(inflate_lanes=request.param)
    yield request.param
    eng.set_decoder_options(**old)


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


# ---- dynamic Huffman (HuffmanEncoding::DYNAMIC, the reference default) ---------------------
# (compress parity does not depend on the decoder: the dynamic-Huffman tests run under the
# lanes4 decoder, and the reference's 59460-B segments under the other two as well)
def _by_decoders(*ds):
    ids = {4: "lanes4", 16: "lanes16", 0: "wave"}
    return pytest.mark.parametrize("inflate_decoder", list(ds), indirect=True,
                                   ids=[ids[d] for d in ds])


@_by_decoders(4)
@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("seg", [59460, 65536, 2048, 100, 13, 8])
def test_deflate_dynamic_bit_exact_vs_oracle(eng, kind, seg):
    """deflate_dyn_parse_kernel + deflate_dyn_emit_kernel emit the oracle's exact stream
    (dynamic, fixed or stored block, whichever is smallest); zlib decodes every segment and
    our inflaters round-trip it."""
    _dynamic_bit_exact(eng, kind, seg)


@_by_decoders(16, 0)
@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4, 5, 6])
def test_deflate_dynamic_bit_exact_other_decoders(eng, kind):
    _dynamic_bit_exact(eng, kind, 59460)


def _dynamic_bit_exact(eng, kind, seg):
    import bitar_amd
    n = 3 * seg + seg // 3 + 1 if seg > 100 else 700
    data = O.fill(kind, 93, n)
    slab, stride, sizes = eng.compress(bitar_amd.CODEC_DEFLATE_DYNAMIC, up(data)[:n], seg)
    eng.sync()
    r, oslab, osizes = O.compress_segments(O.CODEC_DEFLATE_DYN, data, seg, stride)
    assert r == 0
    gsizes = down(sizes).astype(np.uint32)
    assert np.array_equal(gsizes, osizes)
    gslab = down(slab)
    for i in range(gsizes.size):
        a = gslab[i * stride:i * stride + gsizes[i]]
        b = oslab[i * stride:i * stride + osizes[i]]
        assert np.array_equal(a, b), f"segment {i}"
        plain = data[i * seg:(i + 1) * seg].tobytes()
        assert zlib.decompress(a.tobytes(), -15) == plain
    out, prod = eng.decompress(bitar_amd.CODEC_DEFLATE_DYNAMIC, slab, stride, sizes, seg)
    eng.sync()
    assert np.array_equal(down(out)[:n], data)


@_by_decoders(4)
def test_deflate_dynamic_covers_every_block_type(eng):
    """Inputs that make the encoder choose stored (random), fixed (tiny) and dynamic blocks,
    in one ragged batch, including a 65536-B stored segment (two stored blocks)."""
    import bitar_amd
    seg = 65536
    parts = [O.fill(0, 1, seg), O.fill(1, 2, 40), O.fill(6, 3, seg), O.fill(3, 4, seg),
             O.fill(0, 5, 5000), bytes([7]) * 1 + b"", O.fill(2, 6, 20000)]
    modes = set()
    for p in parts:
        p = bytes(p)
        modes.add(O.deflate_dynamic_mode(p))
        data = np.frombuffer(p, np.uint8)
        slab, stride, sizes = eng.compress(bitar_amd.CODEC_DEFLATE_DYNAMIC, up(data)[:len(p)], seg)
        eng.sync()
        g = down(slab)[:int(down(sizes)[0])].tobytes()
        assert (0, g) == O.deflate_dynamic(p)
        assert zlib.decompress(g, -15) == p
    assert modes == {0, 1, 2}


@_by_decoders(4)
def test_deflate_dynamic_scattered_slots(eng):
    """compress_scattered (the C++ slot pool's form) writes the same streams."""
    import bitar_amd
    seg = 59460
    n = 5 * seg + 99
    data = O.fill(2, 8, n)
    stride = bitar_amd.slot_size(bitar_amd.CODEC_DEFLATE_DYNAMIC, seg)
    nseg = (n + seg - 1) // seg
    slots = eng.empty(nseg * stride * 2)
    order = [3, 0, 5, 1, 4, 2]  # slot k of segment i: a permuted, non-contiguous layout
    ptrs = torch.tensor([slots.data_ptr() + order[i] * 2 * stride for i in range(nseg)],
                        dtype=torch.int64).cuda()
    sizes = eng.empty(nseg, dtype=torch.int32)
    L = bitar_amd.lib()
    import ctypes
    bitar_amd.check(L.bitar_hip_compress_scattered(
        eng.ctx, eng._stream(None), bitar_amd.CODEC_DEFLATE_DYNAMIC,
        ctypes.c_void_p(up(data).data_ptr()), n, seg, ctypes.c_void_p(ptrs.data_ptr()), stride,
        ctypes.c_void_p(sizes.data_ptr())))
    eng.sync()
    gs = down(sizes).astype(np.uint32)
    s = down(slots)
    for i in range(nseg):
        plain = data[i * seg:(i + 1) * seg].tobytes()
        blob = s[order[i] * 2 * stride:order[i] * 2 * stride + gs[i]].tobytes()
        assert (0, blob) == O.deflate_dynamic(plain), i


@_by_decoders(4, 0)
@pytest.mark.parametrize("kind", [1, 2])
def test_full_size_deflate_dynamic_roundtrip(eng, kind):
    """1 GiB at 59460-B segments with dynamic Huffman: round trip + zlib + oracle samples."""
    import bitar_amd
    n = 1 << 30
    seg = 59460
    data = eng.empty(n)
    eng.fill(kind, 6, data)
    slab, stride, sizes = eng.compress(bitar_amd.CODEC_DEFLATE_DYNAMIC, data, seg)
    eng.sync()
    out, prod = eng.decompress(bitar_amd.CODEC_DEFLATE_DYNAMIC, slab, stride, sizes, seg)
    eng.sync()
    assert torch.equal(out[:n], data)
    gs = down(sizes).astype(np.uint32)
    for i in (0, 1, 9000, gs.size - 1):
        blob = down(slab[i * stride:i * stride + int(gs[i])]).tobytes()
        plain = down(data[i * seg:min(n, (i + 1) * seg)]).tobytes()
        assert zlib.decompress(blob, -15) == plain
        assert (0, blob) == O.deflate_dynamic(plain)
    del data, slab, out
    torch.cuda.empty_cache()
