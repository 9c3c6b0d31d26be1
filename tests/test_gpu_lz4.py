"""GPU parity tests for the LZ4 path, through the C ABI (libbitar_hip.so).

The checker is the oracle (oracle/bitar_oracle.c) pinned by the golden vectors: the HIP
decoder must reproduce every liblz4 golden vector; the HIP encoder must emit exactly the
oracle's bytes (same window-scan parse) and those bytes must round-trip.  Full-size
(1 GiB) runs are checked through size-independent properties (round trip equality,
oracle agreement on sampled segments).
"""
from contextlib import nullcontext

import numpy as np
import pytest

import golden_lib
import oracle_lib as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def eng():
    import bitar_amd
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    e = bitar_amd.Engine(0)
    yield e
    e.close()


def up(a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    t = torch.empty(max(a.size, 1), dtype=torch.uint8)
    if a.size:
        t[:a.size] = torch.from_numpy(a)
    return t.cuda()


def down(t, n=None):
    torch.cuda.synchronize()
    a = t.cpu().numpy()
    return a if n is None else a[:n]


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("n", [1, 63, 64, 65, 4096 + 7, (3 << 20) + 129])
def test_fill_matches_oracle(eng, kind, n):
    d = eng.empty(n)
    eng.fill(kind, 1234, d)
    assert np.array_equal(down(d), O.fill(kind, 1234, n))


def _decode_blobs(eng, codec, blobs, seg):
    """Run the HIP decoder over a list of byte strings as one segment batch (ragged)."""
    import bitar_amd
    nseg = len(blobs)
    stride = max(256, max(len(b) for b in blobs) + 64)
    slab = np.zeros(nseg * stride, np.uint8)
    for i, b in enumerate(blobs):
        slab[i * stride:i * stride + len(b)] = np.frombuffer(b, np.uint8)
    d_slab = up(slab)
    d_sizes = torch.tensor([len(b) for b in blobs], dtype=torch.int32).cuda()
    out = eng.empty(nseg * seg)
    prod = eng.empty(nseg, dtype=torch.int32)
    eng.decompress_slab_into(codec, d_slab, stride, d_sizes, nseg, seg, out, prod)
    torch.cuda.synchronize()
    try:
        eng.sync()
        ok = True
    except bitar_amd.BitarError as ex:
        assert ex.code == -5
        ok = False
    return ok, down(out), down(prod).astype(np.uint32)


def test_decode_all_golden_lz4(eng):
    vecs = [(e, blob, plain) for e, blob, plain in golden_lib.vectors("lz4")
            if len(plain) <= 65536]  # one segment each (larger inputs: oracle tests)
    seg = 65536
    blobs = [blob for _, blob, _ in vecs]
    ok, out, prod = _decode_blobs(eng, O.CODEC_LZ4, blobs, seg)
    assert ok
    for k, (e, blob, plain) in enumerate(vecs):
        assert prod[k] == len(plain), (e["producer"], e["input"])
        assert out[k * seg:k * seg + len(plain)].tobytes() == plain, (e["producer"], e["input"])


@pytest.mark.parametrize("kind", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("seg", [65536, 59460, 2048, 13, 8])
def test_compress_bit_exact_vs_oracle(eng, kind, seg):
    import bitar_amd
    n = 5 * seg + seg // 3 + 1 if seg > 100 else 1000
    data = O.fill(kind, 77, n)
    slab, stride, sizes = eng.compress(bitar_amd.CODEC_LZ4, up(data)[:n], seg)
    eng.sync()
    r, oslab, osizes = O.compress_segments(O.CODEC_LZ4, data, seg, stride)
    assert r == 0
    gsizes = down(sizes).astype(np.uint32)
    assert np.array_equal(gsizes, osizes)
    gslab = down(slab)
    for i in range(gsizes.size):
        a = gslab[i * stride:i * stride + gsizes[i]]
        b = oslab[i * stride:i * stride + osizes[i]]
        assert np.array_equal(a, b), f"segment {i}"
    out, prod = eng.decompress(bitar_amd.CODEC_LZ4, slab, stride, sizes, seg)
    eng.sync()
    assert np.array_equal(down(out)[:n], data)
    assert int(down(prod).astype(np.int64).sum()) == n


def test_malformed_streams_fail_like_oracle(eng):
    data = O.fill(O.KIND_MIXED, 3, 5000).tobytes()
    _, comp = O.lz4_compress(data)
    cases = [comp[:1], comp[:2], comp[:len(comp) // 2], comp[:-1], comp,
             bytes([0x10, 0x41, 0x00, 0x00, 0x00]), bytes([0x10, 0x41, 0x02, 0x00, 0x00]),
             bytes([0xF0]) + bytes([255] * 300), bytes([0x0F, 0x01, 0x00]) + bytes([255] * 40)]
    seg = 5000
    for c in cases:
        ok, out, prod = _decode_blobs(eng, O.CODEC_LZ4, [c, comp], seg)
        r, ref = O.lz4_decompress(c, seg)
        if r == 0:
            assert prod[0] == len(ref) and out[:len(ref)].tobytes() == ref
        else:
            assert prod[0] == 0xFFFFFFFF and not ok
        assert prod[1] == 5000 and out[seg:2 * seg].tobytes() == data


def test_capacity_error(eng):
    import bitar_amd
    data = up(O.fill(0, 1, 10000))
    slab, stride, sizes = eng.compress(bitar_amd.CODEC_LZ4, data[:10000], 4096)
    out = eng.empty(3 * 4096 - 1)
    prod = eng.empty(3, dtype=torch.int32)
    with pytest.raises(bitar_amd.BitarError) as ex:
        eng.decompress_slab_into(bitar_amd.CODEC_LZ4, slab, stride, sizes, 3, 4096, out, prod)
    assert ex.value.code == -6


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_full_size_roundtrip_1gib(eng, kind):
    """BASELINE configs 2/3 at full size: 1 GiB, 64 KiB segments, round trip + samples."""
    import bitar_amd
    n = 1 << 30
    seg = 65536
    data = eng.empty(n)
    eng.fill(kind, 0, data)
    slab, stride, sizes = eng.compress(bitar_amd.CODEC_LZ4, data, seg)
    eng.sync()
    out, prod = eng.decompress(bitar_amd.CODEC_LZ4, slab, stride, sizes, seg)
    eng.sync()
    assert torch.equal(out[:n], data)
    assert int(prod.to(torch.int64).sum().item()) == n
    # sampled segments agree with the oracle byte for byte
    host = None
    gs = down(sizes).astype(np.uint32)
    for i in (0, 1, 4097, 8191, 16383):
        if host is None:
            host = {}
        plain = down(data[i * seg:(i + 1) * seg])
        r, comp = O.lz4_compress(plain.tobytes())
        assert r == 0 and len(comp) == gs[i]
        got = down(slab[i * stride:i * stride + int(gs[i])]).tobytes()
        assert got == comp, f"segment {i}"
    del data, slab, out
    torch.cuda.empty_cache()


# ---- cost-ordered dispatch (calls of >= 2048 segments) -----------------------------------
@pytest.mark.parametrize("codec_name", ["LZ4", "LZ4_WIDE", "DEFLATE", "DEFLATE_DYNAMIC", "ZSTD"])
def test_cost_ordered_dispatch_same_output(eng, codec_name):
    """Calls of >= 2048 segments dispatch the segments most-expensive-first (runtime.hip
    SegOrder; every wave-per-segment compress and decode kernel): the slab, sizes and decoded
    output must equal a plain-order context's (whose kernels the other tests pin to the
    oracle), and for LZ4 sampled segments the oracle's.  Kind 1 at 2048-byte segments mixes all three of its input
    types within the call, so the order is far from the identity."""
    import bitar_amd
    codec = getattr(bitar_amd, "CODEC_" + codec_name)
    plain = bitar_amd.Engine(0, flags=bitar_amd.FLAG_PLAIN_ORDER)
    try:
        seg, nseg = 2048, 6000
        n = seg * nseg - 77  # a short last segment
        data = eng.empty(n)
        eng.fill(1, 7, data)
        # (1 MiB regions of kind 1 hold 512 segments of 2048 bytes: the call crosses 5 regions)
        s1, st1, z1 = eng.compress(codec, data, seg)
        s2, st2, z2 = plain.compress(codec, data, seg)
        eng.sync()
        plain.sync()
        assert st1 == st2
        assert torch.equal(z1, z2)
        h1, h2, gs = down(s1), down(s2), down(z1).astype(np.uint32)
        for i in range(nseg):  # (slot bytes past a segment's size are not written)
            a = i * st1
            assert np.array_equal(h1[a:a + int(gs[i])], h2[a:a + int(gs[i])]), f"segment {i}"
        o1, p1 = eng.decompress(codec, s1, st1, z1, seg)
        o2, p2 = plain.decompress(codec, s1, st1, z1, seg)
        eng.sync()
        plain.sync()
        assert torch.equal(o1[:n], data) and torch.equal(o2[:n], data)
        assert torch.equal(p1, p2)
        if codec_name == "LZ4":
            for i in (0, 511, 512, 1500, 2999, nseg - 1):
                raw = down(data[i * seg:min((i + 1) * seg, n)])
                r, comp = O.lz4_compress(raw.tobytes())
                assert r == 0 and len(comp) == gs[i], f"segment {i}"
                assert h1[i * st1:i * st1 + int(gs[i])].tobytes() == comp, f"segment {i}"
    finally:
        plain.close()


# ---- the wide LZ4 parse (BITAR_HIP_CODEC_LZ4_WIDE: the ratio operating point) -------------
@pytest.mark.parametrize("kind", [0, 1, 2, 3, 5, 6])
@pytest.mark.parametrize("seg", [65536, 59460, 2048, 13])
def test_wide_compress_bit_exact_vs_oracle(eng, kind, seg):
    """lz4_compress_kernel<16384, 12> writes the oracle's bo_lz4_wide_compress_block stream
    byte for byte; our decoder (its far-history kernel: distances up to 14848) and liblz4's
    semantics (the oracle decoder) round-trip it."""
    import bitar_amd
    n = 5 * seg + seg // 3 + 1 if seg > 100 else 1000
    data = O.fill(kind, 78, n)
    slab, stride, sizes = eng.compress(bitar_amd.CODEC_LZ4_WIDE, up(data)[:n], seg)
    eng.sync()
    r, oslab, osizes = O.compress_segments(O.CODEC_LZ4_WIDE, data, seg, stride)
    assert r == 0
    gsizes = down(sizes).astype(np.uint32)
    assert np.array_equal(gsizes, osizes)
    gslab = down(slab)
    for i in range(gsizes.size):
        a = gslab[i * stride:i * stride + gsizes[i]]
        b = oslab[i * stride:i * stride + osizes[i]]
        assert np.array_equal(a, b), f"segment {i}"
    out, prod = eng.decompress(bitar_amd.CODEC_LZ4_WIDE, slab, stride, sizes, seg)
    eng.sync()
    assert np.array_equal(down(out)[:n], data)


def test_wide_full_size_roundtrip_and_ratio(eng):
    """1 GiB of the headline input through the wide parse: round trip, sampled segments equal
    the oracle's, and the ratio gains over the fast parse."""
    import bitar_amd
    n, seg = 1 << 30, 65536
    data = eng.empty(n)
    eng.fill(1, 0, data)
    ratios = {}
    for codec in (bitar_amd.CODEC_LZ4, bitar_amd.CODEC_LZ4_WIDE):
        slab, stride, sizes = eng.compress(codec, data, seg)
        eng.sync()
        out, prod = eng.decompress(codec, slab, stride, sizes, seg)
        eng.sync()
        assert torch.equal(out[:n], data)
        ratios[codec] = n / float(sizes.to(torch.int64).sum().item())
        if codec == bitar_amd.CODEC_LZ4_WIDE:
            gs = down(sizes).astype(np.uint32)
            for i in (0, 5, 16383):
                plain = down(data[i * seg:(i + 1) * seg]).tobytes()
                r, comp = O.lz4_wide_compress(plain)
                assert r == 0 and comp == down(slab[i * stride:i * stride + int(gs[i])]).tobytes()
        del slab, out
    assert ratios[bitar_amd.CODEC_LZ4_WIDE] > 1.03 * ratios[bitar_amd.CODEC_LZ4], ratios
    torch.cuda.empty_cache()


@pytest.mark.parametrize("flags", [0, "plain"])
def test_far_history_large_mixed_call(eng, flags):
    """Large calls (>= 2048 segments, cost-ordered or plain) in which the near kernel defers the
    segments whose matches reach past its LDS ring to the far kernel: a call mixing stock
    liblz4 segments (64 KiB history: they defer), our own (never defer) and a few corrupted
    stock segments (rejected by the far kernel) must decode exactly as the oracle does."""
    import bitar_amd
    import stock_lib as S
    seg, nseg = 65536, 3000
    n = nseg * seg
    host = O.fill(1, 77, n)
    sslab, sstride, ssz = S.compress(S.LZ4, host, seg, 1)
    stride = max(sstride, bitar_amd.slot_size(bitar_amd.CODEC_LZ4, seg))
    e = eng if flags == 0 else bitar_amd.Engine(0, flags=bitar_amd.FLAG_PLAIN_ORDER | bitar_amd.FLAG_COUNT_PATHS)
    try:
        if flags == 0:
            old = e.set_decoder_options(count_paths=1)
        data = up(host)
        gslab, gstride, gsz = e.compress(bitar_amd.CODEC_LZ4, data, seg)
        gslab_h, gsz_h = down(gslab), down(gsz).astype(np.uint32)
        slab = np.zeros(nseg * stride, np.uint8)
        sizes = np.zeros(nseg, np.uint32)
        rng = np.random.default_rng(5)
        bad = set(rng.choice(np.arange(0, nseg, 2), 7, replace=False).tolist())
        for i in range(nseg):
            if i % 2 == 0:  # stock (far matches)
                b = sslab[i * sstride:i * sstride + ssz[i]].copy()
                if i in bad:
                    b[len(b) // 2] ^= 0xA5
            else:
                b = gslab_h[i * gstride:i * gstride + gsz_h[i]]
            slab[i * stride:i * stride + b.size] = b
            sizes[i] = b.size
        out = e.empty(n)
        prod = e.empty(nseg, dtype=torch.int32)
        e.decompress_slab_into(bitar_amd.CODEC_LZ4, up(slab), stride,
                               up(sizes.view(np.uint8)).view(torch.int32), nseg, seg, out, prod,
                               capacity=n)
        blobs = [slab[i * stride:i * stride + sizes[i]] for i in range(nseg)]
        # the oracle's verdicts: the intact segments decode to the input (checked for a
        # sample here, all of them below); a corrupted one is decoded by the oracle alone
        ref = host.copy()
        verdict = np.full(nseg, seg, np.uint32)
        for i in sorted(bad) + list(range(0, nseg, 97)):
            r, dec = O.lz4_decompress(blobs[i], seg)
            if i in bad:
                verdict[i] = 0xFFFFFFFF if r != 0 else len(dec)
                if r == 0:
                    ref[i * seg:i * seg + len(dec)] = np.frombuffer(dec, np.uint8)
            else:
                assert r == 0 and dec == host[i * seg:(i + 1) * seg].tobytes(), i
        rejected = int((verdict == 0xFFFFFFFF).sum())
        try:
            e.sync()
            failed = False
        except bitar_amd.BitarError:
            failed = True
        c = e.path_counters()
        p = down(prod).view(np.uint32)
        o = down(out)
        diff = np.nonzero(p != verdict)[0]
        assert diff.size == 0, (diff[:10].tolist(), p[diff[:10]].tolist(),
                                verdict[diff[:10]].tolist(), sorted(bad), c)
        assert failed == (rejected > 0)
        assert c["lz4_far"] >= nseg // 4  # (stock segments of random data have no far match)
        for i in range(nseg):
            if verdict[i] != 0xFFFFFFFF:
                assert np.array_equal(o[i * seg:i * seg + p[i]], ref[i * seg:i * seg + p[i]]), i
    finally:
        if flags == 0:
            e.set_decoder_options(**old)
        else:
            e.close()
