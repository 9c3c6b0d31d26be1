"""GPU tests of the runtime around the kernels, through the C ABI: per-stream error words
(a failure on one queue pair is reported by that queue pair only, reference
device.cc:84-110, 512-520), bitar_hip_pack's handling of failed segments, and seeded
mutations of LZ4 streams long enough to reach the decoder's batch fast path (accept / reject
and output exactly as the oracle's bo_lz4_decompress_block)."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
from test_gpu_lz4 import _decode_blobs, down, eng, up  # noqa: F401  (fixture reuse)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _slab(blobs, stride):
    slab = np.zeros(len(blobs) * stride, np.uint8)
    for i, b in enumerate(blobs):
        slab[i * stride:i * stride + len(b)] = np.frombuffer(b, np.uint8)
    return up(slab), torch.tensor([len(b) for b in blobs], dtype=torch.int32).cuda()


def test_error_word_is_per_stream():
    """qp 1 decodes a malformed segment, qp 0 a valid one, concurrently: sync(qp0) is OK,
    sync(qp1) is IOError, and qp1's error survives qp0's sync (it is not cleared by it)."""
    import bitar_amd
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    e = bitar_amd.Engine(0, num_streams=2)
    try:
        s0, s1 = e.queue_pair_stream(0), e.queue_pair_stream(1)
        seg = 65536
        data = O.fill(O.KIND_MIXED, 9, 8 * seg)
        r, comp = O.lz4_compress(data[:seg].tobytes())
        assert r == 0
        good = [comp] * 8
        bad = [bytes([0, 0, 0])]  # token 0, offset 0: invalid
        for rep in range(4):
            gs, gz = _slab(good, 65536 + 512)
            bs, bz = _slab(bad, 512)
            torch.cuda.synchronize()
            go, gp = e.empty(8 * seg), e.empty(8, dtype=torch.int32)
            bo, bp = e.empty(seg), e.empty(1, dtype=torch.int32)
            e.decompress_slab_into(O.CODEC_LZ4, bs, 512, bz, 1, seg, bo, bp, stream=s1)
            e.decompress_slab_into(O.CODEC_LZ4, gs, 65536 + 512, gz, 8, seg, go, gp, stream=s0)
            e.sync(s0)  # must not see qp 1's failure, nor clear it
            with pytest.raises(bitar_amd.BitarError) as ex:
                e.sync(s1)
            assert ex.value.code == -5
            e.sync(s1)  # cleared by its own sync
            assert np.array_equal(down(gp).astype(np.uint32), [seg] * 8)
            assert down(bp).astype(np.uint32)[0] == 0xFFFFFFFF
            assert np.array_equal(down(go)[:seg], data[:seg])
        # a failure on a foreign stream (torch's) is reported by sync(NULL) too
        bs, bz = _slab(bad, 512)
        bo, bp = e.empty(seg), e.empty(1, dtype=torch.int32)
        e.decompress_slab_into(O.CODEC_LZ4, bs, 512, bz, 1, seg, bo, bp)
        with pytest.raises(bitar_amd.BitarError):
            e.sync(False)
        e.sync(False)
    finally:
        e.close()


def test_pack_skips_failed_segments(eng):
    """A SEGMENT_ERROR (or any size above the slot stride) packs as 0 bytes and makes the
    next sync return IOError instead of copying out of bounds."""
    import bitar_amd
    stride = 256
    nseg = 4
    slab = up(np.arange(nseg * stride, dtype=np.uint32).astype(np.uint8))
    sizes = torch.tensor([10, -1, 20, stride + 1], dtype=torch.int32).cuda()
    offsets = eng.empty(nseg + 1, dtype=torch.int64)
    frame = eng.empty(64)
    eng.pack(slab, stride, sizes, nseg, offsets, frame)
    with pytest.raises(bitar_amd.BitarError) as ex:
        eng.sync()
    assert ex.value.code == -5
    assert down(offsets).tolist() == [0, 10, 10, 30, 30]
    s = down(slab)
    f = down(frame)
    assert np.array_equal(f[:10], s[:10])
    assert np.array_equal(f[10:30], s[2 * stride:2 * stride + 20])
    eng.sync()
    # offsets only (no frame): same clamp
    sizes2 = torch.tensor([5, -1], dtype=torch.int32).cuda()
    off2 = eng.empty(3, dtype=torch.int64)
    eng.pack(None, 0, sizes2, 2, off2)
    with pytest.raises(bitar_amd.BitarError):
        eng.sync()
    assert down(off2).tolist() == [0, 5, 5]


def test_pack_rejects_null_slab(eng):
    import bitar_amd
    sizes = torch.tensor([5], dtype=torch.int32).cuda()
    off = eng.empty(2, dtype=torch.int64)
    with pytest.raises(bitar_amd.BitarError) as ex:
        eng.pack(None, 256, sizes, 1, off, eng.empty(16))
    assert ex.value.code == -4


def _lz4_sequences(comp):
    """(token position, offset position or None) of every sequence of an LZ4 block."""
    seqs, ip, n = [], 0, len(comp)
    while ip < n:
        tok = comp[ip]
        t0 = ip
        ip += 1
        lit = tok >> 4
        if lit == 15:
            while True:
                b = comp[ip]
                ip += 1
                lit += b
                if b != 255:
                    break
        ip += lit
        if ip >= n:
            seqs.append((t0, None))
            break
        seqs.append((t0, ip))
        ip += 2
        if tok & 15 == 15:
            while comp[ip] == 255:
                ip += 1
            ip += 1
    return seqs


def _lz4_cases(rng):
    """Valid streams of >= 200 bytes (ours and liblz4's, which has far offsets), their
    seeded byte mutations, and targeted bad offsets / lengths in the first and in middle
    sequences of a batch."""
    bases = []
    for kind, seed, n in ((1, 1, 3000), (2, 2, 6000), (5, 3, 4000), (6, 4, 8000), (4, 5, 2500)):
        plain = O.fill(kind, seed, n).tobytes()
        r, c = O.lz4_compress(plain)
        assert r == 0 and len(c) >= 200
        bases.append(c)
    try:
        L = ctypes.CDLL("liblz4.so.1")
        L.LZ4_compress_default.restype = ctypes.c_int
        for kind, seed, n in ((1, 6, 30000), (6, 7, 20000), (2, 8, 40000)):
            plain = O.fill(kind, seed, n).tobytes()
            buf = ctypes.create_string_buffer(n + n // 255 + 16)
            r = L.LZ4_compress_default(plain, buf, n, len(buf))
            assert r > 0
            bases.append(buf.raw[:r])
    except OSError:
        pass
    cases = []
    for c in bases:
        cases.append(c)
        for _ in range(24):
            b = bytearray(c)
            k = int(rng.integers(0, 3))
            i = int(rng.integers(0, len(b)))
            if k == 0:
                b[i] ^= 1 << int(rng.integers(0, 8))
            elif k == 1:
                b[i] = int(rng.integers(0, 256))
            else:
                b = b[:max(1, i)]
            cases.append(bytes(b))
        seqs = [s for s in _lz4_sequences(c) if s[1] is not None]
        picks = [0, 1, 2, len(seqs) // 3, len(seqs) // 2, len(seqs) - 1]
        for j in sorted(set(p for p in picks if 0 <= p < len(seqs))):
            t, o = seqs[j]
            for off in (0, 0xFFFF, 1, 4097):  # zero, too far, overlap, beyond the ring
                b = bytearray(c)
                b[o], b[o + 1] = off & 255, off >> 8
                cases.append(bytes(b))
            b = bytearray(c)
            b[t] = (b[t] & 0xF0) | 15  # match length extension where there was none
            cases.append(bytes(b))
            b = bytearray(c)
            b[t] = 0xF0 | (b[t] & 15)  # literal length extension where there was none
            cases.append(bytes(b))
    return cases


def test_lz4_mutations_match_oracle(eng):
    rng = np.random.default_rng(11)
    cases = _lz4_cases(rng)
    seg = 65536
    for lo in range(0, len(cases), 128):
        chunk = cases[lo:lo + 128]
        ok, out, prod = _decode_blobs(eng, O.CODEC_LZ4, chunk, seg)
        n_bad = 0
        for k, c in enumerate(chunk):
            r, ref = O.lz4_decompress(c, seg)
            if r == 0:
                assert prod[k] == len(ref), (lo + k, len(c))
                assert out[k * seg:k * seg + len(ref)].tobytes() == ref, lo + k
            else:
                n_bad += 1
                assert prod[k] == 0xFFFFFFFF, (lo + k, r, int(prod[k]))
        assert ok == (n_bad == 0)


@pytest.mark.parametrize("kind", [0, 1, 6])
@pytest.mark.parametrize("seg", [65536, 59460, 4096, 100, 1])
def test_checksums_match_zlib(eng, kind, seg):
    """bitar_hip_checksum: per-segment CRC32 / Adler32 / both (DPDK's CRC32_ADLER32 layout)
    equal zlib's, over contiguous segments (a compress's input) and over segments of given
    lengths (a decompress's produced sizes, SEGMENT_ERROR -> 0)."""
    import zlib
    import bitar_amd
    n = 3 * seg + seg // 2 + 1 if seg > 1 else 77
    data = O.fill(kind, 5, n)
    d = up(data)[:n]
    nseg = (n + seg - 1) // seg
    for ck in (1, 2, 3):
        sums = eng.empty(nseg, dtype=torch.int64)
        eng.checksum(ck, d, seg, sums, n=n)
        got = down(sums).view(np.uint64)
        for i in range(nseg):
            part = data[i * seg:(i + 1) * seg].tobytes()
            c, a = zlib.crc32(part), zlib.adler32(part)
            want = c if ck == 1 else a if ck == 2 else c | (a << 32)
            assert int(got[i]) == want, (ck, i)
    # per-segment lengths (shorter than seg, zero, and a failed segment)
    lens = np.array([min(seg, (7 * i + 3) % (seg + 1)) for i in range(nseg)], np.uint32)
    lens[0] = 0
    if nseg > 2:
        lens[2] = 0xFFFFFFFF
    dl = torch.from_numpy(lens.view(np.int32)).cuda()
    sums = eng.empty(nseg, dtype=torch.int64)
    eng.checksum(3, d, seg, sums, n=n, lens=dl, nseg=nseg)
    got = down(sums).view(np.uint64)
    for i in range(nseg):
        if lens[i] == 0xFFFFFFFF:
            assert int(got[i]) == 0
            continue
        part = data[i * seg:i * seg + int(lens[i])].tobytes()
        assert int(got[i]) == zlib.crc32(part) | (zlib.adler32(part) << 32), i


def test_checksum_rejects_bad_kind(eng):
    import bitar_amd
    d = eng.empty(100)
    s = eng.empty(1, dtype=torch.int64)
    with pytest.raises(bitar_amd.BitarError):
        eng.checksum(4, d, 100, s)


def test_copy_batch_any_alignment(eng):
    """bitar_hip_copy_batch (chained ops' split / join): entries of any size and alignment,
    zero-size entries, neighbours untouched."""
    rng = np.random.default_rng(3)
    src = up(rng.integers(0, 256, 1 << 20, dtype=np.uint8))
    dst = eng.empty(1 << 20)
    dst.zero_()
    base_s, base_d = src.data_ptr(), dst.data_ptr()
    entries, at = [], 0
    for k in range(300):
        n = int(rng.choice([0, 1, 15, 16, 17, 63, 64, 1000, 4096, 5000]))
        so = int(rng.integers(0, (1 << 20) - n))
        entries.append((so, at, n))
        at += n + int(rng.integers(1, 40))
    srcs = torch.tensor([base_s + e[0] for e in entries], dtype=torch.int64).cuda()
    dsts = torch.tensor([base_d + e[1] for e in entries], dtype=torch.int64).cuda()
    sizes = torch.tensor([e[2] for e in entries], dtype=torch.int32).cuda()
    eng.copy_batch(srcs, dsts, sizes, len(entries))
    eng.sync()
    s, d = down(src), down(dst)
    want = np.zeros_like(d)
    for so, do, n in entries:
        want[do:do + n] = s[so:so + n]
    assert np.array_equal(d, want)


def test_sync_null_leaves_foreign_stream_errors():
    """sync(NULL) reads and clears only the default stream's and the queue pairs' error words:
    a failure on a foreign (torch side) stream is reported exactly once, by a sync of that
    stream, whether or not a sync(NULL) came first (a NULL sync that cleared it could lose it
    to work still running there)."""
    import bitar_amd
    e = bitar_amd.Engine(0, num_streams=1)
    try:
        seg = 65536
        side = torch.cuda.Stream()
        bs, bz = _slab([bytes([0, 0, 0])], 512)
        torch.cuda.synchronize()
        bo, bp = e.empty(seg), e.empty(1, dtype=torch.int32)
        e.decompress_slab_into(O.CODEC_LZ4, bs, 512, bz, 1, seg, bo, bp, stream=side)
        side.synchronize()
        e.sync(False)  # NULL: not this stream's word
        with pytest.raises(bitar_amd.BitarError) as ex:
            e.sync(side)
        assert ex.value.code == -5
        e.sync(side)  # reported once
        e.sync(False)
    finally:
        e.close()


@pytest.mark.parametrize("codec", [O.CODEC_ZSTD, O.CODEC_DEFLATE_DYN])
def test_two_scratch_chunks_bit_exact(codec):
    """Calls above 32768 segments run in chunks over one scratch allocation (runtime.hip
    kChunkSegs): 64 MiB at seg 1024 = 65536 segments = two chunks; every segment's stream
    equals the oracle's, and the decode of the whole call is byte-exact."""
    import bitar_amd
    e = bitar_amd.Engine(0)
    try:
        seg, n = 1024, 64 << 20
        data = O.fill(O.KIND_ARROW, 77, n)
        d = up(data)
        slab, stride, sizes = e.compress(codec, d, seg)
        out, prod = e.decompress(codec, slab, stride, sizes, seg)
        e.sync()
        assert torch.equal(out[:n], d)
        assert np.array_equal(down(prod).astype(np.uint32), np.full(n // seg, seg, np.uint32))
        r, oslab, osz = O.compress_segments(codec, data, seg, stride, 16)
        assert r == 0
        gsz = down(sizes).astype(np.uint32)
        assert np.array_equal(gsz, osz)
        g = down(slab).reshape(-1, stride)
        o = oslab.reshape(-1, stride)
        col = np.arange(stride)[None, :]
        mask = col < osz[:, None]
        assert np.array_equal(g[mask], o[mask])
    finally:
        e.close()


@pytest.mark.parametrize("pinned", [True, False], ids=["pinned", "pageable"])
@pytest.mark.parametrize("codec", [O.CODEC_LZ4, O.CODEC_ZSTD, O.CODEC_DEFLATE_DYN])
def test_host_memory_calls_overlap_and_match(codec, pinned):
    """bitar_hip_compress_host / _decompress_host: host input staged chunk by chunk with each
    chunk's compress overlapping the next chunk's copy, and the decode copied out chunk by
    chunk -- the same slab and sizes as a compress of the HBM copy, and the input back in host
    memory (the reference attaches host slices zero-copy, src/memory.cc:380-399, 482-493)."""
    import bitar_amd
    e = bitar_amd.Engine(0)
    try:
        seg = 59460 if codec == O.CODEC_DEFLATE_DYN else 65536
        # ~12 MiB: one chunk; 96 MiB: three chunks of >= 32 MiB (the last one short)
        for n in (200 * seg + 777, (96 << 20) + 12345):
            data = O.fill(O.KIND_MIXED, 61, n)
            host = torch.from_numpy(data)
            if pinned:
                host = host.pin_memory()
            nseg = (n + seg - 1) // seg
            stride = bitar_amd.slot_size(codec, seg)
            stage = e.empty(nseg * seg)
            slab = e.empty(nseg * stride)
            sizes = e.empty(nseg, dtype=torch.int32)
            e.compress_host_into(codec, host.data_ptr(), n, seg, stage, slab, stride, sizes)
            e.sync()
            d = up(data)
            slab2, stride2, sizes2 = e.compress(codec, d[:n], seg)
            e.sync()
            assert torch.equal(sizes, sizes2)
            g1, g2, gs = down(slab), down(slab2), down(sizes).astype(np.uint32)
            for i in range(nseg):
                assert np.array_equal(g1[i * stride:i * stride + gs[i]],
                                      g2[i * stride:i * stride + gs[i]]), i
            srcs = torch.tensor([slab.data_ptr() + i * stride for i in range(nseg)],
                                dtype=torch.int64).cuda()
            out = torch.zeros(nseg * seg, dtype=torch.uint8)
            if pinned:
                out = out.pin_memory()
            prod = e.empty(nseg, dtype=torch.int32)
            e.decompress_host_into(codec, srcs, sizes, nseg, seg, stage, out.data_ptr(), prod)
            e.sync()
            assert np.array_equal(out.numpy()[:n], data)
            assert int(prod.to(torch.int64).sum().item()) == n
    finally:
        e.close()
