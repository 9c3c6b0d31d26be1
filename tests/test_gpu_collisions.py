"""Same-slot hash inserts: every compressor against the oracle on inputs where whole windows
of positions hash to ONE slot of the parse's 1024-entry table.

The window parse (bitar_amd/csrc/window_parse.hip.h) inserts a window's 64 positions with
one ds_write_b16 and relies on the hardware keeping the highest lane's value when lanes hit
the same address -- the oracle's rule is that the largest position wins (ascending inserts,
oracle/bitar_oracle.c bo_window_parse).  Here every 4-byte string of a stretch maps to the
same slot, and later stretches repeat bytes from random earlier positions, so which position
a slot ended with decides which matches exist: any other winner changes the output.
"""
import numpy as np
import pytest

import gpu_parity as P

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

K = 2654435761  # the parse's multiplicative hash (hash4), table of 2^10 slots


@pytest.fixture(scope="module")
def eng():
    import bitar_amd
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    e = bitar_amd.Engine(0)
    yield e
    e.close()


def same_slot_stream(n, seed):
    """n bytes of stretches in which a window's 64 positions fall into few table slots: random
    strings over 2- and 4-letter alphabets (every 4-byte string recurs, so each lookup's match
    distance is set by which earlier position won its slot) and short periodic bursts (period
    1..16, one slot per phase), between random bytes."""
    rng = np.random.default_rng(seed)
    parts, total = [], 0
    while total < n:
        kind = int(rng.integers(0, 4))
        m = int(rng.integers(200, 3000))
        if kind == 0:
            a = rng.choice(np.frombuffer(rng.bytes(2), np.uint8), m)
        elif kind == 1:
            a = rng.choice(np.frombuffer(rng.bytes(4), np.uint8), m)
        elif kind == 2:
            per = int(rng.integers(1, 17))
            a = np.resize(np.frombuffer(rng.bytes(per), np.uint8), int(rng.integers(70, 400)))
        else:
            a = np.frombuffer(rng.bytes(int(rng.integers(16, 200))), np.uint8)
        parts.append(a)
        total += a.size
    return np.concatenate(parts)[:n].copy()


def slots_per_window(host):
    """mean positions per distinct slot within aligned 64-position windows"""
    v = (host[:-3].astype(np.uint64) | (host[1:-2].astype(np.uint64) << np.uint64(8)) |
         (host[2:-1].astype(np.uint64) << np.uint64(16)) |
         (host[3:].astype(np.uint64) << np.uint64(24)))
    h = ((v * np.uint64(K)) & np.uint64(0xFFFFFFFF)) >> np.uint64(22)
    w = h[:h.size // 64 * 64].reshape(-1, 64)
    return float(np.mean([64.0 / np.unique(r).size for r in w]))


@pytest.mark.parametrize("seed", [7, 11, 23])
@pytest.mark.parametrize("name,seg", [("LZ4", 65536), ("LZ4_WIDE", 65536), ("ZSTD", 65536),
                                      ("DEFLATE", 59460), ("DEFLATE_DYNAMIC", 59460)])
def test_same_slot_windows_vs_oracle(eng, name, seg, seed):
    import bitar_amd
    codec = getattr(bitar_amd, "CODEC_" + name)
    n = (16 << 16) + 777
    host = same_slot_stream(n, seed)
    assert slots_per_window(host) > 2.5  # (positions per distinct slot in a window)
    data = torch.from_numpy(host).cuda()
    slab, stride, sizes = eng.compress(codec, data, seg)
    out, prod = eng.decompress(codec, slab, stride, sizes, seg)
    eng.sync()
    assert torch.equal(out[:n], data)
    P.assert_every_segment_matches_oracle(codec, data, n, seg, slab, stride, sizes)


def structured_stream(n, seed):
    """n bytes of randomly chosen stretches: runs of one byte, small-alphabet strings, periodic
    bursts, random bytes, copies from 1 B .. 60 KiB back (near, far and overlapping), zero
    pages and word-like text -- shapes whose boundaries the synthetic kinds rarely put side by
    side."""
    rng = np.random.default_rng(seed)
    out = bytearray(rng.bytes(16))
    words = [bytes(rng.integers(97, 123, int(rng.integers(2, 9)), dtype=np.uint8)) for _ in range(64)]
    while len(out) < n:
        k = int(rng.integers(0, 7))
        if k == 0:
            out += bytes([int(rng.integers(0, 256))]) * int(rng.integers(1, 600))
        elif k == 1:
            al = np.frombuffer(rng.bytes(int(rng.integers(2, 9))), np.uint8)
            out += rng.choice(al, int(rng.integers(20, 2000))).tobytes()
        elif k == 2:
            per = rng.bytes(int(rng.integers(1, 40)))
            out += (per * 200)[:int(rng.integers(8, 3000))]
        elif k == 3:
            out += rng.bytes(int(rng.integers(1, 1500)))
        elif k == 4:
            back = int(rng.integers(1, min(len(out), 61440) + 1))
            m = int(rng.integers(4, 700))
            s = len(out) - back
            for j in range(m):  # byte by byte: the copy may overlap itself
                out.append(out[s + j])
        elif k == 5:
            out += bytes(int(rng.integers(64, 5000)))
        else:
            out += b" ".join(words[int(i)] for i in rng.integers(0, 64, int(rng.integers(5, 300))))
    return np.frombuffer(bytes(out[:n]), np.uint8).copy()


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("name,seg", [("LZ4", 65536), ("LZ4_WIDE", 65536), ("ZSTD", 65536),
                                      ("DEFLATE", 59460), ("DEFLATE_DYNAMIC", 59460)])
def test_structured_fuzz_vs_oracle_and_stock(eng, name, seg, seed):
    """our frames: bit-exact against the oracle, decoded by the GPU and by the stock library"""
    import bitar_amd
    import stock_lib as S
    codec = getattr(bitar_amd, "CODEC_" + name)
    n = (24 << 16) + 12345
    host = structured_stream(n, seed)
    data = torch.from_numpy(host).cuda()
    slab, stride, sizes = eng.compress(codec, data, seg)
    out, prod = eng.decompress(codec, slab, stride, sizes, seg)
    eng.sync()
    assert torch.equal(out[:n], data)
    P.assert_every_segment_matches_oracle(codec, data, n, seg, slab, stride, sizes)
    stock = {"LZ4": S.LZ4, "LZ4_WIDE": S.LZ4, "ZSTD": S.ZSTD}.get(name, S.DEFLATE)
    P.stock_decodes_every_frame(stock, slab, stride, sizes, data, n, seg)


@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("name,levels", [("LZ4", [1]), ("DEFLATE_DYNAMIC", [1, 6, 9]),
                                         ("ZSTD", [1, 3, 9, 19])])
def test_structured_fuzz_stock_streams_decode(eng, name, levels, seed):
    """streams the stock libraries write from the same shapes, at several levels: the GPU
    decoders reproduce the input"""
    import bitar_amd
    import stock_lib as S
    codec = getattr(bitar_amd, "CODEC_" + name)
    sc = {"LZ4": S.LZ4, "ZSTD": S.ZSTD}.get(name, S.DEFLATE)
    seg = 59460 if name.startswith("DEFLATE") else 65536
    n = (12 << 16) + 999
    host = structured_stream(n, 100 + seed)
    for level in levels:
        slab_h, stride, sizes_h = S.compress(sc, host, seg, level, P.THREADS)
        nseg = sizes_h.size
        slab = torch.from_numpy(slab_h).cuda()
        sizes = torch.from_numpy(sizes_h.view(np.int32)).cuda()
        out = eng.empty(nseg * seg)
        prod = eng.empty(nseg, dtype=torch.int32)
        eng.decompress_slab_into(codec, slab, stride, sizes, nseg, seg, out, prod,
                                 capacity=nseg * seg)
        eng.sync()
        assert np.array_equal(out[:n].cpu().numpy(), host), f"level {level}"
