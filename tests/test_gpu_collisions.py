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


@pytest.mark.parametrize("name,seg", [("LZ4", 65536), ("LZ4_WIDE", 65536), ("ZSTD", 65536),
                                      ("DEFLATE", 59460), ("DEFLATE_DYNAMIC", 59460)])
def test_same_slot_windows_vs_oracle(eng, name, seg):
    import bitar_amd
    codec = getattr(bitar_amd, "CODEC_" + name)
    n = (16 << 16) + 777
    host = same_slot_stream(n, 7)
    assert slots_per_window(host) > 2.5  # (positions per distinct slot in a window)
    data = torch.from_numpy(host).cuda()
    slab, stride, sizes = eng.compress(codec, data, seg)
    out, prod = eng.decompress(codec, slab, stride, sizes, seg)
    eng.sync()
    assert torch.equal(out[:n], data)
    P.assert_every_segment_matches_oracle(codec, data, n, seg, slab, stride, sizes)
