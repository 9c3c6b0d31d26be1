"""Whole-call parity helpers for the GPU tests: every segment of a (full-size) GPU compress
call against the oracle's encoder, in chunks of <= 1 GiB of input so host memory stays
bounded; every GPU frame decoded by the stock library.  Test infrastructure only."""
import os

import numpy as np

import oracle_lib as O
import stock_lib as S

THREADS = min(16, os.cpu_count() or 1)  # the GPU box grants 16 cores (cgroup quota)


def _down(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def assert_every_segment_matches_oracle(codec, data, n, seg, slab, stride, sizes,
                                        chunk=1 << 30):
    """data: device uint8 tensor (>= n bytes), slab: device slab (stride per segment), sizes:
    device int32 tensor -- the GPU's output of one compress call.  Compares the sizes of all
    segments and the bytes of every slot with the oracle's encoding of the same input."""
    nseg = (n + seg - 1) // seg
    gs_all = _down(sizes).astype(np.uint32)[:nseg]
    per = max(1, chunk // seg)
    col = np.arange(stride, dtype=np.uint32)[None, :]
    for a in range(0, nseg, per):
        b = min(nseg, a + per)
        lo, hi = a * seg, min(n, b * seg)
        host = _down(data[lo:hi])
        r, oslab, osz = O.compress_segments(codec, host, seg, stride, THREADS)
        assert r == 0
        gs = gs_all[a:b]
        bad = np.nonzero(gs != osz)[0]
        assert bad.size == 0, f"segment {a + int(bad[0])}: size {gs[bad[0]]} != {osz[bad[0]]}"
        g = _down(slab[a * stride:b * stride]).reshape(-1, stride)
        o = oslab.reshape(-1, stride)
        for r0 in range(0, b - a, 2048):
            r1 = min(b - a, r0 + 2048)
            m = col < osz[r0:r1, None]
            if not np.array_equal(g[r0:r1][m], o[r0:r1][m]):
                for i in range(r0, r1):
                    k = int(osz[i])
                    assert np.array_equal(g[i, :k], o[i, :k]), f"segment {a + i}"
        del host, oslab, g, o
    return gs_all


def stock_decodes_every_frame(stock_codec, slab, stride, sizes, data, n, seg):
    """Decode every GPU frame of the call with the stock library (zlib raw inflate, liblz4
    LZ4_decompress_safe, libzstd ZSTD_decompress, multi-threaded) and compare with the input."""
    s = _down(slab)
    z = _down(sizes).astype(np.uint32)[:(n + seg - 1) // seg]
    out = S.decompress(stock_codec, s, stride, z, n, seg, threads=THREADS)
    assert np.array_equal(out, _down(data[:n]))
