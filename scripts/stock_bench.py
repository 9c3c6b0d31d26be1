#!/usr/bin/env python3
"""GPU decode time of streams a stock library wrote on the host (HIP events, byte-checked).
usage: python scripts/stock_bench.py [--codec lz4] [--kind 1] [--bytes N] [--level 1]"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--codec", default="lz4")
    ap.add_argument("--kind", type=int, default=1)
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--level", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import numpy as np
    import torch
    import bitar_amd
    import stock_lib as S
    eng = bitar_amd.Engine(0)
    sc = {"lz4": S.LZ4, "zstd": S.ZSTD, "deflate": S.DEFLATE}[a.codec]
    codec = {"lz4": bitar_amd.CODEC_LZ4, "zstd": bitar_amd.CODEC_ZSTD,
             "deflate": bitar_amd.CODEC_DEFLATE_DYNAMIC}[a.codec]
    seg = 59460 if a.codec == "deflate" else 65536
    n = a.bytes
    data = eng.empty(n)
    eng.fill(a.kind, 0, data)
    host = data.cpu().numpy()
    slab_h, stride, sizes_h = S.compress(sc, host, seg, a.level, 16)
    nseg = sizes_h.size
    slab = torch.from_numpy(slab_h).cuda()
    sizes = torch.from_numpy(sizes_h.view(np.int32)).cuda()
    out = eng.empty(nseg * seg)
    prod = eng.empty(nseg, dtype=torch.int32)
    s = torch.cuda.current_stream()
    ts = []
    for r in range(a.reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        eng.decompress_slab_into(codec, slab, stride, sizes, nseg, seg, out, prod, capacity=nseg * seg)
        e1.record(s)
        torch.cuda.synchronize()
        if r:
            ts.append(e0.elapsed_time(e1))
    eng.sync()
    ok = bool(torch.equal(out[:n], data))
    print(f'{{"codec": "{a.codec}", "kind": {a.kind}, "level": {a.level}, "ok": {str(ok).lower()}, '
          f'"decompress_ms": {min(ts):.3f}, "gib_s": {n / 2**30 / (min(ts) / 1e3):.1f}}}')


if __name__ == "__main__":
    main()
