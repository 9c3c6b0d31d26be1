#!/usr/bin/env python3
"""Run one codec kernel a few times on one input kind (for rocprofv3 PMC passes).
usage: python scripts/prof_one.py --kind 5 --codec lz4 --which decompress"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", type=int, default=5)
    ap.add_argument("--codec", default="lz4")
    ap.add_argument("--which", default="decompress")
    ap.add_argument("--bytes", type=int, default=256 << 20)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    import torch
    import bitar_amd
    eng = bitar_amd.Engine(0)
    codec = {"lz4": bitar_amd.CODEC_LZ4, "deflate": bitar_amd.CODEC_DEFLATE,
             "deflate_dyn": bitar_amd.CODEC_DEFLATE_DYNAMIC, "zstd": bitar_amd.CODEC_ZSTD}[a.codec]
    seg = 59460 if a.codec.startswith("deflate") else 65536
    n = a.bytes
    nseg = (n + seg - 1) // seg
    stride = bitar_amd.slot_size(codec, seg)
    data = eng.empty(n)
    slab = eng.empty(nseg * stride)
    sizes = eng.empty(nseg, dtype=torch.int32)
    out = eng.empty(nseg * seg)
    prod = eng.empty(nseg, dtype=torch.int32)
    eng.fill(a.kind, 0, data)
    eng.compress_into(codec, data, seg, slab, stride, sizes, n=n)
    for _ in range(a.reps):
        if a.which == "compress":
            eng.compress_into(codec, data, seg, slab, stride, sizes, n=n)
        else:
            eng.decompress_slab_into(codec, slab, stride, sizes, nseg, seg, out, prod,
                                     capacity=nseg * seg)
    eng.sync()
    assert torch.equal(out[:n], data) or a.which == "compress"


if __name__ == "__main__":
    main()
