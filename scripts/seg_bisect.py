#!/usr/bin/env python3
"""Where a decompress launch spends its time: time the decode of contiguous ranges of the
segments (HIP events), bisecting into the slowest range.
usage: python scripts/seg_bisect.py --codec deflate --kind 1 --seed 2000"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--codec", default="deflate")
    ap.add_argument("--kind", type=int, default=1)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--phase", default="decompress", choices=("compress", "decompress"))
    a = ap.parse_args()
    import torch
    import bitar_amd
    eng = bitar_amd.Engine(0)
    codec = {"lz4": bitar_amd.CODEC_LZ4, "deflate": bitar_amd.CODEC_DEFLATE,
             "zstd": bitar_amd.CODEC_ZSTD, "deflate_dyn": bitar_amd.CODEC_DEFLATE_DYNAMIC}[a.codec]
    seg = 59460 if a.codec.startswith("deflate") else 65536
    n = a.bytes
    nseg = (n + seg - 1) // seg
    stride = bitar_amd.slot_size(codec, seg)
    data = eng.empty(n)
    slab = eng.empty(nseg * stride)
    sizes = eng.empty(nseg, dtype=torch.int32)
    out = eng.empty(nseg * seg)
    prod = eng.empty(nseg, dtype=torch.int32)
    eng.fill(a.kind, a.seed, data)
    eng.compress_into(codec, data, seg, slab, stride, sizes, n=n)
    eng.sync()
    s = torch.cuda.current_stream()

    def t(lo, hi, reps=3):
        best = 1e9
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            if a.phase == "decompress":
                eng.decompress_slab_into(codec, slab[lo * stride:], stride, sizes[lo:], hi - lo,
                                         seg, out[lo * seg:], prod[lo:],
                                         capacity=(hi - lo) * seg)
            else:  # (the slots of segments lo.. are rewritten with the same bytes)
                nb = min(hi * seg, n) - lo * seg
                eng.compress_into(codec, data[lo * seg:], seg, slab[lo * stride:], stride,
                                  sizes[lo:], n=nb)
            e1.record(s)
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        return best

    print(json.dumps({"all": nseg, "ms": round(t(0, nseg), 3)}))
    lo, hi = 0, nseg
    while hi - lo > 64:
        mid = (lo + hi) // 2
        ta, tb = t(lo, mid), t(mid, hi)
        print(json.dumps({"range": [lo, hi], "lo_ms": round(ta, 3), "hi_ms": round(tb, 3)}))
        lo, hi = (lo, mid) if ta >= tb else (mid, hi)
    singles = sorted(((t(i, i + 1, 1), i) for i in range(lo, hi)), reverse=True)[:8]
    sz = sizes.cpu().tolist()
    print(json.dumps({"slowest_single": [(round(ms, 3), i, sz[i]) for ms, i in singles]}))


if __name__ == "__main__":
    main()
