#!/usr/bin/env python3
"""Per-kernel throughput sweep over input kinds (HBM-resident, HIP-event timed).
usage: python scripts/kernel_bench.py [--kinds 0,1,5,6] [--codec lz4] [--bytes N]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kinds", default="0,1,2,5,6")
    ap.add_argument("--codec", default="lz4")
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--seg", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    import torch
    import bitar_amd
    eng = bitar_amd.Engine(0)
    codec = {"lz4": bitar_amd.CODEC_LZ4, "deflate": bitar_amd.CODEC_DEFLATE,
             "zstd": bitar_amd.CODEC_ZSTD, "deflate_dyn": bitar_amd.CODEC_DEFLATE_DYNAMIC}[a.codec]
    seg = a.seg or (59460 if a.codec.startswith("deflate") else 65536)
    n = a.bytes
    nseg = (n + seg - 1) // seg
    stride = bitar_amd.slot_size(codec, seg)
    data = eng.empty(n)
    slab = eng.empty(nseg * stride)
    sizes = eng.empty(nseg, dtype=torch.int32)
    out = eng.empty(nseg * seg)
    prod = eng.empty(nseg, dtype=torch.int32)
    s = torch.cuda.current_stream()
    for kind in [int(k) for k in a.kinds.split(",")]:
        eng.fill(kind, a.seed, data)
        tc, td = [], []
        for r in range(a.reps + 1):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record(s)
            eng.compress_into(codec, data, seg, slab, stride, sizes, n=n)
            e[1].record(s)
            eng.decompress_slab_into(codec, slab, stride, sizes, nseg, seg, out, prod,
                                     capacity=nseg * seg)
            e[2].record(s)
            torch.cuda.synchronize()
            if r:
                tc.append(e[0].elapsed_time(e[1]))
                td.append(e[1].elapsed_time(e[2]))
        try:
            eng.sync()
            ok = bool(torch.equal(out[:n], data))
        except bitar_amd.BitarError:  # (timing variants that cut the encoder short)
            ok = False
        C = int(sizes.to(torch.int64).sum().item())
        tcm, tdm = min(tc), min(td)
        print(json.dumps({"kind": kind, "codec": a.codec, "ratio": round(n / C, 3), "ok": ok,
                          "compress_ms": round(tcm, 3), "decompress_ms": round(tdm, 3),
                          "compress_GiBs": round(n / 2**30 / (tcm / 1e3), 2),
                          "decompress_GiBs": round(n / 2**30 / (tdm / 1e3), 2),
                          "decompress_alg_GBs": round((n + C) / (tdm / 1e3) / 1e9, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
