#!/usr/bin/env python3
"""Timing experiment: one 1 GiB call against the same 1 GiB as K concurrent calls of 1/K each
on K queue-pair streams (compress and decompress phases timed separately, bracketed by
device syncs).  usage: python scripts/split_bench.py [--codec zstd] [--kind 2] [--k 2]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--codec", default="zstd")
    ap.add_argument("--kind", type=int, default=2)
    ap.add_argument("--ks", default="1,2,4")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    import bitar_amd
    eng = bitar_amd.Engine(0, num_streams=4)
    codec = {"lz4": bitar_amd.CODEC_LZ4, "zstd": bitar_amd.CODEC_ZSTD,
             "deflate": bitar_amd.CODEC_DEFLATE,
             "deflate_dyn": bitar_amd.CODEC_DEFLATE_DYNAMIC}[a.codec]
    seg = 59460 if a.codec.startswith("deflate") else 65536
    n = 1 << 30
    nseg = (n + seg - 1) // seg
    stride = bitar_amd.slot_size(codec, seg)
    data, slab = eng.empty(n), eng.empty(nseg * stride)
    sizes = eng.empty(nseg, dtype=torch.int32)
    out, prod = eng.empty(nseg * seg), eng.empty(nseg, dtype=torch.int32)
    eng.fill(a.kind, 0, data)
    for k in [int(x) for x in a.ks.split(",")]:
        per = (nseg + k - 1) // k
        parts = [(j * per, min(per, nseg - j * per)) for j in range(k)]
        streams = [None] if k == 1 else [eng.queue_pair_stream(j) for j in range(k)]
        tc, td = [], []
        for r in range(a.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for (s0, c), st in zip(parts, streams):
                nb = min(c * seg, n - s0 * seg)
                eng.compress_into(codec, data[s0 * seg:], seg, slab[s0 * stride:], stride,
                                  sizes[s0:], n=nb, stream=st)
            for st in streams:
                eng.sync(st)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            for (s0, c), st in zip(parts, streams):
                eng.decompress_slab_into(codec, slab[s0 * stride:], stride, sizes[s0:], c, seg,
                                         out[s0 * seg:], prod[s0:], capacity=c * seg, stream=st)
            for st in streams:
                eng.sync(st)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            if r:
                tc.append(t1 - t0)
                td.append(t2 - t1)
        ok = bool(torch.equal(out[:n], data))
        print(json.dumps({"codec": a.codec, "kind": a.kind, "k": k, "ok": ok,
                          "compress_ms": round(min(tc) * 1e3, 3),
                          "decompress_ms": round(min(td) * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
