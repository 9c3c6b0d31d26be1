#!/usr/bin/env python3
"""LZ4 decoder batch diagnostics: run with a -DBITAR_LZ4D_PROFILE=1 library
   (scripts/build_variant.sh prof "-DBITAR_LZ4D_PROFILE=1"; BITAR_HIP_LIB=...) and print, per
   input kind, batches per segment, output bytes per batch, the share of output the batches
   produced, general-path sequences and why walks ended."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bitar_amd
    kinds = [int(k) for k in (sys.argv[1] if len(sys.argv) > 1 else "1,2,5,6").split(",")]
    eng = bitar_amd.Engine(0, flags=bitar_amd.FLAG_COUNT_PATHS)
    n, seg = 256 << 20, 65536
    nseg = n // seg
    codec = bitar_amd.CODEC_LZ4
    stride = bitar_amd.slot_size(codec, seg)
    data, slab = eng.empty(n), eng.empty(nseg * stride)
    sizes = eng.empty(nseg, dtype=torch.int32)
    out, prod = eng.empty(n), eng.empty(nseg, dtype=torch.int32)
    for kind in kinds:
        eng.fill(kind, 0, data)
        eng.compress_into(codec, data, seg, slab, stride, sizes, n=n)
        eng.path_counters()
        eng.decompress_slab_into(codec, slab, stride, sizes, nseg, seg, out, prod, capacity=n)
        c = eng.path_counters()
        assert torch.equal(out, data)
        b = max(c["lz4_batches"], 1)
        print(json.dumps({"kind": kind, "batches_per_seg": round(c["lz4_batches"] / nseg, 1),
                          "bytes_per_batch": round(c["lz4_batch_bytes"] / b, 1),
                          "batch_share": round(c["lz4_batch_bytes"] / n, 3),
                          "general_seqs_per_seg": round(c["lz4_general_seqs"] / nseg, 1),
                          "stop_parse": round(c["lz4_stop_parse"] / b, 3),
                          "stop_ineligible": round(c["lz4_stop_ineligible"] / b, 3)}))
    eng.close()


if __name__ == "__main__":
    main()
