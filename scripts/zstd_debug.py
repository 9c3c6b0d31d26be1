#!/usr/bin/env python3
"""Debug aid: Zstd round trip of kind-K input under each decoder option, listing the segments
whose decode differs from the input with their frame structure."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))


def main():
    import torch
    import bitar_amd
    from test_oracle import _zstd_blocks
    kind = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    n = int(sys.argv[2]) if len(sys.argv) > 2 else (256 << 20)
    seg = 65536
    eng = bitar_amd.Engine(0)
    data = eng.empty(n)
    eng.fill(kind, 0, data)
    slab, stride, sizes = eng.compress(bitar_amd.CODEC_ZSTD, data, seg)
    eng.sync()
    host = data.cpu().numpy()
    sl = slab.cpu().numpy()
    sz = sizes.cpu().numpy().astype(np.uint32)
    for lanes, seq in ((16, 1), (64, 0), (0, 1), (0, 0), (16, 0)):
        eng.set_decoder_options(zstd_lanes=lanes, zstd_seq=seq, count_paths=1)
        out, prod = eng.decompress(bitar_amd.CODEC_ZSTD, slab, stride, sizes, seg)
        try:
            eng.sync()
            err = None
        except bitar_amd.BitarError as e:
            err = str(e)
        c = eng.path_counters()
        o = out.cpu().numpy()
        p = prod.cpu().numpy().view(np.uint32)
        bad = []
        for i in range(sz.size):
            a = o[i * seg:(i + 1) * seg]
            b = host[i * seg:(i + 1) * seg]
            if p[i] != b.size or not np.array_equal(a[:b.size], b):
                bad.append(i)
        print(f"lanes={lanes} seq={seq} err={err} bad={len(bad)} paths={ {k: v for k, v in c.items() if v} }")
        for i in bad[:4]:
            f = sl[i * stride:i * stride + sz[i]].tobytes()
            b = host[i * seg:(i + 1) * seg]
            a = o[i * seg:(i + 1) * seg]
            d = np.nonzero(a[:b.size] != b)[0]
            bl = _zstd_blocks(f)
            print(f"  seg {i} produced {p[i]} first diff {d[:1].tolist()} ndiff {d.size} blocks",
                  [(x['block'], x.get('lit_type'), x.get('nlit'), x.get('nseq'), x.get('modes')) for x in bl])
    eng.close()


if __name__ == "__main__":
    main()
