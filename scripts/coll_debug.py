#!/usr/bin/env python3
"""Debug aid: the collision-test input (tests/test_gpu_collisions.py) through each codec:
per segment, GPU frame vs the oracle's encoding, oracle decode of the GPU frame, GPU decode."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))


def main():
    import torch
    import bitar_amd
    import oracle_lib as O
    from test_gpu_collisions import same_slot_stream
    name = sys.argv[1] if len(sys.argv) > 1 else "ZSTD"
    codec = getattr(bitar_amd, "CODEC_" + name)
    seg = 59460 if name.startswith("DEFLATE") else 65536
    n = (16 << 16) + 777
    host = same_slot_stream(n, 7)
    eng = bitar_amd.Engine(0)
    data = torch.from_numpy(host).cuda()
    slab, stride, sizes = eng.compress(codec, data, seg)
    eng.sync()
    sl = slab.cpu().numpy()
    sz = sizes.cpu().numpy().astype(np.uint32)
    nseg = (n + seg - 1) // seg
    r, oslab, osz = O.compress_segments(codec, host, seg, stride, 1)
    print("compress rc", r, "gpu sizes", sz[:nseg].tolist())
    print("oracle sizes", osz[:nseg].tolist())
    for i in range(nseg):
        g = sl[i * stride:i * stride + sz[i]]
        o = oslab[i * stride:i * stride + osz[i]]
        same = sz[i] == osz[i] and np.array_equal(g, o)
        first = -1
        if not same:
            m = min(sz[i], osz[i])
            d = np.nonzero(g[:m] != o[:m])[0]
            first = int(d[0]) if d.size else m
        plain = host[i * seg:(i + 1) * seg]
        rc, dec = O.zstd_decompress(g.tobytes(), plain.size) if name == "ZSTD" else (None, None)
        ok = None if rc is None else (rc == 0 and np.array_equal(np.frombuffer(dec, np.uint8), plain))
        print(f"seg {i}: same_as_oracle {same} first_diff {first} oracle_decodes_gpu_frame {ok} rc {rc}")
    out, prod = eng.decompress(codec, slab, stride, sizes, seg)
    torch.cuda.synchronize()
    p = prod.cpu().numpy().view(np.uint32)
    print("gpu decode produced", p[:nseg].tolist())
    try:
        eng.sync()
    except bitar_amd.BitarError as e:
        print("gpu decode error", e)


if __name__ == "__main__":
    main()
