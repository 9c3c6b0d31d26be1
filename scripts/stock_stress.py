"""Repeat the bench's stock-stream GPU decodes (1 GiB each: liblz4, zlib-1, libzstd-1) many
times and report any failing segment with the oracle's verdict on it (diagnostics for an
intermittent failure seen once in bench.py's stock_decode leg)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, '.')
sys.path.insert(0, 'tests')
import bitar_amd  # noqa: E402
import oracle_lib as O  # noqa: E402
import stock_lib as S  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
eng = bitar_amd.Engine(0, num_streams=4)
n = 1 << 30
for name, sc, seg, kind, codec in (("zstd", S.ZSTD, 65536, 2, 3), ("lz4", S.LZ4, 65536, 1, 1),
                                   ("deflate", S.DEFLATE, 59460, 1, 2)):
    data = eng.empty(n)
    eng.fill(kind, 0, data)
    host = data.cpu().numpy()
    slab_h, stride, sizes_h = S.compress(sc, host, seg, 1, 16)
    nseg = sizes_h.size
    slab = torch.from_numpy(slab_h).cuda()
    sizes = torch.from_numpy(sizes_h.view(np.int32)).cuda()
    out = eng.empty(nseg * seg)
    prod = eng.empty(nseg, dtype=torch.int32)
    fails = 0
    t0 = time.time()
    for r in range(reps):
        eng.decompress_slab_into(codec, slab, stride, sizes, nseg, seg, out, prod,
                                 capacity=nseg * seg)
        torch.cuda.synchronize()
        try:
            eng.sync()
            if not torch.equal(out[:n], data):
                print(name, r, "WRONG BYTES", flush=True)
                fails += 1
        except bitar_amd.BitarError as e:
            fails += 1
            p = prod.cpu().numpy().view(np.uint32)
            bad = np.nonzero(p == 0xFFFFFFFF)[0]
            print(name, r, "FAILED", e, "segments", bad[:10].tolist(), bad.size, flush=True)
            for i in bad[:3]:
                blob = slab_h[i * stride:i * stride + sizes_h[i]].tobytes()
                f = {1: O.lz4_decompress, 2: O.inflate, 3: O.zstd_decompress}[codec]
                rr, ref = f(blob, seg)
                print("   oracle on segment", int(i), rr, len(ref), flush=True)
    print(name, "reps", reps, "fails", fails, "secs %.1f" % (time.time() - t0), flush=True)
