import sys, os, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import bitar_amd, stock_lib as S, oracle_lib as O
eng = bitar_amd.Engine(0)
n = 1 << 30
for name, sc, seg, kind, codec in (("lz4", S.LZ4, 65536, 1, 1), ("deflate", S.DEFLATE, 59460, 1, 2), ("zstd", S.ZSTD, 65536, 2, 3)):
    data = eng.empty(n); eng.fill(kind, 0, data)
    host = data.cpu().numpy()
    slab_h, stride, sizes_h = S.compress(sc, host, seg, 1, 16)
    nseg = sizes_h.size
    slab = torch.from_numpy(slab_h).cuda(); sizes = torch.from_numpy(sizes_h.view(np.int32)).cuda()
    out = eng.empty(nseg * seg); prod = eng.empty(nseg, dtype=torch.int32)
    for _ in range(4): eng.decompress_slab_into(codec, slab, stride, sizes, nseg, seg, out, prod, capacity=nseg * seg)
    torch.cuda.synchronize()
    try:
        eng.sync(); print(name, "ok", bool(torch.equal(out[:n], data)))
    except Exception as e:
        p = prod.cpu().numpy().view(np.uint32)
        bad = np.nonzero(p == 0xFFFFFFFF)[0]
        print(name, "FAILED", e, "bad segs", bad[:10], len(bad))
        for i in bad[:3]:
            blob = slab_h[i*stride:i*stride+sizes_h[i]].tobytes()
            if codec == 1: r, ref = O.lz4_decompress(blob, seg)
            elif codec == 2: r, ref = O.inflate(blob, seg)
            else: r, ref = O.zstd_decompress(blob, seg)
            print("  oracle on seg", i, r, len(ref))
