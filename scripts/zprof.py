#!/usr/bin/env python3
"""Phase breakdown of zstd_decompress_kernel from a ZPROF build:
BITAR_HIP_LIB=bitar_amd/lib/variants/libbitar_hip_zprof.so python scripts/zprof.py [kinds] [--stock]
--stock: decode libzstd level-1 frames (compressed on the host) instead of our own."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import bitar_amd  # noqa: E402

NAMES = ["total", "block", "lit_hdr", "tables", "seq_loop", "exec_chunk", "general_seq",
         "raw_block", "", "", "n_chunks", "n_seq", "n_general", "n_cblocks", "n_raw", ""]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    stock = "--stock" in sys.argv
    L = bitar_amd.lib()
    f = L.bitar_hip_debug_zstd_prof
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    eng = bitar_amd.Engine(0)
    eng.set_decoder_options(zstd_lanes=0)  # the wave decoder alone
    n, seg = 64 << 20, 65536
    nseg = n // seg
    for kind in [int(k) for k in (args[0] if args else "1,2,6").split(",")]:
        d = eng.empty(n)
        eng.fill(kind, 0, d)
        if stock:
            import numpy as np
            import stock_lib as S
            slab_h, stride, sizes_h = S.compress(S.ZSTD, d.cpu().numpy(), seg, 1, 16)
            slab = torch.from_numpy(slab_h).cuda()
            sizes = torch.from_numpy(sizes_h.view(np.int32)).cuda()
        else:
            slab, stride, sizes = eng.compress(bitar_amd.CODEC_ZSTD, d, seg)
        eng.sync()
        buf = (ctypes.c_ulonglong * 16)()
        f(buf, 1)
        out, prod = eng.decompress(bitar_amd.CODEC_ZSTD, slab, stride, sizes, seg)
        eng.sync()
        f(buf, 1)
        ok = torch.equal(out[:n], d)
        print(f"kind {kind} stock={stock} ok={ok} per segment:", ", ".join(
            f"{NAMES[i]}={buf[i] / nseg:.4g}" for i in range(16) if NAMES[i]), flush=True)


if __name__ == "__main__":
    main()
