#!/usr/bin/env python3
"""Phase cycles of zstd_decompress_kernel from a ZPROF build (scripts/build_variant.sh zprof
-DZPROF; BITAR_HIP_LIB=bitar_amd/lib/variants/libbitar_hip_zprof.so): one 1 GiB decode of
kind $KIND, per-phase s_memtime cycles summed over waves (lane 0), per segment.
Phases: 0 all, 1 compressed blocks, 2 literal sections, 3 sequence table headers,
4 sequences decoded in the wave, 5 exec chunks, 6 general-path copies, 7 raw blocks;
counts 10 exec chunks, 11 sequences, 12 general copies, 13 compressed blocks, 14 raw."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bitar_amd  # noqa: E402

kind = int(os.environ.get("KIND", "2"))
L = bitar_amd.lib()
f = L.bitar_hip_debug_zstd_prof
f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
eng = bitar_amd.Engine(0)
seg, n = 65536, 1 << 30
nseg = n // seg
codec = bitar_amd.CODEC_ZSTD
stride = bitar_amd.slot_size(codec, seg)
data, slab = eng.empty(n), eng.empty(nseg * stride)
sizes = eng.empty(nseg, dtype=torch.int32)
out, prod = eng.empty(n), eng.empty(nseg, dtype=torch.int32)
eng.fill(kind, 0, data)
eng.compress_into(codec, data, seg, slab, stride, sizes, n=n)
buf = (ctypes.c_ulonglong * 16)()
for rep in range(2):
    f(buf, 1)
    eng.decompress_slab_into(codec, slab, stride, sizes, nseg, seg, out, prod, capacity=n)
    eng.sync()
    torch.cuda.synchronize()
    f(buf, 0)
print({k: round(buf[k] / nseg, 1) for k in range(16) if buf[k]})
print("ok", bool(torch.equal(out, data)))
