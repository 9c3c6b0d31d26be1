"""ctypes wrapper over oracle/_build/libbitar_stock.so: the stock liblz4 / zlib / libzstd of
this image, segment-parallel on host threads (oracle/stock_codecs.c).

Baseline / test infrastructure only: bench.py's cpu_baseline leg and the host-side
preparation of stock streams for the GPU decode legs; tests use it for stock-stream parity.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
STOCK_SO = os.path.join(ORACLE_DIR, "_build", "libbitar_stock.so")

LZ4, DEFLATE, ZSTD = 1, 2, 3
NAMES = {LZ4: "liblz4 1.9.3 LZ4_compress_default", DEFLATE: "zlib 1.2.11 raw deflate",
         ZSTD: "libzstd"}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(STOCK_SO):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = ctypes.CDLL(STOCK_SO)
        vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        L.sc_bound.restype = u64
        L.sc_bound.argtypes = [i32, u32]
        L.sc_compress.restype = i32
        L.sc_compress.argtypes = [i32, i32, vp, u64, u32, vp, u64, vp, i32]
        L.sc_decompress.restype = i32
        L.sc_decompress.argtypes = [i32, vp, u64, vp, u64, u32, vp, i32]
        _lib = L
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(0)


def stride_for(codec, seg):
    """A slot stride (256-B multiple) that holds any compressed segment of seg bytes."""
    return (int(lib().sc_bound(codec, seg)) + 255) & ~255


def compress(codec, data, seg, level=1, threads=1, stride=None):
    """-> (slab uint8 [nseg*stride], stride, sizes uint32 [nseg])."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    nseg = (data.size + seg - 1) // seg
    stride = stride or stride_for(codec, seg)
    slab = np.empty(max(nseg * stride, 1), np.uint8)
    sizes = np.zeros(max(nseg, 1), np.uint32)
    r = lib().sc_compress(codec, level, _p(data), data.size, seg, _p(slab), stride, _p(sizes),
                          threads)
    if r != 0:
        raise RuntimeError(f"stock compress failed ({NAMES[codec]})")
    return slab, stride, sizes[:nseg]


def decompress(codec, slab, stride, sizes, n, seg, threads=1, out=None):
    out = np.empty(max(n, 1), np.uint8) if out is None else out
    r = lib().sc_decompress(codec, _p(slab), stride, _p(sizes), n, seg, _p(out), threads)
    if r != 0:
        raise RuntimeError(f"stock decompress failed ({NAMES[codec]})")
    return out[:n]
