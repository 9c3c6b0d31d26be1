"""ctypes wrapper over oracle/_build/libbitar_oracle.so -- the CPU checker.

Test infrastructure only (see oracle/bitar_oracle.h): the product never imports this.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "_build", "libbitar_oracle.so")

CODEC_LZ4 = 1
CODEC_DEFLATE = 2
CODEC_ZSTD = 3
CODEC_DEFLATE_DYN = 4
CODEC_LZ4_WIDE = 5  # the wide LZ4 parse (16 KiB history, 4096-entry table)

BO_OK = 0
BO_ERR_INVALID = -4
BO_ERR_IO = -5
BO_ERR_CAPACITY = -6

KIND_RANDOM, KIND_MIXED, KIND_ARROW, KIND_CONST, KIND_PERIODIC = 0, 1, 2, 3, 4

_lib = None


def lib():
    global _lib
    if _lib is None:
        # make is a no-op when the library is current (rebuilds a stale one)
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = ctypes.CDLL(ORACLE_SO)
        u8p = ctypes.c_void_p
        L.bo_compressed_seg_size.restype = ctypes.c_uint32
        L.bo_compressed_seg_size.argtypes = [ctypes.c_uint32]
        L.bo_lz4_bound.restype = ctypes.c_uint32
        L.bo_lz4_bound.argtypes = [ctypes.c_uint32]
        L.bo_deflate_bound.restype = ctypes.c_uint32
        L.bo_deflate_bound.argtypes = [ctypes.c_uint32]
        L.bo_zstd_bound.restype = ctypes.c_uint32
        L.bo_zstd_bound.argtypes = [ctypes.c_uint32]
        for name in ("bo_lz4_decompress_block", "bo_lz4_compress_block", "bo_inflate_raw",
                     "bo_deflate_fixed_block", "bo_zstd_decompress", "bo_zstd_compress_block",
                     "bo_deflate_dynamic_block", "bo_lz4_wide_compress_block"):
            f = getattr(L, name)
            f.restype = ctypes.c_int
            f.argtypes = [u8p, ctypes.c_uint32, u8p, ctypes.c_uint32,
                          ctypes.POINTER(ctypes.c_uint32)]
        L.bo_compress.restype = ctypes.c_int
        L.bo_compress.argtypes = [ctypes.c_int, u8p, ctypes.c_uint64, ctypes.c_uint32, u8p,
                                  ctypes.c_uint64, u8p, ctypes.POINTER(ctypes.c_uint32),
                                  ctypes.c_int]
        L.bo_decompress.restype = ctypes.c_int
        L.bo_decompress.argtypes = [ctypes.c_int, u8p, u8p, ctypes.c_uint32, ctypes.c_uint32,
                                    u8p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64),
                                    u8p, ctypes.c_int]
        L.bo_deflate_dynamic_mode.restype = ctypes.c_int
        L.bo_deflate_dynamic_mode.argtypes = [u8p, ctypes.c_uint32]
        L.bo_huff_lengths.restype = None
        L.bo_huff_lengths.argtypes = [u8p, ctypes.c_int, ctypes.c_int, u8p]
        L.bo_fill.restype = None
        L.bo_fill.argtypes = [ctypes.c_int, ctypes.c_uint64, u8p, ctypes.c_uint64]
        _lib = L
    return _lib


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(0)


def fill(kind, seed, n):
    out = np.empty(max(n, 1), dtype=np.uint8)
    lib().bo_fill(kind, seed, _ptr(out), n)
    return out[:n]


def compressed_seg_size(seg):
    return lib().bo_compressed_seg_size(seg)


def lz4_bound(n):
    return lib().bo_lz4_bound(n)


def deflate_bound(n):
    return lib().bo_deflate_bound(n)


def _block(fn, src, cap):
    src = np.ascontiguousarray(np.frombuffer(bytes(src), dtype=np.uint8)) \
        if not isinstance(src, np.ndarray) else np.ascontiguousarray(src)
    dst = np.zeros(max(cap, 1), dtype=np.uint8)
    out = ctypes.c_uint32(0)
    r = fn(_ptr(src), src.size, _ptr(dst), cap, ctypes.byref(out))
    return r, (dst[:out.value].tobytes() if r == 0 else None)


def lz4_decompress(src, cap):
    return _block(lib().bo_lz4_decompress_block, src, cap)


def lz4_compress(src):
    n = len(src)
    return _block(lib().bo_lz4_compress_block, src, lz4_bound(n))


def lz4_wide_compress(src):
    """the wide LZ4 parse (BITAR_HIP_CODEC_LZ4_WIDE)"""
    n = len(src)
    return _block(lib().bo_lz4_wide_compress_block, src, lz4_bound(n))


def inflate(src, cap):
    return _block(lib().bo_inflate_raw, src, cap)


def deflate_fixed(src):
    return _block(lib().bo_deflate_fixed_block, src, deflate_bound(len(src)))


def deflate_dynamic(src):
    return _block(lib().bo_deflate_dynamic_block, src, deflate_bound(len(src)))


def deflate_dynamic_mode(src):
    a = np.ascontiguousarray(np.frombuffer(bytes(src), dtype=np.uint8))
    return lib().bo_deflate_dynamic_mode(_ptr(a), a.size)


def huff_lengths(freq, maxlen):
    f = np.ascontiguousarray(freq, dtype=np.uint32)
    out = np.zeros(f.size, np.uint8)
    lib().bo_huff_lengths(_ptr(f), f.size, maxlen, _ptr(out))
    return out


def zstd_bound(n):
    return int(lib().bo_zstd_bound(n))


def zstd_decompress(src, cap):
    return _block(lib().bo_zstd_decompress, src, cap)


def zstd_compress(src):
    return _block(lib().bo_zstd_compress_block, src, zstd_bound(len(src)))


def compress_segments(codec, data, seg, stride, threads=1):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    nseg = (data.size + seg - 1) // seg
    slab = np.zeros(max(nseg * stride, 1), dtype=np.uint8)
    sizes = np.zeros(max(nseg, 1), dtype=np.uint32)
    n_out = ctypes.c_uint32(0)
    r = lib().bo_compress(codec, _ptr(data), data.size, seg, _ptr(slab), stride, _ptr(sizes),
                          ctypes.byref(n_out), threads)
    return r, slab, sizes[:n_out.value]


def decompress_segments(codec, blobs, seg, capacity, threads=1):
    """blobs: list of numpy uint8 arrays (compressed segments)."""
    nseg = len(blobs)
    keep = [np.ascontiguousarray(b, dtype=np.uint8) for b in blobs]
    ptrs = np.array([b.ctypes.data for b in keep] or [0], dtype=np.uint64)
    sizes = np.array([b.size for b in keep] or [0], dtype=np.uint32)
    out = np.zeros(max(capacity, 1), dtype=np.uint8)
    produced = np.zeros(max(nseg, 1), dtype=np.uint32)
    total = ctypes.c_uint64(0)
    r = lib().bo_decompress(codec, _ptr(ptrs), _ptr(sizes), nseg, seg, _ptr(out), capacity,
                            ctypes.byref(total), _ptr(produced), threads)
    return r, out[:total.value], produced[:nseg]
