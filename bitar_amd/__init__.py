"""bitar_amd -- MI355X-native segment codec engine (Python host side).

The product is libbitar_hip.so (C ABI in include/bitar_hip.h, HIP kernels in csrc/); the
bitar-shaped C++ front-end lives in cpp/.  This module binds the C ABI with ctypes for the
Python callers (tests, bench.py, __graft_entry__).  torch is used only as plumbing:
device memory and streams.  There is no CPU fallback: if the HIP library is missing or
no gfx950 device is visible, the calls raise.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BITAR_HIP_LIB") or os.path.join(_HERE, "lib", "libbitar_hip.so")

CODEC_LZ4 = 1
CODEC_DEFLATE = 2
CODEC_ZSTD = 3
CODEC_DEFLATE_DYNAMIC = 4  # HuffmanEncoding::DYNAMIC (decoded as CODEC_DEFLATE)
CODEC_LZ4_WIDE = 5  # LZ4 blocks from the wide parse (16 KiB history): the ratio operating point
SEGMENT_ERROR = 0xFFFFFFFF
CHECKSUM_CRC32, CHECKSUM_ADLER32, CHECKSUM_CRC32_ADLER32 = 1, 2, 3
MAX_SEG_SIZE = 65536
# bitar_hip_config.flags (initial decoder options of a context)
FLAG_INFLATE_WAVE_ONLY, FLAG_ZSTD_WAVE_ONLY, FLAG_ZSTD_LANE_EXEC, FLAG_COUNT_PATHS = 1, 2, 4, 8
FLAG_PLAIN_ORDER = 0x10  # segment i is workgroup i (no cost-ordered dispatch; same output)
FLAG_ZSTD_SERIAL = 0x20  # Zstd literals and phase A in series (default: side by side)
# bitar_hip_path_counter indices
PATHS = ("inflate_wave", "inflate_wave_reject", "inflate_batch_segs", "inflate_batches",
         "zstd_wave", "zstd_handed", "zstd_seqdec", "zstd_seqdec_reject", "zstd_exec",
         "zstd_exec_reject", "lz4_far",
         # LZ4 batch diagnostics (a -DBITAR_LZ4D_PROFILE=1 build only)
         "lz4_batches", "lz4_batch_bytes", "lz4_general_seqs", "lz4_stop_parse",
         "lz4_stop_ineligible")
PATH_COUNT = 16


class DecoderOptions(ctypes.Structure):
    """bitar_hip_decoder_options (include/bitar_hip.h)"""
    _fields_ = [("inflate_lanes", ctypes.c_uint32), ("zstd_lanes", ctypes.c_uint32),
                ("zstd_seq", ctypes.c_uint32), ("count_paths", ctypes.c_uint32)]

# negated arrow::StatusCode (reference src/include/util.h:157-205)
STATUS_NAMES = {0: "OK", -1: "OutOfMemory", -4: "Invalid", -5: "IOError", -6: "CapacityError",
                -8: "Cancelled", -9: "UnknownError", -10: "NotImplemented"}


class BitarError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{STATUS_NAMES.get(code, code)}: {msg}")
        self.code = code


_lib = None


def build(verbose=False):
    """Compile libbitar_hip.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    import subprocess
    out = None if verbose else subprocess.DEVNULL
    subprocess.check_call(["make", "-s", "-j8", "-C", _HERE], stdout=out)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise BitarError(-10, f"{LIB_PATH} is not built (run bitar_amd.build())")
    L = ctypes.CDLL(LIB_PATH)
    vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    sig = {
        "bitar_hip_abi_version": (i32, []),
        "bitar_hip_last_error": (ctypes.c_char_p, []),
        "bitar_hip_device_count": (i32, [ctypes.POINTER(i32)]),
        "bitar_hip_open": (i32, [i32, vp, ctypes.POINTER(vp)]),
        "bitar_hip_close": (i32, [vp]),
        "bitar_hip_stream": (i32, [vp, u32, ctypes.POINTER(vp)]),
        "bitar_hip_device": (i32, [vp, ctypes.POINTER(i32)]),
        "bitar_hip_slot_size": (u64, [u32, u32]),
        "bitar_hip_max_distance": (u32, [u32]),
        "bitar_hip_alloc": (i32, [vp, u64, ctypes.POINTER(vp)]),
        "bitar_hip_free": (i32, [vp, vp]),
        "bitar_hip_host_alloc": (i32, [vp, u64, ctypes.POINTER(vp)]),
        "bitar_hip_host_free": (i32, [vp, vp]),
        "bitar_hip_memcpy": (i32, [vp, vp, vp, u64, vp]),
        "bitar_hip_compress": (i32, [vp, vp, u32, vp, u64, u32, vp, u64, vp]),
        "bitar_hip_compress_scattered": (i32, [vp, vp, u32, vp, u64, u32, vp, u64, vp]),
        "bitar_hip_pointer_info": (i32, [vp, ctypes.POINTER(i32), ctypes.POINTER(i32)]),
        "bitar_hip_decompress": (i32, [vp, vp, u32, vp, vp, u32, u32, vp, u64, vp]),
        "bitar_hip_decompress_slab": (i32, [vp, vp, u32, vp, u64, vp, u32, u32, vp, u64, vp]),
        "bitar_hip_sync": (i32, [vp, vp]),
        "bitar_hip_pack": (i32, [vp, vp, vp, u64, vp, u32, vp, vp]),
        "bitar_hip_fill": (i32, [vp, vp, i32, u64, vp, u64]),
        "bitar_hip_fill_at": (i32, [vp, vp, i32, u64, u64, vp, u64]),
        "bitar_hip_checksum": (i32, [vp, vp, u32, vp, u64, u32, vp, u32, vp]),
        "bitar_hip_copy_batch": (i32, [vp, vp, vp, vp, vp, u32]),
        "bitar_hip_lz4_chain": (i32, [vp, vp, vp, u32, vp, u32, vp, u64, vp]),
        "bitar_hip_get_decoder_options": (i32, [vp, ctypes.POINTER(DecoderOptions)]),
        "bitar_hip_set_decoder_options": (i32, [vp, ctypes.POINTER(DecoderOptions)]),
        "bitar_hip_path_counters": (i32, [vp, ctypes.POINTER(ctypes.c_uint64), u32]),
        "bitar_hip_compress_host": (i32, [vp, vp, u32, vp, u64, u32, vp, vp, vp, u64, vp]),
        "bitar_hip_decompress_host": (i32, [vp, vp, u32, vp, vp, u32, u32, vp, vp, u64, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


# every symbol include/bitar_hip.h declares (checked by tests/test_abi.py)
ABI_SYMBOLS = ("bitar_hip_abi_version", "bitar_hip_last_error", "bitar_hip_device_count",
               "bitar_hip_open", "bitar_hip_close", "bitar_hip_stream", "bitar_hip_device",
               "bitar_hip_slot_size", "bitar_hip_max_distance", "bitar_hip_alloc", "bitar_hip_free",
               "bitar_hip_host_alloc", "bitar_hip_host_free", "bitar_hip_memcpy",
               "bitar_hip_compress", "bitar_hip_compress_scattered", "bitar_hip_pointer_info",
               "bitar_hip_decompress", "bitar_hip_decompress_slab",
               "bitar_hip_sync", "bitar_hip_pack", "bitar_hip_pack_lz4f", "bitar_hip_fill",
               "bitar_hip_fill_at", "bitar_hip_checksum", "bitar_hip_copy_batch",
               "bitar_hip_lz4_chain", "bitar_hip_get_decoder_options",
               "bitar_hip_set_decoder_options", "bitar_hip_path_counters",
               "bitar_hip_compress_host", "bitar_hip_decompress_host")


def check(rc):
    if rc != 0:
        raise BitarError(rc, lib().bitar_hip_last_error().decode())
    return rc


def slot_size(codec, seg):
    return int(lib().bitar_hip_slot_size(codec, seg))


def max_distance(codec):
    """largest match distance the encoder of `codec` emits (its window's reach)"""
    return int(lib().bitar_hip_max_distance(codec))


def device_count():
    n = ctypes.c_int(0)
    check(lib().bitar_hip_device_count(ctypes.byref(n)))
    return n.value


def _ptr(t):
    """device pointer of a torch tensor (or an int address, or None)."""
    if t is None:
        return None
    if isinstance(t, int):
        return ctypes.c_void_p(t)
    return ctypes.c_void_p(t.data_ptr())


class Engine:
    """One context on one gfx950 device: the CompressDevice analogue.

    Calls are asynchronous on `stream` (default: torch's current stream on that device, so
    torch copies and our kernels stay ordered).  Buffers are torch uint8 tensors in HBM.
    """

    def __init__(self, device=0, num_streams=1, flags=0):
        import torch  # plumbing only
        self.torch = torch
        self.device = device

        class Cfg(ctypes.Structure):
            _fields_ = [("num_streams", ctypes.c_uint32), ("flags", ctypes.c_uint32)]

        cfg = Cfg(num_streams, flags)
        ctx = ctypes.c_void_p()
        check(lib().bitar_hip_open(device, ctypes.byref(cfg), ctypes.byref(ctx)))
        self.ctx = ctx

    def close(self):
        if self.ctx:
            lib().bitar_hip_close(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self, stream):
        if stream is None:
            return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)
        if isinstance(stream, int):
            return ctypes.c_void_p(stream)
        return ctypes.c_void_p(stream.cuda_stream)

    def decoder_options(self):
        o = DecoderOptions()
        check(lib().bitar_hip_get_decoder_options(self.ctx, ctypes.byref(o)))
        return {f: getattr(o, f) for f, _ in DecoderOptions._fields_}

    def set_decoder_options(self, **kw):
        """change this context's decoders (inflate_lanes / zstd_lanes / zstd_seq /
        count_paths); returns the previous options"""
        old = self.decoder_options()
        new = dict(old, **kw)
        check(lib().bitar_hip_set_decoder_options(
            self.ctx, ctypes.byref(DecoderOptions(*(new[f] for f, _ in DecoderOptions._fields_)))))
        return old

    def path_counters(self):
        """{path: segments} since the last call (waits for the device, then resets)"""
        v = (ctypes.c_uint64 * PATH_COUNT)()
        check(lib().bitar_hip_path_counters(self.ctx, v, PATH_COUNT))
        return {name: int(v[k]) for k, name in enumerate(PATHS)}

    def queue_pair_stream(self, qp):
        s = ctypes.c_void_p()
        check(lib().bitar_hip_stream(self.ctx, qp, ctypes.byref(s)))
        return s.value

    def empty(self, nbytes, dtype=None):
        t = self.torch
        return t.empty(nbytes, dtype=dtype or t.uint8, device=f"cuda:{self.device}")

    # --- hot path ------------------------------------------------------------------
    def compress_into(self, codec, data, seg, slab, stride, sizes, n=None, stream=None):
        n = data.numel() * data.element_size() if n is None else n
        check(lib().bitar_hip_compress(self.ctx, self._stream(stream), codec, _ptr(data), n, seg,
                                       _ptr(slab), stride, _ptr(sizes)))

    def compress_host_into(self, codec, host, n, seg, stage, slab, stride, sizes, stream=None):
        """compress n bytes of host memory (a pinned torch CPU tensor, or an address) through
        the HBM staging tensor `stage`, link and kernels overlapped"""
        check(lib().bitar_hip_compress_host(self.ctx, self._stream(stream), codec, _ptr(host),
                                            n, seg, _ptr(stage), _ptr(slab), None, stride,
                                            _ptr(sizes)))

    def decompress_host_into(self, codec, srcs, sizes, nseg, seg, stage, host, produced,
                             capacity=None, stream=None):
        """decompress into host memory (nseg*seg bytes at `host`) through `stage`"""
        cap = nseg * seg if capacity is None else capacity
        check(lib().bitar_hip_decompress_host(self.ctx, self._stream(stream), codec, _ptr(srcs),
                                              _ptr(sizes), nseg, seg, _ptr(stage), _ptr(host),
                                              cap, _ptr(produced)))

    def decompress_slab_into(self, codec, slab, stride, sizes, nseg, seg, out, produced,
                             capacity=None, stream=None):
        cap = out.numel() if capacity is None else capacity
        check(lib().bitar_hip_decompress_slab(self.ctx, self._stream(stream), codec, _ptr(slab),
                                              stride, _ptr(sizes), nseg, seg, _ptr(out), cap,
                                              _ptr(produced)))

    def decompress_into(self, codec, srcs, sizes, nseg, seg, out, produced, capacity=None,
                        stream=None):
        """srcs: device int64 tensor of segment addresses."""
        cap = out.numel() if capacity is None else capacity
        check(lib().bitar_hip_decompress(self.ctx, self._stream(stream), codec, _ptr(srcs),
                                         _ptr(sizes), nseg, seg, _ptr(out), cap, _ptr(produced)))

    def pack(self, slab, stride, sizes, nseg, offsets, frame=None, stream=None):
        check(lib().bitar_hip_pack(self.ctx, self._stream(stream), _ptr(slab), stride,
                                   _ptr(sizes), nseg, _ptr(offsets), _ptr(frame)))

    def fill(self, kind, seed, out, n=None, stream=None, offset=0):
        """bytes [offset, offset + n) of the synthetic stream `kind` into `out`."""
        n = out.numel() if n is None else n
        check(lib().bitar_hip_fill_at(self.ctx, self._stream(stream), kind, seed, offset,
                                      _ptr(out), n))

    def checksum(self, kind, data, seg, sums, n=None, lens=None, nseg=None, stream=None):
        """per-segment CRC32 / Adler32 (uint64 tensor `sums`) of uncompressed data"""
        n = data.numel() if n is None else n
        nseg = (n + seg - 1) // seg if nseg is None else nseg
        check(lib().bitar_hip_checksum(self.ctx, self._stream(stream), kind, _ptr(data), n, seg,
                                       _ptr(lens), nseg, _ptr(sums)))

    def copy_batch(self, srcs, dsts, sizes, n, stream=None):
        """entry i: sizes[i] bytes from srcs[i] to dsts[i] (int64 / int32 device tensors)"""
        check(lib().bitar_hip_copy_batch(self.ctx, self._stream(stream), _ptr(srcs), _ptr(dsts),
                                         _ptr(sizes), n))

    def sync(self, stream=None):
        s = self._stream(stream) if stream is not False else None
        check(lib().bitar_hip_sync(self.ctx, s))

    # --- convenience: whole-buffer round trip (the CompressDevice call pair) -----------
    def compress(self, codec, data, seg, stream=None):
        """-> (slab, stride, sizes) ; data: uint8 HBM tensor.  sizes stays on device."""
        n = data.numel()
        nseg = (n + seg - 1) // seg
        stride = slot_size(codec, seg)
        slab = self.empty(max(nseg * stride, 1))
        sizes = self.empty(max(nseg, 1), dtype=self.torch.int32)
        self.compress_into(codec, data, seg, slab, stride, sizes, n=n, stream=stream)
        return slab, stride, sizes[:nseg]

    def decompress(self, codec, slab, stride, sizes, seg, stream=None):
        nseg = sizes.numel()
        out = self.empty(max(nseg * seg, 1))
        produced = self.empty(max(nseg, 1), dtype=self.torch.int32)
        self.decompress_slab_into(codec, slab, stride, sizes, nseg, seg, out, produced,
                                  capacity=nseg * seg, stream=stream)
        return out, produced[:nseg]
