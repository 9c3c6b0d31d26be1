"""The bitar C++ front-end (namespace bitar, bitar_amd/cpp) -- driver / device / config /
memory-pool / async API of the reference, over libbitar_hip.so.

CPU: the library and test binary build against Arrow 25 and the configuration rules hold.
GPU: Compress / Decompress / Recycle / async through a real device; every compressed
segment it returns must decode with the third-party decoder (zlib for DEFLATE, the pinned
oracle for LZ4 and Zstd) to the matching input slice.
"""
import ctypes
import os
import struct
import subprocess
import zlib

import numpy as np

import pytest

import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "bitar_amd", "cpp")
BIN = os.path.join(CPP, "build", "bitar_frontend_test")


def _build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "bitar_amd")])
    subprocess.check_call(["make", "-s", "-j8", "-C", CPP])


def test_frontend_builds_and_cpu_rules():
    _build()
    r = subprocess.run([BIN, "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


def test_release_and_debug_builds():
    """The shipped libbitar.so is the release build (-DNDEBUG): its pools do not poison memory
    (the reference poisons only without NDEBUG, memory_pool.cc:190-263); lib/debug/libbitar.so
    is the debug variant that does."""
    _build()
    for path, want in ((os.path.join(CPP, "lib", "libbitar.so"), False),
                       (os.path.join(CPP, "lib", "debug", "libbitar.so"), True)):
        L = ctypes.CDLL(path)
        f = L._ZN5bitar11PoolPoisonsEv
        f.restype = ctypes.c_bool
        assert f() is want, path
    r = subprocess.run([BIN + "_debug", "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


def test_integration_example_is_the_tested_code():
    """INTEGRATION.md's minimal program is the function frontend_test runs in GPU mode, word
    for word (so the documented flow is the tested one)."""
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        doc = f.read()
    a = doc.index('```cpp\n#include "bitar/bitar.h"\n\n// `data`')
    block = doc[a + len("```cpp\n"):doc.index("```", a + 6)]
    body = block.split("\n", 2)[2]
    with open(os.path.join(ROOT, "tests", "cpp", "frontend_test.cc")) as f:
        src = f.read()
    s = src.index("// --- INTEGRATION.md minimal program ---\n") + len(
        "// --- INTEGRATION.md minimal program ---\n")
    assert src[s:src.index("// --- end ---", s)] == body
    assert "CHECK_OK(RoundTrip(" in src


def _segments(path):
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack_from("<I", data, i)
        out.append(data[i + 4:i + 4 + n])
        i += 4 + n
    return out


@pytest.mark.gpu
def test_frontend_on_gpu(tmp_path):
    if not os.path.exists(BIN):
        _build()
    data = O.fill(O.KIND_ARROW, 11, 3 * 65536 * 4 + 777).tobytes()
    inp = tmp_path / "input.bin"
    inp.write_bytes(data)
    r = subprocess.run([BIN, "gpu", str(inp), str(tmp_path)], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    seg = 59460
    # DYNAMIC (the reference default) is the oracle's dynamic stream; FIXED the fixed one
    for name, enc in (("deflate.segs", O.deflate_dynamic), ("deflate_fixed.segs", O.deflate_fixed)):
        segs = _segments(tmp_path / name)
        assert len(segs) == (len(data) + seg - 1) // seg
        for i, s in enumerate(segs):
            plain = data[i * seg:(i + 1) * seg]
            assert zlib.decompress(s, -15) == plain
            assert enc(plain) == (0, s), (name, i)
    segs = _segments(tmp_path / "lz4.segs")
    seg = 65536
    assert len(segs) == (len(data) + seg - 1) // seg
    for i, s in enumerate(segs):
        rc, plain = O.lz4_decompress(s, seg)
        assert rc == 0 and plain == data[i * seg:(i + 1) * seg]
        assert O.lz4_compress(plain) == (0, s), ("lz4", i)
    # Codec::LZ4 at level 2: the wide parse, bit-exact with the oracle's, smaller in total
    wide = _segments(tmp_path / "lz4_wide.segs")
    assert len(wide) == len(segs)
    for i, s in enumerate(wide):
        assert O.lz4_wide_compress(data[i * seg:(i + 1) * seg]) == (0, s), ("lz4_wide", i)
    assert sum(map(len, wide)) < sum(map(len, segs))
    # configured checksums: CRC32 | Adler32 << 32 of every 64 KiB segment (vs zlib)
    cs = np.fromfile(tmp_path / "checksums.bin", dtype=np.uint64)
    assert cs.size == (len(data) + 65535) // 65536
    for i, v in enumerate(cs.tolist()):
        part = data[i * 65536:(i + 1) * 65536]
        assert v == zlib.crc32(part) | (zlib.adler32(part) << 32), i
    segs = _segments(tmp_path / "zstd.segs")
    assert len(segs) == (len(data) + seg - 1) // seg
    for i, s in enumerate(segs):
        rc, plain = O.zstd_decompress(s, seg)
        assert rc == 0 and plain == data[i * seg:(i + 1) * seg]
        assert O.zstd_compress(plain) == (0, s), ("zstd", i)
    # chained ops (max_sgl_segs = 4 over 16 KiB segments): the 4 buffers of op j joined are
    # one stream of input bytes [j*64Ki, (j+1)*64Ki), the oracle's own encoding of them
    seg, k = 16384, 4
    for name, enc, dec in (("sgl_lz4.segs", O.lz4_compress, O.lz4_decompress),
                           ("sgl_deflate.segs", O.deflate_dynamic, None),
                           ("sgl_zstd.segs", O.zstd_compress, O.zstd_decompress)):
        segs = _segments(tmp_path / name)
        assert len(segs) == (len(data) + seg - 1) // seg, name
        for j in range(0, len(segs), k):
            stream = b"".join(segs[j:j + k])
            plain = data[j * seg:(j + k) * seg]
            assert all(len(p) > 0 for p in segs[j:j + k][:1])
            if dec is None:
                assert zlib.decompress(stream, -15) == plain
            else:
                rc, got = dec(stream, k * seg)
                assert rc == 0 and got == plain, (name, j)
            assert enc(plain) == (0, stream), (name, j)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["release", "debug"])
def test_frontend_pools_on_gpu(tmp_path, variant):
    """Pool poisoning read back (debug: 0xBC / 0xBD at the ends of fresh and grown HBM and host
    allocations; release: none), and Compress / Decompress of LZ4, DEFLATE and Zstd over
    buffers the front-end did not allocate: hipHostRegister'd host memory (staged by copy:
    its device address may differ) and HBM owned by another bitar context."""
    binary = BIN + ("_debug" if variant == "debug" else "")
    if not os.path.exists(binary):
        _build()
    inp = tmp_path / "input.bin"
    inp.write_bytes(O.fill(O.KIND_ARROW, 17, 5 * 65536 + 4321).tobytes())
    r = subprocess.run([binary, "pool", "1" if variant == "debug" else "0", str(inp)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


def _lz4f_compress(plain, independent, block_checksum, content_checksum, content_size):
    """liblz4's frame API with explicit preferences (LZ4F_compressFrame)."""
    L = ctypes.CDLL("liblz4.so.1")

    class FrameInfo(ctypes.Structure):
        _fields_ = [("blockSizeID", ctypes.c_int), ("blockMode", ctypes.c_int),
                    ("contentChecksumFlag", ctypes.c_int), ("frameType", ctypes.c_int),
                    ("contentSize", ctypes.c_ulonglong), ("dictID", ctypes.c_uint),
                    ("blockChecksumFlag", ctypes.c_int)]

    class Prefs(ctypes.Structure):
        _fields_ = [("frameInfo", FrameInfo), ("compressionLevel", ctypes.c_int),
                    ("autoFlush", ctypes.c_uint), ("favorDecSpeed", ctypes.c_uint),
                    ("reserved", ctypes.c_uint * 3)]

    p = Prefs()
    p.frameInfo.blockSizeID = 4  # 64 KiB
    p.frameInfo.blockMode = 1 if independent else 0
    p.frameInfo.contentChecksumFlag = int(content_checksum)
    p.frameInfo.blockChecksumFlag = int(block_checksum)
    p.frameInfo.contentSize = len(plain) if content_size else 0
    L.LZ4F_compressFrameBound.restype = ctypes.c_size_t
    L.LZ4F_compressFrame.restype = ctypes.c_size_t
    cap = L.LZ4F_compressFrameBound(ctypes.c_size_t(len(plain)), ctypes.byref(p))
    out = ctypes.create_string_buffer(cap)
    r = L.LZ4F_compressFrame(out, ctypes.c_size_t(cap), plain, ctypes.c_size_t(len(plain)),
                             ctypes.byref(p))
    assert r < cap
    return out.raw[:r]


def _stock_streams(pa):
    """(kind, stream, plain): the per-buffer frames pyarrow's codecs write (Arrow's default
    LZ4F preferences: linked 64 KiB blocks; zstd level 1 frames of the whole buffer) for the
    column buffers of an Arrow-like table, and liblz4 / libzstd frames with checksums and
    content sizes."""
    out = []
    cols = [O.fill(2, 31, 300000).tobytes(), O.fill(6, 32, 200000).tobytes(),
            O.fill(5, 33, 1 << 20).tobytes(), O.fill(0, 34, 70000).tobytes(), b"x" * 5]
    for plain in cols:
        out.append(("zstd", pa.Codec("zstd").compress(plain).to_pybytes(), plain))
        out.append(("lz4f", pa.Codec("lz4").compress(plain).to_pybytes(), plain))
    plain = cols[0]
    for ind, bc, cc, cs in ((True, True, True, True), (False, True, True, False),
                            (False, False, True, True), (True, False, False, False)):
        out.append(("lz4f", _lz4f_compress(plain, ind, bc, cc, cs), plain))
    try:
        Z = ctypes.CDLL("libzstd.so.1")
        Z.ZSTD_createCCtx.restype = ctypes.c_void_p
        Z.ZSTD_CCtx_setParameter.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        Z.ZSTD_compress2.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_void_p, ctypes.c_size_t]
        Z.ZSTD_compress2.restype = ctypes.c_size_t
        cc = Z.ZSTD_createCCtx()
        for level, cks in ((1, 1), (3, 0), (9, 1)):
            Z.ZSTD_CCtx_setParameter(cc, 100, level)
            Z.ZSTD_CCtx_setParameter(cc, 201, cks)  # checksum flag
            buf = ctypes.create_string_buffer(len(plain) + 4096)
            r = Z.ZSTD_compress2(cc, buf, len(buf), plain, len(plain))
            assert r < len(buf)
            out.append(("zstd", buf.raw[:r], plain))
    except OSError:
        pass
    return out


@pytest.mark.gpu
def test_arrow_codec_adapter_on_gpu(tmp_path):
    """bitar::MakeArrowCodec (ZSTD, LZ4_FRAME): GPU round trips and stock-codec decoding are
    checked in C++; here pyarrow decodes the GPU streams and reads the IPC streams written
    with GPU body compression."""
    pa = pytest.importorskip("pyarrow")
    import pyarrow.ipc  # noqa: F401
    if not os.path.exists(BIN):
        _build()
    data = O.fill(O.KIND_MIXED, 5, 9 * 65536 + 1234).tobytes()
    inp = tmp_path / "input.bin"
    inp.write_bytes(data)
    # stock streams for the GPU decoder (DecompressZstd / DecompressLz4f of arrow_codec.cc)
    man = []
    for k, (kind, blob, plain) in enumerate(_stock_streams(pa)):
        (tmp_path / f"stock_{k}.bin").write_bytes(blob)
        (tmp_path / f"plain_{k}.bin").write_bytes(plain)
        man.append(f"{kind} stock_{k}.bin plain_{k}.bin")
    (tmp_path / "stock.txt").write_text("\n".join(man) + "\n")
    r = subprocess.run([BIN, "arrow", str(inp), str(tmp_path)], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    n_lz4 = sum(1 for m in man if m.startswith("lz4f"))
    assert f"stock streams decoded: {len(man) - n_lz4}" in r.stdout
    assert f"stock streams decoded: {n_lz4}" in r.stdout
    for tag, name in (("zstd", "zstd"), ("lz4f", "lz4")):
        comp = (tmp_path / f"arrow_{tag}.bin").read_bytes()
        assert len(comp) < len(data)
        out = pa.Codec(name).decompress(comp, decompressed_size=len(data))
        assert out.to_pybytes() == data, tag
        table = pa.ipc.open_stream((tmp_path / f"ipc_{tag}.arrows").read_bytes()).read_all()
        n = 200000
        assert table.column("v").to_pylist() == [i * 7 % 1000 for i in range(n)], tag
        assert table.column("s").to_pylist() == [f"row{i % 977}" for i in range(n)], tag


@pytest.mark.gpu
@pytest.mark.parametrize("fmt,ipc", [("parquet", "none"), ("feather", "zstd"), ("raw", "none")])
def test_demo_app_modes(tmp_path, fmt, ipc):
    """demo_app (reference apps/demo_app.cc): mode 1 reads a Parquet / Feather table and
    serializes it to an Arrow IPC stream (optionally GPU-compressed bodies), mode 0 reads raw
    bytes; then EvaluateSync and EvaluateAsync (2 devices' worth of queue pairs on one GPU)
    must report byte-identical round trips."""
    pa = pytest.importorskip("pyarrow")
    n = 300000
    table = pa.table({"v": pa.array([i * 7 % 1000 for i in range(n)], pa.int64()),
                      "s": pa.array([f"row{i % 977}" for i in range(n)])})
    if fmt == "parquet":
        import pyarrow.parquet as pq
        path = tmp_path / "t.parquet"
        pq.write_table(table, path)
        args = ["--mode", "1"]
    elif fmt == "feather":
        import pyarrow.feather as pf
        path = tmp_path / "t.feather"
        pf.write_feather(table, path)
        args = ["--mode", "1"]
    else:
        path = tmp_path / "t.bin"
        path.write_bytes(O.fill(O.KIND_ARROW, 3, 3 << 20).tobytes())
        args = ["--mode", "0", "--bytes", str(2 << 20)]
    demo = os.path.join(CPP, "build", "demo_app")
    if not os.path.exists(demo):
        _build()
    r = subprocess.run([demo, "--file", str(path), *args, "--codec", "lz4", "--seg", "65536",
                        "--workers", "3", "--ipc-codec", ipc],
                       capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out
    assert "The decompressed data is equivalent to the input buffer" in out, out
    assert "parts is equivalent to the input buffer" in out, out
    if fmt != "raw":
        assert "Deserialize Table" in out, out
