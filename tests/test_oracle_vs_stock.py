"""The oracle's decoders against the stock decoders of this image over seeded mutation
corpora (CPU only): bo_inflate_raw vs zlib 1.2.11 raw inflate, bo_lz4_decompress_block vs
liblz4 1.9.3 LZ4_decompress_safe, bo_zstd_decompress vs libzstd 1.4.9 ZSTD_decompress --
every mutated stream gets the same accept / reject verdict and, when accepted, the same bytes.

This pins the oracle's ACCEPTANCE rules (the GPU decoders are pinned to the oracle by
tests/test_gpu_mutations.py over the same corpora), so at this boundary the chain is
GPU == oracle == stock.  Where a stock decoder's verdict is an implementation artefact that
yields wrong bytes, the oracle is stricter, and each such case must belong to one of these
named classes (anything else fails the test):
  * lz4_offset0 -- liblz4 1.9.3 accepts a match offset of 0 ("the value 0 is invalid",
    lz4_Block_format.md) and copies undefined bytes;
  * lz4_capacity -- liblz4 checks the end-of-block conditions (last 5 bytes literals, last
    match >= 12 bytes before the end) against its output capacity, so a short block that
    violates them passes; the same call with capacity = the block's size rejects it;
  * zstd_huf_last -- libzstd's double-symbol Huffman decoder clamps the bit count of a
    stream's last symbol (huf_decompress.c HUF_decodeLastSymbolX2), accepting streams that
    are not consumed exactly (RFC 8878 4.2.2); the oracle reports which stream and by how
    many bits (bo_zstd_last_reject);
  * zstd_seq_overread -- libzstd accepts a sequence bitstream read past its start (its end
    test passes BIT_DStream_overflow), whose values then differ from any RFC 8878 reading.
Rules the oracle took from the stock decoders through this test: zlib's inflate_table
completeness rule for dynamic codes, liblz4's end-of-block conditions and its two
length-extension input limits, libzstd's "weight-1 codes come in pairs" Huffman rule."""
import ctypes
import zlib

import numpy as np
import pytest

import mutation_corpora as M
import oracle_lib as O

SEG = M.SEG


def _zlib(s):
    d = zlib.decompressobj(-15)
    try:
        out = d.decompress(s, SEG + 1)
    except zlib.error:
        return None
    return out if d.eof and len(out) <= SEG else None


def _lz4(L, s, cap=SEG):
    buf = ctypes.create_string_buffer(max(cap, 1))
    r = L.LZ4_decompress_safe(s, buf, len(s), cap)
    return buf.raw[:r] if r >= 0 else None


def _zstd(Z, s):
    buf = ctypes.create_string_buffer(SEG)
    r = Z.ZSTD_decompress(buf, SEG, s, len(s))
    return None if Z.ZSTD_isError(r) else buf.raw[:r]


def _verdict(fn, s):
    r, out = fn(s, SEG)
    return out if r == 0 else None


def _lz4_offsets(s):
    """the match offsets of an LZ4 block, parsed until the stream stops making sense"""
    ip, offs = 0, []
    while ip < len(s):
        tok = s[ip]
        ip += 1
        ll = tok >> 4
        if ll == 15:
            while ip < len(s):
                ll += s[ip]
                ip += 1
                if s[ip - 1] != 255:
                    break
        ip += ll
        if ip + 2 > len(s):
            break
        offs.append(s[ip] | s[ip + 1] << 8)
        ip += 2
        if tok & 15 == 15:
            while ip < len(s) and s[ip] == 255:
                ip += 1
            ip += 1
    return offs


def _compare(cases, oracle, stock, classify):
    seen = {}
    for k, c in enumerate(cases):
        a, b = _verdict(oracle, c), stock(c)
        if a == b:
            continue
        why = classify(c, a, b)
        assert why, (k, "oracle", None if a is None else len(a), "stock",
                     None if b is None else len(b))
        seen[why] = seen.get(why, 0) + 1
    return seen


def _corpus(srcs, rng, count, hot):
    cases = []
    for s, _ in srcs:
        cases += M.mutations(s, rng, count, hot=hot(s))
    return cases


@pytest.mark.parametrize("which", ["gpu_corpora", "extended"])
def test_inflate_verdicts_match_zlib(which):
    if which == "gpu_corpora":
        cases = M.inflate_dynamic_cases() + M.inflate_fixed_cases()
    else:
        rng = np.random.default_rng(4000)
        srcs = M.dynamic_sources() + M.fixed_sources()
        cases = _corpus(srcs, rng, 150, lambda s: (0, 80)) + _corpus(srcs, rng, 50, lambda s: (len(s) * 9 // 10, len(s)))
    seen = _compare(cases, O.inflate, _zlib, lambda c, a, b: None)
    assert not seen


@pytest.mark.parametrize("which", ["gpu_corpora", "extended"])
def test_lz4_verdicts_match_liblz4(which):
    L = M.liblz4()
    if L is None:
        pytest.skip("liblz4 not present")
    if which == "gpu_corpora":
        cases = M.lz4_far_cases()
    else:
        rng = np.random.default_rng(4001)
        srcs = M.lz4_far_sources()
        cases = _corpus(srcs, rng, 300, lambda s: (len(s) // 2, len(s))) + _corpus(srcs, rng, 100, lambda s: (len(s) - 64, len(s)))

    def classify(c, a, b):
        if a is None and b is not None:
            if 0 in _lz4_offsets(c):
                return "lz4_offset0"
            if len(b) < SEG and _lz4(L, c, len(b)) is None:
                return "lz4_capacity"
        return None

    seen = _compare(cases, O.lz4_decompress, lambda c: _lz4(L, c), classify)
    print("lz4 stricter-than-liblz4 classes:", seen)


@pytest.mark.parametrize("which", ["gpu_corpora", "extended"])
def test_zstd_verdicts_match_libzstd(which):
    Z = M.libzstd()
    if Z is None:
        pytest.skip("libzstd not present")
    Lo = O.lib()
    Lo.bo_zstd_last_reject.restype = ctypes.c_int
    Lo.bo_zstd_last_reject.argtypes = [ctypes.POINTER(ctypes.c_int64)]
    if which == "gpu_corpora":
        cases = M.zstd_cases()
    else:
        rng = np.random.default_rng(4002)
        srcs = M.zstd_sources()
        cases = _corpus(srcs, rng, 200, lambda s: (len(s) * 2 // 3, len(s))) + _corpus(srcs, rng, 100, lambda s: (0, 200))

    def classify(c, a, b):
        if a is not None or b is None:
            return None
        O.zstd_decompress(c, SEG)  # (re-run: the reject reason of this case)
        d = ctypes.c_int64()
        why = Lo.bo_zstd_last_reject(ctypes.byref(d))
        if why == 1 and abs(d.value) <= 11:  # (11: the longest Huffman code)
            return "zstd_huf_last"
        if why == 2:
            return "zstd_seq_overread"
        return None

    seen = _compare(cases, O.zstd_decompress, lambda c: _zstd(Z, c), classify)
    print("zstd stricter-than-libzstd classes:", seen)


def test_lz4_near_and_end_rule_verdicts_match_liblz4():
    """Our own blocks mutated near their end, and crafted blocks around the end-of-block
    conditions (final literals 0..20, last match 4..40): the oracle's verdicts equal liblz4's
    when liblz4's capacity is the block's size (its end checks are capacity-relative), and
    with a 64 KiB capacity they differ only in the lz4_capacity class."""
    L = M.liblz4()
    if L is None:
        pytest.skip("liblz4 not present")
    crafted = M.lz4_end_rule_cases()
    n_acc = 0
    for c in crafted:
        r, out = O.lz4_decompress(c, SEG)
        n = len(out) if r == 0 else None
        if r == 0:
            n_acc += 1
            assert _lz4(L, c, n) == out
        else:  # whatever size liblz4 would produce, at that exact capacity it rejects too
            b = _lz4(L, c)
            assert b is None or _lz4(L, c, len(b)) is None, c.hex()
    assert 0 < n_acc < len(crafted)

    def classify(c, a, b):
        if a is None and b is not None:
            if 0 in _lz4_offsets(c):
                return "lz4_offset0"
            if len(b) < SEG and _lz4(L, c, len(b)) is None:
                return "lz4_capacity"
        return None
    seen = _compare(M.lz4_near_cases(), O.lz4_decompress, lambda c: _lz4(L, c), classify)
    print("lz4 (near) stricter-than-liblz4 classes:", seen)
