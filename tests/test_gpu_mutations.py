"""Adversarial parity for the branch-free decoder paths (seeded mutations), through the C ABI.

Targets the two decode paths whose hot loops run without exec-mask branches and write
through per-lane trash slots, where an out-of-bounds write or a wrong verdict would hide:
  * the inflate_kernel batch walk (inflate.hip huff_batch: speculative symbol records,
    v_writelane walk, prefix max) on dynamic-Huffman streams long enough to run many batches
    -- our own encoder's and stock zlib level 1's (the reference's frame, config.cc:83-105);
  * the Zstd hand-off -> zstd_seqdec_kernel -> zstd_exec_kernel path (frames whose last block
    holds >= 16 sequences and no checksum): our level-1-class frames and libzstd level 1's.
Every mutated stream (bit flips, byte sets, truncations, corrupted block / table headers)
must decode exactly as the oracle decides (oracle/bitar_oracle.c bo_inflate_raw,
oracle/bitar_zstd.c bo_zstd_decompress): the same accept / reject verdict per segment, and
byte-equal output when accepted -- the reference's per-op rule (src/device.cc:512-520: a
failed op fails the call, never yields wrong bytes).  The context's path counters
(bitar_hip_path_counters) show that the mutations reached the targeted kernels.
"""
import numpy as np
import pytest

import mutation_corpora as M
import oracle_lib as O
from test_gpu_lz4 import _decode_blobs, eng  # noqa: F401  (fixture reuse)

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

SEG = 65536


_mutations = M.mutations  # (tests/mutation_corpora.py: the corpora the CPU test pins to stock)


def _check_like_oracle(eng, codec, cases, oracle):
    ok, out, prod = _decode_blobs(eng, codec, cases, SEG)
    n_ok = 0
    for k, c in enumerate(cases):
        r, ref = oracle(c, SEG)
        if r == 0:
            n_ok += 1
            assert prod[k] == len(ref), (k, int(prod[k]), len(ref))
            assert out[k * SEG:k * SEG + len(ref)].tobytes() == ref, k
        else:
            assert prod[k] == 0xFFFFFFFF, (k, r, int(prod[k]))
    return n_ok


# ---- DEFLATE: the wave inflater's batch walk ----------------------------------------------
@pytest.fixture(params=[4, 0], ids=["lanes4", "wave"])
def counting_inflate(request, eng):
    old = eng.set_decoder_options(inflate_lanes=request.param, count_paths=1)
    eng.path_counters()  # reset
    yield request.param
    eng.set_decoder_options(**old)


_dynamic_sources = M.dynamic_sources


@pytest.mark.parametrize("codec", [O.CODEC_DEFLATE_DYN, O.CODEC_DEFLATE], ids=["dyn", "fixed-hint"])
def test_inflate_batch_mutations_like_oracle(eng, counting_inflate, codec):
    """Both inflaters: inflate_kernel (the DYNAMIC hint) and inflate_fixed_kernel (the FIXED
    hint, whose 9 / 8-bit fast tables send these streams' longer codes to the slow path)."""
    srcs = _dynamic_sources()
    # the unmutated streams decode and run the batch path
    _check_like_oracle(eng, codec, [s for s, _ in srcs], O.inflate)
    c0 = eng.path_counters()
    assert c0["inflate_wave"] == len(srcs) and c0["inflate_wave_reject"] == 0
    assert c0["inflate_batch_segs"] == len(srcs), c0
    rng = np.random.default_rng(1951)
    cases = []
    for stream, _ in srcs:
        # hot range: the block header and the code-length / literal-length tables
        cases += _mutations(stream, rng, 48, hot=(0, 80))
    n_ok = _check_like_oracle(eng, codec, cases, O.inflate)
    c = eng.path_counters()
    # every mutated stream went to inflate_kernel (dynamic blocks: the lane inflater defers
    # them all), most of them ran batches, and the oracle both accepted and rejected some
    assert c["inflate_wave"] == len(cases), c
    assert c["inflate_batch_segs"] >= len(cases) // 3, c
    assert 0 < c["inflate_wave_reject"] < len(cases), c
    assert c["inflate_wave_reject"] == len(cases) - n_ok
    print(f"inflate mutations: {len(cases)} cases, {n_ok} accepted, counters {c}")


def test_inflate_fixed_and_stored_mutations_like_oracle(eng, counting_inflate):
    """Fixed-Huffman (the lane inflater's own path) and stored streams, mutated."""
    _check_like_oracle(eng, O.CODEC_DEFLATE, M.inflate_fixed_cases(), O.inflate)


# ---- Zstd: hand-off -> phase A (seqdec) -> phase B (exec) ---------------------------------
@pytest.fixture(params=[16, 0], ids=["lanes16-seq", "wave-seq"])
def counting_zstd(request, eng):
    old = eng.set_decoder_options(zstd_lanes=request.param, zstd_seq=1, count_paths=1)
    eng.path_counters()
    yield request.param
    eng.set_decoder_options(**old)


_zstd_sources = M.zstd_sources
_fcs_flip = M.fcs_flip


def test_zstd_sequence_path_mutations_like_oracle(eng, counting_zstd):
    srcs = _zstd_sources()
    _check_like_oracle(eng, O.CODEC_ZSTD, [s for s, _ in srcs], O.zstd_decompress)
    c0 = eng.path_counters()
    # every source frame takes the hand-off -> seqdec -> exec path (with the lane decoder in
    # front, those it does not defer excepted)
    assert c0["zstd_handed"] == c0["zstd_exec"] == c0["zstd_wave"], c0
    if counting_zstd == 0:
        assert c0["zstd_handed"] == len(srcs), c0
    rng = np.random.default_rng(8878)
    cases = []
    for frame, _ in srcs:
        # hot range: the last third of the frame -- the sequence section's headers and the
        # backward FSE bitstream (its first bytes are read first)
        cases += _mutations(frame, rng, 48, hot=(2 * len(frame) // 3, len(frame)))
    # the frame content size off by one: the sequences decode, phase B's final check rejects
    cases += [_fcs_flip(frame) for frame, _ in srcs]
    n_ok = _check_like_oracle(eng, O.CODEC_ZSTD, cases, O.zstd_decompress)
    c = eng.path_counters()
    assert c["zstd_handed"] >= len(cases) // 3, c
    assert 0 < c["zstd_seqdec"] <= c["zstd_handed"], c
    assert c["zstd_exec"] > 0 and c["zstd_seqdec_reject"] > 0, c
    assert c["zstd_exec_reject"] > 0, c  # (the content-size flips of the < 64 KiB frames)
    assert n_ok < len(cases)
    print(f"zstd mutations: {len(cases)} cases, {n_ok} accepted, counters {c}")


def test_zstd_literal_mutations_forked_and_serial(eng):
    """The Huffman literal streams (zstd_hlit_kernel) decode beside the sequences' phase A
    (zstd_seqdec_kernel), on a side stream; the only word they share is produced[i] (phase A
    moves it kHanded -> kRecs by compare-and-swap, a literal failure overwrites it).
    Mutations aimed at the literal section must get the oracle's verdicts with the kernels
    side by side, and a context that runs them in series (BITAR_HIP_FLAG_ZSTD_SERIAL) must
    produce the same bytes and verdicts."""
    import bitar_amd
    srcs = _zstd_sources()
    rng = np.random.default_rng(8879)
    cases = []
    for frame, _ in srcs:
        # hot range: the middle third -- the last block's literal section (Huffman tree and
        # streams) sits before its sequence section
        cases += _mutations(frame, rng, 32, hot=(len(frame) // 3, 2 * len(frame) // 3))
    n_ok = _check_like_oracle(eng, O.CODEC_ZSTD, cases, O.zstd_decompress)
    assert 0 < n_ok < len(cases)
    ok_a, out_a, prod_a = _decode_blobs(eng, O.CODEC_ZSTD, cases, SEG)
    serial = bitar_amd.Engine(0, num_streams=1, flags=bitar_amd.FLAG_ZSTD_SERIAL)
    ok_b, out_b, prod_b = _decode_blobs(serial, O.CODEC_ZSTD, cases, SEG)
    assert ok_a == ok_b
    assert np.array_equal(prod_a, prod_b)
    for k in range(len(cases)):
        if prod_a[k] != 0xFFFFFFFF:
            n = int(prod_a[k])
            assert out_a[k * SEG:k * SEG + n].tobytes() == out_b[k * SEG:k * SEG + n].tobytes(), k
    del serial


def test_two_engines_with_different_decoders_concurrently(eng):
    """Decoder options are per context: two engines, one with the lane decoders and one with
    the wave decoders alone, decode the same batch at the same time on their own streams;
    each context's counters show its own path."""
    import bitar_amd
    a = bitar_amd.Engine(0, num_streams=1, flags=bitar_amd.FLAG_COUNT_PATHS)
    b = bitar_amd.Engine(0, num_streams=1, flags=bitar_amd.FLAG_COUNT_PATHS
                         | bitar_amd.FLAG_INFLATE_WAVE_ONLY | bitar_amd.FLAG_ZSTD_WAVE_ONLY)
    try:
        assert a.decoder_options()["inflate_lanes"] == 0  # the default since round 3
        a.set_decoder_options(inflate_lanes=4)
        assert a.decoder_options()["inflate_lanes"] == 4
        assert b.decoder_options()["inflate_lanes"] == 0 and b.decoder_options()["zstd_lanes"] == 0
        n, seg = 64 * 59460, 59460
        data = a.empty(n)
        a.fill(1, 3, data)
        torch.cuda.synchronize()
        slab, stride, sizes = a.compress(bitar_amd.CODEC_DEFLATE, data, seg)  # fixed Huffman
        a.sync()
        nseg = sizes.numel()
        outs = []
        for e in (a, b):
            out = e.empty(nseg * seg)
            prod = e.empty(nseg, dtype=torch.int32)
            outs.append((e, out, prod))
        for e, out, prod in outs:  # queued back to back on two different streams
            e.decompress_slab_into(bitar_amd.CODEC_DEFLATE, slab, stride, sizes, nseg, seg, out,
                                   prod, stream=e.queue_pair_stream(0))
        for e, out, prod in outs:
            e.sync(e.queue_pair_stream(0))
            assert torch.equal(out[:n], data)
        ca, cb = a.path_counters(), b.path_counters()
        assert ca["inflate_wave"] == 0, ca  # the lane inflater took every fixed stream
        assert cb["inflate_wave"] == nseg, cb  # the wave inflater alone
    finally:
        a.close()
        b.close()


# ---- LZ4: the far-history kernel (lz4_decompress_kernel<true>) ------------------------------
def test_lz4_far_path_mutations_like_oracle(eng):
    """Streams whose matches reach past the decoder's LDS ring -- the wide parse's (<= 14848
    back) and liblz4's (<= 65535) -- are deferred to lz4_decompress_kernel<true>, whose FAR
    batches read history back from HBM after a wave fence.  Mutated, they must decode as the
    oracle's bo_lz4_decompress_block decides; the counters show the far kernel ran."""
    old = eng.set_decoder_options(count_paths=1)
    try:
        eng.path_counters()
        bases = [b for b, _ in M.lz4_far_sources()]
        _check_like_oracle(eng, O.CODEC_LZ4, bases, O.lz4_decompress)
        c0 = eng.path_counters()
        assert c0["lz4_far"] > 0, c0
        cases = M.lz4_far_cases()
        n_ok = _check_like_oracle(eng, O.CODEC_LZ4, cases, O.lz4_decompress)
        c = eng.path_counters()
        assert c["lz4_far"] > len(cases) // 4, c
        assert n_ok < len(cases)
        print(f"lz4 far mutations: {len(cases)} cases, {n_ok} accepted, counters {c}")
    finally:
        eng.set_decoder_options(**old)


def test_lz4_near_mutations_and_end_rules_like_oracle(eng):
    """Our own LZ4 blocks mutated near their end (the batch -> general path hand-over) and
    crafted blocks around the block format's end conditions (final literal run >= 5, last
    match >= 12 bytes before the end; the oracle's bo_lz4_decompress_block, pinned to liblz4
    by tests/test_oracle_vs_stock.py): the near kernel's verdicts and bytes are the oracle's,
    including blocks whose last match was decoded inside a batch (re-walked at the end)."""
    cases = M.lz4_near_cases()
    n_ok = _check_like_oracle(eng, O.CODEC_LZ4, cases, O.lz4_decompress)
    assert 0 < n_ok < len(cases)
    crafted = M.lz4_end_rule_cases()
    n_ok = _check_like_oracle(eng, O.CODEC_LZ4, crafted, O.lz4_decompress)
    assert 0 < n_ok < len(crafted)
