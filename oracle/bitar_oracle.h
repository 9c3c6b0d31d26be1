/*
 * bitar_oracle.h -- CPU restatement of the bitar hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline.  The product
 * (libbitar_hip.so, bitar_amd/) never links or calls it.
 *
 * What it restates (see DESIGN.md "Oracle"):
 *   - segmentation / ordering / capacity / resize rules of CompressDevice::Compress and
 *     ::Decompress      (reference src/device.cc:156-318, src/memory.cc:350-505)
 *   - output slot sizing (Configuration::UpdateCompressedSegSize, src/config.cc:59-73)
 *   - the per-segment codec op.  In the reference this is the BlueField-2 DEFLATE engine
 *     behind DPDK compressdev 22.07 (third-party, absent from /root/reference); its
 *     published algorithm is RFC 1951 raw DEFLATE (config.cc:83-105).  The north-star
 *     LZ4 block codec follows the published LZ4 block format (lz4 1.9.3,
 *     doc/lz4_Block_format.md).
 *
 * Parity pinning: the reference has no tests and no golden vectors and
 * cannot be built here (needs DPDK + BlueField HW).  The decoders below are pinned against
 * golden vectors produced by the third-party implementations present in this image
 * (liblz4 1.9.3, zlib 1.2.11, libdeflate 1.8) -- tests/golden/gen_golden.py -- and
 * against the reference's only behavioural check, the round-trip memcmp of
 * apps/demo_app.cc:534-543, 671-686.  Compressed bitstreams are not a reference contract
 * (the HW bitstream is unspecified); compressed parity = "decodes byte-exactly with the
 * third-party decoder".
 */
#ifndef BITAR_ORACLE_H_
#define BITAR_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes: negated arrow::StatusCode, as carried in an int by the reference
 * (src/include/util.h:157-205). */
enum {
  BO_OK = 0,
  BO_ERR_OUT_OF_MEMORY = -1,
  BO_ERR_INVALID = -4,
  BO_ERR_IO = -5,
  BO_ERR_CAPACITY = -6,
  BO_ERR_CANCELLED = -8,
  BO_ERR_UNKNOWN = -9,
  BO_ERR_NOT_IMPLEMENTED = -10
};

/* DEFLATE = fixed-Huffman blocks (HuffmanEncoding::FIXED); DEFLATE_DYN = dynamic Huffman
 * (HuffmanEncoding::DYNAMIC, the reference default, config.h:151) */
enum { BO_CODEC_LZ4 = 1, BO_CODEC_DEFLATE = 2, BO_CODEC_ZSTD = 3, BO_CODEC_DEFLATE_DYN = 4,
       BO_CODEC_LZ4_WIDE = 5 };

/* Configuration::UpdateCompressedSegSize (src/config.cc:59-73). */
uint32_t bo_compressed_seg_size(uint32_t decompressed_seg_size);

/* ---- LZ4 block format ---------------------------------------------------------- */
uint32_t bo_lz4_bound(uint32_t n);
/* Decode one raw LZ4 block.  Returns BO_OK and *produced, or BO_ERR_IO on malformed input
 * or if the output would exceed cap (the OUT_OF_SPACE rule of device.cc:512-520). */
int bo_lz4_decompress_block(const uint8_t* src, uint32_t csize, uint8_t* dst, uint32_t cap,
                            uint32_t* produced);
/* Encode one block with the bitar window-scan parse (the exact parse the HIP kernel
 * runs; DESIGN.md "LZ4 compress").  n <= 65536.  cap must be >= bo_lz4_bound(n). */
int bo_lz4_compress_block(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap,
                          uint32_t* csize);
/* the wide LZ4 parse (16 KiB history, 4096-entry table): BITAR_HIP_CODEC_LZ4_WIDE */
int bo_lz4_wide_compress_block(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap,
                               uint32_t* csize);

/* ---- raw DEFLATE (RFC 1951) ----------------------------------------------------- */
uint32_t bo_deflate_bound(uint32_t n);
/* Inflate one raw DEFLATE stream (stored / fixed / dynamic blocks). */
int bo_inflate_raw(const uint8_t* src, uint32_t csize, uint8_t* dst, uint32_t cap,
                   uint32_t* produced);
/* Deflate one segment with fixed Huffman codes and the bitar window-scan LZ77 parse
 * (the exact stream the HIP kernel emits). */
int bo_deflate_fixed_block(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap,
                           uint32_t* csize);

/* Deflate one segment with dynamic Huffman codes (bitar_deflate_dyn.c): the exact stream the
 * HIP kernels deflate_dyn_parse_kernel + deflate_dyn_emit_kernel write (dynamic, fixed or
 * stored block, whichever is smallest).  cap >= bo_deflate_bound(n). */
int bo_deflate_dynamic_block(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap,
                             uint32_t* csize);
/* the block type that encoder chooses: 0 stored, 1 fixed, 2 dynamic (-1 on error) */
int bo_deflate_dynamic_mode(const uint8_t* src, uint32_t n);
/* length-limited Huffman code lengths as the dynamic encoder builds them */
void bo_huff_lengths(const uint32_t* freq, int nsym, int maxlen, uint8_t* lens);

/* ---- Zstandard (RFC 8878), bitar_zstd.c ------------------------------------------ */
/* Decode one Zstandard frame (no dictionary; content checksum verified). */
int bo_zstd_decompress(const uint8_t* src, uint32_t csize, uint8_t* dst, uint32_t cap,
                       uint32_t* produced);
uint64_t bo_xxh64(const uint8_t* p, uint64_t len, uint64_t seed);
/* tests: why the last bo_zstd_decompress on this thread rejected (0: another reason) */
#define BO_ZSTD_REJECT_HUF_END 1      /* a Huffman stream not consumed exactly (detail: bits left) */
#define BO_ZSTD_REJECT_SEQ_OVERREAD 2 /* the sequence bitstream read past its start */
int bo_zstd_last_reject(int64_t* detail);
/* Encode one segment as one Zstandard frame, exactly as the HIP kernel does (bitar
 * window-scan parse; blocks of <= 512 sequences; raw literals; predefined FSE sequence
 * codes; no repeat offsets; a block that does not shrink is stored raw).  cap must be
 * >= bo_zstd_bound(n). */
uint32_t bo_zstd_bound(uint32_t n);
int bo_zstd_compress_block(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap,
                           uint32_t* csize);

/* internal: the shared window-scan parse (bitar_oracle.c) */
typedef void (*bo_emit_fn)(void* ctx, uint32_t lit_start, uint32_t lit_len, uint32_t off,
                           uint32_t mlen);
void bo_window_parse(const uint8_t* src, uint32_t n, uint32_t max_dist, uint32_t max_mlen,
                     bo_emit_fn emit, void* ctx);
#define BO_MAX_DIST_ALL 2560u
/* DEFLATE encoders: a coded block is kept over stored blocks only if smaller by >= n / 16 */
#define BO_STORE_MARGIN(n) ((uint64_t)(n) >> 4)
#define BO_PARSE_REP 1u
#define BO_PARSE_SKIP 2u
#define BO_PARSE_HLOG(h) ((uint32_t)(h) << 8) /* hash table log2 size (0: 10) */
/* test hook: before each window it scans, the parse reports the positions [done, x) that
 * skipped probe windows covered since the last scanned window, as emit(ctx, done, x - done,
 * BO_GAP_OFF, 0) */
#define BO_PARSE_GAPS (1u << 16)
#define BO_GAP_OFF 0xFFFFFFFFu
uint32_t bo_set_lz4_parse_flags(uint32_t flags);
/* Zstd parse flags (default BO_PARSE_REP | BO_PARSE_SKIP, the shipped zstd_parse_kernel).
 * BO_ZSTD_DROP_GAP_LITERALS reproduces the round-3 experimental GPU emitter (its literal
 * section lacked the bytes of skipped probe windows): the tests check that such frames are
 * rejected by libzstd and by bo_zstd_decompress alike. */
#define BO_ZSTD_DROP_GAP_LITERALS (1u << 17)
uint32_t bo_set_zstd_parse_flags(uint32_t flags);
/* Blocks per Zstd frame.  Default (0): frames with >= 64 sequences are written as 4 blocks of
 * equal sequence counts sharing one literal code and one set of tables, 8 when they also hold
 * >= 32 KiB of literals; 1..8: that many for every frame with >= 64
 * sequences (1: the single-block frames of rounds 1-4).  Returns the previous setting. */
uint32_t bo_set_zstd_blocks(uint32_t blocks);
void bo_window_parse_flags(const uint8_t* src, uint32_t n, uint32_t max_dist, uint32_t max_mlen,
                           uint32_t flags, bo_emit_fn emit, void* ctx);

/* ---- segment-level restatement of CompressDevice ------------------------------- */
/* Compress (device.cc:156-238): cut `in` into ceil(n/seg) segments in order, compress each
 * independently into slot i of `slab` (stride slot_stride), sizes[i] = compressed size.
 * n == 0 yields zero segments (device.cc:161-164). */
int bo_compress(int codec, const uint8_t* in, uint64_t n, uint32_t seg, uint8_t* slab,
                uint64_t slot_stride, uint32_t* sizes, uint32_t* nseg_out, int threads);
/* Decompress (device.cc:240-318): capacity >= nseg*seg else CapacityError (248-254);
 * segment i inflates into out + i*seg (memory.cc:482-493); *out_size = sum(produced)
 * (resize without shrink, 312-315).  srcs[i]/sizes[i] describe compressed segment i. */
int bo_decompress(int codec, const uint8_t* const* srcs, const uint32_t* sizes, uint32_t nseg,
                  uint32_t seg, uint8_t* out, uint64_t capacity, uint64_t* out_size,
                  uint32_t* produced, int threads);

/* ---- deterministic synthetic inputs ------------------------------ */
/* kind: 0 = random (SplitMix64), 1 = "Silesia-style" 3 MiB period mix, 2 = Arrow-like
 * record-batch body (int64 small range | float64 | dictionary-index int32 | utf8),
 * 3 = constant, 4 = periodic, 5 = int64 small-range only, 6 = log text only. */
void bo_fill(int kind, uint64_t seed, uint8_t* out, uint64_t n);

#ifdef __cplusplus
}
#endif
#endif /* BITAR_ORACLE_H_ */
