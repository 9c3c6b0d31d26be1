/*
 * bitar_oracle.c -- CPU restatement of the bitar hot path.  TEST INFRASTRUCTURE ONLY.
 * See bitar_oracle.h for scope, pinning and the import rule (tests / smoke / cpu_baseline).
 *
 * Nothing here is shared with the product: the HIP kernels in bitar_amd/csrc are an
 * independent implementation that must agree with this file bit for bit.
 */
#include "bitar_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ================================================================================ */
/* Slot sizing -- restates Configuration::UpdateCompressedSegSize (config.cc:59-73):  */
/* the highest set bit of 2*seg (capped at 65536); if that exceeds 32 KiB the slot is */
/* seg * kExpanseRatio (1.1, config.h:41) truncated to uint16.                        */
/* ================================================================================ */
uint32_t bo_compressed_seg_size(uint32_t seg) {
  uint32_t lower_bound = (seg << 1u) & 0x1FFFFu; /* decompressed_seg_size_ is uint16 */
  uint32_t num = 65536u;
  if (lower_bound == 0) return 0;
  while ((num & lower_bound) == 0) num >>= 1u;
  if (num > (65536u >> 1u)) return (uint16_t)((double)seg * 1.1);
  return num;
}

/* ================================================================================ */
/* LZ4 block format (lz4 1.9.3 doc/lz4_Block_format.md).                             */
/* ================================================================================ */
uint32_t bo_lz4_bound(uint32_t n) { return n + n / 255u + 16u; }

/* LZ4 block decode with the block format's rules (lz4 1.9.3 doc/lz4_Block_format.md):
 * offset 0 and offsets before the block start are invalid, and the end-of-block conditions
 * hold for any block with a match -- the last sequence is literals only, at least 5 of them
 * ("the last 5 bytes are always literals"), and the last match starts at least 12 bytes
 * before the end of the block.  liblz4's LZ4_decompress_safe checks the same conditions
 * against its output capacity (equal to the block size for a full segment); its two
 * input-side limits on length-extension bytes are applied as it applies them
 * (read_variable_length: a literal-length extension must start more than 15 bytes before
 * the end of the input, and a match-length extension byte must end more than 4 bytes before
 * it).  tests/test_oracle_vs_stock.py pins these verdicts to liblz4's over mutation corpora. */
int bo_lz4_decompress_block(const uint8_t* src, uint32_t csize, uint8_t* dst, uint32_t cap,
                            uint32_t* produced) {
  uint64_t ip = 0, op = 0, last_ml = 0;
  if (csize == 0) return BO_ERR_IO;
  for (;;) {
    if (ip >= csize) return BO_ERR_IO; /* truncated: no token */
    uint32_t token = src[ip++];
    uint64_t lit = token >> 4;
    if (lit == 15) {
      if (ip + 15 >= csize) return BO_ERR_IO;
      uint32_t b;
      do {
        if (ip >= csize) return BO_ERR_IO;
        b = src[ip++];
        lit += b;
      } while (b == 255);
    }
    if (ip + lit > csize) return BO_ERR_IO;  /* literals run past the block */
    if (op + lit > cap) return BO_ERR_IO;    /* OUT_OF_SPACE */
    memcpy(dst + op, src + ip, (size_t)lit);
    ip += lit;
    op += lit;
    if (ip == csize) { /* last sequence: literals only */
      if (op > lit && (lit < 5 || lit + last_ml < 12)) return BO_ERR_IO; /* end of block */
      break;
    }
    if (ip + 2 > csize) return BO_ERR_IO;
    uint32_t off = (uint32_t)src[ip] | ((uint32_t)src[ip + 1] << 8);
    ip += 2;
    if (off == 0 || off > op) return BO_ERR_IO; /* reference before segment start */
    uint64_t mlen = token & 15u;
    if (mlen == 15) {
      uint32_t b;
      do {
        if (ip >= csize) return BO_ERR_IO;
        b = src[ip++];
        if (ip + 4 >= csize) return BO_ERR_IO;
        mlen += b;
      } while (b == 255);
    }
    mlen += 4;
    if (op + mlen > cap) return BO_ERR_IO;
    for (uint64_t i = 0; i < mlen; ++i) dst[op + i] = dst[op - off + i]; /* overlap-safe */
    op += mlen;
    last_ml = mlen;
  }
  *produced = (uint32_t)op;
  return BO_OK;
}

/* ---- the bitar window-scan parse (shared by the LZ4 and fixed-DEFLATE encoders) --- *
 * Restated exactly as the HIP kernels run it (DESIGN.md "Window-scan parse"):
 *   positions 0..n-12 (legal match starts) are visited in FIXED windows of 64, one per
 *   wavefront lane: window w covers [64w, 64w+64);
 *   every window position looks up hash(read32(p)) in a 1024-entry table holding the most
 *   recent position inserted by an EARLIER window, then all window positions are inserted
 *   (the largest position wins a shared slot) -- the table never depends on the parse;
 *   greedily, from the current position, the first window position whose candidate c
 *   satisfies c < p, p - c <= max_dist and read32(c) == read32(p) starts a match,
 *   extended forward while bytes agree, never past n-5 nor max_mlen; the search resumes
 *   at the match end (possibly several windows later).                                  */
/* 1024 entries: the kernel keeps the table in 2 KiB of LDS so 14 waves fit a CU (12 with
 * 2048 entries, 8 with 4096); measured on kind 1 / 2 / 5 / 6 input: ratio -1.8 / -1.3 /
 * -4.6 / -2.8 % against 2048 entries, LZ4 compress 12 % faster. */
#define BO_HASH_LOG 10
#define BO_WIN 64
#define BO_MINMATCH 4
#define BO_LASTLITERALS 5
#define BO_MFLIMIT 12

static inline uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
         ((uint32_t)p[3] << 24);
}
static inline uint32_t bo_hash_n(uint32_t v, uint32_t hlog) { return (v * 2654435761u) >> (32 - hlog); }

void bo_window_parse(const uint8_t* src, uint32_t n, uint32_t max_dist,
                            uint32_t max_mlen, bo_emit_fn emit, void* ctx) {
  bo_window_parse_flags(src, n, max_dist, max_mlen, 0, emit, ctx);
}

/* flags & BO_PARSE_REP (the Zstd parse): the parse keeps a history of its 3 most recent
 * distinct match distances h (initially 1 4 8, Zstd's repeat offsets; updated per match:
 * a distance already in h moves to the front, a new one is pushed), fixed for the duration
 * of a window.  Every window position first tries the repeat candidates p - h0, p - h1,
 * p - h2 (the first whose 4 bytes agree is its candidate), then the hash candidate; and a
 * position holding only a hash match is not a match start when one of the next 3 positions
 * holds a repeat match (Zstd's fast parse checks the repeat offset at ip + 1 first; looking
 * 3 ahead keeps the parse on repeat offsets through the short literal runs of columnar
 * data: kind-2 ratio 2.378 -> 2.451, libzstd-1 2.475). */
/* one of the next BO_REP_AHEAD window positions holds a repeat match */
#define BO_REP_AHEAD 3
static int repnear(const int* isrep, uint32_t l, uint32_t cnt) {
  for (uint32_t k = 1; k <= BO_REP_AHEAD; ++k)
    if (l + k < cnt && isrep[l + k]) return 1;
  return 0;
}
/* flags & BO_PARSE_SKIP (the LZ4 parse): windows the parse has no use for are skipped, as
 * liblz4 skips positions (LZ4_compress_generic's search step grows with consecutive misses
 * and positions inside a match are never searched nor inserted).  With g = the gate (the
 * parse position, or -- after a probe hit -- the end of the probed span, whichever is later):
 *   - a window lying entirely inside the current match (pos >= x + 64) is skipped: no
 *     lookups, no inserts;
 *   - a window starting >= 128 positions past g (two windows with no match start) is a PROBE
 *     of stride s = 2 (s = 4 from 640 past g): the 64 positions x + s*l (<= last_start) look
 *     up their candidates exactly as a window does; if none of them holds a match, those
 *     positions are inserted (ascending: the largest wins) and the scan moves on to
 *     x + 64 s; if any does, nothing is inserted, g moves to x + 64 (s - 1) - 127 (so the
 *     probed span is scanned by ordinary windows), and ordinary windows go on from x;
 *   - after every ordinary window g = max(g, pos).
 * (The GPU tests all three conditions with one scalar compare per window.) */
#define BO_SKIP_PROBE 128u
#define BO_SKIP_WIDE 640u
void bo_window_parse_flags(const uint8_t* src, uint32_t n, uint32_t max_dist,
                           uint32_t max_mlen, uint32_t flags, bo_emit_fn emit, void* ctx) {
  uint32_t anchor = 0;
  uint32_t hist[3] = {1, 4, 8};
  const int rep = (flags & BO_PARSE_REP) != 0;
  const int skip = (flags & BO_PARSE_SKIP) != 0;
  if (n >= BO_MFLIMIT + 1) {
    /* table log2 size: BO_PARSE_HLOG(flags), default BO_HASH_LOG */
    const uint32_t hlog = (flags >> 8) & 31u ? (flags >> 8) & 31u : BO_HASH_LOG;
    static __thread uint32_t table[1u << 16];
    memset(table, 0, sizeof(uint32_t) << hlog);
    const uint32_t last_start = n - BO_MFLIMIT;        /* match start must be <= n-12 */
    const uint32_t match_limit = n - BO_LASTLITERALS;  /* match end must be <= n-5 */
    uint32_t pos = 0, g = 0, done = 0;
    for (uint32_t x = 0; x <= last_start; x += BO_WIN) {
      if (skip) {
        if (pos >= x + BO_WIN) continue; /* inside the current match */
        if (x >= g + BO_SKIP_PROBE) {    /* (g >= pos: see below) */
          const uint32_t s = x >= g + BO_SKIP_WIDE ? 4u : 2u;
          int hit = 0;
          for (uint32_t l = 0; l < BO_WIN && x + s * l <= last_start; ++l) {
            const uint32_t p = x + s * l, c = table[bo_hash_n(rd32(src + p), hlog)];
            if (c < p && p - c <= max_dist && rd32(src + c) == rd32(src + p)) hit = 1;
          }
          if (!hit) {
            for (uint32_t l = 0; l < BO_WIN && x + s * l <= last_start; ++l)
              table[bo_hash_n(rd32(src + x + s * l), hlog)] = x + s * l;
            x += (s - 1) * BO_WIN; /* (+ BO_WIN by the loop) */
            continue;
          }
          g = x + BO_WIN * (s - 1) - 127u;
        }
      }
      if ((flags & BO_PARSE_GAPS) && done < x) emit(ctx, done, x - done, BO_GAP_OFF, 0);
      uint32_t cnt = last_start - x + 1;
      if (cnt > BO_WIN) cnt = BO_WIN;
      uint32_t cand[BO_WIN], h[BO_WIN];
      int isrep[BO_WIN];
      for (uint32_t l = 0; l < cnt; ++l) {
        const uint32_t p = x + l;
        h[l] = bo_hash_n(rd32(src + p), hlog);
        cand[l] = table[h[l]];
        isrep[l] = 0;
        if (rep) {
          for (int k = 0; k < 3; ++k) {
            const uint32_t d = hist[k];
            if (d <= p && d <= max_dist && rd32(src + p - d) == rd32(src + p)) {
              cand[l] = p - d;
              isrep[l] = 1;
              break;
            }
          }
        }
      }
      for (uint32_t l = 0; l < cnt; ++l) table[h[l]] = x + l; /* ascending: max wins */
      for (;;) {
        uint32_t i = 0, found = 0;
        for (uint32_t l = (pos > x ? pos - x : 0); l < cnt; ++l) {
          uint32_t c = cand[l], p = x + l;
          if (c < p && p - c <= max_dist && rd32(src + c) == rd32(src + p) &&
              !(rep && !isrep[l] && repnear(isrep, l, cnt))) {
            i = p;
            found = 1;
            break;
          }
        }
        if (!found) break;
        uint32_t c = cand[i - x];
        uint32_t len = BO_MINMATCH;
        uint32_t lim = match_limit - i;
        if (lim > max_mlen) lim = max_mlen;
        while (len < lim && src[c + len] == src[i + len]) ++len;
        emit(ctx, anchor, i - anchor, i - c, len);
        pos = i + len;
        anchor = pos;
        if (rep) {
          const uint32_t d = i - c;
          if (d == hist[1]) {
            hist[1] = hist[0];
            hist[0] = d;
          } else if (d == hist[2]) {
            hist[2] = hist[1];
            hist[1] = hist[0];
            hist[0] = d;
          } else if (d != hist[0]) {
            hist[2] = hist[1];
            hist[1] = hist[0];
            hist[0] = d;
          }
        }
      }
      if (pos > g) g = pos;
      done = pos > x + BO_WIN ? pos : x + BO_WIN;
    }
  }
  emit(ctx, anchor, n - anchor, 0, 0); /* last sequence: literals only */
}

typedef struct {
  const uint8_t* src;
  uint8_t* dst;
  uint32_t cap, op;
  int err;
} lz4_emit_ctx;

static void lz4_put_len(lz4_emit_ctx* c, uint32_t v) { /* v >= 15 already subtracted */
  while (v >= 255) {
    if (c->op >= c->cap) { c->err = 1; return; }
    c->dst[c->op++] = 255;
    v -= 255;
  }
  if (c->op >= c->cap) { c->err = 1; return; }
  c->dst[c->op++] = (uint8_t)v;
}

static void lz4_emit(void* vctx, uint32_t lit_start, uint32_t lit_len, uint32_t off,
                     uint32_t mlen) {
  lz4_emit_ctx* c = (lz4_emit_ctx*)vctx;
  if (c->err) return;
  uint32_t ml = mlen ? mlen - BO_MINMATCH : 0;
  uint8_t token = (uint8_t)(((lit_len < 15 ? lit_len : 15) << 4) | (ml < 15 ? ml : 15));
  if (c->op >= c->cap) { c->err = 1; return; }
  c->dst[c->op++] = token;
  if (lit_len >= 15) lz4_put_len(c, lit_len - 15);
  if (c->err || c->op + lit_len > c->cap) { c->err = 1; return; }
  memcpy(c->dst + c->op, c->src + lit_start, lit_len);
  c->op += lit_len;
  if (!mlen) return;
  if (c->op + 2 > c->cap) { c->err = 1; return; }
  c->dst[c->op++] = (uint8_t)(off & 0xFF);
  c->dst[c->op++] = (uint8_t)(off >> 8);
  if (ml >= 15) lz4_put_len(c, ml - 15);
}

/* Match distance cap of the bitar parse (all codecs): 2560 B.  The compressor streams its
 * input through a 4 KiB LDS ring that runs up to 1.5 KiB ahead of the scan, so every
 * candidate of a window is in LDS; the LZ4 decoder's 8 KiB history ring reaches 8048 B back,
 * so every match of our own streams decodes from LDS.  Standard LZ4 allows 65535 and
 * DEFLATE 32768; against a 6656-B cap (8 KiB ring) it costs 0.7-1.4 % ratio on the
 * synthetic corpora for 12-18 % faster compression (DESIGN.md "Window-scan parse"). */
#define BO_MAX_DIST 2560u
_Static_assert(BO_MAX_DIST == BO_MAX_DIST_ALL, "one distance cap for all codecs");

/* LZ4 parse flags: BO_PARSE_SKIP (the shipped LZ4 kernel); bo_set_lz4_parse_flags lets the
 * tests measure the ratio the skipping costs */
static uint32_t g_lz4_parse_flags = BO_PARSE_SKIP;
uint32_t bo_set_lz4_parse_flags(uint32_t flags) {
  const uint32_t old = g_lz4_parse_flags;
  g_lz4_parse_flags = flags;
  return old;
}

int bo_lz4_compress_block(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap,
                          uint32_t* csize) {
  if (n > 65536u) return BO_ERR_INVALID;
  lz4_emit_ctx c = {src, dst, cap, 0, 0};
  bo_window_parse_flags(src, n, BO_MAX_DIST, 0xFFFFFFFFu, g_lz4_parse_flags, lz4_emit, &c);
  if (c.err) return BO_ERR_IO;
  *csize = c.op;
  return BO_OK;
}

/* The wide LZ4 parse (BITAR_HIP_CODEC_LZ4_WIDE: lz4_compress_kernel<16384, 12>): the same
 * parse over a 16 KiB input ring -- match distance <= 16384 - 1536 = 14848 -- and a
 * 4096-entry table.  Measured on 8 MiB of the synthetic kinds 1 / 2 / 5 / 6: ratio +7 / +4 /
 * +19 / +6 % against the 2560 / 1024 parse. */
#define BO_WIDE_MAX_DIST 14848u
#define BO_WIDE_HLOG 12u
int bo_lz4_wide_compress_block(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap,
                               uint32_t* csize) {
  if (n > 65536u) return BO_ERR_INVALID;
  lz4_emit_ctx c = {src, dst, cap, 0, 0};
  bo_window_parse_flags(src, n, BO_WIDE_MAX_DIST, 0xFFFFFFFFu,
                        g_lz4_parse_flags | BO_PARSE_HLOG(BO_WIDE_HLOG), lz4_emit, &c);
  if (c.err) return BO_ERR_IO;
  *csize = c.op;
  return BO_OK;
}

/* ================================================================================ */
/* raw DEFLATE (RFC 1951)                                                            */
/* ================================================================================ */
uint32_t bo_deflate_bound(uint32_t n) {
  /* fixed-Huffman worst case: 9 bits per literal + block header + end code */
  return (uint32_t)(((uint64_t)n * 9 + 7) / 8) + 16u;
}

static const uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                      2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t kDistBase[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                       33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                       1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2,  3,  3,  4,  4,  5,  5,  6,
                                       6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static const uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

typedef struct {
  const uint8_t* src;
  uint32_t csize;
  uint64_t bitpos; /* absolute bit position */
} bo_bits;

/* read n (<= 16) bits LSB-first; returns -1 past the end */
static inline int64_t bits_get(bo_bits* b, int n) {
  if (n == 0) return 0;
  if (b->bitpos + (uint64_t)n > (uint64_t)b->csize * 8) return -1;
  uint32_t v = 0;
  for (int i = 0; i < n; ++i) {
    uint64_t p = b->bitpos + (uint64_t)i;
    v |= (uint32_t)((b->src[p >> 3] >> (p & 7)) & 1u) << i;
  }
  b->bitpos += (uint64_t)n;
  return v;
}

/* Canonical Huffman code: count[len], symbols sorted by (len, symbol). */
typedef struct {
  uint16_t count[16];
  uint16_t symbol[320];
} bo_huff;

/* Build from code lengths.  Over-subscribed sets are an error.  type < 0 (the fixed codes):
 * incomplete sets are accepted.  Dynamic blocks follow zlib 1.2.11's inflate_table: an
 * incomplete set is an error too, except a code with no symbols at all (decoding one is then
 * an error) and -- type 1 literal/length, type 2 distance codes, not type 0 the code-length
 * code -- a code whose longest length is 1 (a single one-bit code). */
static int huff_build(bo_huff* h, const uint8_t* lens, int n, int type) {
  uint16_t offs[16];
  memset(h->count, 0, sizeof(h->count));
  for (int s = 0; s < n; ++s) h->count[lens[s]]++;
  h->count[0] = 0;
  int left = 1;
  for (int len = 1; len <= 15; ++len) {
    left <<= 1;
    left -= h->count[len];
    if (left < 0) return -1;
  }
  int max = 15;
  while (max >= 1 && !h->count[max]) --max;
  if (type >= 0 && left > 0 && max > 0 && (type == 0 || max != 1)) return -1;
  offs[1] = 0;
  for (int len = 1; len < 15; ++len) offs[len + 1] = (uint16_t)(offs[len] + h->count[len]);
  for (int s = 0; s < n; ++s)
    if (lens[s]) h->symbol[offs[lens[s]]++] = (uint16_t)s;
  return 0;
}

/* Decode one symbol bit by bit (codes are stored MSB-first of the code value). */
static int huff_decode(bo_bits* b, const bo_huff* h) {
  int code = 0, first = 0, index = 0;
  for (int len = 1; len <= 15; ++len) {
    int64_t bit = bits_get(b, 1);
    if (bit < 0) return -1;
    code |= (int)bit;
    int count = h->count[len];
    if (code - count < first) return h->symbol[index + (code - first)];
    index += count;
    first += count;
    first <<= 1;
    code <<= 1;
  }
  return -2; /* unassigned code */
}

static int inflate_codes(bo_bits* b, const bo_huff* lit, const bo_huff* dist, uint8_t* dst,
                         uint32_t cap, uint64_t* op) {
  for (;;) {
    int sym = huff_decode(b, lit);
    if (sym < 0) return BO_ERR_IO;
    if (sym < 256) {
      if (*op >= cap) return BO_ERR_IO;
      dst[(*op)++] = (uint8_t)sym;
      continue;
    }
    if (sym == 256) return BO_OK;
    sym -= 257;
    if (sym >= 29) return BO_ERR_IO;
    int64_t e = bits_get(b, kLenExtra[sym]);
    if (e < 0) return BO_ERR_IO;
    uint32_t len = kLenBase[sym] + (uint32_t)e;
    int ds = huff_decode(b, dist);
    if (ds < 0 || ds >= 30) return BO_ERR_IO;
    e = bits_get(b, kDistExtra[ds]);
    if (e < 0) return BO_ERR_IO;
    uint32_t d = kDistBase[ds] + (uint32_t)e;
    if (d > *op) return BO_ERR_IO;
    if (*op + len > cap) return BO_ERR_IO;
    for (uint32_t i = 0; i < len; ++i) dst[*op + i] = dst[*op - d + i];
    *op += len;
  }
}

static void fixed_lengths(uint8_t* litlen, uint8_t* distlen) {
  int s = 0;
  for (; s < 144; ++s) litlen[s] = 8;
  for (; s < 256; ++s) litlen[s] = 9;
  for (; s < 280; ++s) litlen[s] = 7;
  for (; s < 288; ++s) litlen[s] = 8;
  for (s = 0; s < 30; ++s) distlen[s] = 5;
}

int bo_inflate_raw(const uint8_t* src, uint32_t csize, uint8_t* dst, uint32_t cap,
                   uint32_t* produced) {
  bo_bits b = {src, csize, 0};
  uint64_t op = 0;
  bo_huff lit, dist;
  int last;
  do {
    int64_t hdr = bits_get(&b, 3);
    if (hdr < 0) return BO_ERR_IO;
    last = (int)(hdr & 1);
    int type = (int)(hdr >> 1);
    if (type == 0) {
      b.bitpos = (b.bitpos + 7) & ~(uint64_t)7;
      uint64_t p = b.bitpos >> 3;
      if (p + 4 > csize) return BO_ERR_IO;
      uint32_t len = (uint32_t)src[p] | ((uint32_t)src[p + 1] << 8);
      uint32_t nlen = (uint32_t)src[p + 2] | ((uint32_t)src[p + 3] << 8);
      if (len != (~nlen & 0xFFFFu)) return BO_ERR_IO;
      p += 4;
      if (p + len > csize) return BO_ERR_IO;
      if (op + len > cap) return BO_ERR_IO;
      memcpy(dst + op, src + p, len);
      op += len;
      b.bitpos = (p + len) * 8;
    } else if (type == 1) {
      uint8_t ll[288], dl[30];
      fixed_lengths(ll, dl);
      huff_build(&lit, ll, 288, -1);
      huff_build(&dist, dl, 30, -1);
      int r = inflate_codes(&b, &lit, &dist, dst, cap, &op);
      if (r) return r;
    } else if (type == 2) {
      int64_t hlit = bits_get(&b, 5), hdist = bits_get(&b, 5), hclen = bits_get(&b, 4);
      if (hlit < 0 || hdist < 0 || hclen < 0) return BO_ERR_IO;
      int nlen = (int)hlit + 257, ndist = (int)hdist + 1, ncode = (int)hclen + 4;
      if (nlen > 286 || ndist > 30) return BO_ERR_IO;
      uint8_t cl[19];
      memset(cl, 0, sizeof(cl));
      for (int i = 0; i < ncode; ++i) {
        int64_t v = bits_get(&b, 3);
        if (v < 0) return BO_ERR_IO;
        cl[kClOrder[i]] = (uint8_t)v;
      }
      bo_huff clh;
      if (huff_build(&clh, cl, 19, 0)) return BO_ERR_IO;
      uint8_t lens[320];
      int idx = 0;
      while (idx < nlen + ndist) {
        int sym = huff_decode(&b, &clh);
        if (sym < 0) return BO_ERR_IO;
        if (sym < 16) {
          lens[idx++] = (uint8_t)sym;
          continue;
        }
        uint8_t val = 0;
        int64_t rep;
        if (sym == 16) {
          if (idx == 0) return BO_ERR_IO;
          val = lens[idx - 1];
          rep = bits_get(&b, 2);
          if (rep < 0) return BO_ERR_IO;
          rep += 3;
        } else if (sym == 17) {
          rep = bits_get(&b, 3);
          if (rep < 0) return BO_ERR_IO;
          rep += 3;
        } else {
          rep = bits_get(&b, 7);
          if (rep < 0) return BO_ERR_IO;
          rep += 11;
        }
        if (idx + rep > nlen + ndist) return BO_ERR_IO;
        while (rep--) lens[idx++] = val;
      }
      if (lens[256] == 0) return BO_ERR_IO; /* no end-of-block code */
      if (huff_build(&lit, lens, nlen, 1)) return BO_ERR_IO;
      if (huff_build(&dist, lens + nlen, ndist, 2)) return BO_ERR_IO;
      int r = inflate_codes(&b, &lit, &dist, dst, cap, &op);
      if (r) return r;
    } else {
      return BO_ERR_IO;
    }
  } while (!last);
  *produced = (uint32_t)op;
  return BO_OK;
}

/* ---- fixed-Huffman DEFLATE encoder over the window-scan parse -------------------- */
typedef struct {
  const uint8_t* src;
  uint8_t* dst;
  uint32_t cap;
  uint64_t bitpos;
  int err;
} dfl_ctx;

static void put_bits(dfl_ctx* c, uint32_t v, int n) { /* LSB-first */
  for (int i = 0; i < n; ++i) {
    uint64_t p = c->bitpos + (uint64_t)i;
    if ((p >> 3) >= c->cap) { c->err = 1; return; }
    if ((p & 7) == 0) c->dst[p >> 3] = 0;
    c->dst[p >> 3] |= (uint8_t)(((v >> i) & 1u) << (p & 7));
  }
  c->bitpos += (uint64_t)n;
}
static uint32_t rev_bits(uint32_t v, int n) {
  uint32_t r = 0;
  for (int i = 0; i < n; ++i) r |= ((v >> i) & 1u) << (n - 1 - i);
  return r;
}
/* fixed literal/length code of symbol s: (reversed code, length) */
static void fixed_lit_code(uint32_t s, uint32_t* code, int* len) {
  if (s < 144) { *code = rev_bits(0x30 + s, 8); *len = 8; }
  else if (s < 256) { *code = rev_bits(0x190 + (s - 144), 9); *len = 9; }
  else if (s < 280) { *code = rev_bits(s - 256, 7); *len = 7; }
  else { *code = rev_bits(0xC0 + (s - 280), 8); *len = 8; }
}
static void dfl_put_lit(dfl_ctx* c, uint32_t s) {
  uint32_t code;
  int len;
  fixed_lit_code(s, &code, &len);
  put_bits(c, code, len);
}
static void dfl_emit(void* vctx, uint32_t lit_start, uint32_t lit_len, uint32_t off,
                     uint32_t mlen) {
  dfl_ctx* c = (dfl_ctx*)vctx;
  for (uint32_t i = 0; i < lit_len && !c->err; ++i) dfl_put_lit(c, c->src[lit_start + i]);
  if (!mlen || c->err) return;
  int ls = 28;
  while (kLenBase[ls] > mlen) --ls;
  dfl_put_lit(c, 257u + (uint32_t)ls);
  put_bits(c, mlen - kLenBase[ls], kLenExtra[ls]);
  int ds = 29;
  while (kDistBase[ds] > off) --ds;
  put_bits(c, rev_bits((uint32_t)ds, 5), 5);
  put_bits(c, off - kDistBase[ds], kDistExtra[ds]);
}

/* One fixed-Huffman block -- or stored blocks of <= 65535 bytes (stored = 5 * ceil(n / 65535)
 * + n bytes) unless the fixed block, (bits + 7) / 8 bytes, is smaller by at least n / 16
 * (BO_STORE_MARGIN; the dynamic encoder's rule too).  A nearly incompressible segment coded
 * anyway decodes one literal symbol at a time: on the GPU such a segment took 2.4x the decode
 * time of a well compressed one and bounded its whole launch. */
int bo_deflate_fixed_block(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap,
                           uint32_t* csize) {
  dfl_ctx c = {src, dst, cap, 0, 0};
  put_bits(&c, 1u | (1u << 1), 3); /* BFINAL=1, BTYPE=01 */
  bo_window_parse(src, n, BO_MAX_DIST, 258u, dfl_emit, &c);
  dfl_put_lit(&c, 256);
  if (c.err) return BO_ERR_IO;
  const uint64_t fixed = (c.bitpos + 7) >> 3;
  const uint64_t nblk = n ? (n + 65534u) / 65535u : 1;
  const uint64_t stored = nblk * 5 + n;
  if (stored < fixed + BO_STORE_MARGIN(n)) {
    /* (stored can exceed a cap the fixed block just fit in by up to n / 16 bytes) */
    if (stored > cap) return BO_ERR_IO;
    uint64_t o = 0;
    uint32_t p = 0;
    for (uint64_t b = 0; b < nblk; ++b) {
      const uint32_t len = n - p < 65535u ? n - p : 65535u;
      dst[o] = (uint8_t)(b + 1 == nblk);
      dst[o + 1] = (uint8_t)len;
      dst[o + 2] = (uint8_t)(len >> 8);
      dst[o + 3] = (uint8_t)~len;
      dst[o + 4] = (uint8_t)(~len >> 8);
      memcpy(dst + o + 5, src + p, len);
      o += 5 + len;
      p += len;
    }
    *csize = (uint32_t)stored;
    return BO_OK;
  }
  *csize = (uint32_t)fixed;
  return BO_OK;
}

/* ================================================================================ */
/* Segment-level restatement of CompressDevice::Compress / ::Decompress.             */
/* ================================================================================ */
typedef struct {
  int codec, mode; /* mode 0 = compress, 1 = decompress */
  const uint8_t* in;
  uint64_t n;
  uint32_t seg;
  uint8_t* slab;
  uint64_t stride;
  uint32_t* sizes;
  const uint8_t* const* srcs;
  const uint32_t* csizes;
  uint8_t* out;
  uint32_t* produced;
  uint32_t nseg;
  int threads, tid;
  int status;
} bo_job;

static void* bo_worker(void* arg) {
  bo_job* j = (bo_job*)arg;
  /* static round-robin over segments, one thread per host core (the lcore-per-queue-pair
   * model of driver.cc:100-157) */
  for (uint32_t i = (uint32_t)j->tid; i < j->nseg; i += (uint32_t)j->threads) {
    int r;
    if (j->mode == 0) {
      uint64_t off = (uint64_t)i * j->seg;
      uint32_t len = (uint32_t)((j->n - off) < j->seg ? (j->n - off) : j->seg);
      uint32_t cap = (uint32_t)(j->stride > 0xFFFFFFFFull ? 0xFFFFFFFFu : j->stride);
      if (j->codec == BO_CODEC_LZ4)
        r = bo_lz4_compress_block(j->in + off, len, j->slab + (uint64_t)i * j->stride, cap,
                                  &j->sizes[i]);
      else if (j->codec == BO_CODEC_LZ4_WIDE)
        r = bo_lz4_wide_compress_block(j->in + off, len, j->slab + (uint64_t)i * j->stride,
                                       cap, &j->sizes[i]);
      else if (j->codec == BO_CODEC_ZSTD)
        r = bo_zstd_compress_block(j->in + off, len, j->slab + (uint64_t)i * j->stride, cap,
                                   &j->sizes[i]);
      else if (j->codec == BO_CODEC_DEFLATE_DYN)
        r = bo_deflate_dynamic_block(j->in + off, len, j->slab + (uint64_t)i * j->stride, cap,
                                     &j->sizes[i]);
      else
        r = bo_deflate_fixed_block(j->in + off, len, j->slab + (uint64_t)i * j->stride, cap,
                                   &j->sizes[i]);
    } else {
      uint64_t off = (uint64_t)i * j->seg;
      if (j->codec == BO_CODEC_LZ4 || j->codec == BO_CODEC_LZ4_WIDE)
        r = bo_lz4_decompress_block(j->srcs[i], j->csizes[i], j->out + off, j->seg,
                                    &j->produced[i]);
      else if (j->codec == BO_CODEC_ZSTD)
        r = bo_zstd_decompress(j->srcs[i], j->csizes[i], j->out + off, j->seg, &j->produced[i]);
      else
        r = bo_inflate_raw(j->srcs[i], j->csizes[i], j->out + off, j->seg, &j->produced[i]);
    }
    if (r && !j->status) j->status = r;
  }
  return NULL;
}

static int bo_run(bo_job* proto, int threads) {
  if (threads < 1) threads = 1;
  bo_job* jobs = (bo_job*)calloc((size_t)threads, sizeof(bo_job));
  pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
  if (!jobs || !th) { free(jobs); free(th); return BO_ERR_OUT_OF_MEMORY; }
  for (int t = 0; t < threads; ++t) {
    jobs[t] = *proto;
    jobs[t].tid = t;
    jobs[t].threads = threads;
    if (threads > 1) pthread_create(&th[t], NULL, bo_worker, &jobs[t]);
  }
  if (threads == 1) bo_worker(&jobs[0]);
  int status = BO_OK;
  for (int t = 0; t < threads; ++t) {
    if (threads > 1) pthread_join(th[t], NULL);
    if (jobs[t].status && !status) status = jobs[t].status;
  }
  free(jobs);
  free(th);
  return status;
}

int bo_compress(int codec, const uint8_t* in, uint64_t n, uint32_t seg, uint8_t* slab,
                uint64_t slot_stride, uint32_t* sizes, uint32_t* nseg_out, int threads) {
  if (seg == 0) return BO_ERR_INVALID;
  if ((codec == BO_CODEC_LZ4 || codec == BO_CODEC_LZ4_WIDE || codec == BO_CODEC_ZSTD) &&
      seg > 65536u)
    return BO_ERR_INVALID;
  if (codec != BO_CODEC_LZ4 && codec != BO_CODEC_DEFLATE && codec != BO_CODEC_ZSTD &&
      codec != BO_CODEC_DEFLATE_DYN && codec != BO_CODEC_LZ4_WIDE)
    return BO_ERR_NOT_IMPLEMENTED;
  uint32_t nseg = (uint32_t)((n + seg - 1) / seg); /* device.cc:169-172 */
  *nseg_out = nseg;
  if (n == 0) return BO_OK; /* empty input -> empty BufferVector (device.cc:161-164) */
  bo_job j;
  memset(&j, 0, sizeof(j));
  j.codec = codec; j.mode = 0; j.in = in; j.n = n; j.seg = seg; j.slab = slab;
  j.stride = slot_stride; j.sizes = sizes; j.nseg = nseg;
  return bo_run(&j, threads);
}

int bo_decompress(int codec, const uint8_t* const* srcs, const uint32_t* sizes, uint32_t nseg,
                  uint32_t seg, uint8_t* out, uint64_t capacity, uint64_t* out_size,
                  uint32_t* produced, int threads) {
  *out_size = 0;
  if (nseg == 0) return BO_OK; /* device.cc:244-246 */
  if (capacity < (uint64_t)nseg * seg) return BO_ERR_CAPACITY; /* device.cc:248-254 */
  if (codec != BO_CODEC_LZ4 && codec != BO_CODEC_DEFLATE && codec != BO_CODEC_ZSTD &&
      codec != BO_CODEC_DEFLATE_DYN && codec != BO_CODEC_LZ4_WIDE)
    return BO_ERR_NOT_IMPLEMENTED;
  bo_job j;
  memset(&j, 0, sizeof(j));
  j.codec = codec; j.mode = 1; j.seg = seg; j.srcs = srcs; j.csizes = sizes; j.out = out;
  j.produced = produced; j.nseg = nseg;
  int r = bo_run(&j, threads);
  if (r) return r;
  uint64_t total = 0;
  for (uint32_t i = 0; i < nseg; ++i) total += produced[i]; /* device.cc:271-273, 312-315 */
  *out_size = total;
  return BO_OK;
}

/* ================================================================================ */
/* Synthetic inputs.  Every 64-byte line is a pure function of its   */
/* index so the HIP generator (bitar_hip_fill) can compute lines independently.      */
/* ================================================================================ */
static inline uint64_t sm64(uint64_t seed, uint64_t k) { /* k-th SplitMix64 output */
  uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static void put_dec(char* p, uint32_t v, int width) {
  for (int i = width - 1; i >= 0; --i) { p[i] = (char)('0' + v % 10); v /= 10; }
}

/* 64-byte log line #j: "HH:MM:SS.mmm LEVEL component  qp=NN seg=NNNNN status=XXXXXX\n" */
static void log_line(uint64_t seed, uint64_t j, uint8_t* out) {
  static const char* kLevel[4] = {"INFO ", "WARN ", "DEBUG", "ERROR"};
  static const char* kComp[8] = {"device   ", "driver   ", "memory   ", "pool     ",
                                 "queuepair", "config   ", "burst    ", "dequeue  "};
  static const char* kStat[4] = {"OK    ", "OK    ", "EAGAIN", "OK    "};
  uint64_t h = sm64(seed ^ 0x5bd1e995ull, j);
  char l[64];
  memset(l, ' ', sizeof(l));
  uint64_t ms = j * 7;
  put_dec(l + 0, (uint32_t)((ms / 3600000) % 24), 2); l[2] = ':';
  put_dec(l + 3, (uint32_t)((ms / 60000) % 60), 2); l[5] = ':';
  put_dec(l + 6, (uint32_t)((ms / 1000) % 60), 2); l[8] = '.';
  put_dec(l + 9, (uint32_t)(ms % 1000), 3);
  uint32_t lv = (uint32_t)(h & 15);
  memcpy(l + 13, kLevel[lv < 12 ? 0 : lv < 14 ? 1 : lv < 15 ? 2 : 3], 5);
  memcpy(l + 19, kComp[(h >> 4) & 7], 9);
  memcpy(l + 29, "qp=", 3);
  put_dec(l + 32, (uint32_t)((h >> 8) % 32), 2);
  memcpy(l + 35, "seg=", 4);
  put_dec(l + 39, (uint32_t)((h >> 16) % 100000), 5);
  memcpy(l + 45, "status=", 7);
  memcpy(l + 52, kStat[(h >> 40) & 3], 6);
  l[63] = '\n';
  memcpy(out, l, 64);
}

/* one 64-byte line of kind `kind` at line index j (byte offset 64*j) */
static void bo_line(int kind, uint64_t seed, uint64_t j, uint8_t* out) {
  uint64_t w[8];
  uint64_t k0 = j * 8;
  switch (kind) {
    case 0: /* random bytes */
      for (int i = 0; i < 8; ++i) w[i] = sm64(seed, k0 + (uint64_t)i);
      break;
    case 1: { /* Silesia-style: 3 MiB period of [int64 small range | log text | random] */
      uint64_t region = ((j * 64) >> 20) % 3;
      if (region == 0) {
        for (int i = 0; i < 8; ++i) w[i] = sm64(seed ^ 0x1111ull, k0 + (uint64_t)i) % 1000;
      } else if (region == 1) {
        log_line(seed, j, out);
        return;
      } else {
        for (int i = 0; i < 8; ++i) w[i] = sm64(seed ^ 0x2222ull, k0 + (uint64_t)i);
      }
      break;
    }
    case 2: { /* Arrow RecordBatch-like body: 4 MiB period of 1 MiB column buffers */
      uint64_t col = ((j * 64) >> 20) & 3;
      for (int i = 0; i < 8; ++i) {
        uint64_t k = k0 + (uint64_t)i, r = sm64(seed ^ (0x3333ull + col), k);
        if (col == 0) { /* int64 in [0, 1000) */
          w[i] = r % 1000;
        } else if (col == 1) { /* float64 ~ N(0,1) by Irwin-Hall(4), exact in binary */
          int64_t s = (int64_t)(r & 0xFFFF) + (int64_t)((r >> 16) & 0xFFFF) +
                      (int64_t)((r >> 32) & 0xFFFF) + (int64_t)(r >> 48) - 131070;
          double d = (double)s / 37837.0; /* sd of the 4-sum is ~37837 */
          memcpy(&w[i], &d, 8);
        } else if (col == 2) { /* two int32 dictionary indices in [0, 64) */
          w[i] = (r & 63) | (((r >> 32) & 63) << 32);
        } else {
          w[i] = 0; /* replaced by text below */
        }
      }
      if (col == 3) { log_line(seed ^ 0x4444ull, j, out); return; }
      break;
    }
    case 5: /* int64 in [0, 1000) only (region 0 of kind 1) */
      for (int i = 0; i < 8; ++i) w[i] = sm64(seed ^ 0x1111ull, k0 + (uint64_t)i) % 1000;
      break;
    case 6: /* log text only (region 1 of kind 1) */
      log_line(seed, j, out);
      return;
    case 3: /* constant */
      for (int i = 0; i < 8; ++i) w[i] = 0x6161616161616161ull;
      break;
    default: /* periodic with a 251-byte period */
      for (int b = 0; b < 64; ++b) out[b] = (uint8_t)(((j * 64 + (uint64_t)b) % 251) * 7);
      return;
  }
  for (int i = 0; i < 8; ++i)
    for (int b = 0; b < 8; ++b) out[i * 8 + b] = (uint8_t)(w[i] >> (8 * b));
}

void bo_fill(int kind, uint64_t seed, uint8_t* out, uint64_t n) {
  uint8_t line[64];
  uint64_t full = n / 64;
  for (uint64_t j = 0; j < full; ++j) bo_line(kind, seed, j, out + j * 64);
  if (n % 64) {
    bo_line(kind, seed, full, line);
    memcpy(out + full * 64, line, (size_t)(n % 64));
  }
}
