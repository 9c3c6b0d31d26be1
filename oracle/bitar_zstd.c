/*
 * bitar_zstd.c -- CPU restatement of Zstandard (RFC 8878) for the oracle.  TEST
 * INFRASTRUCTURE ONLY (see bitar_oracle.h): only tests/ and bench.py's cpu_baseline leg load
 * it, as the checker.
 *
 * Decoder: one frame per segment (the engine's unit), no dictionary; raw / RLE /
 * compressed blocks; literals raw / RLE / Huffman (1 or 4 streams, FSE-compressed or direct
 * weights, treeless reuse); sequences with predefined / RLE / FSE / repeat tables; repeat
 * offsets; content checksum (XXH64) verified.  Pinned by the libzstd 1.4.9 golden vectors
 * (tests/golden/gen_golden.py): it must decode every one of them byte-exactly.
 *
 * Encoder: the exact frame the HIP kernel emits (DESIGN.md "Zstd"): the bitar window-scan
 * parse (bitar_oracle.c bo_window_parse), one compressed block per segment, raw literals,
 * sequences coded with the predefined FSE distributions (RFC 8878 3.1.1.3.2.2).  libzstd
 * must decode it (tests/test_oracle.py).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "bitar_oracle.h"

/* ================================================================================ */
/* tables (RFC 8878 3.1.1.3.2.1 / 3.1.1.3.2.2)                                       */
/* ================================================================================ */
static const uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,   7,   8,   9,    10,   11,
                                     12, 13, 14, 15, 16, 18, 20,  22,  24,  28,   32,   40,
                                     48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384,
                                     32768, 65536};
static const uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13,   14,   15,   16,
                                     17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27,   28,   29,   30,
                                     31, 32, 33, 34, 35, 37, 39, 41, 43, 47, 51,   59,   67,   83,
                                     99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771,
                                     65539};
static const uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                                    2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const int16_t kLLDefault[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                       2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
static const int16_t kMLDefault[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                       1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                       1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
static const int16_t kOFDefault[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                       1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
#define ZS_LL_AL 6
#define ZS_ML_AL 6
#define ZS_OF_AL 5

static inline uint32_t zs_highbit(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

/* ---- XXH64 (the content checksum keeps its low 32 bits) ---------------------------- */
#define XP1 11400714785074694791ull
#define XP2 14029467366897019727ull
#define XP3 1609587929392839161ull
#define XP4 9650029242287828579ull
#define XP5 2870177450012600261ull
static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint32_t rd32le(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t xround(uint64_t acc, uint64_t in) {
  acc += in * XP2;
  acc = rotl64(acc, 31);
  return acc * XP1;
}
static inline uint64_t xmerge(uint64_t acc, uint64_t v) {
  acc ^= xround(0, v);
  return acc * XP1 + XP4;
}
uint64_t bo_xxh64(const uint8_t* p, uint64_t len, uint64_t seed) {
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
    const uint8_t* limit = end - 32;
    do {
      v1 = xround(v1, rd64(p)); p += 8;
      v2 = xround(v2, rd64(p)); p += 8;
      v3 = xround(v3, rd64(p)); p += 8;
      v4 = xround(v4, rd64(p)); p += 8;
    } while (p <= limit);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xmerge(h, v1); h = xmerge(h, v2); h = xmerge(h, v3); h = xmerge(h, v4);
  } else {
    h = seed + XP5;
  }
  h += len;
  while (p + 8 <= end) {
    h ^= xround(0, rd64(p));
    h = rotl64(h, 27) * XP1 + XP4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= (uint64_t)rd32le(p) * XP1;
    h = rotl64(h, 23) * XP2 + XP3;
    p += 4;
  }
  while (p < end) {
    h ^= (*p) * XP5;
    h = rotl64(h, 11) * XP1;
    p++;
  }
  h ^= h >> 33; h *= XP2; h ^= h >> 29; h *= XP3; h ^= h >> 32;
  return h;
}

/* ================================================================================ */
/* bit readers                                                                        */
/* ================================================================================ */
/* backward: bits [0, pos) of the stream remain; bit i = byte i>>3, bit i&7.  read(n)
 * returns bits [pos-n, pos) as a little-endian integer (zeros below bit 0), pos -= n. */
typedef struct {
  const uint8_t* s;
  int64_t pos;
} zs_bwd;

static int zs_bwd_init(zs_bwd* b, const uint8_t* s, uint32_t len) {
  if (len == 0 || s[len - 1] == 0) return -1;  /* the last byte carries the start marker */
  b->s = s;
  b->pos = (int64_t)len * 8 - 8 + zs_highbit(s[len - 1]);
  return 0;
}
static uint64_t zs_peek(const zs_bwd* b, uint32_t n) {
  uint64_t v = 0;
  for (uint32_t k = 0; k < n; ++k) {
    const int64_t i = b->pos - (int64_t)n + k;
    if (i >= 0) v |= (uint64_t)((b->s[i >> 3] >> (i & 7)) & 1u) << k;
  }
  return v;
}
static uint64_t zs_read(zs_bwd* b, uint32_t n) {
  const uint64_t v = zs_peek(b, n);
  b->pos -= n;
  return v;
}

/* ================================================================================ */
/* FSE                                                                                */
/* ================================================================================ */
typedef struct {
  uint16_t sym;
  uint8_t nbits;
  uint16_t base;
} zs_fse_cell;

typedef struct {
  uint32_t al;  /* accuracy log */
  zs_fse_cell t[1u << 9];
} zs_fse;

static uint64_t zs_fwd_peek(const uint8_t* s, uint32_t len, uint64_t pos, uint32_t n) {
  uint64_t v = 0;
  for (uint32_t k = 0; k < n; ++k) {
    const uint64_t i = pos + k;
    if (i < (uint64_t)len * 8) v |= (uint64_t)((s[i >> 3] >> (i & 7)) & 1u) << k;
  }
  return v;
}

/* FSE_readNCount: the normalized counts at src; returns bytes used or -1 */
static int zs_read_ncount(int16_t* norm, uint32_t* max_sym, uint32_t* al, const uint8_t* src,
                          uint32_t len, uint32_t max_al) {
  uint64_t bitpos = 0;
#define ZS_FPEEK(n) zs_fwd_peek(src, len, bitpos, (n))
  const uint32_t hdr = (uint32_t)ZS_FPEEK(4);
  uint32_t log = hdr + 5;
  if (log > max_al) return -1;
  bitpos += 4;
  int remaining = (1 << log) + 1;
  int threshold = 1 << log;
  uint32_t nbits = log + 1;
  uint32_t sym = 0;
  int prev0 = 0;
  while (remaining > 1 && sym <= *max_sym) {
    if (prev0) {
      uint32_t n0 = sym;
      while ((ZS_FPEEK(16) & 0xFFFF) == 0xFFFF) { n0 += 24; bitpos += 16; }
      while ((ZS_FPEEK(2) & 3) == 3) { n0 += 3; bitpos += 2; }
      n0 += (uint32_t)(ZS_FPEEK(2) & 3);
      bitpos += 2;
      if (n0 > *max_sym) return -1;
      while (sym < n0) norm[sym++] = 0;
    }
    const int max = (2 * threshold - 1) - remaining;
    int count;
    const uint32_t v = (uint32_t)ZS_FPEEK(nbits);
    if ((int)(v & (uint32_t)(threshold - 1)) < max) {
      count = (int)(v & (uint32_t)(threshold - 1));
      bitpos += nbits - 1;
    } else {
      count = (int)(v & (uint32_t)(2 * threshold - 1));
      if (count >= threshold) count -= max;
      bitpos += nbits;
    }
    count--;
    remaining -= count < 0 ? -count : count;
    norm[sym++] = (int16_t)count;
    prev0 = count == 0;
    while (remaining < threshold) { nbits--; threshold >>= 1; }
  }
#undef ZS_FPEEK
  if (remaining != 1 || bitpos > (uint64_t)len * 8) return -1;
  *max_sym = sym - 1;
  *al = log;
  return (int)((bitpos + 7) >> 3);
}

/* FSE_buildDTable */
static int zs_fse_build(zs_fse* f, const int16_t* norm, uint32_t max_sym, uint32_t al) {
  const uint32_t size = 1u << al;
  uint32_t high = size - 1;
  uint16_t next[256];
  for (uint32_t s = 0; s <= max_sym; ++s) {
    if (norm[s] == -1) {
      f->t[high--].sym = (uint16_t)s;
      next[s] = 1;
    } else {
      next[s] = (uint16_t)norm[s];
    }
  }
  const uint32_t step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
  uint32_t pos = 0;
  for (uint32_t s = 0; s <= max_sym; ++s) {
    for (int i = 0; i < norm[s]; ++i) {
      f->t[pos].sym = (uint16_t)s;
      do { pos = (pos + step) & mask; } while (pos > high);
    }
  }
  if (pos != 0) return -1;
  for (uint32_t u = 0; u < size; ++u) {
    const uint32_t s = f->t[u].sym;
    const uint32_t ns = next[s]++;
    const uint32_t nb = al - zs_highbit(ns);
    f->t[u].nbits = (uint8_t)nb;
    f->t[u].base = (uint16_t)((ns << nb) - size);
  }
  f->al = al;
  return 0;
}

static void zs_fse_rle(zs_fse* f, uint32_t sym) {
  f->al = 0;
  f->t[0].sym = (uint16_t)sym;
  f->t[0].nbits = 0;
  f->t[0].base = 0;
}

/* ================================================================================ */
/* Huffman literals                                                                   */
/* ================================================================================ */
typedef struct {
  uint32_t log;  /* max code length */
  uint8_t sym[1u << 11];
  uint8_t nbits[1u << 11];
  int valid;
} zs_huf;

/* Huffman tree description at src; returns bytes used or -1 */
static int zs_huf_read(zs_huf* h, const uint8_t* src, uint32_t len) {
  if (len < 1) return -1;
  uint8_t w[256];
  uint32_t nw = 0;
  const uint32_t hb = src[0];
  int used;
  if (hb < 128) {  /* FSE-compressed weights, hb bytes */
    if (1 + hb > len) return -1;
    int16_t norm[256];
    uint32_t max_sym = 255, al;
    const int n = zs_read_ncount(norm, &max_sym, &al, src + 1, hb, 6);
    if (n < 0) return -1;
    zs_fse f;
    if (zs_fse_build(&f, norm, max_sym, al)) return -1;
    zs_bwd b;
    if (zs_bwd_init(&b, src + 1 + n, hb - (uint32_t)n)) return -1;
    uint32_t s1 = (uint32_t)zs_read(&b, al), s2 = (uint32_t)zs_read(&b, al);
    for (;;) {
      if (nw > 254) return -1;
      w[nw++] = (uint8_t)f.t[s1].sym;
      s1 = f.t[s1].base + (uint32_t)zs_read(&b, f.t[s1].nbits);
      if (b.pos < 0) { w[nw++] = (uint8_t)f.t[s2].sym; break; }
      if (nw > 254) return -1;
      w[nw++] = (uint8_t)f.t[s2].sym;
      s2 = f.t[s2].base + (uint32_t)zs_read(&b, f.t[s2].nbits);
      if (b.pos < 0) { w[nw++] = (uint8_t)f.t[s1].sym; break; }
    }
    used = 1 + (int)hb;
  } else {  /* direct 4-bit weights */
    nw = hb - 127;
    const uint32_t nb = (nw + 1) / 2;
    if (1 + nb > len) return -1;
    for (uint32_t i = 0; i < nw; ++i) w[i] = (i & 1) ? (src[1 + i / 2] & 15) : (src[1 + i / 2] >> 4);
    used = 1 + (int)nb;
  }
  /* the last symbol's weight completes the total to a power of two */
  uint32_t total = 0;
  for (uint32_t i = 0; i < nw; ++i) {
    if (w[i] > 11) return -1;
    if (w[i]) total += 1u << (w[i] - 1);
  }
  if (total == 0) return -1;
  const uint32_t maxb = zs_highbit(total) + 1;
  if (maxb > 11) return -1;
  const uint32_t rest = (1u << maxb) - total;
  if (rest & (rest - 1)) return -1;  /* not a power of two */
  w[nw++] = (uint8_t)(zs_highbit(rest) + 1);
  /* HUF_readDTableX1 */
  uint32_t rank[13] = {0};
  for (uint32_t i = 0; i < nw; ++i) rank[w[i]]++;
  /* the longest codes (weight 1) come in pairs, at least one: libzstd's HUF_readStats
   * rejects any other description ("tree construction validity"), though such weights can
   * still form a complete code (e.g. 2 2 3: lengths 2 2 1 under a table log of 3) */
  if (rank[1] < 2 || (rank[1] & 1)) return -1;
  uint32_t next = 0;
  for (uint32_t n = 1; n <= maxb; ++n) {
    const uint32_t cur = next;
    next += rank[n] << (n - 1);
    rank[n] = cur;
  }
  if (next != (1u << maxb)) return -1;
  for (uint32_t s = 0; s < nw; ++s) {
    const uint32_t wt = w[s];
    if (!wt) continue;
    const uint32_t l = (1u << wt) >> 1;
    for (uint32_t u = rank[wt]; u < rank[wt] + l; ++u) {
      h->sym[u] = (uint8_t)s;
      h->nbits[u] = (uint8_t)(maxb + 1 - wt);
    }
    rank[wt] += l;
  }
  h->log = maxb;
  h->valid = 1;
  return used;
}

/* why the last bo_zstd_decompress on this thread rejected its frame (tests only): a Huffman
 * literal stream that was not consumed exactly records BO_ZSTD_REJECT_HUF_END and the
 * remaining bit count (negative: read past the stream's start) */
static __thread int g_zs_reject;
static __thread int64_t g_zs_reject_detail;
int bo_zstd_last_reject(int64_t* detail) {
  if (detail) *detail = g_zs_reject_detail;
  return g_zs_reject;
}

static int zs_huf_stream(const zs_huf* h, const uint8_t* src, uint32_t len, uint8_t* out,
                         uint32_t n) {
  zs_bwd b;
  if (zs_bwd_init(&b, src, len)) return -1;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t v = (uint32_t)zs_peek(&b, h->log);
    out[i] = h->sym[v];
    b.pos -= h->nbits[v];
  }
  if (b.pos != 0) {
    g_zs_reject = BO_ZSTD_REJECT_HUF_END;
    g_zs_reject_detail = b.pos;
    return -1;
  }
  return 0;
}

/* ================================================================================ */
/* frame / block decode                                                               */
/* ================================================================================ */
typedef struct {
  zs_huf huf;
  zs_fse ll, of, ml;
  int have_ll, have_of, have_ml;
  uint32_t rep[3];
} zs_ctx;

static int zs_table(zs_fse* f, int* have, uint32_t mode, const int16_t* def, uint32_t def_max,
                    uint32_t def_al, uint32_t max_sym, uint32_t max_al, const uint8_t* src,
                    uint32_t len, uint32_t* used) {
  *used = 0;
  if (mode == 0) {
    if (zs_fse_build(f, def, def_max, def_al)) return -1;
  } else if (mode == 1) {
    if (len < 1 || src[0] > max_sym) return -1;
    zs_fse_rle(f, src[0]);
    *used = 1;
  } else if (mode == 2) {
    int16_t norm[256];
    uint32_t ms = max_sym, al;
    const int n = zs_read_ncount(norm, &ms, &al, src, len, max_al);
    if (n < 0) return -1;
    if (zs_fse_build(f, norm, ms, al)) return -1;
    *used = (uint32_t)n;
  } else {
    if (!*have) return -1;
  }
  *have = 1;
  return 0;
}

static int zs_block(zs_ctx* z, const uint8_t* src, uint32_t len, uint8_t* dst, uint32_t cap,
                    uint32_t op0, uint32_t* op_io) {
  /* ---- literals section ---- */
  if (len < 1) return -1;
  const uint32_t lt = src[0] & 3, sf = (src[0] >> 2) & 3;
  uint32_t regen, csz = 0, hsz, nstreams = 1;
  if (lt < 2) {
    if (sf == 0 || sf == 2) { regen = src[0] >> 3; hsz = 1; }
    else if (sf == 1) { if (len < 2) return -1; regen = (src[0] >> 4) + ((uint32_t)src[1] << 4); hsz = 2; }
    else { if (len < 3) return -1; regen = (src[0] >> 4) + ((uint32_t)src[1] << 4) + ((uint32_t)src[2] << 12); hsz = 3; }
  } else {
    if (sf <= 1) {
      if (len < 3) return -1;
      const uint32_t c = src[0] | ((uint32_t)src[1] << 8) | ((uint32_t)src[2] << 16);
      regen = (c >> 4) & 0x3FF; csz = (c >> 14) & 0x3FF; hsz = 3; nstreams = sf == 0 ? 1 : 4;
    } else if (sf == 2) {
      if (len < 4) return -1;
      const uint32_t c = rd32le(src);
      regen = (c >> 4) & 0x3FFF; csz = (c >> 18) & 0x3FFF; hsz = 4; nstreams = 4;
    } else {
      if (len < 5) return -1;
      const uint64_t c = (uint64_t)rd32le(src) | ((uint64_t)src[4] << 32);
      regen = (uint32_t)(c >> 4) & 0x3FFFF; csz = (uint32_t)(c >> 22) & 0x3FFFF; hsz = 5; nstreams = 4;
    }
  }
  if (regen > (128u << 10)) return -1;
  uint8_t* lit = (uint8_t*)malloc(regen ? regen : 1);
  if (!lit) return -1;
  uint32_t p = hsz;
  int rc = -1;
  if (lt == 0) {
    if (p + regen > len) goto out;
    memcpy(lit, src + p, regen);
    p += regen;
  } else if (lt == 1) {
    if (p + 1 > len) goto out;
    memset(lit, src[p], regen);
    p += 1;
  } else {
    if (p + csz > len) goto out;
    const uint8_t* cs = src + p;
    uint32_t cl = csz;
    if (lt == 2) {
      const int n = zs_huf_read(&z->huf, cs, cl);
      if (n < 0) goto out;
      cs += n;
      cl -= (uint32_t)n;
    } else if (!z->huf.valid) {
      goto out;
    }
    if (nstreams == 1) {
      if (zs_huf_stream(&z->huf, cs, cl, lit, regen)) goto out;
    } else {
      if (cl < 6) goto out;
      const uint32_t s1 = cs[0] | (cs[1] << 8), s2 = cs[2] | (cs[3] << 8), s3 = cs[4] | (cs[5] << 8);
      if ((uint64_t)6 + s1 + s2 + s3 > cl) goto out;
      const uint32_t s4 = cl - 6 - s1 - s2 - s3;
      const uint32_t q = (regen + 3) / 4;
      if (3 * q > regen) goto out;
      const uint8_t* st = cs + 6;
      if (zs_huf_stream(&z->huf, st, s1, lit, q)) goto out;
      if (zs_huf_stream(&z->huf, st + s1, s2, lit + q, q)) goto out;
      if (zs_huf_stream(&z->huf, st + s1 + s2, s3, lit + 2 * q, q)) goto out;
      if (zs_huf_stream(&z->huf, st + s1 + s2 + s3, s4, lit + 3 * q, regen - 3 * q)) goto out;
    }
    p += csz;
  }
  /* ---- sequences section ---- */
  {
    if (p >= len) goto out;
    uint32_t nseq = src[p];
    if (nseq == 0) {
      p += 1;
    } else if (nseq < 128) {
      p += 1;
    } else if (nseq < 255) {
      if (p + 2 > len) goto out;
      nseq = ((nseq - 128) << 8) + src[p + 1];
      p += 2;
    } else {
      if (p + 3 > len) goto out;
      nseq = src[p + 1] + ((uint32_t)src[p + 2] << 8) + 0x7F00;
      p += 3;
    }
    uint32_t op = *op_io, lp = 0;
    if (nseq) {
      if (p >= len) goto out;
      const uint32_t modes = src[p++];
      if (modes & 3) goto out;
      uint32_t used;
      if (zs_table(&z->ll, &z->have_ll, modes >> 6, kLLDefault, 35, ZS_LL_AL, 35, 9, src + p, len - p, &used)) goto out;
      p += used;
      if (zs_table(&z->of, &z->have_of, (modes >> 4) & 3, kOFDefault, 28, ZS_OF_AL, 31, 8, src + p, len - p, &used)) goto out;
      p += used;
      if (zs_table(&z->ml, &z->have_ml, (modes >> 2) & 3, kMLDefault, 52, ZS_ML_AL, 52, 9, src + p, len - p, &used)) goto out;
      p += used;
      zs_bwd b;
      if (p >= len || zs_bwd_init(&b, src + p, len - p)) goto out;
      uint32_t sll = (uint32_t)zs_read(&b, z->ll.al), sof = (uint32_t)zs_read(&b, z->of.al),
               sml = (uint32_t)zs_read(&b, z->ml.al);
      for (uint32_t k = 0; k < nseq; ++k) {
        const uint32_t llc = z->ll.t[sll].sym, ofc = z->of.t[sof].sym, mlc = z->ml.t[sml].sym;
        if (llc > 35 || mlc > 52 || ofc > 31) goto seq_fail;
        const uint32_t ofv = (1u << ofc) + (uint32_t)zs_read(&b, ofc);
        const uint32_t ml = kMLBase[mlc] + (uint32_t)zs_read(&b, kMLBits[mlc]);
        const uint32_t ll = kLLBase[llc] + (uint32_t)zs_read(&b, kLLBits[llc]);
        if (k + 1 < nseq) {
          sll = z->ll.t[sll].base + (uint32_t)zs_read(&b, z->ll.t[sll].nbits);
          sml = z->ml.t[sml].base + (uint32_t)zs_read(&b, z->ml.t[sml].nbits);
          sof = z->of.t[sof].base + (uint32_t)zs_read(&b, z->of.t[sof].nbits);
        }
        uint32_t off;
        if (ofv > 3) {
          off = ofv - 3;
          z->rep[2] = z->rep[1]; z->rep[1] = z->rep[0]; z->rep[0] = off;
        } else {
          const uint32_t idx = ofv + (ll == 0 ? 1u : 0u);
          if (idx == 1) {
            off = z->rep[0];
          } else if (idx == 2) {
            off = z->rep[1];
            z->rep[1] = z->rep[0]; z->rep[0] = off;
          } else if (idx == 3) {
            off = z->rep[2];
            z->rep[2] = z->rep[1]; z->rep[1] = z->rep[0]; z->rep[0] = off;
          } else {
            off = z->rep[0] - 1;
            if (off == 0) goto seq_fail;
            z->rep[2] = z->rep[1]; z->rep[1] = z->rep[0]; z->rep[0] = off;
          }
        }
        if (lp + ll > regen || (uint64_t)op + ll + ml > cap) goto seq_fail;
        memcpy(dst + op, lit + lp, ll);
        op += ll;
        lp += ll;
        if (off == 0 || off > op) goto seq_fail;  /* no dictionary: history is this frame */
        for (uint32_t i = 0; i < ml; ++i) dst[op + i] = dst[op - off + i];
        op += ml;
      }
      if (b.pos == 0) goto seq_done;
    seq_fail:
      if (b.pos < 0) { /* the sequence bitstream was read past its start */
        g_zs_reject = BO_ZSTD_REJECT_SEQ_OVERREAD;
        g_zs_reject_detail = b.pos;
      }
      goto out;
    seq_done:;
    } else if (p != len) {
      goto out;
    }
    if ((uint64_t)op + (regen - lp) > cap) goto out;
    memcpy(dst + op, lit + lp, regen - lp);
    op += regen - lp;
    *op_io = op;
    (void)op0;
  }
  rc = 0;
out:
  free(lit);
  return rc;
}

int bo_zstd_decompress(const uint8_t* src, uint32_t csize, uint8_t* dst, uint32_t cap,
                       uint32_t* produced) {
  g_zs_reject = 0;
  g_zs_reject_detail = 0;
  if (csize < 6 || rd32le(src) != 0xFD2FB528u) return BO_ERR_IO;
  uint32_t p = 4;
  const uint32_t fhd = src[p++];
  const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, cks = (fhd >> 2) & 1,
                 did_flag = fhd & 3;
  if (fhd & 8) return BO_ERR_IO;  /* reserved bit */
  if (!single) {
    if (p >= csize) return BO_ERR_IO;
    p++;  /* window descriptor: the whole frame is one segment, history = the frame */
  }
  static const uint32_t did_sz[4] = {0, 1, 2, 4};
  if (p + did_sz[did_flag] > csize) return BO_ERR_IO;
  uint32_t did = 0;
  for (uint32_t i = 0; i < did_sz[did_flag]; ++i) did |= (uint32_t)src[p + i] << (8 * i);
  p += did_sz[did_flag];
  if (did) return BO_ERR_IO;  /* dictionaries are not supported */
  static const uint32_t fcs_sz[4] = {0, 2, 4, 8};
  uint32_t fsz = fcs_sz[fcs_flag];
  if (fcs_flag == 0 && single) fsz = 1;
  if (p + fsz > csize) return BO_ERR_IO;
  uint64_t fcs = 0;
  int has_fcs = fsz != 0;
  for (uint32_t i = 0; i < fsz; ++i) fcs |= (uint64_t)src[p + i] << (8 * i);
  if (fsz == 2) fcs += 256;
  p += fsz;
  if (has_fcs && fcs > cap) return BO_ERR_IO;
  zs_ctx* z = (zs_ctx*)calloc(1, sizeof(zs_ctx));
  if (!z) return BO_ERR_OUT_OF_MEMORY;
  z->rep[0] = 1; z->rep[1] = 4; z->rep[2] = 8;
  uint32_t op = 0;
  int rc = BO_ERR_IO;
  for (;;) {
    if (p + 3 > csize) goto done;
    const uint32_t bh = src[p] | ((uint32_t)src[p + 1] << 8) | ((uint32_t)src[p + 2] << 16);
    p += 3;
    const uint32_t last = bh & 1, type = (bh >> 1) & 3, bsz = bh >> 3;
    if (type == 0) {
      if (p + bsz > csize || (uint64_t)op + bsz > cap) goto done;
      memcpy(dst + op, src + p, bsz);
      op += bsz;
      p += bsz;
    } else if (type == 1) {
      if (p + 1 > csize || (uint64_t)op + bsz > cap) goto done;
      memset(dst + op, src[p], bsz);
      op += bsz;
      p += 1;
    } else if (type == 2) {
      if (bsz > (128u << 10) || p + bsz > csize) goto done;
      if (zs_block(z, src + p, bsz, dst, cap, op, &op)) goto done;
      p += bsz;
    } else {
      goto done;
    }
    if (last) break;
  }
  if (cks) {
    if (p + 4 > csize) goto done;
    if ((uint32_t)bo_xxh64(dst, op, 0) != rd32le(src + p)) goto done;
    p += 4;
  }
  if (p != csize) goto done;            /* one frame per segment */
  if (has_fcs && fcs != op) goto done;
  *produced = op;
  rc = BO_OK;
done:
  free(z);
  return rc;
}

/* ================================================================================ */
/* encoder: the frame the HIP kernels write (zstd_compress.hip)                       */
/* ================================================================================ */
/* One frame per segment: single-segment header with the content size, then ONE block (a
 * segment is <= 64 KiB, below the 128 KiB block limit), compressed or -- when that is not
 * smaller than the input -- raw.  Inside the compressed block:
 *
 *   parse      the bitar window-scan parse (bo_window_parse, distance <= 2560);
 *   offsets    repeat offsets (RFC 8878 3.1.2.5, history 1 4 8): a match whose distance is
 *              in the history is coded as its repeat code, else as distance + 3;
 *   literals   nlit == 0: raw; one distinct byte: RLE; else Huffman (code lengths by
 *              bo_huff_lengths limited to 11 bits; weights direct when <= 128 are sent and
 *              not larger than their FSE form, else FSE-compressed with two interleaved
 *              states), 1 stream below 256 literals, else 4; raw when the Huffman section
 *              is not at least nlit/64 + 2 bytes smaller;
 *   sequences  per table (literal lengths, offsets, match lengths): one distinct code ->
 *              RLE; else FSE_Compressed with counts normalized by zs_normalize when its
 *              estimated size (fixed-point log2 costs + table description) is below the
 *              predefined distribution's, else predefined.
 * Every choice is integer arithmetic, so the kernels reproduce it bit for bit. */

/* 256 * log2(1 + i / 64), rounded */
static const uint8_t kLog2Frac[64] = {
    0,   6,   11,  17,  22,  28,  33,  38,  44,  49,  54,  59,  63,  68,  73,  78,
    82,  87,  92,  96,  100, 105, 109, 113, 118, 122, 126, 130, 134, 138, 142, 146,
    150, 154, 157, 161, 165, 169, 172, 176, 179, 183, 186, 190, 193, 197, 200, 203,
    207, 210, 213, 216, 220, 223, 226, 229, 232, 235, 238, 241, 244, 247, 250, 253};

/* 256 * log2(x) in fixed point, x >= 1 */
static uint32_t zs_log2fix(uint32_t x) {
  const uint32_t hb = zs_highbit(x);
  const uint32_t f = (hb >= 6 ? x >> (hb - 6) : x << (6 - hb)) & 63u;
  return (hb << 8) + kLog2Frac[f];
}

/* FSE table log for `total` symbols of alphabet [0, max_sym] (FSE_optimalTableLog's rule):
 * at most the source size's bits - 2, at least what the alphabet and source need, in
 * [5, max_log].  total >= 2, max_sym >= 1. */
static uint32_t zs_table_log(uint32_t max_log, uint32_t total, uint32_t max_sym) {
  int tl = (int)max_log;
  const int src_bits = (int)zs_highbit(total - 1) - 2;
  if (src_bits < tl) tl = src_bits;
  const int a = (int)zs_highbit(total) + 1, b = (int)zs_highbit(max_sym) + 2;
  const int min_bits = a < b ? a : b;
  if (min_bits > tl) tl = min_bits;
  if (tl < 5) tl = 5;
  if (tl > (int)max_log) tl = (int)max_log;
  return (uint32_t)tl;
}

/* counts -> normalized counts summing to 2^tl: rounded shares, at least 1 per used symbol;
 * a shortfall goes to the most frequent symbol, an excess is taken from the largest
 * normalized counts (first symbol on ties) down to 1 */
static void zs_normalize(const uint32_t* cnt, uint32_t max_sym, uint32_t total, uint32_t tl,
                         int16_t* norm) {
  const uint32_t size = 1u << tl;
  int32_t sum = 0;
  for (uint32_t s = 0; s <= max_sym; ++s) {
    uint32_t v = 0;
    if (cnt[s]) {
      v = (cnt[s] * size + total / 2) / total;
      if (v == 0) v = 1;
    }
    norm[s] = (int16_t)v;
    sum += (int32_t)v;
  }
  int32_t delta = (int32_t)size - sum;
  if (delta > 0) {
    uint32_t best = 0;
    for (uint32_t s = 1; s <= max_sym; ++s) if (cnt[s] > cnt[best]) best = s;
    norm[best] = (int16_t)(norm[best] + delta);
  }
  while (delta < 0) {
    uint32_t best = 0;
    for (uint32_t s = 1; s <= max_sym; ++s) if (norm[s] > norm[best]) best = s;
    int32_t take = norm[best] - 1;
    if (take > -delta) take = -delta;
    norm[best] = (int16_t)(norm[best] - take);
    delta += take;
  }
}

typedef struct {  /* forward bit writer (BIT_CStream) */
  uint8_t* out;
  uint32_t pos, cap;
  uint64_t acc;
  uint32_t nb;
  int err;
} zs_bw;

static void zs_bw_add(zs_bw* w, uint64_t v, uint32_t n) {
  if (n == 0) return;
  w->acc |= (v & ((1ull << n) - 1)) << w->nb;
  w->nb += n;
  while (w->nb >= 8) {
    if (w->pos >= w->cap) { w->err = 1; return; }
    w->out[w->pos++] = (uint8_t)w->acc;
    w->acc >>= 8;
    w->nb -= 8;
  }
}
/* pad to a byte boundary (no end mark) */
static void zs_bw_pad(zs_bw* w) {
  if (w->nb) {
    if (w->pos >= w->cap) { w->err = 1; return; }
    w->out[w->pos++] = (uint8_t)w->acc;
    w->acc = 0;
    w->nb = 0;
  }
}
static void zs_bw_close(zs_bw* w) {
  zs_bw_add(w, 1, 1);  /* end mark */
  zs_bw_pad(w);
}

/* FSE_writeNCount: the table description of norm[0..max_sym]; returns its size in bytes */
static uint32_t zs_write_ncount(zs_bw* w, const int16_t* norm, uint32_t max_sym, uint32_t tl) {
  const uint32_t p0 = w->pos;
  zs_bw_add(w, tl - 5, 4);
  int remaining = (1 << tl) + 1, threshold = 1 << tl;
  uint32_t nbits = tl + 1, s = 0;
  int prev0 = 0;
  while (s <= max_sym && remaining > 1) {
    if (prev0) {
      uint32_t start = s;
      while (norm[s] == 0) ++s;
      while (s >= start + 3) { zs_bw_add(w, 3, 2); start += 3; }
      zs_bw_add(w, s - start, 2);
    }
    int count = norm[s++];
    const int max = (2 * threshold - 1) - remaining;
    remaining -= count < 0 ? -count : count;
    ++count;
    if (count >= threshold) count += max;
    zs_bw_add(w, (uint32_t)count, nbits - (count < max ? 1u : 0u));
    prev0 = count == 1;
    while (remaining < threshold) { --nbits; threshold >>= 1; }
  }
  zs_bw_pad(w);
  return w->pos - p0;
}

typedef struct {
  uint16_t state[1u << 9];
  int32_t dnb[64];   /* deltaNbBits */
  int32_t dfs[64];   /* deltaFindState */
  uint32_t al;
} zs_ctable;

/* FSE_buildCTable for a normalized distribution (-1 = "less than 1" allowed) */
static void zs_build_ctable(zs_ctable* c, const int16_t* norm, uint32_t max_sym, uint32_t al) {
  const uint32_t size = 1u << al, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
  uint32_t high = size - 1;
  uint8_t sym_at[1u << 9];
  uint32_t cumul[65];
  cumul[0] = 0;
  for (uint32_t s = 1; s <= max_sym + 1; ++s) {
    if (norm[s - 1] == -1) {
      cumul[s] = cumul[s - 1] + 1;
      sym_at[high--] = (uint8_t)(s - 1);
    } else {
      cumul[s] = cumul[s - 1] + (uint32_t)norm[s - 1];
    }
  }
  uint32_t pos = 0;
  for (uint32_t s = 0; s <= max_sym; ++s)
    for (int i = 0; i < norm[s]; ++i) {
      sym_at[pos] = (uint8_t)s;
      do { pos = (pos + step) & mask; } while (pos > high);
    }
  for (uint32_t u = 0; u < size; ++u) c->state[cumul[sym_at[u]]++] = (uint16_t)(size + u);
  int32_t total = 0;
  for (uint32_t s = 0; s <= max_sym; ++s) {
    if (norm[s] == 0) {
      c->dnb[s] = (int32_t)(((al + 1) << 16) - size);
      c->dfs[s] = 0;
    } else if (norm[s] == -1 || norm[s] == 1) {
      c->dnb[s] = (int32_t)((al << 16) - size);
      c->dfs[s] = total - 1;
      total += 1;
    } else {
      const uint32_t mbo = al - zs_highbit((uint32_t)norm[s] - 1);
      const uint32_t msp = (uint32_t)norm[s] << mbo;
      c->dnb[s] = (int32_t)((mbo << 16) - msp);
      c->dfs[s] = total - norm[s];
      total += norm[s];
    }
  }
  c->al = al;
}

static void zs_enc_init(const zs_ctable* c, uint32_t* st, uint32_t s) {  /* FSE_initCState2 */
  const uint32_t nbo = (uint32_t)((c->dnb[s] + (1 << 15)) >> 16);
  const uint32_t value = (nbo << 16) - (uint32_t)c->dnb[s];
  *st = c->state[(value >> nbo) + c->dfs[s]];
}
static void zs_enc_sym(zs_bw* w, const zs_ctable* c, uint32_t* st, uint32_t s) {
  const uint32_t nbo = (uint32_t)((*st + (uint32_t)c->dnb[s]) >> 16);
  zs_bw_add(w, *st, nbo);
  *st = c->state[(*st >> nbo) + c->dfs[s]];
}

uint32_t bo_zstd_ll_code(uint32_t ll) {
  uint32_t c = 35;
  while (kLLBase[c] > ll) --c;
  return c;
}
uint32_t bo_zstd_ml_code(uint32_t ml) {  /* ml >= 3 */
  uint32_t c = 52;
  while (kMLBase[c] > ml) --c;
  return c;
}

/* ---- literals section ---- */
static void zs_lit_header(uint8_t* d, uint32_t type, uint32_t n, uint32_t* hsz) {
  if (n < 32) {
    d[0] = (uint8_t)(type | (n << 3));
    *hsz = 1;
  } else if (n < 4096) {
    d[0] = (uint8_t)(type | (1u << 2) | ((n & 15u) << 4));
    d[1] = (uint8_t)(n >> 4);
    *hsz = 2;
  } else {
    d[0] = (uint8_t)(type | (3u << 2) | ((n & 15u) << 4));
    d[1] = (uint8_t)(n >> 4);
    d[2] = (uint8_t)(n >> 12);
    *hsz = 3;
  }
}

/* Huffman tree description of weights w[0..nw-1] (FSE form); 0 if it cannot be FSE-coded
 * (fewer than 2 weights, one distinct weight, or >= 128 bytes).  out: >= 128 bytes. */
static uint32_t zs_weights_fse(const uint8_t* w, uint32_t nw, uint8_t* out) {
  if (nw < 2) return 0;
  uint32_t cnt[13] = {0}, max_w = 0, distinct = 0;
  for (uint32_t i = 0; i < nw; ++i) {
    if (!cnt[w[i]]++) ++distinct;
    if (w[i] > max_w) max_w = w[i];
  }
  if (distinct < 2) return 0;
  const uint32_t tl = zs_table_log(6, nw, max_w);
  int16_t norm[13];
  zs_normalize(cnt, max_w, nw, tl, norm);
  uint8_t buf[512];
  zs_bw bw = {buf + 1, 0, 500, 0, 0, 0};
  zs_write_ncount(&bw, norm, max_w, tl);
  zs_ctable ct;
  zs_build_ctable(&ct, norm, max_w, tl);
  /* FSE_compress_usingCTable: weights from the last, two states, state 1 flushed last */
  uint32_t s1, s2;
  int32_t i = (int32_t)nw;
  if (nw & 1) {
    zs_enc_init(&ct, &s1, w[--i]);
    zs_enc_init(&ct, &s2, w[--i]);
    zs_enc_sym(&bw, &ct, &s1, w[--i]);
  } else {
    zs_enc_init(&ct, &s2, w[--i]);
    zs_enc_init(&ct, &s1, w[--i]);
  }
  while (i > 0) {
    zs_enc_sym(&bw, &ct, &s2, w[--i]);
    zs_enc_sym(&bw, &ct, &s1, w[--i]);
  }
  zs_bw_add(&bw, s2, tl);
  zs_bw_add(&bw, s1, tl);
  zs_bw_close(&bw);
  if (bw.err || bw.pos >= 128) return 0;
  buf[0] = (uint8_t)bw.pos;
  memcpy(out, buf, bw.pos + 1);
  return bw.pos + 1;
}

/* The literal code of a frame: built once from all of the segment's literals and shared by
 * its blocks (the first Huffman-coded block carries the tree, later ones are Treeless). */
typedef struct {
  uint32_t mode;     /* 0 raw, 1 RLE (one distinct byte), 2 Huffman-capable */
  uint32_t nlit;     /* all of the frame's literals */
  uint64_t tb;       /* their Huffman-coded bits: sum of length x count */
  uint8_t rle;
  uint8_t len[256];
  uint32_t code[256];
  uint8_t desc[130];
  uint32_t dsz;
} zs_littab;

static void zs_littab_build(const uint8_t* lit, uint32_t n, zs_littab* H) {
  uint32_t hist[256] = {0}, distinct = 0;
  for (uint32_t i = 0; i < n; ++i)
    if (!hist[lit[i]]++) ++distinct;
  H->mode = 0;
  H->dsz = 0;
  H->nlit = n;
  H->tb = 0;
  if (n == 0) return;
  if (distinct == 1) {
    H->mode = 1;
    H->rle = lit[0];
    return;
  }
  /* ---- Huffman ---- */
  bo_huff_lengths(hist, 256, 11, H->len);
  uint32_t L = 0, max_sym = 0;
  for (uint32_t s = 0; s < 256; ++s) {
    if (H->len[s] > L) L = H->len[s];
    if (H->len[s]) max_sym = s;
  }
  uint8_t w[256];
  uint32_t rank_cnt[13] = {0};
  for (uint32_t s = 0; s < 256; ++s) {
    w[s] = H->len[s] ? (uint8_t)(L + 1 - H->len[s]) : 0;
    if (H->len[s]) rank_cnt[w[s]]++;
  }
  /* codes: table index ranges by increasing weight, then symbol (HUF_readDTableX1) */
  uint32_t start[13], next = 0;
  for (uint32_t k = 1; k <= L; ++k) {
    start[k] = next;
    next += rank_cnt[k] << (k - 1);
  }
  for (uint32_t s = 0; s < 256; ++s) {
    if (!H->len[s]) continue;
    H->code[s] = start[w[s]] >> (w[s] - 1);
    start[w[s]] += 1u << (w[s] - 1);
  }
  /* tree description: direct when possible and not larger than the FSE form */
  const uint32_t nw = max_sym;
  const uint32_t fsz = zs_weights_fse(w, nw, H->desc);
  const uint32_t direct = nw <= 128 ? 1 + (nw + 1) / 2 : 0;
  if (direct && (!fsz || direct <= fsz)) {
    H->desc[0] = (uint8_t)(127 + nw);
    for (uint32_t i = 0; i < nw; i += 2)
      H->desc[1 + i / 2] = (uint8_t)((w[i] << 4) | (i + 1 < nw ? w[i + 1] : 0));
    H->dsz = direct;
  } else {
    H->dsz = fsz;
  }
  if (H->dsz) H->mode = 2;
  for (uint32_t s = 0; s < 256; ++s) H->tb += (uint64_t)H->len[s] * hist[s];
}

/* literals section of one block, lit[0..n), into d; returns its size.  Huffman when the
 * block's section -- the tree included while *tree_sent is 0 -- is at least n/64 + 2 bytes
 * smaller than n, both by an estimate from the frame's statistics (the block's share of all
 * coded bits, n tb / nlit) and exactly (then *tree_sent = 1; the block is Treeless when it
 * already was 1); RLE for an RLE code and n > 0; raw otherwise.  (The estimate lets the
 * kernel encode the streams once and write their sizes afterwards: it only encodes what the
 * estimate admits and rewinds to raw when the exact rule fails.) */
static uint32_t zs_literals_block(const uint8_t* lit, uint32_t n, const zs_littab* H,
                                  int* tree_sent, uint8_t* d, uint32_t cap, int* err) {
  uint32_t hsz;
  if (H->mode == 1 && n > 0) {
    if (cap < 4) { *err = 1; return 0; }
    zs_lit_header(d, 1, n, &hsz);
    d[hsz] = H->rle;
    return hsz + 1;
  }
  if (H->mode == 2 && n > 0) {
    const uint32_t ns = n < 256 ? 1 : 4, q = (n + 3) / 4;
    const uint32_t dsz = *tree_sent ? 0u : H->dsz;
    const int32_t limit = (int32_t)n - (int32_t)((n >> 6) + 2);
    const uint64_t est_bits = (uint64_t)n * H->tb / H->nlit;
    const uint32_t est = dsz + (ns == 4 ? 6 : 0) + (uint32_t)((est_bits + 8u * ns) / 8u);
    uint32_t bytes[4] = {0}, total = dsz + (ns == 4 ? 6 : 0);
    for (uint32_t k = 0; k < ns; ++k) {
      const uint32_t a = ns == 1 ? 0 : k * q, b = ns == 1 ? n : (k == 3 ? n : (k + 1) * q);
      uint64_t bits = 0;
      for (uint32_t i = a; i < b; ++i) bits += H->len[lit[i]];
      bytes[k] = (uint32_t)((bits + 1 + 7) / 8);
      total += bytes[k];
    }
    if ((int32_t)est < limit && (int32_t)total < limit) {
      const uint32_t hs = ns == 1 || n < 1024 ? 3 : n < 16384 ? 4 : 5;
      if (hs + total > cap) { *err = 1; return 0; }
      const uint32_t sf = ns == 1 ? 0 : n < 1024 ? 1 : n < 16384 ? 2 : 3;
      const uint64_t type = *tree_sent ? 3u : 2u;  /* Treeless / Compressed_Literals */
      const uint64_t h = type | (sf << 2) |
                         ((uint64_t)n << 4) | ((uint64_t)total << (hs == 3 ? 14 : hs == 4 ? 18 : 22));
      for (uint32_t k = 0; k < hs; ++k) d[k] = (uint8_t)(h >> (8 * k));
      uint32_t p = hs;
      memcpy(d + p, H->desc, dsz);
      p += dsz;
      if (ns == 4) {
        for (uint32_t k = 0; k < 3; ++k) {
          d[p + 2 * k] = (uint8_t)bytes[k];
          d[p + 2 * k + 1] = (uint8_t)(bytes[k] >> 8);
        }
        p += 6;
      }
      for (uint32_t k = 0; k < ns; ++k) {
        const uint32_t a = ns == 1 ? 0 : k * q, b = ns == 1 ? n : (k == 3 ? n : (k + 1) * q);
        zs_bw bw = {d, p, cap, 0, 0, 0};
        for (uint32_t i = b; i-- > a;) zs_bw_add(&bw, H->code[lit[i]], H->len[lit[i]]);
        zs_bw_close(&bw);
        if (bw.err) { *err = 1; return 0; }
        p = bw.pos;
      }
      *tree_sent = 1;
      return p;
    }
  }
  /* ---- raw ---- */
  zs_lit_header(d, 0, n, &hsz);
  if (hsz + n > cap) { *err = 1; return 0; }
  memcpy(d + hsz, lit, n);
  return hsz + n;
}

/* ---- sequences section ---- */
typedef struct {
  uint32_t mode;   /* 0 predefined, 1 RLE, 2 FSE_Compressed */
  uint32_t rle;    /* the symbol of an RLE table */
  zs_ctable ct;
} zs_seqtab;

/* choose and describe one table (codes[0..nseq)); appends the description to w */
static void zs_choose(zs_seqtab* t, const uint8_t* codes, uint32_t nseq, uint32_t max_code,
                      uint32_t max_log, const int16_t* def, uint32_t def_max, uint32_t def_al,
                      zs_bw* w) {
  uint32_t cnt[64] = {0}, max_sym = 0, distinct = 0;
  for (uint32_t i = 0; i < nseq; ++i) {
    if (!cnt[codes[i]]++) ++distinct;
    if (codes[i] > max_sym) max_sym = codes[i];
  }
  (void)max_code;
  if (distinct == 1) {
    t->mode = 1;
    t->rle = max_sym;
    zs_bw_add(w, max_sym, 8);
    return;
  }
  /* estimated bits (x256) of the symbols' FSE states under each distribution */
  uint64_t cost_pre = 0;
  for (uint32_t s = 0; s <= max_sym; ++s) {
    if (!cnt[s]) continue;
    const uint32_t nd = def[s] == -1 ? 1u : (uint32_t)def[s];
    cost_pre += (uint64_t)cnt[s] * ((def_al << 8) - zs_log2fix(nd));
  }
  const uint32_t tl = zs_table_log(max_log, nseq, max_sym);
  int16_t norm[64];
  zs_normalize(cnt, max_sym, nseq, tl, norm);
  uint64_t cost_fse = 0;
  for (uint32_t s = 0; s <= max_sym; ++s)
    if (cnt[s]) cost_fse += (uint64_t)cnt[s] * ((tl << 8) - zs_log2fix((uint32_t)norm[s]));
  uint8_t tmp[128];
  zs_bw tw = {tmp, 0, sizeof tmp, 0, 0, 0};
  const uint32_t nb = zs_write_ncount(&tw, norm, max_sym, tl);
  cost_fse += (uint64_t)nb * 8 * 256;
  if (cost_fse < cost_pre) {
    t->mode = 2;
    for (uint32_t k = 0; k < nb; ++k) zs_bw_add(w, tmp[k], 8);
    zs_build_ctable(&t->ct, norm, max_sym, tl);
  } else {
    t->mode = 0;
    zs_build_ctable(&t->ct, def, def_max, def_al);
  }
}

typedef struct {
  uint8_t* lit;
  uint32_t nlit;
  uint32_t nseq;
  uint32_t* ll;
  uint32_t* ml;
  uint32_t* off;
  uint8_t* drop;  /* BO_ZSTD_DROP_GAP_LITERALS: positions whose literal byte is left out */
} zs_parsed;

static void zs_collect(void* vctx, uint32_t lit_start, uint32_t lit_len, uint32_t off,
                       uint32_t mlen) {
  zs_parsed* z = (zs_parsed*)vctx;
  if (off == BO_GAP_OFF && !mlen) { /* (BO_PARSE_GAPS: only with a drop map) */
    memset(z->drop + lit_start, 1, lit_len);
    return;
  }
  z->nlit += lit_len;  /* bytes are gathered from the positions afterwards */
  if (mlen) {
    z->ll[z->nseq] = lit_len;
    z->ml[z->nseq] = mlen;
    z->off[z->nseq] = off;
    z->nseq++;
  }
}

/* The parse of the Zstd encoder: the repeat-offset form with window skipping (the shipped
 * zstd_parse_kernel).  Round 3 tried this combination on the GPU and its frames failed
 * libzstd: the kernel's literal collector staged literal bytes window by window and had no
 * case for the positions of skipped probe windows (BO_ZSTD_DROP_GAP_LITERALS restates it). */
static uint32_t g_zstd_parse_flags = BO_PARSE_REP | BO_PARSE_SKIP;
uint32_t bo_set_zstd_parse_flags(uint32_t flags) {
  const uint32_t old = g_zstd_parse_flags;
  g_zstd_parse_flags = flags;
  return old;
}

uint32_t bo_zstd_bound(uint32_t n) {
  /* frame header 4+1+2 + block header 3 + at most the raw input (a block that does not
   * shrink is stored raw); the slack covers the kernels' staging */
  return n + 7 + 3 + 8 + 512;
}

/* Blocks of a frame (round 5): a frame with >= ZS_MULTI_MIN sequences is written as
 * B = 4 compressed blocks of equal sequence counts -- block b takes sequences
 * [b nseq / B, (b + 1) nseq / B) and their literals, the last one the trailing literals too --
 * or B = 8 when it also has >= ZS_WIDE_LIT literal bytes (the near-incompressible columns of
 * a record batch: ~64 KiB of literals whose Huffman streams, 4 per block, are a decoder's
 * longest serial chains).
 * The blocks share one literal code (the first Huffman-coded block carries the tree, the
 * others are Treeless) and one set of sequence tables (described in the first block,
 * Repeat_Mode in the others); repeat offsets run on across blocks (RFC 8878 3.1.2.5).  Each
 * block's FSE state chains start from its own last sequence, so a decoder walks the blocks'
 * chains -- and decodes their literal streams -- in parallel.  bo_set_zstd_blocks(1) writes
 * the single-block frames of rounds 1-4. */
#define ZS_MAX_BLOCKS 8u
#define ZS_MULTI_MIN 64u
#define ZS_WIDE_LIT 32768u
/* 0: the rule above; else every frame with >= ZS_MULTI_MIN sequences has this many blocks */
static uint32_t g_zstd_blocks = 0;
uint32_t bo_set_zstd_blocks(uint32_t b) {
  const uint32_t old = g_zstd_blocks;
  g_zstd_blocks = b > ZS_MAX_BLOCKS ? ZS_MAX_BLOCKS : b;
  return old;
}
static uint32_t zs_nblocks(uint32_t nseq, uint32_t nlit, int drop) {
  if (drop || nseq < ZS_MULTI_MIN) return 1u;
  if (g_zstd_blocks) return g_zstd_blocks;
  return nlit >= ZS_WIDE_LIT ? 8u : 4u;
}
/* sequence starts sb[0..nb] and literal starts lb[0..nb] of the blocks */
static void zs_block_split(const uint32_t* ll, uint32_t nseq, uint32_t nlit, uint32_t nb,
                           uint32_t* sb, uint32_t* lb) {
  uint32_t acc = 0, k = 0;
  for (uint32_t b = 0; b < nb; ++b) {
    sb[b] = (uint32_t)((uint64_t)b * nseq / nb);
    while (k < sb[b]) acc += ll[k++];
    lb[b] = acc;
  }
  sb[nb] = nseq;
  lb[nb] = nlit;
}

int bo_zstd_compress_block(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap,
                           uint32_t* csize) {
  if (n > 65536 || cap < bo_zstd_bound(n)) return BO_ERR_INVALID;
  const uint32_t maxseq = n / 4 + 2;
  zs_parsed z = {0};
  z.lit = (uint8_t*)malloc(n + 1);
  z.ll = (uint32_t*)malloc(4u * maxseq);
  z.ml = (uint32_t*)malloc(4u * maxseq);
  z.off = (uint32_t*)malloc(4u * maxseq);
  uint8_t* codes = (uint8_t*)malloc(3u * maxseq);
  uint32_t* ov = (uint32_t*)malloc(4u * maxseq);
  int rc = BO_ERR_OUT_OF_MEMORY;
  if (!z.lit || !z.ll || !z.ml || !z.off || !codes || !ov) goto out;
  {
    const uint32_t fl = g_zstd_parse_flags;
    if (fl & BO_ZSTD_DROP_GAP_LITERALS) {
      z.drop = (uint8_t*)calloc(n + 1, 1);
      if (!z.drop) goto out;
    }
    bo_window_parse_flags(src, n, BO_MAX_DIST_ALL, 0xFFFFFFFFu,
                          (fl & 0xFFFFu) | (z.drop ? BO_PARSE_GAPS : 0u), zs_collect, &z);
  }
  {
    /* literal bytes: everything outside the matches */
    uint32_t ip = 0, lp = 0;
    for (uint32_t i = 0; i < z.nseq; ++i) {
      memcpy(z.lit + lp, src + ip, z.ll[i]);
      lp += z.ll[i];
      ip += z.ll[i] + z.ml[i];
    }
    memcpy(z.lit + lp, src + ip, n - ip);
    lp += n - ip;
    if (lp != z.nlit) { rc = BO_ERR_IO; goto out; }
    if (z.drop) { /* the broken collector: literal bytes of the gaps never reached the section */
      uint32_t q = 0;
      ip = 0;
      for (uint32_t i = 0; i <= z.nseq; ++i) {
        const uint32_t ll = i < z.nseq ? z.ll[i] : n - ip;
        for (uint32_t k = 0; k < ll; ++k) {
          if (!z.drop[ip + k]) z.lit[q++] = src[ip + k];
        }
        ip += ll + (i < z.nseq ? z.ml[i] : 0);
      }
      z.nlit = q;
    }
  }
  /* repeat offsets (RFC 8878 3.1.2.5) */
  {
    uint32_t r0 = 1, r1 = 4, r2 = 8;
    for (uint32_t i = 0; i < z.nseq; ++i) {
      const uint32_t o = z.off[i];
      uint32_t v;
      if (z.ll[i]) {
        v = o == r0 ? 1 : o == r1 ? 2 : o == r2 ? 3 : o + 3;
      } else {
        v = o == r1 ? 1 : o == r2 ? 2 : o == r0 - 1 ? 3 : o + 3;
      }
      ov[i] = v;
      const uint32_t idx = v > 3 ? 3 : v - 1 + (z.ll[i] ? 0 : 1);  /* 3: a new offset */
      if (v > 3 || idx == 3) {
        r2 = r1;
        r1 = r0;
        r0 = o;
      } else if (idx == 1) {
        r1 = r0;
        r0 = o;
      } else if (idx == 2) {
        r2 = r1;
        r1 = r0;
        r0 = o;
      }
    }
  }
  {
    /* frame header: magic, Single_Segment with the content size (1 byte below 256, else 2) */
    dst[0] = 0x28; dst[1] = 0xB5; dst[2] = 0x2F; dst[3] = 0xFD;
    uint32_t fh;
    if (n < 256) {
      dst[4] = 0x20;
      dst[5] = (uint8_t)n;
      fh = 6;
    } else {
      dst[4] = 0x60;
      dst[5] = (uint8_t)(n - 256);
      dst[6] = (uint8_t)((n - 256) >> 8);
      fh = 7;
    }
    const uint32_t nseq = z.nseq;
    /* blocks: 4 or 8 of equal sequence counts when the frame has >= ZS_MULTI_MIN sequences
     * (each block's FSE state chains, and its literal streams, are then independent of the
     * others': a decoder walks them in parallel), else one */
    const uint32_t nb = zs_nblocks(nseq, z.nlit, z.drop != 0);
    uint32_t sb[ZS_MAX_BLOCKS + 1], lb[ZS_MAX_BLOCKS + 1];
    zs_block_split(z.ll, nseq, z.nlit, nb, sb, lb);
    zs_littab H;
    zs_littab_build(z.lit, z.nlit, &H);
    int err = 0, tree_sent = 0;
    uint32_t p = fh;
    zs_seqtab* tll = NULL;
    static __thread zs_seqtab tabs3[3];  /* (large: not on the stack; per thread) */
    for (uint32_t b = 0; b < nb && !err; ++b) {
      const uint32_t blk = p;
      p = blk + 3;
      if (p + 8 > cap) { err = 1; break; }
      p += zs_literals_block(z.lit + lb[b], lb[b + 1] - lb[b], &H, &tree_sent, dst + p, cap - p,
                             &err);
      if (err || p + 4 > cap) { err = 1; break; }
      const uint32_t s0 = sb[b], s1 = sb[b + 1], ns = s1 - s0;
      if (ns < 128) {
        dst[p++] = (uint8_t)ns;
      } else {
        dst[p++] = (uint8_t)((ns >> 8) + 128);
        dst[p++] = (uint8_t)ns;
      }
      if (ns) {
        uint8_t* llc = codes;
        uint8_t* mlc = codes + maxseq;
        uint8_t* ofc = codes + 2 * maxseq;
        zs_bw w = {dst, p + 1, cap, 0, 0, 0};
        if (!tll) {
          /* the tables: chosen over all of the frame's sequences, described in the first
           * block; the later blocks repeat them (Repeat_Mode) */
          for (uint32_t i = 0; i < nseq; ++i) {
            llc[i] = (uint8_t)bo_zstd_ll_code(z.ll[i]);
            mlc[i] = (uint8_t)bo_zstd_ml_code(z.ml[i]);
            ofc[i] = (uint8_t)zs_highbit(ov[i]);
          }
          tll = tabs3;
          zs_choose(&tabs3[0], llc, nseq, 35, 9, kLLDefault, 35, ZS_LL_AL, &w);
          zs_choose(&tabs3[1], ofc, nseq, 31, 8, kOFDefault, 28, ZS_OF_AL, &w);
          zs_choose(&tabs3[2], mlc, nseq, 52, 9, kMLDefault, 52, ZS_ML_AL, &w);
          dst[p] = (uint8_t)((tabs3[0].mode << 6) | (tabs3[1].mode << 4) | (tabs3[2].mode << 2));
        } else {
          dst[p] = 0xFC;  /* Repeat_Mode for all three */
        }
        const zs_seqtab *tl = &tabs3[0], *to = &tabs3[1], *tm = &tabs3[2];
        /* the bitstream: the block's last sequence first */
        uint32_t sml = 0, sof = 0, sll = 0;
        const uint32_t k = s1 - 1;
        if (tm->mode != 1) zs_enc_init(&tm->ct, &sml, mlc[k]);
        if (to->mode != 1) zs_enc_init(&to->ct, &sof, ofc[k]);
        if (tl->mode != 1) zs_enc_init(&tl->ct, &sll, llc[k]);
        zs_bw_add(&w, z.ll[k], kLLBits[llc[k]]);
        zs_bw_add(&w, z.ml[k] - 3, kMLBits[mlc[k]]);
        zs_bw_add(&w, ov[k], ofc[k]);
        for (uint32_t j = k; j-- > s0;) {
          if (to->mode != 1) zs_enc_sym(&w, &to->ct, &sof, ofc[j]);
          if (tm->mode != 1) zs_enc_sym(&w, &tm->ct, &sml, mlc[j]);
          if (tl->mode != 1) zs_enc_sym(&w, &tl->ct, &sll, llc[j]);
          zs_bw_add(&w, z.ll[j], kLLBits[llc[j]]);
          zs_bw_add(&w, z.ml[j] - 3, kMLBits[mlc[j]]);
          zs_bw_add(&w, ov[j], ofc[j]);
        }
        if (tm->mode != 1) zs_bw_add(&w, sml, tm->ct.al);
        if (to->mode != 1) zs_bw_add(&w, sof, to->ct.al);
        if (tl->mode != 1) zs_bw_add(&w, sll, tl->ct.al);
        zs_bw_close(&w);
        err |= w.err;
        p = w.pos;
      }
      const uint32_t hdr = (b + 1 == nb ? 1u : 0u) | (2u << 1) | ((p - (blk + 3)) << 3);
      dst[blk] = (uint8_t)hdr;
      dst[blk + 1] = (uint8_t)(hdr >> 8);
      dst[blk + 2] = (uint8_t)(hdr >> 16);
    }
    /* did not shrink (or outgrew the slot: the kernels' overflow): one raw block */
    if (err || p - (fh + 3) >= n) {
      memcpy(dst + fh + 3, src, n);
      const uint32_t hdr = 1u | (0u << 1) | (n << 3);
      dst[fh] = (uint8_t)hdr;
      dst[fh + 1] = (uint8_t)(hdr >> 8);
      dst[fh + 2] = (uint8_t)(hdr >> 16);
      p = fh + 3 + n;
    }
    *csize = p;
    rc = BO_OK;
  }
out:
  free(z.lit); free(z.ll); free(z.ml); free(z.off); free(codes); free(ov); free(z.drop);
  return rc;
}
