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

static int zs_huf_stream(const zs_huf* h, const uint8_t* src, uint32_t len, uint8_t* out,
                         uint32_t n) {
  zs_bwd b;
  if (zs_bwd_init(&b, src, len)) return -1;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t v = (uint32_t)zs_peek(&b, h->log);
    out[i] = h->sym[v];
    b.pos -= h->nbits[v];
  }
  return b.pos == 0 ? 0 : -1;
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
        if (llc > 35 || mlc > 52 || ofc > 31) goto out;
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
            if (off == 0) goto out;
            z->rep[2] = z->rep[1]; z->rep[1] = z->rep[0]; z->rep[0] = off;
          }
        }
        if (lp + ll > regen || (uint64_t)op + ll + ml > cap) goto out;
        memcpy(dst + op, lit + lp, ll);
        op += ll;
        lp += ll;
        if (off == 0 || off > op) goto out;  /* no dictionary: history is this frame */
        for (uint32_t i = 0; i < ml; ++i) dst[op + i] = dst[op - off + i];
        op += ml;
      }
      if (b.pos != 0) goto out;
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
/* encoder: the frame the HIP kernel emits                                            */
/* ================================================================================ */
#define ZS_MAX_SEQ 256u /* sequences per block (the kernel keeps a block's sequences in 2 KiB of LDS) */

typedef struct {
  uint16_t state[1u << 6];
  int32_t dnb[64];   /* deltaNbBits */
  int32_t dfs[64];   /* deltaFindState */
  uint32_t al;
} zs_ctable;

/* FSE_buildCTable for a normalized distribution */
static void zs_build_ctable(zs_ctable* c, const int16_t* norm, uint32_t max_sym, uint32_t al) {
  const uint32_t size = 1u << al, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
  uint32_t high = size - 1;
  uint8_t sym_at[64];
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
static void zs_bw_close(zs_bw* w) {
  zs_bw_add(w, 1, 1);  /* end mark */
  if (w->nb) {
    if (w->pos >= w->cap) { w->err = 1; return; }
    w->out[w->pos++] = (uint8_t)w->acc;
    w->acc = 0;
    w->nb = 0;
  }
}
static void zs_enc_init(const zs_ctable* c, uint32_t* st, uint32_t s) {
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

typedef struct {
  const uint8_t* src;
  uint8_t* dst;
  uint32_t cap, op;
  int err;
  uint32_t blk;        /* output offset of the current block header */
  uint32_t in0;        /* input position the current block starts at */
  uint32_t in;         /* input consumed so far */
  uint32_t nlit;
  uint32_t nseq;
  uint32_t ll[ZS_MAX_SEQ], ml[ZS_MAX_SEQ], of[ZS_MAX_SEQ];
  zs_ctable ct_ll, ct_ml, ct_of;
} zs_enc;

static void zs_begin_block(zs_enc* e) {
  e->blk = e->op;
  e->in0 = e->in;
  e->op += 3 + 3;  /* block header + 3-byte raw-literals header */
  e->nlit = 0;
  e->nseq = 0;
  if (e->op > e->cap) e->err = 1;
}

static void zs_close_block(zs_enc* e, uint32_t last) {
  if (e->err) return;
  const uint32_t nlit = e->nlit, nseq = e->nseq;
  uint8_t* d = e->dst;
  const uint32_t lh = e->blk + 3;
  d[lh] = (uint8_t)((3u << 2) | ((nlit & 15u) << 4));  /* raw literals, 20-bit size */
  d[lh + 1] = (uint8_t)(nlit >> 4);
  d[lh + 2] = (uint8_t)(nlit >> 12);
  uint32_t p = e->op;
  if (p + 3 > e->cap) { e->err = 1; return; }
  if (nseq < 128) {
    d[p++] = (uint8_t)nseq;
  } else {
    d[p++] = (uint8_t)((nseq >> 8) + 128);
    d[p++] = (uint8_t)nseq;
  }
  if (nseq) {
    d[p++] = 0;  /* LL, OF, ML: predefined distributions */
    zs_bw w = {d, p, e->cap, 0, 0, 0};
    uint32_t sml, sof, sll;
    const uint32_t k = nseq - 1;
    const uint32_t llc = bo_zstd_ll_code(e->ll[k]), mlc = bo_zstd_ml_code(e->ml[k]),
                   ofc = zs_highbit(e->of[k]);
    zs_enc_init(&e->ct_ml, &sml, mlc);
    zs_enc_init(&e->ct_of, &sof, ofc);
    zs_enc_init(&e->ct_ll, &sll, llc);
    zs_bw_add(&w, e->ll[k], kLLBits[llc]);
    zs_bw_add(&w, e->ml[k] - 3, kMLBits[mlc]);
    zs_bw_add(&w, e->of[k], ofc);
    for (uint32_t j = nseq - 1; j-- > 0;) {
      const uint32_t lc = bo_zstd_ll_code(e->ll[j]), mc = bo_zstd_ml_code(e->ml[j]),
                     oc = zs_highbit(e->of[j]);
      zs_enc_sym(&w, &e->ct_of, &sof, oc);
      zs_enc_sym(&w, &e->ct_ml, &sml, mc);
      zs_enc_sym(&w, &e->ct_ll, &sll, lc);
      zs_bw_add(&w, e->ll[j], kLLBits[lc]);
      zs_bw_add(&w, e->ml[j] - 3, kMLBits[mc]);
      zs_bw_add(&w, e->of[j], oc);
    }
    zs_bw_add(&w, sml, e->ct_ml.al);
    zs_bw_add(&w, sof, e->ct_of.al);
    zs_bw_add(&w, sll, e->ct_ll.al);
    zs_bw_close(&w);
    if (w.err) { e->err = 1; return; }
    p = w.pos;
  }
  const uint32_t csz = p - (e->blk + 3), raw = e->in - e->in0;
  uint32_t hdr;
  if (csz >= raw) {  /* did not shrink: store the block's input raw */
    if (e->blk + 3 + raw > e->cap) { e->err = 1; return; }
    memcpy(d + e->blk + 3, e->src + e->in0, raw);
    hdr = last | (0u << 1) | (raw << 3);
    p = e->blk + 3 + raw;
  } else {
    hdr = last | (2u << 1) | (csz << 3);
  }
  d[e->blk] = (uint8_t)hdr;
  d[e->blk + 1] = (uint8_t)(hdr >> 8);
  d[e->blk + 2] = (uint8_t)(hdr >> 16);
  e->op = p;
}

static void zs_emit(void* vctx, uint32_t lit_start, uint32_t lit_len, uint32_t off, uint32_t mlen) {
  zs_enc* e = (zs_enc*)vctx;
  if (e->err) return;
  if (e->op + lit_len > e->cap) { e->err = 1; return; }
  memcpy(e->dst + e->op, e->src + lit_start, lit_len);
  e->op += lit_len;
  e->nlit += lit_len;
  e->in += lit_len;
  if (mlen) {
    e->ll[e->nseq] = lit_len;
    e->ml[e->nseq] = mlen;
    e->of[e->nseq] = off + 3;  /* Offset_Value: no repeat offsets */
    e->nseq++;
    e->in += mlen;
    /* a block ends right after its ZS_MAX_SEQ-th match: the literals that follow belong to
     * the next block, so the kernel writes every literal byte as soon as it is parsed */
    if (e->nseq == ZS_MAX_SEQ) {
      zs_close_block(e, 0);
      zs_begin_block(e);
    }
  }
}

uint32_t bo_zstd_bound(uint32_t n) {
  /* frame header 4+1+2, then per block of input: 3-byte header + at most the raw input
   * (a block never grows: it is stored raw instead) -- blocks split only at sequence
   * boundaries, at most n/4/ZS_MAX_SEQ+1 of them.  The +512: a block is written compressed
   * before it is judged, and its compressed form may exceed its raw size by < 2 B per
   * sequence (<= 17 state + 16 literal-length + 12 offset bits vs a >= 4-byte match) plus
   * its headers. */
  return n + 7 + 3 * (n / (4 * ZS_MAX_SEQ) + 2) + 8 + 512;
}

int bo_zstd_compress_block(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap,
                           uint32_t* csize) {
  if (n > 65536 || cap < bo_zstd_bound(n)) return BO_ERR_INVALID;
  zs_enc* e = (zs_enc*)calloc(1, sizeof(zs_enc));
  if (!e) return BO_ERR_OUT_OF_MEMORY;
  e->src = src;
  e->dst = dst;
  e->cap = cap;
  zs_build_ctable(&e->ct_ll, kLLDefault, 35, ZS_LL_AL);
  zs_build_ctable(&e->ct_ml, kMLDefault, 52, ZS_ML_AL);
  zs_build_ctable(&e->ct_of, kOFDefault, 28, ZS_OF_AL);
  /* frame header: magic, single segment, content size (1 byte below 256, else 2 bytes) */
  dst[0] = 0x28; dst[1] = 0xB5; dst[2] = 0x2F; dst[3] = 0xFD;
  if (n < 256) {
    dst[4] = 0x20;
    dst[5] = (uint8_t)n;
    e->op = 6;
  } else {
    dst[4] = 0x60;
    dst[5] = (uint8_t)(n - 256);
    dst[6] = (uint8_t)((n - 256) >> 8);
    e->op = 7;
  }
  zs_begin_block(e);
  bo_window_parse(src, n, BO_MAX_DIST_ALL, 0xFFFFFFFFu, zs_emit, e);
  zs_close_block(e, 1);
  const int rc = e->err ? BO_ERR_IO : BO_OK;
  if (!e->err) *csize = e->op;
  free(e);
  return rc;
}
