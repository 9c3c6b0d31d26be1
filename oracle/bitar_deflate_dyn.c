/*
 * bitar_deflate_dyn.c -- raw DEFLATE with DYNAMIC Huffman codes over the bitar window-scan
 * parse, exactly as the HIP kernels deflate_dyn_parse_kernel + deflate_dyn_emit_kernel
 * (bitar_amd/csrc/deflate_dyn.hip) write it.  TEST INFRASTRUCTURE ONLY (see bitar_oracle.h).
 *
 * The reference's default frame is a dynamic-Huffman raw DEFLATE stream per segment
 * (RTE_COMP_HUFFMAN_DYNAMIC: reference src/include/config.h:151, used by the demo through
 * BlueFieldConfiguration::Defaults, apps/app_common.cc:87-88; the BlueField device accepts
 * FIXED or DYNAMIC, src/device.cc:566-574).  Its bitstream is the engine's and unspecified;
 * this restates RFC 1951 3.2.7 with a fully specified (deterministic) code construction:
 *
 *   1. symbols: the window-scan parse (bo_window_parse, distance <= 2560, length <= 258);
 *      literal/length frequencies (EOB counted once) and distance frequencies;
 *   2. code lengths (huff_lengths): a Huffman tree built with two queues over the used
 *      symbols sorted by (frequency, symbol) -- a leaf wins ties against an internal node --
 *      with fewer than two used symbols padded by the lowest unused symbols at frequency 1;
 *      depths limited as zlib's gen_bitlen does (cap, then move leaves down the tree, then
 *      re-assign lengths in the order the nodes left the queues);
 *   3. the code-length sequences of the literal/length (HLIT) and distance (HDIST) codes are
 *      run-length coded separately with symbols 16/17/18 exactly as zlib's send_tree does;
 *      the code-length code is built by the same huff_lengths (limit 7);
 *   4. block choice: dynamic if its size in bits is below the fixed-Huffman size, else fixed;
 *      then stored blocks unless the coded block is smaller by at least n / 16 bytes
 *      (BO_STORE_MARGIN).  One final block (stored: blocks of <= 65535 bytes).
 * Codes are canonical (RFC 1951 3.2.2).  zlib / libdeflate decode every stream (tests).
 */
#include <stdlib.h>
#include <string.h>

#include "bitar_oracle.h"

static const uint16_t kLB[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t kLX[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t kDB[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                 33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const uint8_t kDX[30] = {0, 0, 0, 0, 1, 1, 2, 2,  3,  3,  4,  4,  5,  5,  6,
                                6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static const uint8_t kCLO[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

static int len_sym(uint32_t mlen) { int s = 28; while (kLB[s] > mlen) --s; return s; }
static int dist_sym(uint32_t off) { int s = 29; while (kDB[s] > off) --s; return s; }

/* Code lengths of nsym symbols (nsym <= 286) limited to maxlen; see the header. */
void bo_huff_lengths(const uint32_t* freq, int nsym, int maxlen, uint8_t* lens) {
  uint32_t f[286];
  int leaf[286], m = 0;
  for (int s = 0; s < nsym; ++s) {
    f[s] = freq[s];
    lens[s] = 0;
    if (f[s]) ++m;
  }
  for (int s = 0; s < nsym && m < 2; ++s)
    if (!f[s]) { f[s] = 1; ++m; }
  /* leaves sorted by (frequency, symbol): leaf[rank] */
  for (int s = 0; s < nsym; ++s) {
    if (!f[s]) continue;
    int r = 0;
    for (int t = 0; t < nsym; ++t)
      if (f[t] && (f[t] < f[s] || (f[t] == f[s] && t < s))) ++r;
    leaf[r] = s;
  }
  /* two-queue Huffman: nodes 0..m-1 leaves (in rank order), m..2m-2 internal */
  uint32_t w[571];
  int parent[571], order[571], nlen[571];
  for (int k = 0; k < m; ++k) w[k] = f[leaf[k]];
  int i = 0, j = m, next = m, no = 0;
  for (int step = 0; step < m - 1; ++step) {
    int ab[2];
    for (int t = 0; t < 2; ++t) {
      if (i < m && (j >= next || w[i] <= w[j])) ab[t] = i++;
      else ab[t] = j++;
      order[no++] = ab[t];
    }
    w[next] = w[ab[0]] + w[ab[1]];
    parent[ab[0]] = parent[ab[1]] = next;
    ++next;
  }
  const int root = 2 * m - 2;
  order[no++] = root;
  /* depths, capped at maxlen (zlib gen_bitlen) */
  int bl_count[16] = {0}, overflow = 0;
  nlen[root] = 0;
  for (int k = no - 2; k >= 0; --k) {
    const int nd = order[k];
    int bits = nlen[parent[nd]] + 1;
    if (bits > maxlen) { bits = maxlen; ++overflow; }
    nlen[nd] = bits;
    if (nd < m) bl_count[bits]++;
  }
  if (overflow) {
    do {
      int bits = maxlen - 1;
      while (bl_count[bits] == 0) --bits;
      bl_count[bits]--;
      bl_count[bits + 1] += 2;
      bl_count[maxlen]--;
      overflow -= 2;
    } while (overflow > 0);
    int h = 0;
    for (int bits = maxlen; bits != 0; --bits) {
      int n = bl_count[bits];
      while (n != 0) {
        const int nd = order[h++];
        if (nd >= m) continue;
        nlen[nd] = bits;
        --n;
      }
    }
  }
  for (int k = 0; k < m; ++k) lens[leaf[k]] = (uint8_t)nlen[k];
}

/* canonical codes (RFC 1951 3.2.2), bit-reversed for LSB-first output */
static void canon_codes(const uint8_t* lens, int n, uint16_t* codes) {
  int bl[16] = {0}, next[16];
  for (int s = 0; s < n; ++s) bl[lens[s]]++;
  bl[0] = 0;
  int code = 0;
  for (int b = 1; b <= 15; ++b) {
    code = (code + bl[b - 1]) << 1;
    next[b] = code;
  }
  for (int s = 0; s < n; ++s) {
    codes[s] = 0;
    if (!lens[s]) continue;
    const uint32_t c = (uint32_t)next[lens[s]]++;
    uint32_t r = 0;
    for (int i = 0; i < lens[s]; ++i) r |= ((c >> i) & 1u) << (lens[s] - 1 - i);
    codes[s] = (uint16_t)r;
  }
}

/* zlib send_tree: run-length code lens[0..n) (n = max_code + 1) into (symbol, extra) */
static int rle_lens(const uint8_t* lens, int n, uint16_t* out) {
  int k = 0, prevlen = -1, count = 0, max_count = 7, min_count = 4;
  int nextlen = lens[0];
  if (nextlen == 0) { max_count = 138; min_count = 3; }
  for (int i = 0; i < n; ++i) {
    const int curlen = nextlen;
    nextlen = i + 1 < n ? lens[i + 1] : 0xFFFF;
    if (++count < max_count && curlen == nextlen) continue;
    if (count < min_count) {
      do { out[k++] = (uint16_t)curlen; } while (--count != 0);
    } else if (curlen != 0) {
      if (curlen != prevlen) { out[k++] = (uint16_t)curlen; --count; }
      out[k++] = (uint16_t)(16 | ((count - 3) << 8));
    } else if (count <= 10) {
      out[k++] = (uint16_t)(17 | ((count - 3) << 8));
    } else {
      out[k++] = (uint16_t)(18 | ((count - 11) << 8));
    }
    count = 0;
    prevlen = curlen;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    else if (curlen == nextlen) { max_count = 6; min_count = 3; }
    else { max_count = 7; min_count = 4; }
  }
  return k;
}

typedef struct {
  uint32_t lit_start, lit_len, off, mlen;
} seq_t;

typedef struct {
  seq_t* v;
  uint32_t n, cap;
  int err;
} seq_list;

static void collect(void* vctx, uint32_t lit_start, uint32_t lit_len, uint32_t off,
                    uint32_t mlen) {
  seq_list* L = (seq_list*)vctx;
  if (L->err) return;
  if (L->n == L->cap) {
    uint32_t nc = L->cap ? 2 * L->cap : 1024;
    seq_t* nv = (seq_t*)realloc(L->v, nc * sizeof(seq_t));
    if (!nv) { L->err = 1; return; }
    L->v = nv;
    L->cap = nc;
  }
  seq_t s = {lit_start, lit_len, off, mlen};
  L->v[L->n++] = s;
}

typedef struct {
  uint8_t* dst;
  uint32_t cap;
  uint64_t bitpos;
  int err;
} bw_t;

static void bw_put(bw_t* c, uint32_t v, int n) { /* LSB-first */
  for (int i = 0; i < n; ++i) {
    uint64_t p = c->bitpos + (uint64_t)i;
    if ((p >> 3) >= c->cap) { c->err = 1; return; }
    if ((p & 7) == 0) c->dst[p >> 3] = 0;
    c->dst[p >> 3] |= (uint8_t)(((v >> i) & 1u) << (p & 7));
  }
  c->bitpos += (uint64_t)n;
}

static uint8_t fixed_len(int s) { return s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8; }

/* The plan of one segment (kept for tests via bo_deflate_dyn_plan). */
typedef struct {
  int mode; /* 0 stored, 1 fixed, 2 dynamic */
  uint64_t dyn_bits, fix_bits, stored_bytes;
} dyn_plan;

static int deflate_dyn(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap,
                       uint32_t* csize, dyn_plan* plan) {
  seq_list L = {0};
  bo_window_parse(src, n, BO_MAX_DIST_ALL, 258u, collect, &L);
  if (L.err) { free(L.v); return BO_ERR_OUT_OF_MEMORY; }
  uint32_t lf[286] = {0}, df[30] = {0};
  for (uint32_t k = 0; k < L.n; ++k) {
    const seq_t* s = &L.v[k];
    for (uint32_t i = 0; i < s->lit_len; ++i) lf[src[s->lit_start + i]]++;
    if (s->mlen) {
      lf[257 + len_sym(s->mlen)]++;
      df[dist_sym(s->off)]++;
    }
  }
  lf[256]++;
  uint8_t ll[286], dl[30];
  bo_huff_lengths(lf, 286, 15, ll);
  bo_huff_lengths(df, 30, 15, dl);
  int hlit = 286, hdist = 30;
  while (hlit > 257 && ll[hlit - 1] == 0) --hlit;
  while (hdist > 1 && dl[hdist - 1] == 0) --hdist;
  uint16_t cls[320];
  int ncl = rle_lens(ll, hlit, cls);
  ncl += rle_lens(dl, hdist, cls + ncl);
  uint32_t cf[19] = {0};
  for (int k = 0; k < ncl; ++k) cf[cls[k] & 31]++;
  uint8_t cll[19];
  bo_huff_lengths(cf, 19, 7, cll);
  int hclen = 19;
  while (hclen > 4 && cll[kCLO[hclen - 1]] == 0) --hclen;
  /* sizes */
  uint64_t dyn = 3 + 14 + 3 * (uint64_t)hclen, fix = 3;
  for (int c = 0; c < 19; ++c) dyn += (uint64_t)cf[c] * cll[c];
  dyn += 2 * (uint64_t)cf[16] + 3 * (uint64_t)cf[17] + 7 * (uint64_t)cf[18];
  for (int s = 0; s < 286; ++s) {
    const uint64_t x = s > 256 ? kLX[s - 257] : 0;
    dyn += (uint64_t)lf[s] * (ll[s] + x);
    fix += (uint64_t)lf[s] * (fixed_len(s) + x);
  }
  for (int s = 0; s < 30; ++s) {
    dyn += (uint64_t)df[s] * (dl[s] + kDX[s]);
    fix += (uint64_t)df[s] * (5 + kDX[s]);
  }
  const uint64_t nblk = n ? (n + 65534u) / 65535u : 1;
  const uint64_t stored = nblk * 5 + n;
  int mode = dyn < fix ? 2 : 1;
  const uint64_t best = ((mode == 2 ? dyn : fix) + 7) / 8;
  if (stored < best + BO_STORE_MARGIN(n)) mode = 0;
  if (plan) {
    plan->mode = mode;
    plan->dyn_bits = dyn;
    plan->fix_bits = fix;
    plan->stored_bytes = stored;
  }
  bw_t w = {dst, cap, 0, 0};
  if (mode == 0) {
    uint32_t p = 0;
    for (uint64_t b = 0; b < nblk; ++b) {
      const uint32_t len = n - p < 65535u ? n - p : 65535u;
      const uint64_t o = w.bitpos >> 3;
      if (o + 5 + len > cap) { free(L.v); return BO_ERR_IO; }
      dst[o] = (uint8_t)(b + 1 == nblk);
      dst[o + 1] = (uint8_t)len;
      dst[o + 2] = (uint8_t)(len >> 8);
      dst[o + 3] = (uint8_t)~len;
      dst[o + 4] = (uint8_t)(~len >> 8);
      memcpy(dst + o + 5, src + p, len);
      w.bitpos = (o + 5 + len) * 8;
      p += len;
    }
    free(L.v);
    *csize = (uint32_t)(w.bitpos >> 3);
    return BO_OK;
  }
  /* fixed codes: canonical over all 288 literal/length symbols (RFC 1951 3.2.6) */
  uint8_t lens[288], dlens[30];
  if (mode == 2) {
    memcpy(lens, ll, 286);
    lens[286] = lens[287] = 0;
    memcpy(dlens, dl, sizeof(dlens));
  } else {
    for (int s = 0; s < 288; ++s) lens[s] = fixed_len(s);
    for (int s = 0; s < 30; ++s) dlens[s] = 5;
  }
  uint16_t lc[288], dc[30];
  canon_codes(lens, 288, lc);
  canon_codes(dlens, 30, dc);
  bw_put(&w, 1u | ((uint32_t)mode << 1), 3); /* BFINAL = 1, BTYPE = 01 fixed / 10 dynamic */
  if (mode == 2) {
    uint16_t cc[19];
    canon_codes(cll, 19, cc);
    bw_put(&w, (uint32_t)(hlit - 257), 5);
    bw_put(&w, (uint32_t)(hdist - 1), 5);
    bw_put(&w, (uint32_t)(hclen - 4), 4);
    for (int i = 0; i < hclen; ++i) bw_put(&w, cll[kCLO[i]], 3);
    for (int k = 0; k < ncl; ++k) {
      const int s = cls[k] & 31, x = cls[k] >> 8;
      bw_put(&w, cc[s], cll[s]);
      if (s == 16) bw_put(&w, (uint32_t)x, 2);
      else if (s == 17) bw_put(&w, (uint32_t)x, 3);
      else if (s == 18) bw_put(&w, (uint32_t)x, 7);
    }
  }
  for (uint32_t k = 0; k < L.n && !w.err; ++k) {
    const seq_t* s = &L.v[k];
    for (uint32_t i = 0; i < s->lit_len; ++i) {
      const uint8_t b = src[s->lit_start + i];
      bw_put(&w, lc[b], lens[b]);
    }
    if (s->mlen) {
      const int ls = len_sym(s->mlen), ds = dist_sym(s->off);
      bw_put(&w, lc[257 + ls], lens[257 + ls]);
      bw_put(&w, s->mlen - kLB[ls], kLX[ls]);
      bw_put(&w, dc[ds], dlens[ds]);
      bw_put(&w, s->off - kDB[ds], kDX[ds]);
    }
  }
  bw_put(&w, lc[256], lens[256]);
  free(L.v);
  if (w.err) return BO_ERR_IO;
  *csize = (uint32_t)((w.bitpos + 7) >> 3);
  return BO_OK;
}

int bo_deflate_dynamic_block(const uint8_t* src, uint32_t n, uint8_t* dst, uint32_t cap,
                             uint32_t* csize) {
  return deflate_dyn(src, n, dst, cap, csize, NULL);
}

/* For tests: the block mode (0 stored, 1 fixed, 2 dynamic) the encoder chose. */
int bo_deflate_dynamic_mode(const uint8_t* src, uint32_t n) {
  uint32_t cap = bo_deflate_bound(n), cs = 0;
  uint8_t* tmp = (uint8_t*)malloc(cap ? cap : 1);
  if (!tmp) return -1;
  dyn_plan p = {0};
  const int r = deflate_dyn(src, n, tmp, cap, &cs, &p);
  free(tmp);
  return r ? -1 : p.mode;
}
