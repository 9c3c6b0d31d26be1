// zstd_decompress.hip -- Zstandard (RFC 8878) frame decode, one wavefront per segment
// (gfx950).  Acceptance rules are those of the oracle's bo_zstd_decompress
// (oracle/bitar_zstd.c): one frame per segment, no dictionary, raw / RLE / compressed
// blocks, raw / RLE / Huffman literals (1 or 4 streams, FSE-compressed or direct weights,
// treeless reuse), predefined / RLE / FSE / repeat sequence tables, repeat offsets, and the
// XXH64 content checksum.
//
// Control is wave-uniform (scalar registers); the compressed stream is read through the
// LDS window of stream_ring.hip.h and the output goes through its LDS history ring.  Tables
// (FSE decode cells, the Huffman table) live in LDS and are built lane-parallel where the
// construction allows it.  Huffman-coded literals are decoded into the tail of the
// segment's output slot and copied from there by the sequence executor: output writes never
// overtake the literal reads (op <= cap - remaining literals).
#include "stream_ring.hip.h"
#include "zstd_hand.hip.h"

#include <type_traits>

namespace bitar_hip {

namespace zsd {

using namespace sr;

// ZPROF builds (scripts/build_variant.sh NAME -DZPROF) accumulate s_memtime cycles per phase
// in LDS and add them to g_zprof at wave end (bitar_hip_debug_zstd_prof reads them).
#ifdef ZPROF
__device__ unsigned long long g_zprof[16];
__shared__ unsigned long long zp_lds[16];
#define ZP_T() ((uint64_t)__builtin_amdgcn_s_memtime())
#define ZP_BEGIN(v) const uint64_t v = ZP_T()
#define ZP_ADD(i, x) do { if (lane_id() == 0) zp_lds[i] += (x); } while (0)
#define ZP_END(i, v) ZP_ADD(i, ZP_T() - (v))
#else
#define ZP_BEGIN(v)
#define ZP_ADD(i, x)
#define ZP_END(i, v)
#endif

constexpr uint32_t kHufMaxLog = 11;

__constant__ uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,   7,   8,   9,    10,   11,
                                     12, 13, 14, 15, 16, 18, 20,  22,  24,  28,   32,   40,
                                     48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384,
                                     32768, 65536};
__constant__ uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13,   14,   15,   16,
                                     17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27,   28,   29,   30,
                                     31, 32, 33, 34, 35, 37, 39, 41, 43, 47, 51,   59,   67,   83,
                                     99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771,
                                     65539};
__constant__ uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                                    2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ int16_t kLLDefault[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                       2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t kMLDefault[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                       1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                       1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t kOFDefault[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                       1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

struct Tabs {  // LDS, per wave
  uint32_t fse[3][512];  // decode cells (LL, OF, ML): sym | nbits << 8 | base << 16
  uint32_t wcells[64];   // the Huffman weights' cells (accuracy log <= 6)
  uint16_t huf[1u << kHufMaxLog];  // sym | nbits << 8
  int16_t norm[256];
  uint8_t wts[256];
};

__device__ __forceinline__ uint32_t hb32(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

// ---- scalar stream access ---------------------------------------------------------------
// bytes [pos, pos + n) of the stream (n <= 4, all inside it), little-endian
__device__ __forceinline__ uint32_t load_le(State& s, uint8_t* win, uint32_t pos, uint32_t n) {
  const uint32_t w = win_at(s, win, pos, n);
  lds_order();
  const uint32_t lane = lane_id();
  const uint32_t b = lane < n ? (uint32_t)win[w + lane] : 0u;
  return readlane(b, 0) | (readlane(b, 1) << 8) | (readlane(b, 2) << 16) | (readlane(b, 3) << 24);
}

// forward bit reader (FSE table descriptions): bits past `len` read as zeros
struct Fwd {
  uint32_t start, len;
  uint32_t bitpos;
};
__device__ __forceinline__ uint32_t fwd_peek(State& s, uint8_t* win, const Fwd& f, uint32_t n) {
  const uint32_t byte = f.bitpos >> 3;
  uint32_t avail = byte < f.len ? f.len - byte : 0u;
  if (avail > 4) avail = 4;
  const uint64_t w = avail ? (uint64_t)load_le(s, win, f.start + byte, avail) : 0ull;
  return (uint32_t)(w >> (f.bitpos & 7u)) & ((1u << n) - 1);
}

// backward bit reader: bits [0, bitpos) of a stream remain; read(n) returns bits
// [bitpos - n, bitpos) as a little-endian integer (zeros below bit 0); bitpos < 0 after a
// read = the stream was overrun.  The container holds bits [8 lo, bitpos).
// The stream bytes come from two 256-B register chunks (lane l = one aligned dword), not from
// the LDS window: the window keeps the raw literal section, which the sequence executor reads
// at the other end of the block, staged.  c1 covers absolute [cb, cb + 256), c0 the 256 B
// below it; when the reader moves wholly into c0 the pair slides down and c0 is reloaded,
// so the next chunk's HBM latency overlaps ~60 sequences of decode.
struct Bwd {
  uint32_t start;
  int32_t bitpos;
  uint64_t c;
  int32_t cn;
  uint32_t lo;
  uint32_t c0, c1;  // register chunks (per lane: one dword)
  uint64_t cb;      // absolute address of c1's first byte (4-aligned)
};
// aligned dword `lane` of the 256-B chunk at absolute address a (dwords holding no byte of
// the stream read as zero and are never loaded)
__device__ __forceinline__ uint32_t bwd_chunk(const State& s, uint64_t a) {
  const uint64_t d = a + 4ull * lane_id();
  const uint64_t lo = (uint64_t)(uintptr_t)s.src, hi = lo + s.csize;
  uint32_t v = 0;
  if (d < hi && d + 4 > lo) v = *reinterpret_cast<const GMEM uint32_t*>((uintptr_t)d);
  return v;
}
// stream bytes [pos, pos + 4) (pos decreasing over the reader's life), little-endian
__device__ __forceinline__ uint32_t bwd_dword(const State& s, Bwd& b, uint32_t pos) {
  const uint64_t abs = (uint64_t)(uintptr_t)(s.src + pos);
  while (abs + 4 <= b.cb) {  // wholly inside c0: slide down, prefetch the next chunk
    b.c1 = b.c0;
    b.cb -= 256;
    b.c0 = bwd_chunk(s, b.cb - 256);
  }
  const uint32_t a = uniform((uint32_t)(abs - (b.cb - 256)));  // in [0, 508)
  const uint32_t q = a >> 2, r = a & 3u, q1 = q + 1;
  const uint32_t w0 = q < 64 ? readlane(b.c0, q) : readlane(b.c1, q - 64);
  const uint32_t w1 = q1 < 64 ? readlane(b.c0, q1) : readlane(b.c1, (q1 - 64) & 63u);
  return funnel(w0, w1, r);
}
__device__ __forceinline__ bool bwd_init(State& s, uint8_t* win, Bwd& b, uint32_t start, uint32_t len) {
  if (len == 0) return false;
  const uint32_t last = load_le(s, win, start + len - 1, 1);
  if (last == 0) return false;
  const uint32_t h = hb32(last);
  start = uniform(start);
  len = uniform(len);
  b.start = start;
  b.bitpos = (int32_t)((len - 1) * 8 + h);
  b.c = last & ((1u << h) - 1);
  b.cn = (int32_t)h;
  b.lo = len - 1;
  const uint64_t top = uniform64(((uint64_t)(uintptr_t)(s.src + start + len) + 3) & ~3ull);
  b.cb = top - 256;
  b.c1 = bwd_chunk(s, b.cb);
  b.c0 = bwd_chunk(s, b.cb - 256);
  return true;
}
__device__ __forceinline__ void bwd_fill(State& s, uint8_t*, Bwd& b) {
  if (b.cn <= 32 && b.lo >= 4) {
    b.lo -= 4;
    b.c = (b.c << 32) | uniform(bwd_dword(s, b, b.start + b.lo));
    b.cn += 32;
  }
  while (b.cn <= 56 && b.lo > 0) {
    b.lo -= 1;
    b.c = (b.c << 8) | (uniform(bwd_dword(s, b, b.start + b.lo)) & 0xFFu);
    b.cn += 8;
  }
}
__device__ __forceinline__ uint32_t bwd_peek(State& s, uint8_t* win, Bwd& b, uint32_t n) {
  if (b.cn < (int32_t)n) bwd_fill(s, win, b);
  if (n == 0) return 0;
  const uint64_t m = (1ull << n) - 1;
  return b.cn >= (int32_t)n ? (uint32_t)((b.c >> (b.cn - (int32_t)n)) & m)
                            : (uint32_t)((b.c << ((int32_t)n - b.cn)) & m);
}
__device__ __forceinline__ uint32_t bwd_read(State& s, uint8_t* win, Bwd& b, uint32_t n) {
  const uint32_t v = bwd_peek(s, win, b, n);
  b.cn -= (int32_t)n;
  if (b.cn < 0) { b.cn = 0; b.c = 0; }
  b.bitpos -= (int32_t)n;
  return v;
}
__device__ __forceinline__ void bwd_skip(Bwd& b, uint32_t n) {
  b.cn -= (int32_t)n;
  if (b.cn < 0) { b.cn = 0; b.c = 0; }
  b.bitpos -= (int32_t)n;
}

// ---- FSE ----------------------------------------------------------------------------------
// FSE_readNCount from the stream at [start, start + len); returns bytes used, or -1
__device__ __forceinline__ int read_ncount(State& s, uint8_t* win, Tabs& t, uint32_t start, uint32_t len,
                           uint32_t& max_sym, uint32_t& al, uint32_t max_al) {
  Fwd f = {start, len, 0};
  const uint32_t log = fwd_peek(s, win, f, 4) + 5;
  if (log > max_al) return -1;
  f.bitpos = 4;
  int remaining = (1 << log) + 1;
  int threshold = 1 << log;
  uint32_t nbits = log + 1;
  uint32_t sym = 0;
  bool prev0 = false;
  const uint32_t lane = lane_id();
  while (remaining > 1 && sym <= max_sym) {
    if (prev0) {
      uint32_t n0 = sym;
      while (fwd_peek(s, win, f, 16) == 0xFFFFu) { n0 += 24; f.bitpos += 16; }
      while ((fwd_peek(s, win, f, 2) & 3u) == 3u) { n0 += 3; f.bitpos += 2; }
      n0 += fwd_peek(s, win, f, 2) & 3u;
      f.bitpos += 2;
      if (n0 > max_sym) return -1;
      lds_order();
      for (uint32_t k = sym + lane; k < n0; k += kWave) t.norm[k] = 0;
      lds_order();
      sym = n0;
    }
    const int max = (2 * threshold - 1) - remaining;
    int count;
    const uint32_t v = fwd_peek(s, win, f, nbits);
    if ((int)(v & (uint32_t)(threshold - 1)) < max) {
      count = (int)(v & (uint32_t)(threshold - 1));
      f.bitpos += nbits - 1;
    } else {
      count = (int)(v & (uint32_t)(2 * threshold - 1));
      if (count >= threshold) count -= max;
      f.bitpos += nbits;
    }
    count--;
    remaining -= count < 0 ? -count : count;
    lds_order();
    if (lane == 0) t.norm[sym] = (int16_t)count;
    lds_order();
    sym++;
    prev0 = count == 0;
    while (remaining < threshold) { nbits--; threshold >>= 1; }
  }
  if (remaining != 1 || f.bitpos > len * 8) return -1;
  max_sym = sym - 1;
  al = log;
  return (int)((f.bitpos + 7) >> 3);
}

// FSE_buildDTable from t.norm[0..max_sym] (max_sym <= 255: Huffman-weight tables may
// declare symbols they never decode).  Per-symbol state counters live one per lane, in
// four registers (symbol = 64 j + lane).
__device__ __forceinline__ uint32_t pick4(const uint32_t (&v)[4], uint32_t j) {
  return j == 0 ? v[0] : j == 1 ? v[1] : j == 2 ? v[2] : v[3];
}
__device__ __forceinline__ bool fse_build(Tabs& t, uint32_t* cells, uint32_t max_sym, uint32_t al) {
  const uint32_t lane = lane_id();
  const uint32_t size = 1u << al;
  lds_order();
  uint32_t nextv[4], normv[4];
  uint32_t high = size - 1;
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    const uint32_t sm = 64 * j + lane;
    const int nl = sm <= max_sym ? (int)t.norm[sm] : 0;
    normv[j] = nl > 0 ? (uint32_t)nl : 0u;
    nextv[j] = nl == -1 ? 1u : normv[j];
    // symbols of "less than 1" probability take the top cells, in symbol order
    for (uint64_t m = ballot(sm <= max_sym && nl == -1); m; m &= m - 1) {
      const uint32_t sy = 64 * j + (uint32_t)__builtin_ctzll(m);
      if (lane == 0) cells[high] = sy;
      high--;
    }
  }
  const uint32_t step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
  if (max_sym < kWave) {
    // spread, all lanes (every sequence table and any weights table of <= 64 symbols): the
    // positions k * step & mask, k = 0, 1, ..., that are not reserved; the c-th of them takes
    // the symbol whose run of cells [cum, cum + norm) holds c.  The runs must fill exactly
    // the unreserved cells (the scalar spread's "ends at 0").
    const uint32_t cum = wave_incl_sum(normv[0]) - normv[0];
    if (readlane(cum + normv[0], kWave - 1) != high + 1) return false;
    uint32_t c0 = 0;
    for (uint32_t k0 = 0; k0 < size; k0 += kWave) {
      const uint32_t k = k0 + lane;
      const uint32_t v = (k * step) & mask;
      const bool ok = k < size && v <= high;
      const uint64_t bm = ballot(ok);
      const uint32_t c = c0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
      c0 += (uint32_t)__builtin_popcountll(bm);
      uint32_t sl = 0;  // the last symbol whose run starts at or before c
#pragma unroll
      for (uint32_t d = 32; d != 0; d >>= 1) {
        const uint32_t x = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((sl + d) << 2), (int)cum);
        sl = x <= c ? sl + d : sl;
      }
      if (ok) cells[v] = sl;
    }
  } else {
    // spread (scalar: the step sequence skips the reserved top cells)
    uint32_t pos = 0;
    for (uint32_t sm = 0; sm <= max_sym; ++sm) {
      const uint32_t cnt = readlane(pick4(normv, sm >> 6), sm & 63u);
      for (uint32_t i = 0; i < cnt; ++i) {
        if (lane == 0) cells[pos] = sm;
        do { pos = (pos + step) & mask; } while (pos > high);
      }
    }
    if (pos != 0) return false;
  }
  lds_order();
  // states: cell u of symbol s gets next[s]++ in u order; lanes take 64 cells at a time and
  // rank equal symbols with a ballot
  for (uint32_t u0 = 0; u0 < size; u0 += kWave) {
    const uint32_t u = u0 + lane;
    const bool in = u < size;
    const uint32_t sy = in ? (cells[u] & 0xFFu) : 0u;
    uint64_t pend = ballot(in);
    uint32_t ns = 0;
    while (pend) {
      const uint32_t l0 = (uint32_t)__builtin_ctzll(pend);
      const uint32_t s0 = readlane(sy, l0);
      const uint64_t mk = ballot(in && sy == s0) & pend;
      const uint32_t j0 = s0 >> 6, l1 = s0 & 63u;
      const uint32_t base = readlane(pick4(nextv, j0), l1);
      if ((mk >> lane) & 1) ns = base + (uint32_t)__builtin_popcountll(mk & ((1ull << lane) - 1));
      const uint32_t add = lane == l1 ? (uint32_t)__builtin_popcountll(mk) : 0u;
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) nextv[j] += j == j0 ? add : 0u;
      pend &= ~mk;
    }
    lds_order();
    if (in) {
      const uint32_t nb = al - hb32(ns);
      cells[u] = sy | (nb << 8) | (((ns << nb) - size) << 16);
    }
    lds_order();
  }
  return true;
}

__device__ __forceinline__ void fse_rle(uint32_t* cells, uint32_t sym) {
  lds_order();
  if (lane_id() == 0) cells[0] = sym;  // nbits 0, base 0
  lds_order();
}

__device__ __forceinline__ uint32_t cell(const uint32_t* cells, uint32_t st) {
  lds_order();
  return uniform(cells[st]);
}

// ---- Huffman -------------------------------------------------------------------------------
// tree description at stream [start, start + len); returns bytes used or -1; sets log
__device__ __forceinline__ int huf_read(State& s, uint8_t* win, Tabs& t, uint32_t start, uint32_t len,
                        uint32_t& log) {
  const uint32_t lane = lane_id();
  if (len < 1) return -1;
  const uint32_t hb = load_le(s, win, start, 1);
  uint32_t nw = 0;
  int used;
  if (hb < 128) {  // FSE-compressed weights in hb bytes
    if (1 + hb > len) return -1;
    uint32_t max_sym = 255, al;
    const int n = read_ncount(s, win, t, start + 1, hb, max_sym, al, 6);
    if (n < 0) return -1;
    uint32_t* cells = t.wcells;
    if (!fse_build(t, cells, max_sym, al)) return -1;
    Bwd b;
    if (!bwd_init(s, win, b, start + 1 + (uint32_t)n, hb - (uint32_t)n)) return -1;
    uint32_t s1 = bwd_read(s, win, b, al), s2 = bwd_read(s, win, b, al);
    for (;;) {
      if (nw > 254) return -1;
      uint32_t c1 = cell(cells, s1);
      if (lane == 0) t.wts[nw] = (uint8_t)c1;
      nw++;
      s1 = (c1 >> 16) + bwd_read(s, win, b, (c1 >> 8) & 0xFFu);
      if (b.bitpos < 0) {
        const uint32_t c2 = cell(cells, s2);
        if (lane == 0) t.wts[nw] = (uint8_t)c2;
        nw++;
        break;
      }
      if (nw > 254) return -1;
      const uint32_t c2 = cell(cells, s2);
      if (lane == 0) t.wts[nw] = (uint8_t)c2;
      nw++;
      s2 = (c2 >> 16) + bwd_read(s, win, b, (c2 >> 8) & 0xFFu);
      if (b.bitpos < 0) {
        c1 = cell(cells, s1);
        if (lane == 0) t.wts[nw] = (uint8_t)c1;
        nw++;
        break;
      }
    }
    used = 1 + (int)hb;
  } else {  // direct 4-bit weights
    nw = hb - 127;
    const uint32_t nb = (nw + 1) / 2;
    if (1 + nb > len) return -1;
    for (uint32_t k0 = 0; k0 < nw; k0 += kWave) {  // 64 weights = 32 bytes per step
      const uint32_t k = k0 + lane;
      const uint32_t w = win_at(s, win, start + 1 + k0 / 2, 32);
      lds_order();
      const uint32_t wk = k < nw ? (uint32_t)win[w + lane / 2] : 0u;
      lds_order();
      if (k < nw) t.wts[k] = (uint8_t)((k & 1) ? (wk & 15u) : (wk >> 4));
      lds_order();
    }
    used = 1 + (int)nb;
  }
  lds_order();
  // weights -> total, implied last weight, rank starts (lane-parallel over 4 x 64 symbols)
  uint32_t total = 0;
  bool bad = false;
  for (uint32_t k0 = 0; k0 < nw; k0 += kWave) {
    const uint32_t k = k0 + lane;
    const uint32_t w = k < nw ? t.wts[k] : 0u;
    bad |= ballot(w > 11) != 0;
    uint32_t v = w ? (1u << (w - 1)) : 0u;
    for (uint32_t d = 1; d < 64; d <<= 1) v += __shfl_xor((int)v, (int)d, 64);
    total += readlane(v, 0);
  }
  if (bad || total == 0) return -1;
  const uint32_t maxb = hb32(total) + 1;
  if (maxb > kHufMaxLog) return -1;
  const uint32_t rest = (1u << maxb) - total;
  if (rest & (rest - 1)) return -1;
  lds_order();
  if (lane == 0) t.wts[nw] = (uint8_t)(hb32(rest) + 1);
  lds_order();
  nw++;
  // rank starts: lane w (1..11) holds the first table index of weight w
  uint32_t rankv = 0;  // lane w: count of symbols of weight w
  for (uint32_t k0 = 0; k0 < nw; k0 += kWave) {
    const uint32_t k = k0 + lane;
    const uint32_t w = k < nw ? t.wts[k] : 0u;
    for (uint32_t q = 1; q <= maxb; ++q) {
      const uint32_t c = (uint32_t)__builtin_popcountll(ballot(k < nw && w == q));
      rankv += lane == q ? c : 0u;
    }
  }
  // the longest codes (weight 1) come in pairs, at least one (libzstd HUF_readStats; the
  // oracle's zs_huf_read)
  const uint32_t r1 = readlane(rankv, 1);
  if (r1 < 2 || (r1 & 1u)) return -1;
  uint32_t startv = 0, nxt = 0;
  for (uint32_t q = 1; q <= maxb; ++q) {
    if (lane == q) startv = nxt;
    nxt += readlane(rankv, q) << (q - 1);
  }
  if (nxt != (1u << maxb)) return -1;
  // fill: symbol k of weight w takes 2^(w-1) entries from its rank slot, in symbol order
  for (uint32_t k0 = 0; k0 < nw; k0 += kWave) {
    const uint32_t k = k0 + lane;
    const uint32_t w = k < nw ? t.wts[k] : 0u;
    uint32_t my = 0;
    for (uint32_t q = 1; q <= maxb; ++q) {
      const uint64_t mk = ballot(k < nw && w == q);
      const uint32_t st = readlane(startv, q);
      if (w == q) my = st + ((uint32_t)__builtin_popcountll(mk & ((1ull << lane) - 1)) << (q - 1));
      startv += lane == q ? ((uint32_t)__builtin_popcountll(mk) << (q - 1)) : 0u;
    }
    lds_order();
    if (k < nw && w) {
      const uint16_t e = (uint16_t)(k | ((maxb + 1 - w) << 8));
      for (uint32_t j = 0; j < (1u << (w - 1)); ++j) t.huf[my + j] = e;
    }
    lds_order();
  }
  log = maxb;
  return used;
}

// decode one Huffman stream of n symbols to out[0, n) (global); false if malformed
__device__ __forceinline__ bool huf_stream(State& s, uint8_t* win, Tabs& t, uint32_t log, uint32_t start,
                           uint32_t len, GMEM uint8_t* out, uint32_t n) {
  Bwd b;
  if (!bwd_init(s, win, b, start, len)) return false;
  const uint32_t lane = lane_id();
  uint32_t v = 0, k = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t idx = bwd_peek(s, win, b, log);
    lds_order();
    const uint32_t e = uniform((uint32_t)t.huf[idx]);
    bwd_skip(b, e >> 8);
    if (lane == k) v = e & 0xFFu;
    if (++k == kWave) {
      out[i + 1 - kWave + lane] = (uint8_t)v;
      k = 0;
    }
  }
  if (k && lane < k) out[n - k + lane] = (uint8_t)v;
  return b.bitpos == 0;
}

// The speculative form of huf_stream: every lane decodes "a symbol starting at bit P - lane"
// (its table index = the `log` bits below that position, bits below the stream start read as
// zero) with one LDS table lookup, and a scalar walk follows the real code chain through the
// candidates (one v_readlane + one v_writelane per symbol, the symbol dropped into the lane
// of its output byte); 64 output bytes are stored at once.  Same result and the same
// acceptance rule (the stream consumed exactly) as huf_stream.
__device__ __forceinline__ uint32_t huf_walk(uint32_t ev, uint32_t c0, uint32_t cmax, uint32_t& k,
                                             uint32_t& outv) {
  uint32_t c, e, nb, m0_saved;
  __asm__ volatile(
      "s_mov_b32 %[m0s], m0\n"
      "s_mov_b32 %[k], 0\n"
      "s_mov_b32 m0, %[c0]\n"
      "L_hw_%=:\n"
      "s_cmp_ge_u32 %[k], 64\n"
      "s_cbranch_scc1 L_hd_%=\n"
      "s_cmp_ge_u32 m0, %[cmax]\n"
      "s_cbranch_scc1 L_hd_%=\n"
      "v_readlane_b32 %[e], %[ev], %[k]\n"
      "v_writelane_b32 %[ov], %[e], m0\n"
      "s_lshr_b32 %[nb], %[e], 8\n"
      "s_add_u32 m0, m0, 1\n"
      "s_add_u32 %[k], %[k], %[nb]\n"
      "s_branch L_hw_%=\n"
      "L_hd_%=:\n"
      "s_mov_b32 %[c], m0\n"
      "s_mov_b32 m0, %[m0s]\n"
      : [k] "=&s"(k), [c] "=&s"(c), [e] "=&s"(e), [nb] "=&s"(nb), [m0s] "=&s"(m0_saved),
        [ov] "+v"(outv)
      : [ev] "v"(ev), [c0] "s"(c0), [cmax] "s"(cmax)
      : "scc");
  return c;
}

__device__ __forceinline__ bool huf_stream_fast(State& s, uint8_t* win, Tabs& t, uint32_t log,
                                                uint32_t start, uint32_t len, GMEM uint8_t* out,
                                                uint32_t n) {
  if (len == 0) return false;
  const uint32_t lane = lane_id();
  const uint32_t last = load_le(s, win, start + len - 1, 1);
  if (last == 0) return false;
  int32_t P = (int32_t)((len - 1) * 8 + hb32(last));  // bits [0, P) remain
  const uint64_t sabs = (uint64_t)(uintptr_t)(s.src + start);
  const uint32_t mask = (1u << log) - 1;
  uint32_t produced = 0, cnt = 0, outv = 0;
  while (produced + cnt < n) {
    // stage the bytes holding bits [P - 64 - log, P) (+ a dword of slack), window placed so
    // that the backward reader keeps finding them in it
    const int32_t lo_bit = P - 64 - (int32_t)log;
    const uint32_t lo = lo_bit > 0 ? (uint32_t)lo_bit >> 3 : 0u;
    const uint32_t hi = (uint32_t)(P + 7) >> 3;  // <= len
    const uint64_t alo = sabs + lo, ahi = sabs + hi + 8;
    if (alo < s.wb || ahi > s.wb + kWin) {
      const uint64_t want = ahi > kWin ? ahi - kWin + 16 : 0ull;
      refill_abs(s, win, want > alo ? alo : want);
    }
    const uint32_t wbase = (uint32_t)(sabs - s.wb);  // window index of stream byte 0 (mod 2^32)
    // candidate lane: the `log` bits starting at bit b = P - lane - log
    const int32_t b = P - (int32_t)lane - (int32_t)log;
    const uint32_t bb = b > 0 ? (uint32_t)b : 0u;
    const uint32_t wi = wbase + (bb >> 3);
    lds_order();
    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(win + (wi & ~3u));
    const uint32_t w1 = *reinterpret_cast<const uint32_t*>(win + (wi & ~3u) + 4);
    const uint32_t v = funnel(w0, w1, wi & 3u);
    const uint32_t bits = b >= 0 ? v >> (bb & 7u) : (-b < 32 ? v << (uint32_t)(-b) : 0u);
    const uint32_t ev = t.huf[bits & mask];
    uint32_t k;
    const uint32_t rem = n - produced;
    cnt = huf_walk(ev, cnt, rem < 64u ? rem : 64u, k, outv);
    P -= (int32_t)k;
    if (cnt == 64) {
      out[produced + lane] = (uint8_t)outv;
      produced += 64;
      cnt = 0;
    }
  }
  if (cnt && lane < cnt) out[produced + lane] = (uint8_t)outv;
  return P == 0;
}

// ---- output helpers -------------------------------------------------------------------------
__device__ __forceinline__ void out_fill(State& s, uint8_t* ring, uint32_t v, uint32_t n) {
  const uintptr_t base = (uintptr_t)s.dst;
  while (n) {
    const uint32_t step = n < kWave ? n : kWave;
    make_room(s, ring, step);
    lds_order();
    if (lane_id() < step) ring[(base + s.op + lane_id()) & kRingMask] = (uint8_t)v;
    lds_order();
    s.op += step;
    n -= step;
  }
}
// n bytes from global memory this wave wrote (fenced by the caller) into the output
__device__ __forceinline__ void out_global(State& s, uint8_t* ring, const GMEM uint8_t* src, uint32_t n) {
  const uintptr_t base = (uintptr_t)s.dst;
  while (n) {
    const uint32_t step = n < kWave ? n : kWave;
    make_room(s, ring, step);
    const uint32_t v = lane_id() < step ? (uint32_t)src[lane_id()] : 0u;
    lds_order();
    if (lane_id() < step) ring[(base + s.op + lane_id()) & kRingMask] = (uint8_t)v;
    lds_order();
    s.op += step;
    src += step;
    n -= step;
  }
}

// Fast backward bit reader (sequence sections): C = the 8 stream bytes at [ptr, ptr + 8),
// little-endian, with bytes below the section start zeroed; `used` bits are consumed from
// its top.  reload() moves ptr down by the whole bytes consumed (libzstd's
// BIT_reloadDStream), so after a reload at least 57 bits are readable.  The bytes come from
// two register chunks of 256 B (lane l = one aligned dword) overlapping by 128 B: c1 covers
// [cb, cb + 256), c0 [cb - 128, cb + 128), prefetched one slide ahead.
struct FastBits {
  uint64_t C;
  uint32_t used;
  int32_t ptr, cb;  // stream positions (relative to s.src; may go below 0 on overrun)
  uint32_t c0, c1;
  // aligned dword `lane` of the 256 B at stream position `at` (4-aligned in absolute terms);
  // dwords holding no byte of the segment read as zero and are never loaded
  __device__ __forceinline__ static uint32_t chunk(const State& s, int32_t at) {
    const uint64_t lo = (uint64_t)(uintptr_t)s.src, hi = lo + s.csize;
    const uint64_t d = lo + (uint64_t)(int64_t)at + 4ull * lane_id();
    uint32_t v = 0;
    if (d < hi && d + 4 > lo) v = *reinterpret_cast<const GMEM uint32_t*>((uintptr_t)d);
    return v;
  }
  __device__ __forceinline__ void load(const State& s, uint32_t q) {
    while (ptr < cb) {
      c1 = c0;
      cb -= 128;
      c0 = chunk(s, cb - 128);
    }
    const uint32_t o = (uint32_t)(ptr - cb), qd = o >> 2, r = (o & 3u) * 8;
    const uint32_t w0 = readlane(c1, qd), w1 = readlane(c1, qd + 1), w2 = readlane(c1, qd + 2);
    const uint32_t lo = (uint32_t)((((uint64_t)w1 << 32) | w0) >> r);
    const uint32_t hi = (uint32_t)((((uint64_t)w2 << 32) | w1) >> r);
    C = ((uint64_t)hi << 32) | lo;
    if (ptr < (int32_t)q) {
      const uint32_t k = (uint32_t)((int32_t)q - ptr);
      C = k >= 8 ? 0ull : C & (~0ull << (8 * k));
    }
  }
  // section [q, end): false if empty or its last byte holds no end marker
  __device__ __forceinline__ bool init(State& s, uint32_t q, uint32_t end) {
    // the marker byte, read through the chunk path below (ptr = end - 8)
    ptr = (int32_t)end - 8;
    const int32_t mis = (int32_t)(((uintptr_t)s.src + (uint32_t)ptr) & 3u);
    cb = ptr - mis - 128;
    c1 = chunk(s, cb);
    c0 = chunk(s, cb - 128);
    load(s, q);
    const uint32_t last = (uint32_t)(C >> 56);
    if (last == 0) return false;
    used = 8 - hb32(last);
    return true;
  }
  __device__ __forceinline__ void reload(const State& s, uint32_t q) {
    ptr -= (int32_t)(used >> 3);
    used &= 7u;
    load(s, q);
  }
  __device__ __forceinline__ uint32_t read(uint32_t n) {
    const uint32_t sh = (64 - used - n) & 63u;  // n == used == 0: any shift, masked to 0
    const uint32_t v = (uint32_t)(C >> sh) & ((1u << n) - 1u);
    used += n;
    return v;
  }
  __device__ __forceinline__ int32_t remaining(uint32_t q) const {
    return 8 * (ptr - (int32_t)q) + 64 - (int32_t)used;
  }
};

// Produce a pending chunk of co <= 64 output bytes.  Lane j (< co) is byte j of the chunk:
// rec = first lane of its sequence | literal count << 8 | chunk literal index << 16, roff =
// the sequence's offset; literal bytes are in LDS at w0 + chunk literal index.  Sources:
// a literal, the ring (history before the chunk), or another lane of the chunk (a match
// reaching into it), resolved by pointer doubling; then one LDS gather + one ring store.
// Lanes >= co write ring slots ahead of the output, which are kRing - 64 bytes old,
// already flushed, and rewritten before they are read.
__device__ __forceinline__ void exec_chunk(State& s, uint8_t* win, uint8_t* ring, uint32_t co,
                                           uint32_t rec, uint32_t roff, uint32_t w0) {
  const uint32_t lane = lane_id();
  make_room(s, ring, co);
  const uint32_t base = (uint32_t)(uintptr_t)s.dst;
  const uint32_t o = rec & 0xFFu, ll = (rec >> 8) & 0xFFu, lq = rec >> 16;
  const uint32_t r = lane - o;
  const bool is_lit = r < ll;
  const uint32_t m = (r - ll) & 63u;
  const uint32_t off = roff;
  const float qf = floorf(((float)m + 0.5f) * __builtin_amdgcn_rcpf((float)off));
  const uint32_t mm = off <= m ? m - (uint32_t)qf * off : m;  // m mod off (exact below 64)
  const int32_t srel = (int32_t)(o + ll + mm) - (int32_t)off;  // vs the chunk start
  const uint32_t hist = kWin + ((base + s.op + (uint32_t)srel) & kRingMask);
  uint32_t st = lane >= co ? kWin : is_lit ? w0 + lq + r
                : srel >= 0 ? ((uint32_t)srel | 0x80000000u) : hist;
  while (ballot((st & 0x80000000u) != 0u)) {  // alias chains strictly descend
    const uint32_t other = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((st & 63u) << 2), (int)st);
    st = (st & 0x80000000u) ? other : st;
  }
  uint8_t* lds = win;  // win and ring are one LDS array
  lds_order();
  const uint8_t v = lds[st];
  ring[(base + s.op + lane) & kRingMask] = v;
  lds_order();
  s.op += co;
}

// Hand-off to the lane kernels (zstd_hand.hip.h)
using zhand::kHanded;

struct Frame {
  uint32_t rep0, rep1, rep2;
  uint32_t al[3];      // accuracy logs of the LL / OF / ML tables
  bool have[3];
  bool pre[3];         // table k holds the predefined distribution (built once per frame)
  uint32_t huf_log;    // 0 = no Huffman table yet
};

// one compressed block at stream [p, p + len)
// 0: malformed, 1: decoded, 2: handed off (the frame's last block goes to the lane kernels:
// hand != null, i.e. no checksum, and last block)
__device__ __forceinline__ int block(State& s, uint8_t* win, uint8_t* ring, Tabs& t, Frame& fr, uint32_t p,
                      uint32_t len, GMEM uint32_t* hand, bool last_block, uint32_t fsz,
                      uint32_t fcs, uint32_t& h_nseq, uint32_t& h_regen) {
  const uint32_t lane = lane_id();
  p = uniform(p);
  len = uniform(len);
  const uint32_t end = p + len;
  ZP_BEGIN(th);
  // ---- literals section ----
  const uint32_t b0 = load_le(s, win, p, 1);
  const uint32_t lt = b0 & 3u, sf = (b0 >> 2) & 3u;
  uint32_t regen, csz = 0, hsz, nstreams = 1;
  if (lt < 2) {
    if (sf == 0 || sf == 2) { regen = b0 >> 3; hsz = 1; }
    else if (sf == 1) { if (len < 2) return 0; regen = load_le(s, win, p, 2) >> 4; hsz = 2; }
    else { if (len < 3) return 0; regen = load_le(s, win, p, 3) >> 4; hsz = 3; }
  } else {
    if (sf <= 1) {
      if (len < 3) return 0;
      const uint32_t c = load_le(s, win, p, 3);
      regen = (c >> 4) & 0x3FFu; csz = (c >> 14) & 0x3FFu; hsz = 3; nstreams = sf == 0 ? 1 : 4;
    } else if (sf == 2) {
      if (len < 4) return 0;
      const uint32_t c = load_le(s, win, p, 4);
      regen = (c >> 4) & 0x3FFFu; csz = (c >> 18) & 0x3FFFu; hsz = 4; nstreams = 4;
    } else {
      if (len < 5) return 0;
      const uint64_t c = (uint64_t)load_le(s, win, p, 4) | ((uint64_t)load_le(s, win, p + 4, 1) << 32);
      regen = (uint32_t)(c >> 4) & 0x3FFFFu; csz = (uint32_t)(c >> 22) & 0x3FFFFu; hsz = 5; nstreams = 4;
    }
  }
  if (regen > (128u << 10) || regen > s.cap - s.op) return 0;
  uint32_t q = p + hsz;
  // where the literals come from: the stream (raw), one byte (RLE), or the slot tail
  uint32_t lit_stream = 0, lit_byte = 0;
  GMEM uint8_t* lit_tail = s.dst + (s.cap - regen);
  if (hand && lane == 0) hand[zhand::kLitPend] = 0u;  // set below if the lanes decode them
  if (lt == 0) {
    if (q + regen > end) return 0;
    lit_stream = q;
    q += regen;
  } else if (lt == 1) {
    if (q + 1 > end) return 0;
    lit_byte = load_le(s, win, q, 1);
    q += 1;
  } else {
    if (q + csz > end) return 0;
    uint32_t cs = q, cl = csz;
    if (lt == 2) {
      uint32_t log;
      const int n = huf_read(s, win, t, cs, cl, log);
      if (n < 0) return 0;
      fr.huf_log = log;
      cs += (uint32_t)n;
      cl -= (uint32_t)n;
    } else if (!fr.huf_log) {
      return 0;
    }
    // the streams: one, or four behind a jump table
    uint32_t st = cs, s1 = cl, s2 = 0, s3 = 0, s4 = 0, qq = regen;
    if (nstreams != 1) {
      if (cl < 6) return 0;
      const uint32_t j = load_le(s, win, cs, 4);
      s1 = j & 0xFFFFu;
      s2 = j >> 16;
      s3 = load_le(s, win, cs + 4, 2);
      if (6ull + s1 + s2 + s3 > cl) return 0;
      s4 = cl - 6 - s1 - s2 - s3;
      qq = (regen + 3) / 4;
      if (3 * qq > regen) return 0;
      st = cs + 6;
    }
    // a last block with enough sequences goes to the lane kernels, literals included: peek
    // at its sequence count (the same test as the hand-off below)
    bool lanes_lits = false;
    if (hand && last_block && q + csz < end) {
      const uint32_t qs = q + csz;
      uint32_t ns = load_le(s, win, qs, 1);
      if (ns >= 128 && ns < 255 && qs + 2 <= end) ns = ((ns - 128) << 8) + load_le(s, win, qs + 1, 1);
      else if (ns == 255 && qs + 3 <= end) ns = load_le(s, win, qs + 1, 2) + 0x7F00u;
      else if (ns >= 128) ns = 0;
      (void)ns;
      lanes_lits = true;  // every last block is handed over, with or without sequences
    }
    if (lanes_lits) {
      lds_order();
      const uint32_t ne = 1u << fr.huf_log;
      for (uint32_t u = lane; u < ne / 2; u += kWave)
        hand[zhand::kHufAt + u] = (uint32_t)t.huf[2 * u] | ((uint32_t)t.huf[2 * u + 1] << 16);
      const uint32_t rv = lane == 0 ? 1u : lane == 1 ? fr.huf_log | (nstreams << 8)
                          : lane == 2 ? st : lane == 3 ? s1 : lane == 4 ? s2 : lane == 5 ? s3
                          : lane == 6 ? s4 : qq;
      if (lane < 8) hand[zhand::kLitPend + lane] = rv;
    } else {
      if (nstreams == 1) {
        if (!huf_stream_fast(s, win, t, fr.huf_log, st, s1, lit_tail, regen)) return 0;
      } else {
        if (!huf_stream_fast(s, win, t, fr.huf_log, st, s1, lit_tail, qq)) return 0;
        if (!huf_stream_fast(s, win, t, fr.huf_log, st + s1, s2, lit_tail + qq, qq)) return 0;
        if (!huf_stream_fast(s, win, t, fr.huf_log, st + s1 + s2, s3, lit_tail + 2 * qq, qq)) return 0;
        if (!huf_stream_fast(s, win, t, fr.huf_log, st + s1 + s2 + s3, s4, lit_tail + 3 * qq,
                        regen - 3 * qq)) return 0;
      }
      global_fence_wave();  // the executor reads back what the streams wrote
    }
    q += csz;
  }
  uint32_t lp = 0;  // literals consumed
  auto copy_lits = [&](uint32_t n) __attribute__((always_inline)) {
    if (lt == 0) {
      s.ip = lit_stream + lp;
      if (n >= kLongLit) literals_long(s, win, ring, n);
      else if (n) literals_short(s, win, ring, n);
    } else if (lt == 1) {
      out_fill(s, ring, lit_byte, n);
    } else {
      out_global(s, ring, lit_tail + lp, n);
    }
    lp += n;
  };
  // ---- sequences section ----
  if (q >= end) return 0;
  uint32_t nseq = load_le(s, win, q, 1);
  if (nseq < 128) {
    q += 1;
  } else if (nseq < 255) {
    if (q + 2 > end) return 0;
    nseq = ((nseq - 128) << 8) + load_le(s, win, q + 1, 1);
    q += 2;
  } else {
    if (q + 3 > end) return 0;
    nseq = load_le(s, win, q + 1, 2) + 0x7F00u;
    q += 3;
  }
  ZP_END(2, th);
  if (nseq) {
    if (q >= end) return 0;
    ZP_BEGIN(tm);
    const uint32_t modes = load_le(s, win, q, 1);
    q += 1;
    if (modes & 3u) return 0;
    // tables in order LL, OF, ML (unrolled: fr.al / fr.have stay in registers)
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) {
      const uint32_t mode = (modes >> (6 - 2 * k)) & 3u;
      const uint32_t maxs = k == 0 ? 35u : k == 1 ? 31u : 52u;
      const uint32_t maxal = k == 1 ? 8u : 9u;
      uint32_t* cells = t.fse[k];
      if (mode == 0) {
        const uint32_t dal = k == 1 ? 5u : 6u;
        if (!fr.pre[k]) {
          const uint32_t dmax = k == 0 ? 35u : k == 1 ? 28u : 52u;
          lds_order();
          if (lane <= dmax)
            t.norm[lane] = k == 0 ? kLLDefault[lane] : k == 1 ? kOFDefault[lane] : kMLDefault[lane];
          lds_order();
          if (!fse_build(t, cells, dmax, dal)) return 0;
          fr.pre[k] = true;
        }
        fr.al[k] = dal;
      } else if (mode == 1) {
        if (q >= end) return 0;
        const uint32_t sy = load_le(s, win, q, 1);
        if (sy > maxs) return 0;
        fse_rle(cells, sy);
        fr.pre[k] = false;
        fr.al[k] = 0;
        q += 1;
      } else if (mode == 2) {
        uint32_t ms = maxs, al;
        const int n = read_ncount(s, win, t, q, end - q, ms, al, maxal);
        if (n < 0) return 0;
        fr.pre[k] = false;
        if (!fse_build(t, cells, ms, al)) return 0;
        fr.al[k] = al;
        q += (uint32_t)n;
      } else if (!fr.have[k]) {
        return 0;
      }
      fr.have[k] = true;
    }
    if (q >= end) return 0;
    ZP_END(3, tm);
    if (hand && last_block) {
      // everything before this block is output; the executor continues from s.op
      flush(s, ring, s.op, true);
      global_fence_wave();
#pragma unroll
      for (uint32_t k = 0; k < 3; ++k) {
        const uint32_t nc = 1u << fr.al[k];
        lds_order();
        for (uint32_t u = lane; u < nc; u += kWave) hand[zhand::kCellsAt + k * zhand::kCells + u] = t.fse[k][u];
      }
      const uint32_t rv = lane == 0 ? q : lane == 1 ? end : lane == 2 ? nseq
                          : lane == 3 ? fr.al[0] | (fr.al[1] << 8) | (fr.al[2] << 16) | (lt << 24)
                          : lane == 4 ? (lt == 0 ? lit_stream : lit_byte)
                          : lane == 5 ? regen : lane == 6 ? s.op : lane == 7 ? fr.rep0
                          : lane == 8 ? fr.rep1 : lane == 9 ? fr.rep2 : lane == 10 ? fsz : fcs;
      if (lane < 12) hand[lane] = rv;
      h_nseq = nseq;
      h_regen = regen;
      return 2;
    }
    // FSE tables of <= 64 cells (every predefined one) move into registers: lane u holds cell
    // u and a state lookup is one v_readlane instead of an LDS round trip
    const bool rt = fr.al[0] <= 6 && fr.al[1] <= 6 && fr.al[2] <= 6;
    lds_order();
    const uint32_t tll = t.fse[0][lane], tof = t.fse[1][lane], tml = t.fse[2][lane];
    // baseline | extra-bit count << 24 of every LL / ML code, one code per lane: the loop
    // reads them with v_readlane instead of a dependent constant-memory load per sequence
    const uint32_t llt = lane < 36 ? kLLBase[lane] | ((uint32_t)kLLBits[lane] << 24) : 0u;
    const uint32_t mlt = lane < 53 ? kMLBase[lane] | ((uint32_t)kMLBits[lane] << 24) : 0u;
    // Pending output chunk: short sequences (<= 64 output bytes, history in the ring) are
    // packed into the next 64 output bytes; lane j of the chunk keeps the sequence it falls
    // in (rec = first lane | literal count << 8 | chunk literal index << 16, roff = offset).
    // A full chunk is produced with one gather + one ring store (exec_chunk).
    uint32_t rec = 0, roff = 1, co = 0, lq = 0;
    auto exec = [&]() __attribute__((always_inline)) {
      if (!co) return;
      uint32_t w0;
      const uint32_t lp0 = lp - lq;
      if (lt == 0) {
        w0 = win_at(s, win, lit_stream + lp0, lq ? lq : 1u);
      } else {  // RLE byte or Huffman-decoded literals (slot tail): stage them in the window
        uint32_t v = lit_byte;
        if (lt != 1 && lane < lq) v = lit_tail[lp0 + lane];
        lds_order();
        win[lane] = (uint8_t)v;
        lds_order();
        s.wb = ~0ull;  // the window no longer mirrors the stream
        w0 = 0;
      }
      ZP_BEGIN(tx);
      exec_chunk(s, win, ring, co, rec, roff, w0);
      ZP_END(5, tx);
      ZP_ADD(10, 1);
      co = 0;
      lq = 0;
    };
    // fast sequence loop for tables of <= 64 cells (every predefined one): the tables live in
    // registers, lane u = cell u packed as baseline (17 bits) | extra-bit count << 17 |
    // state bits << 22 | next-state base << 25 (offset table: the code in place of the
    // baseline), so one v_readlane per table and sequence fetches everything; the bit reader
    // is an 8-byte container reloaded from two overlapping 256-B register chunks (FastBits)
    auto fast = [&]() __attribute__((always_inline)) -> bool {
      uint32_t info[3];
#pragma unroll
      for (uint32_t k = 0; k < 3; ++k) {
        const uint32_t c = k == 0 ? tll : k == 1 ? tof : tml;
        const uint32_t sym = c & 0xFFu;
        const uint32_t code = k == 1 ? (sym & 31u) | ((sym & 31u) << 17)
                                     : (uint32_t)__builtin_amdgcn_ds_bpermute((int)(sym << 2), (int)(k == 0 ? llt : mlt));
        const uint32_t bv = k == 1 ? code : (code & 0x1FFFFu) | ((code >> 24) << 17);
        info[k] = bv | (((c >> 8) & 7u) << 22) | (((c >> 16) & 63u) << 25);
      }
      FastBits fb;
      if (!fb.init(s, q, end)) return 0;
      uint32_t sll = fb.read(fr.al[0]), sof = fb.read(fr.al[1]), sml = fb.read(fr.al[2]);
      for (uint32_t k = 0; k < nseq; ++k) {
        fb.reload(s, q);
        const uint32_t il = readlane(info[0], sll), io = readlane(info[1], sof),
                       im = readlane(info[2], sml);
        const uint32_t ofc = (io >> 17) & 31u;
        const uint32_t ofv = (1u << ofc) + fb.read(ofc);
        const uint32_t ml = (im & 0x1FFFFu) + fb.read((im >> 17) & 31u);
        if (fb.used > 31) fb.reload(s, q);
        const uint32_t ll = (il & 0x1FFFFu) + fb.read((il >> 17) & 31u);
        if (k + 1 < nseq) {
          sll = (il >> 25) + fb.read((il >> 22) & 7u);
          sml = (im >> 25) + fb.read((im >> 22) & 7u);
          sof = (io >> 25) + fb.read((io >> 22) & 7u);
        }
        uint32_t off;
        if (ofv > 3) {
          off = ofv - 3;
          fr.rep2 = fr.rep1; fr.rep1 = fr.rep0; fr.rep0 = off;
        } else {
          const uint32_t idx = ofv + (ll == 0 ? 1u : 0u);
          if (idx == 1) {
            off = fr.rep0;
          } else if (idx == 2) {
            off = fr.rep1;
            fr.rep1 = fr.rep0; fr.rep0 = off;
          } else if (idx == 3) {
            off = fr.rep2;
            fr.rep2 = fr.rep1; fr.rep1 = fr.rep0; fr.rep0 = off;
          } else {
            off = fr.rep0 - 1;
            if (off == 0) return 0;
            fr.rep2 = fr.rep1; fr.rep1 = fr.rep0; fr.rep0 = off;
          }
        }
        const uint32_t opv = s.op + co;
        if (lp + ll > regen || (uint64_t)opv + ml + (regen - lp) > s.cap) return 0;
        if (off == 0 || off > opv + ll) return 0;
        const uint32_t ol = ll + ml;
        if (ol <= kWave && off <= kNearOff) {
          if (co + ol > kWave) exec();
          if (lane - co < ol) {
            rec = co | (ll << 8) | (lq << 16);
            roff = off;
          }
          co += ol;
          lq += ll;
          lp += ll;
        } else {
          exec();
          ZP_BEGIN(tg);
          copy_lits(ll);
          match_copy(s, ring, off, ml);
          ZP_END(6, tg);
          ZP_ADD(12, 1);
        }
      }
      exec();
      return fb.remaining(q) == 0;
    };
    // the same loop for larger tables (libzstd's custom FSE tables, accuracy <= 9): the
    // three cells come from LDS (issued together), baselines from the llt / mlt registers
    auto fast_lds = [&]() __attribute__((always_inline)) -> bool {
      FastBits fb;
      if (!fb.init(s, q, end)) return 0;
      uint32_t sll = fb.read(fr.al[0]), sof = fb.read(fr.al[1]), sml = fb.read(fr.al[2]);
      for (uint32_t k = 0; k < nseq; ++k) {
        fb.reload(s, q);
        lds_order();
        const uint32_t cll = uniform(t.fse[0][sll]), cof = uniform(t.fse[1][sof]),
                       cml = uniform(t.fse[2][sml]);
        const uint32_t ofc = cof & 0xFFu;
        const uint32_t ofv = (1u << ofc) + fb.read(ofc);
        const uint32_t mle = readlane(mlt, cml & 0xFFu);
        const uint32_t ml = (mle & 0xFFFFFFu) + fb.read(mle >> 24);
        if (fb.used > 31) fb.reload(s, q);
        const uint32_t lle = readlane(llt, cll & 0xFFu);
        const uint32_t ll = (lle & 0xFFFFFFu) + fb.read(lle >> 24);
        if (k + 1 < nseq) {
          sll = (cll >> 16) + fb.read((cll >> 8) & 0xFFu);
          sml = (cml >> 16) + fb.read((cml >> 8) & 0xFFu);
          sof = (cof >> 16) + fb.read((cof >> 8) & 0xFFu);
        }
        uint32_t off;
        if (ofv > 3) {
          off = ofv - 3;
          fr.rep2 = fr.rep1; fr.rep1 = fr.rep0; fr.rep0 = off;
        } else {
          const uint32_t idx = ofv + (ll == 0 ? 1u : 0u);
          if (idx == 1) {
            off = fr.rep0;
          } else if (idx == 2) {
            off = fr.rep1;
            fr.rep1 = fr.rep0; fr.rep0 = off;
          } else if (idx == 3) {
            off = fr.rep2;
            fr.rep2 = fr.rep1; fr.rep1 = fr.rep0; fr.rep0 = off;
          } else {
            off = fr.rep0 - 1;
            if (off == 0) return 0;
            fr.rep2 = fr.rep1; fr.rep1 = fr.rep0; fr.rep0 = off;
          }
        }
        const uint32_t opv = s.op + co;
        if (lp + ll > regen || (uint64_t)opv + ml + (regen - lp) > s.cap) return 0;
        if (off == 0 || off > opv + ll) return 0;
        const uint32_t ol = ll + ml;
        if (ol <= kWave && off <= kNearOff) {
          if (co + ol > kWave) exec();
          if (lane - co < ol) {
            rec = co | (ll << 8) | (lq << 16);
            roff = off;
          }
          co += ol;
          lq += ll;
          lp += ll;
        } else {
          exec();
          copy_lits(ll);
          match_copy(s, ring, off, ml);
        }
      }
      exec();
      return fb.remaining(q) == 0;
    };
    ZP_BEGIN(tq);
    ZP_ADD(11, nseq);
    if (!(rt ? fast() : fast_lds())) return 0;
    ZP_END(4, tq);
  } else if (q != end) {
    return 0;
  } else if (hand && last_block) {
    // no sequences: the literals go over too (their Huffman streams may be with
    // zstd_hlit_kernel already: a block of 64 Ki literals and no match -- libzstd writes
    // such blocks for incompressible columns -- would be one wave's serial decode)
    flush(s, ring, s.op, true);
    global_fence_wave();
    const uint32_t rv = lane <= 1 ? q : lane == 2 ? 0u : lane == 3 ? (lt << 24)
                        : lane == 4 ? (lt == 0 ? lit_stream : lit_byte)
                        : lane == 5 ? regen : lane == 6 ? s.op : lane == 7 ? fr.rep0
                        : lane == 8 ? fr.rep1 : lane == 9 ? fr.rep2 : lane == 10 ? fsz : fcs;
    if (lane < 12) hand[lane] = rv;
    h_nseq = 0;
    h_regen = regen;
    return 2;
  }
  if ((uint64_t)s.op + (regen - lp) > s.cap) return 0;
  copy_lits(regen - lp);
  return 1;
}

// Frames whose blocks can all be handed over (zstd_hand.hip.h): 2..kMaxBlocks compressed
// blocks ending exactly at the frame's end, where the blocks after the first define no table
// and no Huffman tree (Repeat_Mode or no sequences; Treeless, raw or RLE literals) -- the
// frames of this engine's encoder.  Returns the block count, else 0.  Only the headers are
// read here; every other rule is checked where the blocks run.
__device__ uint32_t multi_blocks(State& s, uint8_t* win, uint32_t p, uint32_t cs) {
  uint32_t nb = 0;
  for (;;) {
    if (nb == zhand::kMaxBlocks || p + 3 > cs) return 0;
    const uint32_t bh = load_le(s, win, p, 3);
    const uint32_t last = bh & 1u, type = (bh >> 1) & 3u, bsz = bh >> 3;
    p += 3;
    if (type != 2 || bsz > (128u << 10) || bsz < 2 || p + bsz > cs) return 0;
    if (nb > 0) {
      const uint32_t end = p + bsz;
      const uint32_t b0 = load_le(s, win, p, 1);
      const uint32_t lt = b0 & 3u, sf = (b0 >> 2) & 3u;
      if (lt == 2) return 0;  // a new tree
      uint32_t hsz, size;
      if (lt < 2) {
        hsz = (sf == 0 || sf == 2) ? 1u : sf == 1 ? 2u : 3u;
        if (p + hsz > end) return 0;
        const uint32_t regen = hsz == 1 ? b0 >> 3 : load_le(s, win, p, hsz) >> 4;
        size = lt == 0 ? regen : 1u;
      } else {
        hsz = sf <= 1 ? 3u : sf == 2 ? 4u : 5u;
        if (p + hsz > end) return 0;
        const uint64_t c = (uint64_t)load_le(s, win, p, hsz < 4 ? hsz : 4u) |
                           (hsz == 5 ? (uint64_t)load_le(s, win, p + 4, 1) << 32 : 0ull);
        size = (uint32_t)(hsz == 3 ? (c >> 14) & 0x3FFu : hsz == 4 ? (c >> 18) & 0x3FFFu
                                                                 : (c >> 22) & 0x3FFFFu);
      }
      const uint32_t q = p + hsz + size;
      if (q >= end) return 0;
      uint32_t nseq = load_le(s, win, q, 1), qm = q + 1;
      if (nseq >= 128) {
        if (nseq < 255) { nseq = 1; qm = q + 2; }
        else { nseq = 1; qm = q + 3; }
      }
      if (nseq && (qm >= end || load_le(s, win, qm, 1) != 0xFCu)) return 0;  // Repeat_Mode
    }
    ++nb;
    p += bsz;
    if (last) return (nb >= 2 && p == cs) ? nb : 0u;
  }
}

// A block after the first of a multi-block hand-off (multi_blocks): its headers into the
// sub-record hb (zstd_hand.hip.h), with the checks the wave decoder would apply to them
// (block()).  False = malformed.
__device__ bool hand_header(State& s, uint8_t* win, const Frame& fr, GMEM uint32_t* hb,
                            uint32_t p, uint32_t len, uint32_t& nseq_o, uint32_t& regen_o) {
  const uint32_t lane = lane_id();
  p = uniform(p);
  len = uniform(len);
  const uint32_t end = p + len;
  const uint32_t b0 = load_le(s, win, p, 1);
  const uint32_t lt = b0 & 3u, sf = (b0 >> 2) & 3u;
  uint32_t regen, csz = 0, hsz, nstreams = 1;
  if (lt < 2) {
    if (sf == 0 || sf == 2) { regen = b0 >> 3; hsz = 1; }
    else if (sf == 1) { if (len < 2) return false; regen = load_le(s, win, p, 2) >> 4; hsz = 2; }
    else { if (len < 3) return false; regen = load_le(s, win, p, 3) >> 4; hsz = 3; }
  } else {
    if (sf <= 1) {
      if (len < 3) return false;
      const uint32_t c = load_le(s, win, p, 3);
      regen = (c >> 4) & 0x3FFu; csz = (c >> 14) & 0x3FFu; hsz = 3; nstreams = sf == 0 ? 1 : 4;
    } else if (sf == 2) {
      if (len < 4) return false;
      const uint32_t c = load_le(s, win, p, 4);
      regen = (c >> 4) & 0x3FFFu; csz = (c >> 18) & 0x3FFFu; hsz = 4; nstreams = 4;
    } else {
      if (len < 5) return false;
      const uint64_t c = (uint64_t)load_le(s, win, p, 4) | ((uint64_t)load_le(s, win, p + 4, 1) << 32);
      regen = (uint32_t)(c >> 4) & 0x3FFFFu; csz = (uint32_t)(c >> 22) & 0x3FFFFu; hsz = 5; nstreams = 4;
    }
  }
  if (regen > (128u << 10)) return false;
  uint32_t q = p + hsz;
  uint32_t litv = 0, st = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0, qq = regen;
  bool pend = false;
  if (lt == 0) {
    if (q + regen > end) return false;
    litv = q;
    q += regen;
  } else if (lt == 1) {
    if (q + 1 > end) return false;
    litv = load_le(s, win, q, 1);
    q += 1;
  } else {  // Treeless: the first block's tree
    if (q + csz > end || !fr.huf_log) return false;
    st = q;
    s1 = csz;
    if (nstreams != 1) {
      if (csz < 6) return false;
      const uint32_t j = load_le(s, win, q, 4);
      s1 = j & 0xFFFFu;
      s2 = j >> 16;
      s3 = load_le(s, win, q + 4, 2);
      if (6ull + s1 + s2 + s3 > csz) return false;
      s4 = csz - 6 - s1 - s2 - s3;
      qq = (regen + 3) / 4;
      if (3 * qq > regen) return false;
      st = q + 6;
    }
    pend = true;
    q += csz;
  }
  if (q >= end) return false;
  uint32_t nseq = load_le(s, win, q, 1);
  if (nseq < 128) {
    q += 1;
  } else if (nseq < 255) {
    if (q + 2 > end) return false;
    nseq = ((nseq - 128) << 8) + load_le(s, win, q + 1, 1);
    q += 2;
  } else {
    if (q + 3 > end) return false;
    nseq = load_le(s, win, q + 1, 2) + 0x7F00u;
    q += 3;
  }
  if (nseq) {
    // Repeat_Mode for all three tables (multi_blocks), which the first block must have had
    if (q >= end || !fr.have[0] || !fr.have[1] || !fr.have[2]) return false;
    q += 1;
    if (q >= end) return false;
  } else if (q != end) {
    return false;
  }
  const uint32_t rv = lane == zhand::kQ ? q : lane == zhand::kEnd ? end
                      : lane == zhand::kNseq ? nseq
                      : lane == zhand::kAls ? fr.al[0] | (fr.al[1] << 8) | (fr.al[2] << 16) | (lt << 24)
                      : lane == zhand::kLitV ? litv : lane == zhand::kRegen ? regen
                      : lane == zhand::kLitPend ? (pend ? 1u : 0u)
                      : lane == zhand::kHufLog ? fr.huf_log | (nstreams << 8)
                      : lane == zhand::kStreams ? st : lane == zhand::kS1 ? s1
                      : lane == zhand::kS2 ? s2 : lane == zhand::kS3 ? s3
                      : lane == zhand::kS4 ? s4 : qq;
  if (lane < zhand::kBlkW && (lane < zhand::kOp || lane >= zhand::kLitPend)) hb[lane] = rv;
  nseq_o = nseq;
  regen_o = regen;
  return true;
}

// XXH64 of the first n output bytes (already flushed to HBM and fenced), low 32 bits
__device__ __forceinline__ uint32_t xxh64_low(const GMEM uint8_t* p, uint32_t n) {
  constexpr uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull,
                     P3 = 1609587929392839161ull, P4 = 9650029242287828579ull,
                     P5 = 2870177450012600261ull;
  auto rotl = [](uint64_t x, int r) { return (x << r) | (x >> (64 - r)); };
  auto round = [&](uint64_t acc, uint64_t in) { acc += in * P2; acc = rotl(acc, 31); return acc * P1; };
  const uint32_t lane = lane_id();
  uint64_t h;
  uint32_t i = 0;
  if (n >= 32) {
    uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
    const uint32_t nstripes = n / 32;
    for (uint32_t s0 = 0; s0 < nstripes; s0 += 32) {  // 32 stripes = 1 KiB per step
      const uint32_t off = s0 * 32 + 16 * lane;
      uint64_t a = 0, c = 0;
      if (off + 16 <= nstripes * 32) {
        uint64_t lo = 0, hi = 0;
        for (uint32_t b = 0; b < 8; ++b) lo |= (uint64_t)p[off + b] << (8 * b);
        for (uint32_t b = 0; b < 8; ++b) hi |= (uint64_t)p[off + 8 + b] << (8 * b);
        a = lo;
        c = hi;
      }
      const uint32_t cnt = nstripes - s0 < 32 ? nstripes - s0 : 32;
      for (uint32_t k = 0; k < cnt; ++k) {
        const uint64_t x1 = ((uint64_t)readlane((uint32_t)(a >> 32), 2 * k) << 32) | readlane((uint32_t)a, 2 * k);
        const uint64_t x2 = ((uint64_t)readlane((uint32_t)(c >> 32), 2 * k) << 32) | readlane((uint32_t)c, 2 * k);
        const uint64_t x3 = ((uint64_t)readlane((uint32_t)(a >> 32), 2 * k + 1) << 32) | readlane((uint32_t)a, 2 * k + 1);
        const uint64_t x4 = ((uint64_t)readlane((uint32_t)(c >> 32), 2 * k + 1) << 32) | readlane((uint32_t)c, 2 * k + 1);
        v1 = round(v1, x1); v2 = round(v2, x2); v3 = round(v3, x3); v4 = round(v4, x4);
      }
    }
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    auto merge = [&](uint64_t acc, uint64_t v) { acc ^= round(0, v); return acc * P1 + P4; };
    h = merge(h, v1); h = merge(h, v2); h = merge(h, v3); h = merge(h, v4);
    i = nstripes * 32;
  } else {
    h = P5;
  }
  h += n;
  // tail (< 32 bytes): lanes fetch, lane 0's scalar loop consumes
  const uint32_t tb = i + lane < n ? (uint32_t)p[i + lane] : 0u;
  uint32_t k = 0;
  const uint32_t rem = n - i;
  for (; k + 8 <= rem; k += 8) {
    uint64_t x = 0;
    for (uint32_t b = 0; b < 8; ++b) x |= (uint64_t)readlane(tb, k + b) << (8 * b);
    h ^= round(0, x);
    h = rotl(h, 27) * P1 + P4;
  }
  if (k + 4 <= rem) {
    uint64_t x = 0;
    for (uint32_t b = 0; b < 4; ++b) x |= (uint64_t)readlane(tb, k + b) << (8 * b);
    h ^= x * P1;
    h = rotl(h, 23) * P2 + P3;
    k += 4;
  }
  for (; k < rem; ++k) {
    h ^= (uint64_t)readlane(tb, k) * P5;
    h = rotl(h, 11) * P1;
  }
  h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
  return (uint32_t)h;
}

}  // namespace zsd

#ifndef BITAR_ZSD_WAVES
#define BITAR_ZSD_WAVES 0
#endif
#if BITAR_ZSD_WAVES
#define BITAR_ZSD_ATTR __attribute__((amdgpu_waves_per_eu(BITAR_ZSD_WAVES)))
#else
#define BITAR_ZSD_ATTR
#endif
__global__ __launch_bounds__(64) BITAR_ZSD_ATTR void zstd_decompress_kernel(
    const uint8_t* const* __restrict__ srcs, const uint8_t* __restrict__ slab,
    uint64_t slot_stride, const uint32_t* __restrict__ csizes, uint32_t nseg, uint32_t seg,
    uint8_t* __restrict__ out, uint32_t* __restrict__ produced, uint32_t* __restrict__ err,
    uint32_t defer_only, uint8_t* __restrict__ hscr, unsigned long long* __restrict__ stats,
    const uint32_t* __restrict__ order, uint32_t multi) {
  using namespace zsd;
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWin + kRing];
  __shared__ __attribute__((aligned(16))) Tabs t;
  uint8_t* win = lds;
  uint8_t* ring = lds + kWin;
  if (blockIdx.x >= nseg) return;
  const uint32_t i = order ? order[blockIdx.x] : blockIdx.x;  // (cost-ordered dispatch)
  if (i >= nseg) return;
  // after zstd_lanes_kernel: only the segments it deferred (zstd_lanes.hip)
  if (defer_only && produced[i] != 0xFFFFFFFEu) return;
  State s;
  s.src = global_ptr(srcs ? srcs[i] : slab + (uint64_t)i * slot_stride);
  s.csize = csizes[i];
  s.dst = global_ptr(out + (uint64_t)i * seg);
  s.cap = seg;
  s.ip = 0;
  s.op = 0;
  s.flushed = 0;
  s.fenced = 0;
  s.wb = ~0ull;
  s.wlen = 0;
#ifdef ZPROF
  if (lane_id() < 16) zp_lds[lane_id()] = 0;
  const uint64_t t_all = ZP_T();
#endif
  bool ok = false;
  do {
    const uint32_t cs = s.csize;
    if (cs < 6 || load_le(s, win, 0, 4) != 0xFD2FB528u) break;
    uint32_t p = 4;
    const uint32_t fhd = load_le(s, win, p++, 1);
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1u, cks = (fhd >> 2) & 1u,
                   did_flag = fhd & 3u;
    if (fhd & 8u) break;
    if (!single) {
      if (p >= cs) break;
      p++;
    }
    const uint32_t did_sz = did_flag == 3 ? 4u : did_flag;
    if (p + did_sz > cs) break;
    const uint32_t did = did_sz ? load_le(s, win, p, did_sz) : 0u;
    p += did_sz;
    if (did) break;
    uint32_t fsz = fcs_flag == 0 ? (single ? 1u : 0u) : fcs_flag == 1 ? 2u : fcs_flag == 2 ? 4u : 8u;
    if (p + fsz > cs) break;
    uint64_t fcs = 0;
    if (fsz == 8) fcs = (uint64_t)load_le(s, win, p, 4) | ((uint64_t)load_le(s, win, p + 4, 4) << 32);
    else if (fsz) fcs = load_le(s, win, p, fsz);
    if (fsz == 2) fcs += 256;
    p += fsz;
    if (fsz && fcs > s.cap) break;
    Frame fr;
    fr.rep0 = 1; fr.rep1 = 4; fr.rep2 = 8;
    fr.have[0] = fr.have[1] = fr.have[2] = false;
    fr.pre[0] = fr.pre[1] = fr.pre[2] = false;
    fr.huf_log = 0;
    bool bad = false, last = false, handed = false;
    GMEM uint32_t* hand = hscr && !cks ? global_ptr(reinterpret_cast<uint32_t*>(hscr + (uint64_t)i * zhand::kStride))
                                       : nullptr;
    // all blocks to the lane kernels (the two-phase sequence path only), else the last one
    const uint32_t nbm = hand && multi ? multi_blocks(s, win, p, cs) : 0u;
    uint32_t h_nseq = 0, h_regen = 0;
    while (!last) {
      if (p + 3 > cs) { bad = true; break; }
      const uint32_t bh = load_le(s, win, p, 3);
      p += 3;
      last = bh & 1u;
      const uint32_t type = (bh >> 1) & 3u, bsz = bh >> 3;
      if (type == 0) {
        if (p + bsz > cs || (uint64_t)s.op + bsz > s.cap) { bad = true; break; }
        s.ip = p;
        ZP_BEGIN(tr);
        if (bsz >= kLongLit) literals_long(s, win, ring, bsz);
        else if (bsz) literals_short(s, win, ring, bsz);
        ZP_END(7, tr);
        ZP_ADD(14, 1);
        p += bsz;
      } else if (type == 1) {
        if (p + 1 > cs || (uint64_t)s.op + bsz > s.cap) { bad = true; break; }
        out_fill(s, ring, load_le(s, win, p, 1), bsz);
        p += 1;
      } else if (type == 2) {
        if (bsz > (128u << 10) || p + bsz > cs) { bad = true; break; }
        ZP_BEGIN(tb);
        const int r = block(s, win, ring, t, fr, p, bsz, hand, last || nbm != 0, fsz, (uint32_t)fcs,
                            h_nseq, h_regen);
        if (r == 0) { bad = true; break; }
        if (r == 2) {
          handed = true;
          // the frame-level words (zstd_hand.hip.h), and the later blocks' sub-records
          uint32_t nsa = h_nseq, lsa = h_regen, nb = 1;
          uint32_t xv = 0;  // lane 8 b + k: block b's extra word k
          if (lane_id() == 0) xv = 0u;  // block 0: records and literals from 0
          for (uint32_t q = p + bsz; nb < nbm; ++nb) {
            const uint32_t bh2 = load_le(s, win, q, 3);
            const uint32_t bsz2 = bh2 >> 3;
            q += 3;
            uint32_t ns2 = 0, rg2 = 0;
            if (!hand_header(s, win, fr, hand + zhand::blk_at(nb), q, bsz2, ns2, rg2)) {
              bad = true;
              break;
            }
            const uint32_t ln = lane_id();
            xv = ln == zhand::kXW * nb + zhand::kXRec ? nsa : ln == zhand::kXW * nb + zhand::kXLit ? lsa : xv;
            nsa += ns2;
            lsa += rg2;
            q += bsz2;
          }
          if (bad) break;
          if (lsa > s.cap - s.op) { bad = true; break; }  // (the slot tail holds them all)
          const uint32_t ln = lane_id();
          const bool xs = ln < zhand::kXW * nb && (ln % zhand::kXW) <= zhand::kXLit;
          if (xs) hand[zhand::kX0 + ln] = xv;
          if (ln == 0) {
            hand[zhand::kNb] = nb;
            hand[zhand::kNseqAll] = nsa;
            hand[zhand::kLitAll] = lsa;
          }
          break;
        }
        ZP_END(1, tb);
        ZP_ADD(13, 1);
        p += bsz;
      } else {
        bad = true;
        break;
      }
    }
    if (bad) break;
    if (handed) {  // the executor finishes the frame (and its final checks)
#ifdef ZPROF
      ZP_ADD(0, ZP_T() - t_all);
      lds_order();
      if (lane_id() < 16) atomicAdd(&g_zprof[lane_id()], zp_lds[lane_id()]);
#endif
      if (lane_id() == 0) {
        produced[i] = kHanded;
        if (stats) {
          atomicAdd(stats + BITAR_HIP_PATH_ZSTD_WAVE, 1ull);
          atomicAdd(stats + BITAR_HIP_PATH_ZSTD_HANDED, 1ull);
        }
      }
      return;
    }
    flush(s, ring, s.op, true);
    if (cks) {
      if (p + 4 > cs) break;
      global_fence_wave();
      if (xxh64_low(s.dst, s.op) != load_le(s, win, p, 4)) break;
      p += 4;
    }
    if (p != cs) break;
    if (fsz && fcs != s.op) break;
    ok = true;
  } while (false);
#ifdef ZPROF
  ZP_ADD(0, ZP_T() - t_all);
  lds_order();
  if (lane_id() < 16) atomicAdd(&g_zprof[lane_id()], zp_lds[lane_id()]);
#endif
  if (ok) {
    if (lane_id() == 0) produced[i] = s.op;
  } else if (lane_id() == 0) {
    produced[i] = 0xFFFFFFFFu;
    atomicOr(err, 1u);
  }
  if (stats && lane_id() == 0) atomicAdd(stats + BITAR_HIP_PATH_ZSTD_WAVE, 1ull);
}

}  // namespace bitar_hip

#ifdef ZPROF
extern "C" int bitar_hip_debug_zstd_prof(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(bitar_hip::zsd::g_zprof), 16 * 8) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(bitar_hip::zsd::g_zprof), z, sizeof z) != hipSuccess) return -1;
  }
  return 0;
}
#endif
