// inflate.hip -- raw DEFLATE (RFC 1951) decode, one wavefront per segment (gfx950).
//
// The reference's frame: one independent raw-DEFLATE stream per segment, produced by the
// BlueField-2 engine with RTE_COMP_ALGO_DEFLATE (reference src/config.cc:83-105) and
// FLUSH_FINAL per op (src/memory.cc:110).  Acceptance rules are those of the oracle's
// bo_inflate_raw (stored / fixed / dynamic blocks; over-subscribed codes rejected,
// incomplete codes accepted until an unassigned code is met).
//
// Decoding is wave-uniform: the bit buffer lives in scalar registers, Huffman symbols come
// from LDS fast tables (10-bit literal/length, 9-bit distance, canonical fallback for longer
// codes), literals gather in a lane vector and land in the history ring 64 at a time, and
// matches / stored blocks reuse the window + ring machinery of stream_ring.hip.h.
#include "stream_ring.hip.h"

namespace bitar_hip {

namespace infl {

using namespace sr;

constexpr uint32_t kLitFast = 10, kDistFast = 9, kClFast = 7;

__device__ __forceinline__ uint32_t bpermute_u32(uint32_t v, uint32_t src_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}

struct Tables {  // LDS
  uint16_t lit_fast[1u << kLitFast];   // sym | len << 9  (0 = not a <= kLitFast-bit code)
  uint16_t dist_fast[1u << kDistFast];
  uint16_t cl_fast[1u << kClFast];
  uint16_t lit_count[16], dist_count[16], cl_count[16];
  uint16_t lit_sym[288], dist_sym[32], cl_sym[19];
  uint32_t base[16];                   // scratch for ranking / next codes
  uint8_t lens[320];
};

__constant__ uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                      2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDistBase[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                       33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                       1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2,  3,  3,  4,  4,  5,  5,  6,
                                       6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Wave-uniform LSB-first bit reader over the staged stream.
struct Bits {
  uint64_t buf;   // next bits, LSB first
  uint32_t cnt;   // valid bits in buf
  uint32_t bp;    // next stream byte to load into buf
  uint64_t used;  // bits consumed so far
};

// 4 stream bytes at bp (zeros past csize), as one little-endian word
__device__ __forceinline__ uint32_t peek4(State& s, uint8_t* win, uint32_t bp) {
  const uint32_t lane = lane_id();
  uint32_t avail = bp < s.csize ? s.csize - bp : 0;
  if (avail > 4) avail = 4;
  uint32_t v = 0;
  if (avail) {
    const uint32_t w = win_at(s, win, bp, avail);
    lds_order();
    v = lane < avail ? (uint32_t)win[w + lane] : 0u;
  }
  const uint32_t b0 = readlane(v, 0), b1 = readlane(v, 1), b2 = readlane(v, 2), b3 = readlane(v, 3);
  return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
}

__device__ __forceinline__ void need(State& s, uint8_t* win, Bits& b, uint32_t n) {
  while (b.cnt < n) {  // n <= 32: at most two refills
    const uint32_t w = peek4(s, win, b.bp);
    b.buf |= (uint64_t)w << b.cnt;
    b.cnt += 32;
    b.bp += 4;
  }
}

// take n (<= 32) bits; false if that runs past the stream (the oracle's bits_get == -1)
__device__ __forceinline__ bool take(State& s, uint8_t* win, Bits& b, uint32_t n, uint32_t& v) {
  if (n == 0) { v = 0; return true; }
  need(s, win, b, n);
  if (b.used + n > (uint64_t)s.csize * 8) return false;
  v = (uint32_t)(b.buf & ((1ull << n) - 1));
  b.buf >>= n;
  b.cnt -= n;
  b.used += n;
  return true;
}

// Build the decoding tables of one code from lens[0..n) (LDS).  Returns false if the code is
// over-subscribed.  fast: 2^fbits entries; count/sym: canonical arrays for long codes.
__device__ __forceinline__ bool build(Tables& t, const uint8_t* lens, uint32_t n, uint16_t* fast, uint32_t fbits,
                      uint16_t* count, uint16_t* sym) {
  const uint32_t lane = lane_id();
  lds_order();
  if (lane < 16) t.base[lane] = 0;
  lds_order();
  for (uint32_t k = lane; k < n; k += kWave) {
    const uint32_t l = lens[k];
    if (l) atomicAdd(&t.base[l], 1u);
  }
  lds_order();
  uint32_t cntv = lane < 16 ? t.base[lane] : 0u;
  if (lane == 0) cntv = 0;
  // over-subscription: left = 1; left = 2*left - count[len]
  int left = 1;
  uint32_t code = 0;
  uint32_t ncv = 0;    // lane L: first canonical code of length L
  uint32_t offs = 0;
  uint32_t offsv = 0;  // lane L: index of the first symbol of length L in sorted order
#pragma unroll
  for (uint32_t len = 1; len <= 15; ++len) {
    const uint32_t c = readlane(cntv, len);
    left = 2 * left - (int)c;
    code = (code + readlane(cntv, len - 1)) << 1;
    if (lane == len) { offsv = offs; ncv = code; }
    offs += c;
  }
  if (left < 0) return false;
  lds_order();
  if (lane < 16) {
    count[lane] = (uint16_t)cntv;
    t.base[lane] = offsv;  // running sorted position per length
  }
  for (uint32_t k = 0; k < (1u << fbits); k += kWave) fast[k + lane] = 0;
  lds_order();
  // rank symbols of each length in symbol order (64 at a time), assign canonical codes
  for (uint32_t k0 = 0; k0 < n; k0 += kWave) {
    const uint32_t k = k0 + lane;
    const uint32_t l = k < n ? lens[k] : 0u;
    uint32_t myidx = 0;
    for (uint32_t len = 1; len <= 15; ++len) {
      const uint64_t m = ballot(l == len);
      if (!m) continue;
      const uint32_t b = uniform(t.base[len]);
      if (l == len) myidx = b + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1));
      lds_order();
      if (lane == 0) t.base[len] = b + (uint32_t)__builtin_popcountll(m);
      lds_order();
    }
    // canonical code = first code of length l + rank within length (all lanes permute:
    // ds_bpermute must run with every lane active)
    const uint32_t first = bpermute_u32(offsv, l), nc = bpermute_u32(ncv, l);
    if (l) {
      sym[myidx] = (uint16_t)k;
      const uint32_t c = nc + (myidx - first);
      if (l <= fbits) {
        const uint32_t r = __builtin_bitreverse32(c) >> (32 - l);
        const uint16_t e = (uint16_t)(k | (l << 9));
        for (uint32_t j = r; j < (1u << fbits); j += (1u << l)) fast[j] = e;
      }
    }
    lds_order();
  }
  return true;
}

// Decode one symbol; returns -1 if the code runs past the stream, -2 if unassigned.
__device__ __forceinline__ int decode(State& s, uint8_t* win, Bits& b, const uint16_t* fast,
                                      uint32_t fbits, const uint16_t* count, const uint16_t* sym) {
  need(s, win, b, 15);
  lds_order();
  const uint32_t e = uniform((uint32_t)fast[b.buf & ((1u << fbits) - 1)]);
  if (e) {
    const uint32_t len = e >> 9;
    if (b.used + len > (uint64_t)s.csize * 8) return -1;
    b.buf >>= len;
    b.cnt -= len;
    b.used += len;
    return (int)(e & 511u);
  }
  int code = 0, first = 0, index = 0;
  for (uint32_t len = 1; len <= 15; ++len) {
    if (b.used + len > (uint64_t)s.csize * 8) return -1;
    code |= (int)((b.buf >> (len - 1)) & 1u);
    const int cnt = (int)uniform((uint32_t)count[len]);
    if (code - cnt < first) {
      b.buf >>= len;
      b.cnt -= len;
      b.used += len;
      return (int)uniform((uint32_t)sym[index + (code - first)]);
    }
    index += cnt;
    first += cnt;
    first <<= 1;
    code <<= 1;
  }
  return -2;
}

// pending literals, one per lane, written to the ring 64 at a time
struct Lits {
  uint32_t v;  // lane j: j-th pending byte
  uint32_t n;
};

__device__ __forceinline__ void lits_flush(State& s, uint8_t* ring, Lits& L) {
  if (!L.n) return;
  make_room(s, ring, L.n);
  const uintptr_t base = (uintptr_t)s.dst;
  lds_order();
  if (lane_id() < L.n) ring[(base + s.op + lane_id()) & kRingMask] = (uint8_t)L.v;
  lds_order();
  s.op += L.n;
  L.n = 0;
}

__device__ __forceinline__ int inflate_codes(State& s, uint8_t* win, uint8_t* ring, Bits& b, Tables& t,
                             Lits& L) {
  for (;;) {
    const int sym = decode(s, win, b, t.lit_fast, kLitFast, t.lit_count, t.lit_sym);
    if (sym < 0) return -1;
    if (sym < 256) {
      if (s.op + L.n >= s.cap) return -1;
      if (lane_id() == L.n) L.v = (uint32_t)sym;
      if (++L.n == kWave) lits_flush(s, ring, L);
      continue;
    }
    if (sym == 256) return 0;
    const uint32_t ls = (uint32_t)sym - 257;
    if (ls >= 29) return -1;
    uint32_t e;
    if (!take(s, win, b, kLenExtra[ls], e)) return -1;
    const uint32_t len = kLenBase[ls] + e;
    const int ds = decode(s, win, b, t.dist_fast, kDistFast, t.dist_count, t.dist_sym);
    if (ds < 0 || ds >= 30) return -1;
    if (!take(s, win, b, kDistExtra[ds], e)) return -1;
    const uint32_t d = kDistBase[ds] + e;
    lits_flush(s, ring, L);
    if (d > s.op) return -1;
    if (s.op + len > s.cap) return -1;
    match_copy(s, ring, d, len);
  }
}

}  // namespace infl

__global__ __launch_bounds__(64) void inflate_kernel(
    const uint8_t* const* __restrict__ srcs, const uint8_t* __restrict__ slab,
    uint64_t slot_stride, const uint32_t* __restrict__ csizes, uint32_t nseg, uint32_t seg,
    uint8_t* __restrict__ out, uint32_t* __restrict__ produced, uint32_t* __restrict__ err) {
  using namespace infl;
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWin + kRing];
  __shared__ __attribute__((aligned(16))) Tables t;
  uint8_t* win = lds;
  uint8_t* ring = lds + kWin;
  const uint32_t i = blockIdx.x;
  if (i >= nseg) return;
  const uint32_t lane = lane_id();

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

  Bits b = {0ull, 0u, 0u, 0ull};
  Lits L = {0u, 0u};
  bool ok = true;
  uint32_t last = 0;
  uint32_t built_fixed = 0;
  do {
    uint32_t hdr;
    if (!take(s, win, b, 3, hdr)) { ok = false; break; }
    last = hdr & 1u;
    const uint32_t type = hdr >> 1;
    if (type == 0) {  // stored: LEN, NLEN at the next byte boundary, then LEN raw bytes
      const uint32_t drop = (uint32_t)(b.used & 7u) ? 8u - (uint32_t)(b.used & 7u) : 0u;
      uint32_t junk;
      if (drop && !take(s, win, b, drop, junk)) { ok = false; break; }
      const uint32_t p = (uint32_t)(b.used >> 3);
      if ((uint64_t)p + 4 > s.csize) { ok = false; break; }
      uint32_t w0;
      take(s, win, b, 32, w0);
      const uint32_t len = w0 & 0xFFFFu, nlen = w0 >> 16;
      if (len != (~nlen & 0xFFFFu)) { ok = false; break; }
      if ((uint64_t)p + 4 + len > s.csize) { ok = false; break; }
      lits_flush(s, ring, L);
      if ((uint64_t)s.op + len > s.cap) { ok = false; break; }
      s.ip = p + 4;
      if (len >= kLongLit) literals_long(s, win, ring, len);
      else if (len) literals_short(s, win, ring, len);
      b.buf = 0;  // restart the bit reader after the raw bytes
      b.cnt = 0;
      b.bp = s.ip;
      b.used = (uint64_t)s.ip * 8;
    } else if (type == 1) {
      if (!built_fixed) {
        lds_order();
        for (uint32_t k = lane; k < 320; k += kWave)
          t.lens[k] = k < 144 ? 8 : k < 256 ? 9 : k < 280 ? 7 : k < 288 ? 8 : 5;
        lds_order();
        build(t, t.lens, 288, t.lit_fast, kLitFast, t.lit_count, t.lit_sym);
        build(t, t.lens + 288, 30, t.dist_fast, kDistFast, t.dist_count, t.dist_sym);
        built_fixed = 1;
      }
      if (inflate_codes(s, win, ring, b, t, L)) { ok = false; break; }
    } else if (type == 2) {
      built_fixed = 0;
      uint32_t hlit, hdist, hclen;
      if (!take(s, win, b, 5, hlit) || !take(s, win, b, 5, hdist) || !take(s, win, b, 4, hclen)) {
        ok = false;
        break;
      }
      const uint32_t nlen = hlit + 257, ndist = hdist + 1, ncode = hclen + 4;
      if (nlen > 286 || ndist > 30) { ok = false; break; }
      lds_order();
      if (lane < 19) t.lens[lane] = 0;
      lds_order();
      bool bad = false;
      for (uint32_t k = 0; k < ncode; ++k) {
        uint32_t v;
        if (!take(s, win, b, 3, v)) { bad = true; break; }
        lds_order();
        if (lane == 0) t.lens[kClOrder[k]] = (uint8_t)v;
        lds_order();
      }
      if (bad) { ok = false; break; }
      if (!build(t, t.lens, 19, t.cl_fast, kClFast, t.cl_count, t.cl_sym)) { ok = false; break; }
      uint32_t idx = 0;
      while (idx < nlen + ndist) {
        const int sym = decode(s, win, b, t.cl_fast, kClFast, t.cl_count, t.cl_sym);
        if (sym < 0) { bad = true; break; }
        if (sym < 16) {
          lds_order();
          if (lane == 0) t.lens[idx] = (uint8_t)sym;
          lds_order();
          ++idx;
          continue;
        }
        uint32_t val = 0, rep;
        if (sym == 16) {
          if (idx == 0) { bad = true; break; }
          lds_order();
          val = uniform((uint32_t)t.lens[idx - 1]);
          if (!take(s, win, b, 2, rep)) { bad = true; break; }
          rep += 3;
        } else if (sym == 17) {
          if (!take(s, win, b, 3, rep)) { bad = true; break; }
          rep += 3;
        } else {
          if (!take(s, win, b, 7, rep)) { bad = true; break; }
          rep += 11;
        }
        if (idx + rep > nlen + ndist) { bad = true; break; }
        lds_order();
        for (uint32_t k = lane; k < rep; k += kWave) t.lens[idx + k] = (uint8_t)val;
        lds_order();
        idx += rep;
      }
      if (bad) { ok = false; break; }
      lds_order();
      if (uniform((uint32_t)t.lens[256]) == 0) { ok = false; break; }
      // the distance lengths must not alias the scratch the literal build uses
      if (!build(t, t.lens, nlen, t.lit_fast, kLitFast, t.lit_count, t.lit_sym)) { ok = false; break; }
      if (!build(t, t.lens + nlen, ndist, t.dist_fast, kDistFast, t.dist_count, t.dist_sym)) {
        ok = false;
        break;
      }
      if (inflate_codes(s, win, ring, b, t, L)) { ok = false; break; }
    } else {
      ok = false;
      break;
    }
  } while (!last);
  if (ok) {
    lits_flush(s, ring, L);
    flush(s, ring, s.op, true);
    if (lane == 0) produced[i] = s.op;
  } else if (lane == 0) {
    produced[i] = 0xFFFFFFFFu;
    atomicOr(err, 1u);
  }
}

}  // namespace bitar_hip
