// compress.hip -- segment compressors, one wavefront per segment (gfx950):
//   lz4_compress_kernel      raw LZ4 block per segment (the north-star codec)
//   deflate_compress_kernel  raw DEFLATE, one fixed-Huffman block per segment (the
//                            reference's frame: RTE_COMP_ALGO_DEFLATE, FLUSH_FINAL, Huffman
//                            FIXED is a legal BlueField config -- device.cc:558-577)
//
// Both replace the compress op the reference hands to the BlueField engine per segment
// (reference src/memory.cc:350-430: one op per <= seg-byte input slice into a slot).
// They share the "window-scan parse" restated in oracle/bitar_oracle.c (bo_window_parse)
// and must match the oracle's output byte for byte.
//
// Per fixed window of 64 positions (one per lane):
//   1. the segment streams through an 8 KiB LDS input ring in 256-B rows loaded 2 KiB ahead
//      (coalesced dword loads held in registers), so every byte a position, a candidate
//      (matches are capped at 7680 B back) or a literal needs is an LDS read;
//   2. look up a 4096-entry LDS table of u16 positions, then insert every position (the
//      largest position wins a slot: deterministic);
//   3. lanes with a candidate verify + measure the match on 8 bytes from the input ring;
//   4. a scalar greedy loop picks matches in lane order (ballot + ctz), extends long ones
//      cooperatively (ring first, then HBM 1 KiB per step), and hands each sequence to the
//      codec's emitter.
// Emitters stage output in LDS and flush it with wide stores:
//   LZ4: one LDS write per sequence (token, length bytes, literals, offset laid out across
//        lanes); a byte ring flushed in 16-B blocks; long literal runs go HBM -> HBM.
//   DEFLATE: a bit ring; each lane's code (a sequence's literals and its match symbol) is
//            placed by a wave prefix sum of code lengths and OR-ed into LDS (ds_or_b32).
#include "wave.hip.h"

namespace bitar_hip {

namespace cmp {

constexpr uint32_t kHashLog = 12;
constexpr uint32_t kMinMatch = 4;
constexpr uint32_t kLastLiterals = 5;
constexpr uint32_t kMfLimit = 12;
// Match distance cap (both codecs): the 8 KiB input ring holds [x + 128 - 8192, x + 128) at
// window x, so every candidate of a window (>= x - 7680) is in LDS; it is also inside the
// LZ4 decoder's 8 KiB history ring (reach 8048), so our streams decode on its LDS path.
constexpr uint32_t kMaxDist = 7680;
constexpr uint32_t kIn = 8192, kInMask = kIn - 1;  // LDS input ring

__device__ __forceinline__ uint32_t hash4(uint32_t v) { return (v * 2654435761u) >> (32 - kHashLog); }

// 4 bytes at p (any alignment).  The dword after the aligned one is loaded only if it
// starts before `end`, so no load leaves the input buffer (an aligned dword holding a valid
// byte never crosses a page).
__device__ __forceinline__ uint32_t ld32u(const uint8_t* p, const uint8_t* end) {
  const uintptr_t a = (uintptr_t)p & ~(uintptr_t)3;
  const uint32_t r = (uint32_t)((uintptr_t)p & 3);
  const uint32_t lo = *reinterpret_cast<const uint32_t*>(a);
  const uint32_t hi = (r && a + 4 < (uintptr_t)end) ? *reinterpret_cast<const uint32_t*>(a + 4) : 0u;
  return funnel(lo, hi, r);
}

// 16 bytes at p (any alignment); aligned blocks at or past `end` are not loaded (zeros)
__device__ __forceinline__ uint4 ld16u(const uint8_t* p, const uint8_t* end) {
  const uintptr_t a = (uintptr_t)p & ~(uintptr_t)15;
  const uint32_t sh = (uint32_t)((uintptr_t)p & 15);
  const uint4 x = *reinterpret_cast<const uint4*>(a);
  uint4 y = make_uint4(0, 0, 0, 0);
  if (sh && a + 16 < (uintptr_t)end) y = *reinterpret_cast<const uint4*>(a + 16);
  const uint32_t w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
  const uint32_t q = sh >> 2, r = sh & 3u;
  const uint32_t s0 = q == 0 ? w[0] : q == 1 ? w[1] : q == 2 ? w[2] : w[3];
  const uint32_t s1 = q == 0 ? w[1] : q == 1 ? w[2] : q == 2 ? w[3] : w[4];
  const uint32_t s2 = q == 0 ? w[2] : q == 1 ? w[3] : q == 2 ? w[4] : w[5];
  const uint32_t s3 = q == 0 ? w[3] : q == 1 ? w[4] : q == 2 ? w[5] : w[6];
  const uint32_t s4 = q == 0 ? w[4] : q == 1 ? w[5] : q == 2 ? w[6] : w[7];
  return make_uint4(funnel(s0, s1, r), funnel(s1, s2, r), funnel(s2, s3, r), funnel(s3, s4, r));
}

__device__ __forceinline__ uint32_t common16(uint4 a, uint4 b) {
  const uint32_t d0 = a.x ^ b.x, d1 = a.y ^ b.y, d2 = a.z ^ b.z, d3 = a.w ^ b.w;
  if (d0) return __builtin_ctz(d0) >> 3;
  if (d1) return 4 + (__builtin_ctz(d1) >> 3);
  if (d2) return 8 + (__builtin_ctz(d2) >> 3);
  if (d3) return 12 + (__builtin_ctz(d3) >> 3);
  return 16;
}

__device__ __forceinline__ uint32_t bpermute(uint32_t v, uint32_t src_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}

// The LDS input ring: byte of segment position q lives at ring[(in_lo + q) & kInMask]
// (absolute-address indexing keeps aligned dwords aligned).
struct InRing {
  uint8_t* ring;
  uint32_t in_lo;  // low 32 bits of the segment's input address
  uint32_t lo;     // positions >= lo are in the ring (< the filled end)

  __device__ __forceinline__ uint32_t byte(uint32_t q) const {
    return ring[(in_lo + q) & kInMask];
  }
  // 8 bytes at position q (q >= lo, q + 8 <= filled end), as a little-endian 64-bit value
  __device__ __forceinline__ uint64_t bytes8(uint32_t q) const {
    const uint32_t a = in_lo + q;
    const uint32_t* r32 = reinterpret_cast<const uint32_t*>(ring);
    const uint32_t d = a >> 2, sh = a & 3u;
    const uint32_t w0 = r32[d & (kInMask >> 2)], w1 = r32[(d + 1) & (kInMask >> 2)],
                   w2 = r32[(d + 2) & (kInMask >> 2)];
    return (uint64_t)funnel(w0, w1, sh) | ((uint64_t)funnel(w1, w2, sh) << 32);
  }
};

// number of equal leading bytes of two 8-byte little-endian values (0..8)
__device__ __forceinline__ uint32_t common8(uint64_t a, uint64_t b) {
  const uint64_t d = a ^ b;
  return d ? (uint32_t)(__builtin_ctzll(d) >> 3) : 8u;
}

// ---- LZ4 emitter: output staged in an LDS byte ring, flushed in aligned 16-B blocks ----
constexpr uint32_t kObuf = 2048, kObufMask = kObuf - 1, kObufFlush = kObuf / 2;

struct Lz4Out {
  uint8_t* ring;  // LDS
  uint8_t* dst;   // slot
  uint64_t cap;
  uint32_t op, flushed;
  bool overflow;

  __device__ __forceinline__ void flush(uint32_t upto, bool final) {
    const uint32_t lane = lane_id();
    const uintptr_t base = (uintptr_t)dst;
    uint32_t f = flushed;
    lds_order();
    uint32_t head = (uint32_t)((16u - ((base + f) & 15u)) & 15u);
    if (head > upto - f) head = upto - f;
    if (head) {
      if (lane < head) dst[f + lane] = ring[(base + f + lane) & kObufMask];
      f += head;
    }
    const uint32_t nb = (upto - f) >> 4;
    for (uint32_t b = lane; b < nb; b += kWave) {
      const uint32_t k = f + 16u * b;
      *reinterpret_cast<uint4*>(dst + k) = *reinterpret_cast<const uint4*>(ring + ((base + k) & kObufMask));
    }
    f += nb << 4;
    if (final && f < upto) {
      if (lane < upto - f) dst[f + lane] = ring[(base + f + lane) & kObufMask];
      f = upto;
    }
    flushed = f;
  }
  __device__ __forceinline__ bool room(uint32_t n) {
    if ((uint64_t)op + n > cap) { overflow = true; return false; }
    if (op + n - flushed > kObufFlush) flush(op, false);
    return true;
  }
  // lanes < n write byte `v` at op + lane
  __device__ __forceinline__ void put(uint32_t v, uint32_t n) {
    lds_order();
    if (lane_id() < n) ring[((uintptr_t)dst + op + lane_id()) & kObufMask] = (uint8_t)v;
    lds_order();
    op += n;
  }
  __device__ __forceinline__ void put_ext(uint32_t v) {  // 255 ... 255, v % 255
    const uint32_t cnt = v / 255u + 1;
    for (uint32_t k = 0; k < cnt; k += kWave) {
      const uint32_t step = cnt - k < kWave ? cnt - k : kWave;
      if (!room(step)) return;
      const uint32_t t = k + lane_id();
      put(t + 1 < cnt ? 255u : v % 255u, step);
    }
  }
  __device__ __forceinline__ void sequence(const uint8_t* in, const InRing& I, uint32_t lit_start,
                                           uint32_t lit_len, uint32_t off, uint32_t mlen) {
    if (overflow) return;
    const uint32_t ml = mlen ? mlen - kMinMatch : 0;
    const uint32_t token = ((lit_len < 15 ? lit_len : 15) << 4) | (ml < 15 ? ml : 15);
    const uint32_t nlx = lit_len >= 15 ? (lit_len - 15) / 255u + 1 : 0;
    const uint32_t nmx = mlen && ml >= 15 ? (ml - 15) / 255u + 1 : 0;
    const uint32_t e = 1 + nlx + lit_len + (mlen ? 2 + nmx : 0);
    if (e <= kWave && lit_start >= I.lo) {
      // the whole sequence in one LDS write: lane t holds encoded byte t
      if (!room(e)) return;
      const uint32_t t = lane_id();
      const uint32_t lit0 = 1 + nlx, offp = lit0 + lit_len;
      lds_order();
      const uint32_t lb = I.byte(lit_start + (t - lit0 < lit_len ? t - lit0 : 0u));
      uint32_t v;
      if (t == 0) v = token;
      else if (t < lit0) v = t + 1 < lit0 ? 255u : (lit_len - 15) - 255u * (nlx - 1);
      else if (t < offp) v = lb;
      else if (t == offp) v = off & 0xFFu;
      else if (t == offp + 1) v = off >> 8;
      else v = t + 1 < e ? 255u : (ml - 15) - 255u * (nmx - 1);
      put(v, e);
      return;
    }
    if (!room(1)) return;
    put(token, 1);
    if (lit_len >= 15) put_ext(lit_len - 15);
    if (overflow) return;
    if (lit_len) {
      if ((uint64_t)op + lit_len > cap) { overflow = true; return; }
      // long run (or not in the input ring): drain the ring, then HBM -> HBM
      flush(op, true);
      wave_copy_global(dst + op, in + lit_start, lit_len);
      op += lit_len;
      flushed = op;
    }
    if (!mlen) return;
    if (!room(2)) return;
    put(lane_id() ? off >> 8 : off & 0xFF, 2);
    if (ml >= 15) put_ext(ml - 15);
  }
  __device__ __forceinline__ uint32_t finish() {
    flush(op, true);
    return op;
  }
};

// ---- fixed-Huffman DEFLATE emitter: LDS bit ring, lane codes placed by prefix sum -----
constexpr uint32_t kBitWords = 512, kBitMask = kBitWords - 1, kBitFlushWords = kBitWords / 2;

__constant__ uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                      31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                      2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDistBase[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                       33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                       1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2,  3,  3,  4,  4,  5,  5,  6,
                                       6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

__device__ __forceinline__ uint32_t rev(uint32_t v, uint32_t n) {
  return __builtin_bitreverse32(v) >> (32 - n);
}
// fixed literal/length code of symbol s, bit-reversed for LSB-first packing; *n = length
__device__ __forceinline__ uint32_t fixed_code(uint32_t s, uint32_t& n) {
  if (s < 144) { n = 8; return rev(0x30 + s, 8); }
  if (s < 256) { n = 9; return rev(0x190 + (s - 144), 9); }
  if (s < 280) { n = 7; return rev(s - 256, 7); }
  n = 8;
  return rev(0xC0 + (s - 280), 8);
}

struct DflOut {
  uint32_t* stage;  // LDS, kBitWords dwords, zero outside the pending range
  uint32_t* dst;    // slot (16-B aligned)
  uint64_t cap;     // bytes
  uint64_t bits;
  uint32_t wflushed;
  bool overflow;

  __device__ __forceinline__ void flush_words(uint32_t upto) {
    const uint32_t lane = lane_id();
    lds_order();
    for (uint32_t w = wflushed + lane; w < upto; w += kWave) {
      dst[w] = stage[w & kBitMask];
      stage[w & kBitMask] = 0;
    }
    lds_order();
    wflushed = upto;
  }
  // append each lane's (val, nb) in lane order (nb <= 32; nb = 0 appends nothing)
  __device__ __forceinline__ void put_lanes(uint32_t val, uint32_t nb) {
    const uint32_t lane = lane_id();
    uint32_t incl = nb;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)incl, d, 64);
      if (lane >= d) incl += y;
    }
    const uint32_t total = readlane(incl, 63);
    if ((bits + total + 7) / 8 > cap) { overflow = true; return; }
    const uint64_t bp = bits + incl - nb;
    const uint32_t w = (uint32_t)(bp >> 5), sh = (uint32_t)(bp & 31);
    lds_order();
    if (nb) {
      atomicOr(&stage[w & kBitMask], val << sh);
      if (sh + nb > 32) atomicOr(&stage[(w + 1) & kBitMask], val >> (32 - sh));
    }
    lds_order();
    bits += total;
    const uint32_t full = (uint32_t)(bits >> 5);
    if (full - wflushed >= kBitFlushWords) flush_words(full);
  }
  __device__ __forceinline__ void put_one(uint32_t val, uint32_t nb) {
    put_lanes(lane_id() == 0 ? val : 0u, lane_id() == 0 ? nb : 0u);
  }
  // literal codes of [s, s+n) and (if mlen) the match symbol, in lane order, 63 per step
  __device__ __forceinline__ void sequence(const uint8_t* in, const InRing& I, uint32_t s,
                                           uint32_t n, uint32_t off, uint32_t mlen) {
    if (overflow) return;
    const uint32_t lane = lane_id();
    uint32_t mv = 0, mb = 0;  // the match symbol: length code + extra + distance code + extra
    if (mlen) {
      uint32_t ls = 28;
      while (kLenBase[ls] > mlen) --ls;
      uint32_t ln;
      const uint32_t lcode = fixed_code(257 + ls, ln);
      uint32_t ds = 29;
      while (kDistBase[ds] > off) --ds;
      const uint32_t le = kLenExtra[ls], de = kDistExtra[ds];
      mv = lcode | ((mlen - kLenBase[ls]) << ln) | (rev(ds, 5) << (ln + le)) |
           ((off - kDistBase[ds]) << (ln + le + 5));
      mb = ln + le + 5 + de;
    }
    const bool ring_ok = s >= I.lo;
    uint32_t k = 0;
    for (;;) {
      const uint32_t step = n - k < kWave - 1 ? n - k : kWave - 1;
      const bool last = k + step == n;
      const uint32_t q = s + k + (lane < step ? lane : 0);
      uint32_t b;
      lds_order();
      if (ring_ok) b = I.byte(q);
      else b = lane < step ? (uint32_t)in[q] : 0u;
      uint32_t nb;
      const uint32_t code = fixed_code(b, nb);
      uint32_t val = lane < step ? code : 0u;
      uint32_t bits_n = lane < step ? nb : 0u;
      if (last && lane == step) { val = mv; bits_n = mb; }
      put_lanes(val, bits_n);
      if (last || overflow) return;
      k += step;
    }
  }
  __device__ __forceinline__ uint32_t finish() {
    uint32_t n;
    const uint32_t eob = fixed_code(256, n);
    put_one(eob, n);
    flush_words((uint32_t)((bits + 31) >> 5));
    return (uint32_t)((bits + 7) >> 3);
  }
};

// The window-scan parse over one segment; calls E.sequence(...) in stream order.
//
// Input staging: the segment is read in 256-B rows (one aligned dword per lane, absolute-
// address aligned) that are loaded kQ rows ahead into registers and written into the 8 KiB
// LDS input ring one row ahead of the window scan.  At window x (row m = x / 256) the ring
// holds positions [F - 8192, F) with F = 256 (m + 2) - (in & 3): every candidate
// (>= x - 7680), every position's 8-byte probe (<= x + 74) and the first >= 256 B of every
// match extension are LDS reads; HBM is only touched by the row prefetch, by extensions past
// F and by literal runs longer than the ring.
// Hash table: 4096 u16 positions (8 KiB).  Lookups read the previous windows' state, then
// every position is written; a read-back loop settles same-slot writes of one window so the
// largest position wins (the oracle's ascending insert order).
constexpr uint32_t kQ = 8;  // rows in flight ahead of the ring (2 KiB)

__device__ __forceinline__ uint32_t common4(uint32_t a, uint32_t b) {
  const uint32_t d = a ^ b;
  return d ? (uint32_t)(__builtin_ctz(d) >> 3) : 4u;
}

template <class E>
__device__ __forceinline__ void parse(const uint8_t* in, uint32_t n, const uint8_t* in_end,
                                      uint16_t* table, uint8_t* inring, uint32_t max_dist,
                                      uint32_t max_mlen, E& em) {
  const uint32_t lane = lane_id();
  uint32_t anchor = 0;
  InRing I;
  I.ring = inring;
  I.in_lo = (uint32_t)(uintptr_t)in;
  I.lo = 0xFFFFFFFFu;  // nothing staged: literal bytes come from HBM
  if (n >= kMfLimit + 1) {
    // empty slot = candidate position 0 (the oracle's zeroed table)
    for (uint32_t k = lane; k < (1u << kHashLog) / 8; k += kWave)
      reinterpret_cast<uint4*>(table)[k] = make_uint4(0, 0, 0, 0);
    const uint32_t last_start = n - kMfLimit;
    const uint32_t match_limit = n - kLastLiterals;
    const uint32_t s0 = I.in_lo & 3u;
    const uint32_t* in32 = reinterpret_cast<const uint32_t*>(in - s0);
    uint32_t* r32 = reinterpret_cast<uint32_t*>(inring);
    const uint32_t rbase = (I.in_lo - s0) >> 2;  // ring dword of in32[0]
    // row r = dwords [64 r, 64 r + 64) of in32 = positions [256 r - s0, 256 r + 256 - s0)
    auto load_row = [&](uint32_t r) -> uint32_t {
      const uint32_t j = 64u * r + lane;
      return 4u * j < n + s0 ? in32[j] : 0u;
    };
    auto write_row = [&](uint32_t r, uint32_t v) { r32[(rbase + 64u * r + lane) & (kInMask >> 2)] = v; };
    uint32_t q[kQ];
    const uint32_t r0 = load_row(0);
#pragma unroll
    for (uint32_t k = 0; k < kQ; ++k) q[k] = load_row(1 + k);
    lds_order();
    write_row(0, r0);
    uint32_t F = 0;
    uint32_t pos = 0;
    for (uint32_t x = 0; x <= last_start; x += kWave) {
      if ((x & 255u) == 0) {  // next row into the ring, one more row in flight
        const uint32_t m = x >> 8;
        lds_order();
        write_row(m + 1, q[0]);
#pragma unroll
        for (uint32_t k = 0; k + 1 < kQ; ++k) q[k] = q[k + 1];
        q[kQ - 1] = load_row(m + 1 + kQ);
        F = 256u * (m + 2) - s0;
        I.lo = F > kIn ? F - kIn : 0u;
      }
      lds_order();
      const uint32_t p = x + lane;
      const bool act = p <= last_start;
      const uint64_t vp = I.bytes8(p);
      const uint32_t h = hash4((uint32_t)vp);
      const uint32_t cand = act ? table[h] : 0u;
      lds_order();
      if (act) table[h] = (uint16_t)p;
      const bool pre = act && cand < p && p - cand <= max_dist;
      uint32_t len = 0;
      if (pre) {  // verify the 4 bytes and measure up to 8, from the input ring
        len = common8(vp, I.bytes8(cand));
        uint32_t lim = match_limit - p;
        if (lim > max_mlen) lim = max_mlen;
        if (len > lim) len = lim;
      }
      // same-slot writes of this window: re-write until the largest position holds the slot
      lds_order();
      bool redo = act && table[h] < p;
      while (ballot(redo)) {
        lds_order();
        if (redo) table[h] = (uint16_t)p;
        lds_order();
        redo = redo && table[h] < p;
      }
      const uint64_t valid = ballot(pre && len >= kMinMatch);
      while (valid) {
        const uint32_t start = pos > x ? pos - x : 0u;
        if (start >= kWave) break;
        const uint64_t mk = valid & (~0ull << start);
        if (!mk) break;
        const uint32_t l = (uint32_t)__builtin_ctzll(mk);
        const uint32_t i = x + l;
        const uint32_t c = readlane(cand, l);
        uint32_t mlen = readlane(len, l);
        uint32_t lim = match_limit - i;
        if (lim > max_mlen) lim = max_mlen;
        if (mlen == 8 && lim > 8) {
          // extension, first from the input ring (4 B per lane per step) up to F ...
          const uint32_t lr = lim < F - i ? lim : F - i;
          uint32_t k = 8;
          bool more = true;
          for (;;) {
            const uint32_t kk = k + 4u * lane;
            uint32_t cl = 4;
            if (kk < lr) {
              cl = common4((uint32_t)I.bytes8(i + kk), (uint32_t)I.bytes8(c + kk));
              if (cl > lr - kk) cl = lr - kk;
            }
            const uint64_t stop = ballot(kk >= lr || cl < 4);
            if (stop) {
              const uint32_t sl = (uint32_t)__builtin_ctzll(stop);
              const uint32_t ks = k + 4u * sl;
              k = ks >= lr ? lr : ks + readlane(cl, sl);
              more = k == lr && lr < lim;  // stopped by the ring's end, not by a mismatch
              break;
            }
            k += 4u * kWave;
          }
          // ... then from HBM, 16 B per lane per step
          while (more) {
            const uint32_t kk = k + 16u * lane;
            uint32_t cl = 16;
            if (kk < lim) {
              const uint4 a = ld16u(in + i + kk, in_end);
              const uint4 b = ld16u(in + c + kk, in_end);
              cl = common16(a, b);
              if (cl > lim - kk) cl = lim - kk;
            }
            const uint64_t stop = ballot(kk >= lim || cl < 16);
            if (stop) {
              const uint32_t sl = (uint32_t)__builtin_ctzll(stop);
              const uint32_t ks = k + 16u * sl;
              k = ks >= lim ? lim : ks + readlane(cl, sl);
              break;
            }
            k += 16u * kWave;
          }
          mlen = k;
        }
        em.sequence(in, I, anchor, i - anchor, i - c, mlen);
        pos = i + mlen;
        anchor = pos;
      }
    }
  }
  em.sequence(in, I, anchor, n - anchor, 0, 0);
}

}  // namespace cmp

__global__ __launch_bounds__(64) void lz4_compress_kernel(
    const uint8_t* __restrict__ input, uint64_t n_total, uint32_t seg,
    uint8_t* __restrict__ slab, uint64_t slot_stride, uint8_t* const* __restrict__ dsts,
    uint32_t* __restrict__ sizes, uint32_t* __restrict__ err) {
  using namespace cmp;
  __shared__ __attribute__((aligned(16))) uint16_t table[1u << kHashLog];
  __shared__ __attribute__((aligned(16))) uint8_t inring[kIn];
  __shared__ __attribute__((aligned(16))) uint8_t obuf[kObuf];
  const uint32_t i_seg = blockIdx.x;
  const uint64_t seg_off = (uint64_t)i_seg * seg;
  if (seg_off >= n_total) return;
  const uint32_t n = (uint32_t)((n_total - seg_off) < seg ? (n_total - seg_off) : seg);
  Lz4Out o;
  o.ring = obuf;
  o.dst = dsts ? dsts[i_seg] : slab + (uint64_t)i_seg * slot_stride;
  o.cap = slot_stride;
  o.op = 0;
  o.flushed = 0;
  o.overflow = false;
  parse(input + seg_off, n, input + n_total, table, inring, kMaxDist, 0xFFFFFFFFu, o);
  const uint32_t size = o.finish();
  if (lane_id() == 0) {
    sizes[i_seg] = o.overflow ? 0xFFFFFFFFu : size;
    if (o.overflow) atomicOr(err, 2u);
  }
}

__global__ __launch_bounds__(64) void deflate_compress_kernel(
    const uint8_t* __restrict__ input, uint64_t n_total, uint32_t seg,
    uint8_t* __restrict__ slab, uint64_t slot_stride, uint8_t* const* __restrict__ dsts,
    uint32_t* __restrict__ sizes, uint32_t* __restrict__ err) {
  using namespace cmp;
  __shared__ __attribute__((aligned(16))) uint16_t table[1u << kHashLog];
  __shared__ __attribute__((aligned(16))) uint8_t inring[kIn];
  __shared__ __attribute__((aligned(16))) uint32_t stage[kBitWords];
  const uint32_t i_seg = blockIdx.x;
  const uint64_t seg_off = (uint64_t)i_seg * seg;
  if (seg_off >= n_total) return;
  const uint32_t n = (uint32_t)((n_total - seg_off) < seg ? (n_total - seg_off) : seg);
  for (uint32_t k = lane_id(); k < kBitWords; k += kWave) stage[k] = 0;
  DflOut o;
  o.stage = stage;
  o.dst = reinterpret_cast<uint32_t*>(dsts ? dsts[i_seg] : slab + (uint64_t)i_seg * slot_stride);
  o.cap = slot_stride;
  o.bits = 0;
  o.wflushed = 0;
  o.overflow = false;
  o.put_one(1u | (1u << 1), 3);  // BFINAL = 1, BTYPE = 01 (fixed Huffman)
  parse(input + seg_off, n, input + n_total, table, inring, kMaxDist, 258u, o);
  const uint32_t size = o.finish();
  if (lane_id() == 0) {
    sizes[i_seg] = o.overflow ? 0xFFFFFFFFu : size;
    if (o.overflow) atomicOr(err, 2u);
  }
}

}  // namespace bitar_hip
