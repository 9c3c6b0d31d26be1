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
//   1. the 4 bytes at every position (coalesced dword loads; the previous window's
//      registers are kept, so literal bytes come from registers via ds_bpermute);
//   2. look up a 4096-entry LDS table of (position << 16 | upper 16 bits of the 4 bytes),
//      then insert every position with ds_max_u32 (largest position wins: deterministic);
//   3. lanes whose 16-bit check matches verify + measure the match on 16 bytes;
//   4. a scalar greedy loop picks matches in lane order (ballot + ctz), extends long ones
//      cooperatively 1 KiB per step, and hands each sequence to the codec's emitter.
// Emitters stage output in LDS and flush it with wide stores:
//   LZ4: a byte ring flushed in 16-B blocks; long literal runs go HBM -> HBM.
//   DEFLATE: a bit ring; each lane's code is placed by a wave prefix sum of code lengths
//            and OR-ed into LDS (ds_or_b32), whole dwords flushed to HBM.
#include "wave.hip.h"

namespace bitar_hip {

namespace cmp {

constexpr uint32_t kHashLog = 12;
constexpr uint32_t kMinMatch = 4;
constexpr uint32_t kLastLiterals = 5;
constexpr uint32_t kMfLimit = 12;

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

// The input bytes the parse has in registers: lane l of `cur` holds the 4 bytes at x+l,
// lane l of `prev` those at x-64+l.  A literal run inside [x-64, x+64) is read from here.
struct Regs {
  uint32_t prev, cur, x;
  // byte at segment position q, x-64 <= q < x+64 (per lane)
  __device__ __forceinline__ uint32_t byte_at(uint32_t q) const {
    const uint32_t rel = q + 64 - x;  // 0..127
    const uint32_t a = bpermute(prev, rel & 63), b = bpermute(cur, rel & 63);
    return (rel >= 64 ? b : a) & 0xFFu;
  }
};

// ---- LZ4 emitter: output staged in an LDS byte ring, flushed in aligned 16-B blocks ----
constexpr uint32_t kObuf = 4096, kObufMask = kObuf - 1, kObufFlush = kObuf / 2;

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
  __device__ __forceinline__ void sequence(const uint8_t* in, const Regs& R, uint32_t lit_start,
                                           uint32_t lit_len, uint32_t off, uint32_t mlen) {
    if (overflow) return;
    const uint32_t ml = mlen ? mlen - kMinMatch : 0;
    const uint32_t token = ((lit_len < 15 ? lit_len : 15) << 4) | (ml < 15 ? ml : 15);
    if (!room(1)) return;
    put(token, 1);
    if (lit_len >= 15) put_ext(lit_len - 15);
    if (overflow) return;
    if (lit_len) {
      if ((uint64_t)op + lit_len > cap) { overflow = true; return; }
      if (lit_len <= kWave && lit_start + 64 >= R.x) {  // from registers
        room(lit_len);
        put(R.byte_at(lit_start + (lane_id() < lit_len ? lane_id() : 0)), lit_len);
      } else {  // long run: drain the ring, then HBM -> HBM
        flush(op, true);
        wave_copy_global(dst + op, in + lit_start, lit_len);
        op += lit_len;
        flushed = op;
      }
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
constexpr uint32_t kBitWords = 1024, kBitMask = kBitWords - 1, kBitFlushWords = kBitWords / 2;

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
  __device__ __forceinline__ void literals(const uint8_t* in, const Regs& R, uint32_t s,
                                           uint32_t n) {
    const uint32_t lane = lane_id();
    for (uint32_t k = 0; k < n && !overflow; k += kWave) {
      const uint32_t step = n - k < kWave ? n - k : kWave;
      const uint32_t q = s + k + (lane < step ? lane : 0);
      uint32_t b;
      if (n <= kWave && s + 64 >= R.x) b = R.byte_at(q);
      else b = lane < step ? (uint32_t)in[q] : 0u;
      uint32_t nb;
      const uint32_t code = fixed_code(b, nb);
      put_lanes(lane < step ? code : 0u, lane < step ? nb : 0u);
    }
  }
  __device__ __forceinline__ void sequence(const uint8_t* in, const Regs& R, uint32_t lit_start,
                                           uint32_t lit_len, uint32_t off, uint32_t mlen) {
    if (overflow) return;
    if (lit_len) literals(in, R, lit_start, lit_len);
    if (!mlen || overflow) return;
    uint32_t ls = 28;
    while (kLenBase[ls] > mlen) --ls;
    uint32_t ln;
    const uint32_t lcode = fixed_code(257 + ls, ln);
    uint32_t ds = 29;
    while (kDistBase[ds] > off) --ds;
    const uint32_t le = kLenExtra[ls], de = kDistExtra[ds];
    const uint32_t v = lcode | ((mlen - kLenBase[ls]) << ln) | (rev(ds, 5) << (ln + le)) |
                       ((off - kDistBase[ds]) << (ln + le + 5));
    put_one(v, ln + le + 5 + de);
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
template <class E>
__device__ __forceinline__ void parse(const uint8_t* in, uint32_t n, const uint8_t* in_end,
                                      uint32_t* table, uint32_t max_dist, uint32_t max_mlen, E& em) {
  const uint32_t lane = lane_id();
  uint32_t anchor = 0;
  Regs R;
  R.prev = 0;
  R.cur = 0;
  R.x = 0;
  if (n >= kMfLimit + 1) {
    // An empty slot means "candidate position 0" (the oracle's zeroed table): it holds
    // position 0 with position 0's own check bits.
    const uint32_t empty = ld32u(in, in_end) >> 16;
    for (uint32_t k = lane; k < (1u << kHashLog); k += kWave) table[k] = empty;
    lds_order();
    const uint32_t last_start = n - kMfLimit;
    const uint32_t match_limit = n - kLastLiterals;
    uint32_t pos = 0;
    for (uint32_t x = 0; x <= last_start; x += kWave) {
      const uint32_t p = x + lane;
      R.prev = R.cur;
      R.cur = p < n ? ld32u(in + p, in_end) : 0u;
      R.x = x;
      const bool act = p <= last_start;
      const uint32_t v = R.cur;
      const uint32_t h = hash4(v);
      lds_order();
      const uint32_t e = act ? table[h] : 0u;
      lds_order();
      if (act) atomicMax(&table[h], (p << 16) | (v >> 16));
      const uint32_t cand = e >> 16;
      const bool pre = act && cand < p && p - cand <= max_dist && (e & 0xFFFFu) == (v >> 16);
      uint32_t len = 0;
      if (pre) {  // verify the 4 bytes and measure up to 16 (gathered loads)
        const uint4 a = ld16u(in + p, in_end);
        const uint4 b = ld16u(in + cand, in_end);
        len = common16(a, b);
        uint32_t lim = match_limit - p;
        if (lim > max_mlen) lim = max_mlen;
        if (len > lim) len = lim;
      }
      const uint64_t valid = ballot(pre && len >= kMinMatch);
      while (valid) {
        const uint32_t start = pos > x ? pos - x : 0u;
        if (start >= kWave) break;
        const uint64_t m = valid & (~0ull << start);
        if (!m) break;
        const uint32_t l = (uint32_t)__builtin_ctzll(m);
        const uint32_t i = x + l;
        const uint32_t c = readlane(cand, l);
        uint32_t mlen = readlane(len, l);
        uint32_t lim = match_limit - i;
        if (lim > max_mlen) lim = max_mlen;
        if (mlen == 16 && lim > 16) {  // cooperative extension, 16 B per lane per step
          uint32_t k = 16;
          for (;;) {
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
              const uint32_t kk_s = k + 16u * sl;
              const uint32_t cl_s = readlane(cl, sl);
              mlen = kk_s >= lim ? lim : kk_s + cl_s;
              break;
            }
            k += 16u * kWave;
          }
        }
        em.sequence(in, R, anchor, i - anchor, i - c, mlen);
        pos = i + mlen;
        anchor = pos;
      }
    }
    R.x = ~0u;  // the final run is past the register window: read it from HBM
  } else {
    R.x = ~0u;
  }
  em.sequence(in, R, anchor, n - anchor, 0, 0);
}

}  // namespace cmp

__global__ __launch_bounds__(64) void lz4_compress_kernel(
    const uint8_t* __restrict__ input, uint64_t n_total, uint32_t seg,
    uint8_t* __restrict__ slab, uint64_t slot_stride, uint8_t* const* __restrict__ dsts,
    uint32_t* __restrict__ sizes, uint32_t* __restrict__ err) {
  using namespace cmp;
  __shared__ __attribute__((aligned(16))) uint32_t table[1u << kHashLog];
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
  parse(input + seg_off, n, input + n_total, table, 65535u, 0xFFFFFFFFu, o);
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
  __shared__ __attribute__((aligned(16))) uint32_t table[1u << kHashLog];
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
  parse(input + seg_off, n, input + n_total, table, 32768u, 258u, o);
  const uint32_t size = o.finish();
  if (lane_id() == 0) {
    sizes[i_seg] = o.overflow ? 0xFFFFFFFFu : size;
    if (o.overflow) atomicOr(err, 2u);
  }
}

}  // namespace bitar_hip
