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
// Input staging.  The segment streams through an 8 KiB LDS input ring in 1 KiB rows (one
// aligned 16-B block per lane): each row is loaded into registers a whole row of windows
// before it is written into the ring, and the ring runs 576..1536 B ahead of the scan.
// Every byte a position, a candidate (matches are capped at 6656 B back) or a literal needs
// is then an LDS read.  One register block in a fixed register: a rotation between
// blocks would make the compiler wait for every load in flight.
//
// Per fixed window of 64 positions (one per lane):
//   1. hash the 4 bytes at every position (from the ring), look up a 2048-entry LDS table of
//      u16 positions, then insert every position (the largest position wins a slot);
//   2. lanes with a candidate verify + measure the match on 8 bytes from the ring, and
//      lanes still matching extend in parallel up to 32 bytes;
//   3. a scalar chain walk picks the greedy matches in lane order (one ctz per match,
//      cooperative extension only for matches reaching 32 bytes);
//   4. the codec's emitter writes the whole window's output lane-parallel:
//      LZ4: every selected match lane writes its token / length bytes / offset, every
//           literal lane writes its own byte, placed by a wave prefix sum of sequence sizes;
//           rare long runs fall back to a per-sequence path (long literal runs go HBM->HBM);
//      DEFLATE: every position lane contributes its literal code or its match symbol; codes
//           are placed by a prefix sum of bit lengths and OR-ed into an LDS bit ring.
// Output is staged in LDS and flushed with aligned 16-B stores once per input row, right
// before the next row's load is issued.
#include "wave.hip.h"

namespace bitar_hip {

namespace cmp {

// Build-time knobs for tuning experiments (scripts/build_variant.sh); the defaults are the
// shipped configuration and the one the oracle restates.
#ifndef BITAR_CMP_HASH_LOG
#define BITAR_CMP_HASH_LOG 11
#endif
#ifndef BITAR_CMP_OBUF
#define BITAR_CMP_OBUF 1024
#endif
#ifndef BITAR_CMP_BITWORDS
#define BITAR_CMP_BITWORDS 256
#endif
constexpr uint32_t kHashLog = BITAR_CMP_HASH_LOG;
constexpr uint32_t kMinMatch = 4;
constexpr uint32_t kLastLiterals = 5;
constexpr uint32_t kMfLimit = 12;
// Match distance cap (both codecs): at window x the input ring holds positions
// [F - 8192, F) with F <= x + 1536, so every candidate (>= x - 6656) is in LDS; it is also
// inside the LZ4 decoder's 8 KiB history ring (reach 8048), so our streams decode from LDS.
constexpr uint32_t kMaxDist = 6656;
constexpr uint32_t kIn = 8192, kInMask = kIn - 1;  // LDS input ring
constexpr uint32_t kInPad = 64;  // mirror of ring[0, 64) after its end: probes never wrap
constexpr uint32_t kRow = 1024;                   // prefetch row: one 16-B block per lane
constexpr uint32_t kPreExt = 32;                  // parallel per-lane match extension limit

__device__ __forceinline__ uint32_t hash4(uint32_t v) { return (v * 2654435761u) >> (32 - kHashLog); }

// 16 bytes at p (any alignment); aligned blocks at or past `end` are not loaded (zeros)
__device__ __forceinline__ uint4 ld16u(const GMEM uint8_t* p, const GMEM uint8_t* end) {
  const uintptr_t a = (uintptr_t)p & ~(uintptr_t)15;
  const uint32_t sh = (uint32_t)((uintptr_t)p & 15);
  const GMEM uint4* xa = reinterpret_cast<const GMEM uint4*>(p - sh);
  const uint4 x = xa[0];
  uint4 y = make_uint4(0, 0, 0, 0);
  if (sh && a + 16 < (uintptr_t)end) y = xa[1];
  const uint32_t w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
  const uint32_t q = sh >> 2, r = sh & 3u;
  const uint32_t s0 = q == 0 ? w[0] : q == 1 ? w[1] : q == 2 ? w[2] : w[3];
  const uint32_t s1 = q == 0 ? w[1] : q == 1 ? w[2] : q == 2 ? w[3] : w[4];
  const uint32_t s2 = q == 0 ? w[2] : q == 1 ? w[3] : q == 2 ? w[4] : w[5];
  const uint32_t s3 = q == 0 ? w[3] : q == 1 ? w[4] : q == 2 ? w[5] : w[6];
  const uint32_t s4 = q == 0 ? w[4] : q == 1 ? w[5] : q == 2 ? w[6] : w[7];
  return make_uint4(funnel(s0, s1, r), funnel(s1, s2, r), funnel(s2, s3, r), funnel(s3, s4, r));
}

// number of equal leading bytes of two 16-byte little-endian values (branch-free: all four
// dwords are compared, so the compiler cannot defer the loads behind data-dependent branches)
__device__ __forceinline__ uint32_t common16(uint4 a, uint4 b) {
  const uint32_t d0 = a.x ^ b.x, d1 = a.y ^ b.y, d2 = a.z ^ b.z, d3 = a.w ^ b.w;
  uint32_t r = 128;
  r = d3 ? 96 + __builtin_ctz(d3) : r;
  r = d2 ? 64 + __builtin_ctz(d2) : r;
  r = d1 ? 32 + __builtin_ctz(d1) : r;
  r = d0 ? __builtin_ctz(d0) : r;
  return r >> 3;
}

// number of equal leading bytes of two little-endian values
__device__ __forceinline__ uint32_t common8(uint64_t a, uint64_t b) {
  const uint64_t d = a ^ b;
  return d ? (uint32_t)(__builtin_ctzll(d) >> 3) : 8u;
}
__device__ __forceinline__ uint32_t common4(uint32_t a, uint32_t b) {
  const uint32_t d = a ^ b;
  return d ? (uint32_t)(__builtin_ctz(d) >> 3) : 4u;
}

__device__ __forceinline__ uint32_t bpermute(uint32_t v, uint32_t src_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}

// inclusive prefix sum over the wave's 64 lanes (DPP row shifts + row broadcasts)
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
  int x = (int)v;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return (uint32_t)x;
}

// inclusive prefix max (unsigned) over the wave's 64 lanes
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
  uint32_t x = v;
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
  return x;
}
// lane l gets lane l-1's value, lane 0 gets 0 (DPP wave_shr:1)
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}

// lowest set bit of a 64-bit mask (64 if none); highest set bit (mask nonzero)
__device__ __forceinline__ uint32_t lowbit(uint64_t m) { return m ? (uint32_t)__builtin_ctzll(m) : 64u; }
__device__ __forceinline__ uint32_t highbit(uint64_t m) { return 63u - (uint32_t)__builtin_clzll(m); }

// The LDS input ring: byte of segment position q lives at ring[(in_lo + q) & kInMask]
// (absolute-address indexing keeps aligned blocks aligned).
struct InRing {
  uint8_t* ring;
  uint32_t in_lo;  // low 32 bits of the segment's input address
  uint32_t lo;     // positions >= lo are in the ring (< the filled end)

  __device__ __forceinline__ uint32_t byte(uint32_t q) const {
    return ring[(in_lo + q) & kInMask];
  }
  // 4 / 16 bytes at position q (little-endian); the pad lets the dword reads run past the
  // ring's end without wrapping
  __device__ __forceinline__ uint32_t dword(uint32_t q) const {
    const uint32_t a = (in_lo + q) & kInMask;
    const uint32_t* r32 = reinterpret_cast<const uint32_t*>(ring) + (a >> 2);
    return funnel(r32[0], r32[1], a & 3u);
  }
  __device__ __forceinline__ uint4 bytes16(uint32_t q) const {
    const uint32_t a = (in_lo + q) & kInMask;
    const uint32_t* r32 = reinterpret_cast<const uint32_t*>(ring) + (a >> 2);
    const uint32_t sh = a & 3u;
    const uint32_t w0 = r32[0], w1 = r32[1], w2 = r32[2], w3 = r32[3], w4 = r32[4];
    return make_uint4(funnel(w0, w1, sh), funnel(w1, w2, sh), funnel(w2, w3, sh),
                      funnel(w3, w4, sh));
  }
};

// One parsed window, as handed to the emitter.  Per-lane fields are meaningful on the
// lanes the masks name.
struct Window {
  uint32_t x;       // window start
  uint64_t chain;   // lanes where a selected match starts
  uint32_t mlen;    // per lane: match length (chain lanes)
  uint32_t off;     // per lane: match distance (chain lanes)
  uint32_t byte;    // per lane: input byte at x + lane
  uint32_t pos_in;  // parse position at window start: [x, pos_in) is covered by a match
};

// ---- LZ4 emitter: output staged in an LDS byte ring, flushed in aligned 16-B blocks ----
constexpr uint32_t kObuf = BITAR_CMP_OBUF, kObufMask = kObuf - 1;

struct Lz4Out {
  uint8_t* ring;      // LDS, kObuf bytes + one trash byte per lane
  GMEM uint8_t* dst;  // slot
  uint64_t cap;
  uint32_t op, flushed;
  bool overflow;

  __device__ __forceinline__ uint32_t at(uint32_t k) const {
    return ((uint32_t)(uintptr_t)dst + k) & kObufMask;
  }
  __device__ __forceinline__ void flush(uint32_t upto, bool final) {
    const uint32_t lane = lane_id();
    const uintptr_t base = (uintptr_t)dst;
    uint32_t f = flushed;
    lds_order();
    uint32_t head = (uint32_t)((16u - ((base + f) & 15u)) & 15u);
    if (head > upto - f) head = upto - f;
    if (head) {
      if (lane < head) dst[f + lane] = ring[at(f + lane)];
      f += head;
    }
    const uint32_t nb = (upto - f) >> 4;
    for (uint32_t b = lane; b < nb; b += kWave) {
      const uint32_t k = f + 16u * b;
      *reinterpret_cast<GMEM uint4*>(dst + k) = *reinterpret_cast<const uint4*>(ring + at(k));
    }
    f += nb << 4;
    if (final && f < upto) {
      if (lane < upto - f) dst[f + lane] = ring[at(f + lane)];
      f = upto;
    }
    flushed = f;
  }
  // once per input row, before the next row's load is issued
  __device__ __forceinline__ void drain() {
    if (op - flushed >= 16) flush(op, false);
  }
  __device__ __forceinline__ bool room(uint32_t n) {
    if ((uint64_t)op + n > cap) { overflow = true; return false; }
    if (op + n - flushed > kObuf - 64) flush(op, false);
    return true;
  }
  // lanes < n write byte `v` at op + lane
  __device__ __forceinline__ void put(uint32_t v, uint32_t n) {
    lds_order();
    if (lane_id() < n) ring[at(op + lane_id())] = (uint8_t)v;
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
  // One sequence, general path: any literal run (long runs HBM -> HBM), any lengths.
  __device__ __forceinline__ void sequence(const GMEM uint8_t* in, const InRing& I,
                                           uint32_t lit_start, uint32_t lit_len, uint32_t off,
                                           uint32_t mlen) {
    if (overflow) return;
    const uint32_t ml = mlen ? mlen - kMinMatch : 0;
    const uint32_t token = ((lit_len < 15 ? lit_len : 15) << 4) | (ml < 15 ? ml : 15);
    if (!room(1)) return;
    put(token, 1);
    if (lit_len >= 15) put_ext(lit_len - 15);
    if (overflow) return;
    if (lit_len) {
      if ((uint64_t)op + lit_len > cap) { overflow = true; return; }
      if (lit_len <= 256 && lit_start >= I.lo) {
        for (uint32_t k = 0; k < lit_len; k += kWave) {
          const uint32_t step = lit_len - k < kWave ? lit_len - k : kWave;
          room(step);
          lds_order();
          const uint32_t b = I.byte(lit_start + k + (lane_id() < step ? lane_id() : 0u));
          put(b, step);
        }
      } else {
        // long run (or not in the input ring): drain the ring, then HBM -> HBM
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
  // the tail sequence starts at the last match's end
  __device__ __forceinline__ uint32_t pending_from(uint32_t anchor, uint32_t) const { return anchor; }

  // All sequences of one window.  Fast path (every literal run < 270 bytes and in the
  // input ring, every match < 274 bytes: at most one length byte each): each match lane
  // writes its header bytes and each literal lane its own byte, all lanes at once, at
  // offsets from a prefix sum of the sequence sizes.
  __device__ __forceinline__ void window(const GMEM uint8_t* in, const InRing& I, const Window& W,
                                         uint32_t anchor, uint32_t) {
    if (!W.chain || overflow) return;
    const uint32_t lane = lane_id();
    const uint32_t q = W.x + lane;
    const bool cl = (W.chain >> lane) & 1;
    // match ends increase along the chain, so "end of the previous match" is a prefix max
    const uint32_t end_incl = wave_incl_max(cl ? q + W.mlen : 0u);
    const uint32_t end_excl = wave_shr1(end_incl);
    const uint32_t lit_start = max(anchor, cl ? end_excl : end_incl);
    const uint32_t lit_len = q - lit_start;  // chain lanes: their literal run
    const uint32_t ml = W.mlen - kMinMatch;
    const bool bad = cl && (lit_len >= 270 || ml >= 270);
    const uint32_t nlx = lit_len >= 15 ? 1u : 0u, nmx = ml >= 15 ? 1u : 0u;
    const uint32_t e = cl ? 1 + nlx + lit_len + 2 + nmx : 0u;
    const uint32_t incl = wave_incl_sum(e);
    const uint32_t total = readlane(incl, 63);
    if (ballot(bad) || anchor < I.lo || (uint64_t)op + total > cap) {
      // general path, one sequence at a time
      uint64_t m = W.chain;
      uint32_t a = anchor;
      while (m) {
        const uint32_t l = (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        const uint32_t i = W.x + l, mlen = readlane(W.mlen, l);
        sequence(in, I, a, i - a, readlane(W.off, l), mlen);
        a = i + mlen;
      }
      return;
    }
    room(total);
    // A literal lane (not a match start, not inside a match) belongs to the sequence of the
    // lowest chain lane s above it: that sequence starts at op + incl (no chain lane lies
    // between), its literal run at lit_start (= this lane's prefix max), and its token is
    // followed by one length byte if the run is >= 15 bytes.
    const uint64_t above = lane == 63 ? 0ull : W.chain & (~0ull << (lane + 1));
    const uint32_t s = lowbit(above);
    const bool lit = !cl && above && q >= lit_start;
    const uint32_t lit_nlx = W.x + s - lit_start >= 15 ? 1u : 0u;
    const uint32_t o = op + incl - e;  // chain lanes: sequence start
    // every lane stores every byte kind; lanes without one store into their trash byte
    // past the ring (no exec-mask branches)
    const uint32_t tr = kObuf + lane;
    const uint32_t h = o + 1 + nlx + lit_len;
    lds_order();
    ring[cl ? at(o) : tr] = (uint8_t)(((lit_len < 15 ? lit_len : 15) << 4) | (ml < 15 ? ml : 15));
    ring[cl && nlx ? at(o + 1) : tr] = (uint8_t)(lit_len - 15);
    ring[cl ? at(h) : tr] = (uint8_t)W.off;
    ring[cl ? at(h + 1) : tr] = (uint8_t)(W.off >> 8);
    ring[cl && nmx ? at(h + 2) : tr] = (uint8_t)(ml - 15);
    ring[lit ? at(op + incl + 1 + lit_nlx + (q - lit_start)) : tr] = (uint8_t)W.byte;
    // literals of the first sequence that precede the window (anchor < x): from the ring
    if (anchor < W.x) {
      const uint32_t l0 = lowbit(W.chain);
      const uint32_t d0 = op + 1 + (W.x + l0 - anchor >= 15 ? 1u : 0u) - anchor;
      for (uint32_t k = anchor; k < W.x; k += kWave) {
        const uint32_t qq = k + lane;
        if (qq < W.x) ring[at(d0 + qq)] = (uint8_t)I.byte(qq);
      }
    }
    lds_order();
    op += total;
  }
};

// ---- fixed-Huffman DEFLATE emitter: LDS bit ring, lane codes placed by prefix sum -----
constexpr uint32_t kBitWords = BITAR_CMP_BITWORDS, kBitMask = kBitWords - 1;

__device__ __forceinline__ uint32_t rev(uint32_t v, uint32_t n) {
  return __builtin_bitreverse32(v) >> (32 - n);
}
// fixed literal/length code of symbol s, bit-reversed for LSB-first packing; *n = length
__device__ __forceinline__ uint32_t fixed_code(uint32_t s, uint32_t& n) {
  // 0-143: 8 bits 0x30+s; 144-255: 9 bits 0x190+s-144; 256-279: 7 bits s-256;
  // 280-287: 8 bits 0xC0+s-280 (RFC 1951 3.2.6), as selects
  const uint32_t code = s < 144 ? 0x30 + s : s < 256 ? 0x190 + (s - 144) : s < 280 ? s - 256 : 0xC0 + (s - 280);
  n = s < 144 ? 8u : s < 256 ? 9u : s < 280 ? 7u : 8u;
  return __builtin_bitreverse32(code) >> (32 - n);
}
// The whole match symbol -- length code, its extra bits, distance code, its extra bits --
// LSB first (RFC 1951 3.2.5); mlen in [3, 258], off in [1, 32768]; *n <= 31.
__device__ __forceinline__ uint32_t match_code(uint32_t mlen, uint32_t off, uint32_t& n) {
  const uint32_t v = mlen - 3;
  // length code (symbol - 257) and extra bit count; distance code and extra bit count
  const uint32_t lev = 29u - __builtin_clz(v | 8u);  // floor(log2 v) - 2 for v >= 8
  const uint32_t le = mlen == 258 || v < 8 ? 0u : lev;
  const uint32_t lc = mlen == 258 ? 28u : v < 8 ? v : 4 * lev + 4 + ((v >> lev) & 3u);
  const uint32_t lx = v & ((1u << le) - 1);
  const uint32_t d = off - 1;
  const uint32_t dev = 30u - __builtin_clz(d | 4u);  // floor(log2 d) - 1 for d >= 4
  const uint32_t de = d < 4 ? 0u : dev;
  const uint32_t dc = d < 4 ? d : 2 * dev + 2 + ((d >> dev) & 1u);
  const uint32_t dx = d & ((1u << de) - 1);
  uint32_t ln;
  const uint32_t code = fixed_code(257 + lc, ln);
  n = ln + le + 5 + de;
  return code | (lx << ln) | (rev(dc, 5) << (ln + le)) | (dx << (ln + le + 5));
}

struct DflOut {
  uint32_t* stage;     // LDS, kBitWords dwords, zero outside the pending range
  GMEM uint32_t* dst;  // slot (16-B aligned)
  uint64_t cap;        // bytes
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
  // once per input row, before the next row's load is issued: complete words only
  __device__ __forceinline__ void drain() {
    const uint32_t full = (uint32_t)(bits >> 5);
    if (full != wflushed) flush_words(full);
  }
  // append each lane's (val, nb) in lane order (nb <= 32; nb = 0 appends nothing)
  __device__ __forceinline__ void put_lanes(uint32_t val, uint32_t nb) {
    if (overflow) return;
    const uint32_t incl = wave_incl_sum(nb);
    const uint32_t total = readlane(incl, 63);
    if ((bits + total + 7) / 8 > cap) { overflow = true; return; }
    const uint64_t bp = bits + incl - nb;
    const uint32_t w = (uint32_t)(bp >> 5), sh = (uint32_t)(bp & 31);
    // every lane ORs into both words (zeros where it has nothing): no exec-mask branches
    const uint32_t spill = sh + nb > 32 ? val >> ((32 - sh) & 31) : 0u;
    lds_order();
    atomicOr(&stage[w & kBitMask], val << sh);
    atomicOr(&stage[(w + 1) & kBitMask], spill);
    lds_order();
    bits += total;
    const uint32_t full = (uint32_t)(bits >> 5);
    if (full - wflushed >= kBitWords - 80) flush_words(full);  // a window adds <= 63 words
  }
  __device__ __forceinline__ void put_one(uint32_t val, uint32_t nb) {
    put_lanes(lane_id() == 0 ? val : 0u, lane_id() == 0 ? nb : 0u);
  }
  // literal codes of [s, s+n) (from the input ring when it holds them, else from HBM)
  __device__ __forceinline__ void sequence(const GMEM uint8_t* in, const InRing& I, uint32_t s,
                                           uint32_t n, uint32_t, uint32_t) {
    const uint32_t lane = lane_id();
    const bool ring_ok = s >= I.lo;
    for (uint32_t k = 0; k < n; k += kWave) {
      const uint32_t step = n - k < kWave ? n - k : kWave;
      const uint32_t q = s + k + (lane < step ? lane : 0);
      uint32_t b;
      lds_order();
      if (ring_ok) b = I.byte(q);
      else b = lane < step ? (uint32_t)in[q] : 0u;
      uint32_t nb;
      const uint32_t code = fixed_code(b, nb);
      put_lanes(lane < step ? code : 0u, lane < step ? nb : 0u);
      if (overflow) return;
    }
  }
  // literals are emitted window by window: the tail starts where output stopped
  __device__ __forceinline__ uint32_t pending_from(uint32_t, uint32_t emitted) const { return emitted; }

  // One window: each position contributes its literal code, its match symbol (a selected
  // match starts there) or nothing (inside a match); one prefix sum places them all.
  __device__ __forceinline__ void window(const GMEM uint8_t*, const InRing&, const Window& W,
                                         uint32_t, uint32_t n) {
    const uint32_t lane = lane_id();
    const uint32_t q = W.x + lane;
    const bool cl = (W.chain >> lane) & 1;
    const uint32_t pend = wave_incl_max(cl ? q + W.mlen : 0u);  // end of the last match <= q
    const bool covered = q < W.pos_in || (!cl && q < pend);
    uint32_t mb, lb;
    const uint32_t mv = match_code(cl ? W.mlen : 3u, cl ? W.off : 1u, mb);
    const uint32_t lv = fixed_code(W.byte, lb);
    const bool lit = !cl && !covered && q < n;
    put_lanes(cl ? mv : lit ? lv : 0u, cl ? mb : lit ? lb : 0u);
  }
};

// The window-scan parse over one segment; hands each window to E::window and the tail to
// E::sequence.
template <class E>
__device__ __forceinline__ void parse(const GMEM uint8_t* in, uint32_t n, const GMEM uint8_t* in_end,
                                      uint16_t* table, uint8_t* inring, uint32_t max_dist,
                                      uint32_t max_mlen, E& em) {
  const uint32_t lane = lane_id();
  uint32_t anchor = 0, emitted = 0;
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
    // Rows cover the 16-B aligned span starting at in - s0: row r, lane l = the block of
    // segment positions [kRow r + 16 l - s0, +16).  Blocks past the segment are not loaded;
    // a block holding a byte before in_end never crosses a page.
    const uint32_t s0 = I.in_lo & 15u;
    const GMEM uint4* in16 = reinterpret_cast<const GMEM uint4*>(in - s0);
    const uint64_t span = (uint64_t)(in_end - (in - s0));
    uint4* ring16 = reinterpret_cast<uint4*>(inring);
    const uint32_t rbase = (I.in_lo - s0) >> 4;  // ring block of in16[0]
    auto load_row = [&](uint32_t r) __attribute__((always_inline)) -> uint4 {
      const uint32_t o = kRow * r + 16u * lane;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (o < n + s0 && o < span) v = in16[o >> 4];
      return v;
    };
    auto write_row = [&](uint32_t r, const uint4& v) __attribute__((always_inline)) {
      const uint32_t blk = (rbase + (kRow / 16) * r + lane) & (kInMask >> 4);
      ring16[blk] = v;
      if (blk < kInPad / 16) ring16[kIn / 16 + blk] = v;  // the pad mirrors the ring's head
    };
    uint32_t pos = 0;
    uint32_t F = 0;  // the ring holds positions [F - kIn, F)
    // one window of 64 positions at x; vp = the 16 bytes at x + lane, read during the
    // previous window (the ring already holds them then)
    uint4 vp = make_uint4(0, 0, 0, 0);
    auto window = [&](uint32_t x) __attribute__((always_inline)) {
      const uint32_t p = x + lane;
      const bool act = p <= last_start;
      const uint4 v = vp;
      const uint32_t h = hash4(v.x);
      // Table and ring accesses are issued on all lanes (no exec-mask branches: the scalar
      // unit is the bottleneck).  Lanes past last_start exist only in the final window;
      // their table writes are never looked up again.
      const uint32_t cand = table[h];
      lds_order();
      table[h] = (uint16_t)p;
      lds_order();
      // read back now, settle same-slot writes at the end of the window
      const uint32_t back = table[h];
      vp = I.bytes16(p + kWave);  // next window's bytes
      const bool pre = act && cand < p && p - cand <= max_dist;
      uint32_t lim = match_limit - p;
      if (lim > max_mlen) lim = max_mlen;
      // verify the 4 bytes and measure up to 16, from the input ring
      const uint32_t c16 = common16(v, I.bytes16(cand));
      uint32_t len = pre ? (c16 < lim ? c16 : lim) : 0u;
      // lanes still matching after 16 bytes extend in parallel, up to kPreExt
      for (uint32_t k = 16; k < kPreExt; k += 16) {
        const bool go = pre && len == k && lim > k;
        if (!ballot(go)) break;
        const uint32_t l2 = k + common16(I.bytes16(p + k), I.bytes16(cand + k));
        len = go ? (l2 < lim ? l2 : lim) : len;
      }
      // lanes at or past the parse position holding a match, and those of them whose match
      // reached kPreExt bytes and may go on (cooperative extension during the walk)
      const uint32_t pos_in = pos;
      const uint32_t start = pos > x ? pos - x : 0u;
      const bool okl = pre && len >= kMinMatch && lane >= start;
      const uint64_t valid = ballot(okl);
      const uint64_t extm = ballot(okl && len == kPreExt && lim > kPreExt);
      uint64_t chain = 0;
      uint32_t mlen_v = len;
      uint64_t m = valid;
      uint32_t e = 0;
      while (m) {  // the greedy chain: the next match is the first valid lane past the end
        const uint32_t l = (uint32_t)__builtin_ctzll(m);
        uint32_t mlen = readlane(len, l);
        if ((extm >> l) & 1) {
          const uint32_t i = x + l;
          uint32_t li = match_limit - i;
          if (li > max_mlen) li = max_mlen;
          const uint32_t c = readlane(cand, l);
          // cooperative extension, first from the input ring (4 B per lane per step) up to F
          const uint32_t lr = li < F - i ? li : F - i;
          uint32_t k = kPreExt;
          bool more = true;
          for (;;) {
            const uint32_t kk = k + 4u * lane;
            uint32_t cl = 4;
            if (kk < lr) {
              cl = common4(I.dword(i + kk), I.dword(c + kk));
              if (cl > lr - kk) cl = lr - kk;
            }
            const uint64_t stop = ballot(kk >= lr || cl < 4);
            if (stop) {
              const uint32_t sl = (uint32_t)__builtin_ctzll(stop);
              const uint32_t ks = k + 4u * sl;
              k = ks >= lr ? lr : ks + readlane(cl, sl);
              more = k == lr && lr < li;  // stopped by the ring's end, not by a mismatch
              break;
            }
            k += 4u * kWave;
          }
          // ... then from HBM, 16 B per lane per step
          while (more) {
            const uint32_t kk = k + 16u * lane;
            uint32_t cl = 16;
            if (kk < li) {
              const uint4 a = ld16u(in + i + kk, in_end);
              const uint4 b = ld16u(in + c + kk, in_end);
              cl = common16(a, b);
              if (cl > li - kk) cl = li - kk;
            }
            const uint64_t stop = ballot(kk >= li || cl < 16);
            if (stop) {
              const uint32_t sl = (uint32_t)__builtin_ctzll(stop);
              const uint32_t ks = k + 16u * sl;
              k = ks >= li ? li : ks + readlane(cl, sl);
              break;
            }
            k += 16u * kWave;
          }
          mlen = k;
          if (lane == l) mlen_v = mlen;
        }
        chain |= 1ull << l;
        e = l + mlen;
        m = e < kWave ? valid & (~0ull << e) : 0ull;
      }
      if (chain) pos = x + e;
      Window W;
      W.x = x;
      W.chain = chain;
      W.mlen = mlen_v;
      W.off = p - cand;
      W.byte = v.x & 0xFFu;
      W.pos_in = pos_in;
      em.window(in, I, W, anchor, n);
      if (chain) anchor = pos;
      emitted = pos > x + kWave ? pos : x + kWave;
      // same-slot writes of this window: re-write until the largest position holds the slot
      // (the empty asm pins the read-back's use, and so its wait, here)
      uint32_t bk = back;
      __asm__ volatile("" : "+v"(bk));
      bool redo = act && bk < p;
      while (ballot(redo)) {
        lds_order();
        if (redo) table[h] = (uint16_t)p;
        lds_order();
        redo = redo && table[h] < p;
      }
    };
    // Row k+1 goes into the ring at x = 1024 k + 512 (the ring then runs 576..1536 B ahead
    // of the scan); right after, the row register block is reloaded with row k+2, which
    // has a whole row of windows (1 KiB of scan) to land.  The output is drained just
    // before that load, so no store queues behind it.
    uint4 nxt = load_row(1);
    {
      const uint4 r0 = load_row(0);
      lds_order();
      write_row(0, r0);
    }
    F = kRow - s0;
    I.lo = 0;
    lds_order();
    vp = I.bytes16(lane);
    for (uint32_t x = 0; x <= last_start; x += kWave) {
      if ((x & (kRow - 1)) == kRow / 2) {
        const uint32_t k = x / kRow;
        lds_order();
        write_row(k + 1, nxt);
        F = kRow * (k + 2) - s0;
        I.lo = F > kIn ? F - kIn : 0u;
        em.drain();
        nxt = load_row(k + 2);
      }
      lds_order();
      window(x);
    }
  }
  const uint32_t t0 = em.pending_from(anchor, emitted);
  if (t0 < n) em.sequence(in, I, t0, n - t0, 0, 0);
}

}  // namespace cmp

__global__ __launch_bounds__(64) void lz4_compress_kernel(
    const uint8_t* __restrict__ input, uint64_t n_total, uint32_t seg,
    uint8_t* __restrict__ slab, uint64_t slot_stride, uint8_t* const* __restrict__ dsts,
    uint32_t* __restrict__ sizes, uint32_t* __restrict__ err) {
  using namespace cmp;
  __shared__ __attribute__((aligned(16))) uint16_t table[1u << kHashLog];
  __shared__ __attribute__((aligned(16))) uint8_t inring[kIn + kInPad];
  __shared__ __attribute__((aligned(16))) uint8_t obuf[kObuf + kWave];  // + trash bytes
  const uint32_t i_seg = blockIdx.x;
  const uint64_t seg_off = (uint64_t)i_seg * seg;
  if (seg_off >= n_total) return;
  const uint32_t n = (uint32_t)((n_total - seg_off) < seg ? (n_total - seg_off) : seg);
  Lz4Out o;
  o.ring = obuf;
  o.dst = global_ptr(dsts ? dsts[i_seg] : slab + (uint64_t)i_seg * slot_stride);
  o.cap = slot_stride;
  o.op = 0;
  o.flushed = 0;
  o.overflow = false;
  parse(global_ptr(input + seg_off), n, global_ptr(input + n_total), table, inring, kMaxDist,
        0xFFFFFFFFu, o);
  o.flush(o.op, true);
  if (lane_id() == 0) {
    sizes[i_seg] = o.overflow ? 0xFFFFFFFFu : o.op;
    if (o.overflow) atomicOr(err, 2u);
  }
}

__global__ __launch_bounds__(64) void deflate_compress_kernel(
    const uint8_t* __restrict__ input, uint64_t n_total, uint32_t seg,
    uint8_t* __restrict__ slab, uint64_t slot_stride, uint8_t* const* __restrict__ dsts,
    uint32_t* __restrict__ sizes, uint32_t* __restrict__ err) {
  using namespace cmp;
  __shared__ __attribute__((aligned(16))) uint16_t table[1u << kHashLog];
  __shared__ __attribute__((aligned(16))) uint8_t inring[kIn + kInPad];
  __shared__ __attribute__((aligned(16))) uint32_t stage[kBitWords];
  const uint32_t i_seg = blockIdx.x;
  const uint64_t seg_off = (uint64_t)i_seg * seg;
  if (seg_off >= n_total) return;
  const uint32_t n = (uint32_t)((n_total - seg_off) < seg ? (n_total - seg_off) : seg);
  for (uint32_t k = lane_id(); k < kBitWords; k += kWave) stage[k] = 0;
  DflOut o;
  o.stage = stage;
  o.dst = reinterpret_cast<GMEM uint32_t*>(
      global_ptr(dsts ? dsts[i_seg] : slab + (uint64_t)i_seg * slot_stride));
  o.cap = slot_stride;
  o.bits = 0;
  o.wflushed = 0;
  o.overflow = false;
  o.put_one(1u | (1u << 1), 3);  // BFINAL = 1, BTYPE = 01 (fixed Huffman)
  parse(global_ptr(input + seg_off), n, global_ptr(input + n_total), table, inring, kMaxDist,
        258u, o);
  uint32_t eb;
  const uint32_t eob = fixed_code(256, eb);
  o.put_one(eob, eb);
  o.flush_words((uint32_t)((o.bits + 31) >> 5));
  if (lane_id() == 0) {
    sizes[i_seg] = o.overflow ? 0xFFFFFFFFu : (uint32_t)((o.bits + 7) >> 3);
    if (o.overflow) atomicOr(err, 2u);
  }
}

}  // namespace bitar_hip
