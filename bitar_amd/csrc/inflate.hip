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

// Fast-table sizes, namespace and kernel name: inflate_fixed.hip builds this file a second
// time with 9 / 8-bit tables for fixed-Huffman streams (inflate_fixed_kernel)
#ifndef BITAR_INFL_NS
#define BITAR_INFL_NS infl
#endif
#ifndef BITAR_INFL_KERNEL
#define BITAR_INFL_KERNEL inflate_kernel
#endif

namespace bitar_hip {

namespace BITAR_INFL_NS {

using namespace sr;

#ifndef BITAR_INFL_LIT_FAST
#define BITAR_INFL_LIT_FAST 10
#endif
#ifndef BITAR_INFL_DIST_FAST
#define BITAR_INFL_DIST_FAST 9
#endif
constexpr uint32_t kLitFast = BITAR_INFL_LIT_FAST, kDistFast = BITAR_INFL_DIST_FAST, kClFast = 7;

__device__ __forceinline__ uint32_t bpermute_u32(uint32_t v, uint32_t src_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src_lane << 2), (int)v);
}

struct Tables {  // LDS
  uint16_t lit_fast[1u << kLitFast];   // lit_entry(sym, len) (0 = not a <= kLitFast-bit code)
  uint16_t dist_fast[1u << kDistFast];
  uint16_t cl_fast[1u << kClFast];
  uint16_t lit_count[16], dist_count[16], cl_count[16];
  uint16_t lit_sym[288], dist_sym[32], cl_sym[19];
  uint32_t base[16];                   // scratch for ranking / next codes
  uint8_t lens[320];
};

// Length and distance symbol bases and extra-bit counts (RFC 1951 3.2.5), computed rather
// than looked up: a table indexed by a value the compiler cannot prove wave-uniform becomes a
// per-match vector load from memory.
__device__ __forceinline__ uint32_t len_extra(uint32_t ls) {  // ls = symbol - 257, 0..28
  return ls < 8 || ls == 28 ? 0u : (ls - 4) >> 2;
}
__device__ __forceinline__ uint32_t len_base(uint32_t ls) {
  return ls < 8 ? 3 + ls : ls == 28 ? 258u : ((4 + ((ls - 4) & 3u)) << len_extra(ls)) + 3;
}
__device__ __forceinline__ uint32_t dist_extra(uint32_t ds) {  // 0..29
  return ds < 4 ? 0u : (ds - 2) >> 1;
}
__device__ __forceinline__ uint32_t dist_base(uint32_t ds) {
  return ds < 4 ? ds + 1 : ((2 + (ds & 1u)) << dist_extra(ds)) + 1;
}
// A literal/length table entry, pre-decoded so the batch path's 256 candidates need no
// symbol arithmetic: bits 9..12 the code length (0 on the slow path), bits 13..15 the kind --
// 7 a literal (bits 0..7 the byte), 6 end of block or an invalid length symbol (bits 0..8 =
// symbol - 256: 0, 30, 31), 0..5 a length symbol with that many extra bits (bits 0..8 its base
// length, 3..258).  A fast entry is never 0 (its code length is not).  The distance and
// code-length table keeps sym | len << 9.
__device__ __forceinline__ uint32_t lit_entry(uint32_t sym, uint32_t l) {
  if (sym < 256) return sym | (l << 9) | (7u << 13);
  const uint32_t ls = sym - 257;
  if (sym == 256 || ls >= 29) return (sym - 256) | (l << 9) | (6u << 13);
  return len_base(ls) | (l << 9) | (len_extra(ls) << 13);
}
// A distance table entry: bits 0..4 the symbol, 5..8 its extra-bit count, 9..12 the code
// length, 13..14 m, the base being (m << extra) + 1 (m = the symbol below 4, else 2 | its low
// bit).
__device__ __forceinline__ uint32_t dist_entry(uint32_t ds, uint32_t l) {
  const uint32_t de = ds < 30 ? dist_extra(ds) : 0u;
  const uint32_t m = ds < 4 ? ds : 2u | (ds & 1u);
  return ds | (de << 5) | (l << 9) | (m << 13);
}
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Wave-uniform LSB-first bit reader.  The bit buffer lives in scalar registers; it is
// refilled 32 bits at a time from a register vector holding 256 stream bytes (lane l:
// bytes vb+4l .. vb+4l+3), itself reloaded from the LDS stream window every ~250 bytes --
// no LDS round trip per refill.
//
// Reads past the stream's end return zero bits and are not checked per symbol: the decoder
// checks once, at the end, that it consumed no more than csize*8 bits (a stream that runs
// short then fails exactly as the oracle's bit-by-bit check makes it fail; zero bits decode
// to bounded work -- every output is capped by the segment size).
struct Bits {
  uint64_t buf;   // next bits, LSB first
  uint32_t cnt;   // valid bits in buf
  uint32_t bp;    // next stream byte to load into buf
  uint32_t v;     // register vector of stream bytes
  uint32_t vb;    // stream position of its byte 0 (modular; may sit up to 3 below 0)
};

__device__ __forceinline__ void bits_reset(Bits& b, uint32_t pos) {
  b.buf = 0;
  b.cnt = 0;
  b.bp = pos;
  b.vb = 0xFFFFFF00u;  // nothing loaded
  b.v = 0;
}

// 4 stream bytes at bp (zeros past csize), as one little-endian word
__device__ __forceinline__ uint32_t peek4(State& s, uint8_t* win, Bits& b, uint32_t bp) {
  if (bp >= s.csize) return 0u;
  if (bp - b.vb > 256u - 8u) {  // modular: also when bp < vb
    const uint64_t abs = (uint64_t)(uintptr_t)(s.src + bp);
    const uint32_t mis = (uint32_t)(abs & 3u);
    uint32_t want = s.csize - bp + mis;
    if (want > 256) want = 256;
    const uint32_t w = win_at_abs(s, win, abs - mis, want);  // 16-B aligned window
    lds_order();
    b.v = *reinterpret_cast<const uint32_t*>(win + w + 4 * lane_id());
    b.vb = bp - mis;
  }
  const uint32_t k = bp - b.vb;
  const uint32_t d = k >> 2;
  const uint64_t w2 = (uint64_t)readlane(b.v, d) | ((uint64_t)readlane(b.v, d + 1) << 32);
  uint32_t w = (uint32_t)(w2 >> ((k & 3u) * 8));
  const uint32_t avail = s.csize - bp;
  if (avail < 4) w &= (1u << (8 * avail)) - 1;
  return w;
}

// The reader's scalars are wave-uniform; saying so (readfirstlane of an SGPR value is free)
// keeps them in SGPRs -- otherwise the divergent per-lane code around them (literal
// gathering, ring copies) can make the compiler carry them in VGPRs and turn every branch
// on them into an exec-mask branch.
__device__ __forceinline__ void bits_uniform(Bits& b) {
  b.buf = uniform64(b.buf);
  b.cnt = uniform(b.cnt);
  b.bp = uniform(b.bp);
  b.vb = uniform(b.vb);
}

__device__ __forceinline__ void need(State& s, uint8_t* win, Bits& b, uint32_t n) {
  while (b.cnt < n) {  // n <= 32: at most two refills
    const uint32_t w = peek4(s, win, b, b.bp);
    b.buf |= (uint64_t)w << b.cnt;
    b.cnt += 32;
    b.bp += 4;
  }
  bits_uniform(b);
}

// take n (<= 32) bits; false if that runs past the stream (the oracle's bits_get == -1)
__device__ __forceinline__ uint64_t used_bits(const Bits& b) { return (uint64_t)b.bp * 8 - b.cnt; }

__device__ __forceinline__ bool take(State& s, uint8_t* win, Bits& b, uint32_t n, uint32_t& v) {
  if (n == 0) { v = 0; return true; }
  need(s, win, b, n);
  v = (uint32_t)(b.buf & ((1ull << n) - 1));
  b.buf >>= n;
  b.cnt -= n;
  return true;
}

// Build the decoding tables of one code from lens[0..n) (LDS).  Returns false if the code is
// over-subscribed, or -- strict, the codes of a dynamic block -- incomplete, except a code
// with no symbols and (kind 1 / 2) one whose longest length is 1: zlib 1.2.11's
// inflate_table rule, as the oracle's huff_build.  fast: 2^fbits entries; count/sym:
// canonical arrays for long codes.
// Inlined (at two sites): an out-of-line call would make every value live across it --
// the bit reader's state included -- sit in callee-saved VGPRs for the whole kernel.
__device__ __forceinline__ bool build(Tables& t, const uint8_t* lens, uint32_t n, uint16_t* fast, uint32_t fbits,
                      uint16_t* count, uint16_t* sym, uint32_t kind, bool strict) {
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
  if (strict && left > 0) {
    const uint64_t nz = ballot(cntv != 0u);  // (lane 0's count is 0)
    const uint32_t maxlen = nz ? 63u - (uint32_t)__builtin_clzll(nz) : 0u;
    if (maxlen != 0 && (kind == 0 || maxlen != 1)) return false;
  }
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
        // (kind 1: the literal/length table, 2: the distance table, 0: code lengths)
        const uint16_t e = (uint16_t)(kind == 1 ? lit_entry(k, l) : kind == 2 ? dist_entry(k, l)
                                                                            : k | (l << 9));
        for (uint32_t j = r; j < (1u << fbits); j += (1u << l)) fast[j] = e;
      }
    }
    lds_order();
  }
  return true;
}

// The literal/length and distance fast tables mirrored in registers (two 16-bit entries
// per dword, dword d in lane d % 64 of register d / 64): a lookup is a register select and a
// v_readlane instead of an LDS round trip.
struct RegTables {
  uint32_t lit[(1u << kLitFast) / 128];
  uint32_t dist[(1u << kDistFast) / 128];
};

__device__ __forceinline__ void load_reg_tables(const Tables& t, RegTables& r) {
  const uint32_t lane = lane_id();
  const uint32_t* lf = reinterpret_cast<const uint32_t*>(t.lit_fast);
  const uint32_t* df = reinterpret_cast<const uint32_t*>(t.dist_fast);
  lds_order();
#pragma unroll
  for (uint32_t j = 0; j < (1u << kLitFast) / 128; ++j) r.lit[j] = lf[j * kWave + lane];
#pragma unroll
  for (uint32_t j = 0; j < (1u << kDistFast) / 128; ++j) r.dist[j] = df[j * kWave + lane];
}

// register j of r (j uniform) by a select tree on j's bits (written out: a linear select
// chain gets turned back into an indexed stack array)
__device__ __forceinline__ uint32_t pick(const uint32_t (&r)[8], uint32_t j) {
  const bool b0 = j & 1u, b1 = j & 2u, b2 = j & 4u;
  const uint32_t a0 = b0 ? r[1] : r[0], a1 = b0 ? r[3] : r[2];
  const uint32_t a2 = b0 ? r[5] : r[4], a3 = b0 ? r[7] : r[6];
  const uint32_t c0 = b1 ? a1 : a0, c1 = b1 ? a3 : a2;
  return b2 ? c1 : c0;
}
__device__ __forceinline__ uint32_t pick(const uint32_t (&r)[2], uint32_t j) {
  return (j & 1u) ? r[1] : r[0];
}
__device__ __forceinline__ uint32_t pick(const uint32_t (&r)[4], uint32_t j) {
  const bool b0 = j & 1u, b1 = j & 2u;
  const uint32_t a0 = b0 ? r[1] : r[0], a1 = b0 ? r[3] : r[2];
  return b1 ? a1 : a0;
}
template <uint32_t N>
__device__ __forceinline__ uint32_t reg_entry(const uint32_t (&r)[N], uint32_t idx) {
  const uint32_t dw = idx >> 1;
  const uint32_t v = readlane(pick(r, dw / kWave), dw % kWave);
  return (idx & 1u) ? v >> 16 : v & 0xFFFFu;
}

// Decode one symbol; returns -1 if the code runs past the stream, -2 if unassigned.
// `e` is the fast-table entry of the next fbits bits (0: code longer than fbits).
__device__ __forceinline__ int decode_entry(State& s, Bits& b, uint32_t e, const uint16_t* count,
                                            const uint16_t* sym) {
  if (e) {
    const uint32_t len = (e >> 9) & 15u;
    b.buf >>= len;
    b.cnt -= len;
    return (int)(e & 511u);
  }
  lds_order();
  int code = 0, first = 0, index = 0;
  for (uint32_t len = 1; len <= 15; ++len) {
    code |= (int)((b.buf >> (len - 1)) & 1u);
    const int cnt = (int)uniform((uint32_t)count[len]);
    if (code - cnt < first) {
      b.buf >>= len;
      b.cnt -= len;
      return (int)uniform((uint32_t)sym[index + (code - first)]);
    }
    index += cnt;
    first += cnt;
    first <<= 1;
    code <<= 1;
  }
  return -2;
}

__device__ __forceinline__ int decode(State& s, uint8_t* win, Bits& b, const uint16_t* fast,
                                      uint32_t fbits, const uint16_t* count, const uint16_t* sym) {
  need(s, win, b, 15);
  lds_order();
  const uint32_t e = uniform((uint32_t)fast[b.buf & ((1u << fbits) - 1)]);
  return decode_entry(s, b, e, count, sym);
}
template <uint32_t N>
__device__ __forceinline__ int decode_reg(State& s, uint8_t* win, Bits& b, const uint32_t (&r)[N],
                                          uint32_t fbits, const uint16_t* count, const uint16_t* sym) {
  need(s, win, b, 15);
  const uint32_t e = reg_entry(r, (uint32_t)b.buf & ((1u << fbits) - 1));
  return decode_entry(s, b, e, count, sym);
}

// The literal/length table: the symbol's pre-decoded entry (lit_entry), < 0 if unassigned.
template <uint32_t N>
__device__ __forceinline__ int decode_lit_reg(State& s, uint8_t* win, Bits& b, const uint32_t (&r)[N],
                                              const uint16_t* count, const uint16_t* sym) {
  need(s, win, b, 15);
  const uint32_t e = reg_entry(r, (uint32_t)b.buf & ((1u << kLitFast) - 1));
  if (e) {
    const uint32_t len = (e >> 9) & 15u;
    b.buf >>= len;
    b.cnt -= len;
    return (int)e;
  }
  const int v = decode_entry(s, b, 0u, count, sym);  // (a code longer than kLitFast bits)
  return v < 0 ? v : (int)lit_entry((uint32_t)v, 0u);
}

// pending literals, one per lane, written to the ring 64 at a time
struct Lits {
  uint32_t v;  // lane j: j-th pending byte
  uint32_t n;
};

// false if the literals would overflow the segment (checked here, once per 64 literals)
__device__ __forceinline__ bool lits_flush(State& s, uint8_t* ring, Lits& L) {
  if (!L.n) return true;
  if (s.op + L.n > s.cap) return false;
  make_room(s, ring, L.n);
  const uintptr_t base = (uintptr_t)s.dst;
  lds_order();
  if (lane_id() < L.n) ring[(base + s.op + lane_id()) & kRingMask] = (uint8_t)L.v;
  lds_order();
  s.op += L.n;
  L.n = 0;
  return true;
}

// Move the reader to absolute stream bit `bit` (the batch path's position).
__device__ __forceinline__ void seek(State& s, uint8_t* win, Bits& b, uint64_t bit) {
  b.buf = 0;
  b.cnt = 0;
  b.bp = (uint32_t)(bit >> 3);
  const uint32_t skip = (uint32_t)(bit & 7u);
  if (skip) {
    need(s, win, b, skip);
    b.buf >>= skip;
    b.cnt -= skip;
  }
  bits_uniform(b);
}

// Batch path for Huffman-coded block bodies: up to 64 output bytes per step.
//   1. every lane decodes, speculatively, the symbol starting at 4 candidate bit offsets
//      (lane, lane+64, lane+128, lane+192 past the current position): literal, or length +
//      distance with their extra bits, from the LDS fast tables -- two LDS round trips for
//      all 256 candidates;
//   2. a scalar walk follows the real symbol chain (one v_readlane per symbol; the walk over
//      candidates of register j is unrolled so each register is read statically);
//   3. each output lane takes its byte from its symbol: the literal itself, history in the
//      ring, or (match source inside this batch) another lane, resolved by pointer doubling;
//      one ds_read gathers, one ds_write stores.
// Symbols it does not take (end of block, codes longer than the fast tables, matches longer
// than 64 or farther than the ring, anything invalid) stop it; the scalar path decodes them.
constexpr uint32_t kBatchStreamBytes = 48;  // stream bytes past the position a batch may read

__device__ __forceinline__ void huff_batch(State& s, uint8_t* win, uint8_t* ring, Bits& b,
                                           const Tables& t) {
  const uint32_t lane = lane_id();
  const uint32_t base = (uint32_t)(uintptr_t)s.dst;  // ring index = absolute address & mask
  const uint64_t src_abs = (uint64_t)(uintptr_t)s.src;
  uint64_t P = used_bits(b);
  bool moved = false;
  for (;;) {
    const uint32_t room = s.cap - s.op;
    const uint32_t byte0 = (uint32_t)(P >> 3);
    if (room == 0 || byte0 + kBatchStreamBytes > s.csize) break;
    make_room(s, ring, 64);
    const uint64_t a0 = (src_abs + byte0) & ~3ull;
    win_at_abs(s, win, a0, kBatchStreamBytes + 8);
    const uint64_t absbit0 = (src_abs + byte0) * 8 + (P & 7u);
    const uint32_t wd = (uint32_t)(s.wb >> 2);  // window base, in absolute dwords
    const uint32_t* w32 = reinterpret_cast<const uint32_t*>(win);
    // (1) speculative decode of 4 candidates per lane
    uint32_t rec[4], mlv[4];
    lds_order();
    // candidate j's bits start 64 j bits (2 j dwords) after candidate 0's: the nine dwords
    // they span are read once
    const uint64_t ab0 = absbit0 + lane;
    const uint32_t di0 = (uint32_t)(ab0 >> 5) - wd, sh = (uint32_t)(ab0 & 31u);
    uint32_t dw[9];
#pragma unroll
    for (uint32_t k = 0; k < 9; ++k) dw[k] = w32[di0 + k];
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t c = lane + kWave * j;
      const uint32_t d0 = dw[2 * j], d1 = dw[2 * j + 1], d2 = dw[2 * j + 2];
      const uint64_t bits = (uint64_t)__builtin_amdgcn_alignbit(d1, d0, sh) |
                            ((uint64_t)__builtin_amdgcn_alignbit(d2, d1, sh) << 32);
      const uint32_t e = t.lit_fast[(uint32_t)bits & ((1u << kLitFast) - 1)];
      const uint32_t l1 = (e >> 9) & 15u, kind = e >> 13, pay = e & 511u;
      const bool is_lit = kind == 7u;
      const bool is_len = (kind < 6u) & (e != 0u);
      const uint32_t le = kind & 7u;  // (only meaningful for a length symbol)
      const uint32_t mlen = pay + ((uint32_t)(bits >> l1) & ((1u << le) - 1));
      const uint32_t o2 = l1 + le;
      const uint32_t e2 = t.dist_fast[(uint32_t)(bits >> o2) & ((1u << kDistFast) - 1)];
      const uint32_t dl = (e2 >> 9) & 15u, ds = e2 & 31u, de = (e2 >> 5) & 15u;
      const uint32_t dist = ((e2 >> 13) << de) + 1u + ((uint32_t)(bits >> (o2 + dl)) & ((1u << de) - 1));
      // any distance (far history -- beyond the ring's reach, stock zlib streams go to
      // 32 KiB -- is read back from HBM below)
      const bool d_ok = is_len && e2 != 0 && ds < 30 && dist <= s.op;
      const bool m_ok = d_ok && mlen <= 64;
      const uint32_t nb = is_lit ? l1 : o2 + dl + de;
      // 126: a match longer than a batch -- the walk stops on it and it is copied below
      const uint32_t olen = is_lit ? 1u : m_ok ? mlen : d_ok ? 126u : 127u;
      mlv[j] = mlen;
      const uint32_t payload = is_lit ? pay : (0x8000u | (dist - 1u));
      // record: next candidate (9 bits) | olen (7 bits, 127 = stop) | payload (16 bits:
      // literal byte, or 0x8000 | distance - 1)
      rec[j] = ((c + nb) & 511u) | (olen << 9) | (payload << 16);
    }
    // (2) scalar walk over the real symbols
    const uint32_t lim = room < 64 ? room : 64;
    // Written out (scalar issue binds the walk): the output position in m0, the room as a
    // remainder whose s_sub_u32 borrow is "does not fit", each symbol's record dropped into
    // the lane of its first output byte by v_writelane (a prefix max below hands every
    // output byte its record); the candidate index k (< 256: lane k & 63 of rec[k >> 6]) is
    // range-checked per vector, v_readlane taking the low 6 bits of its lane select.
    uint32_t k, out, olx, ns, vrec = 0;
    {
      uint32_t e, ol, rem, m0_saved;
      __asm__ volatile(
          "s_mov_b32 %[m0s], m0\n"
          "s_mov_b32 %[k], 0\n"
          "s_mov_b32 %[rem], %[lim]\n"
          "s_mov_b32 %[olx], 0\n"
          "s_mov_b32 %[ns], 0\n"
          "s_mov_b32 m0, 0\n"
          "L_i0_%=:\n"
          "s_cmp_ge_u32 %[k], 64\n"
          "s_cbranch_scc1 L_i1_%=\n"
          "v_readlane_b32 %[e], %[r0], %[k]\n"
          "s_bfe_u32 %[ol], %[e], 0x70009\n"
          "s_sub_u32 %[rem], %[rem], %[ol]\n"
          "s_cbranch_scc1 L_stop_%=\n"
          "v_writelane_b32 %[vr], %[e], m0\n"
          "s_add_u32 %[ns], %[ns], 1\n"
          "s_add_u32 m0, m0, %[ol]\n"
          "s_and_b32 %[k], %[e], 511\n"
          "s_branch L_i0_%=\n"
          "L_i1_%=:\n"
          "s_cmp_ge_u32 %[k], 128\n"
          "s_cbranch_scc1 L_i2_%=\n"
          "v_readlane_b32 %[e], %[r1], %[k]\n"
          "s_bfe_u32 %[ol], %[e], 0x70009\n"
          "s_sub_u32 %[rem], %[rem], %[ol]\n"
          "s_cbranch_scc1 L_stop_%=\n"
          "v_writelane_b32 %[vr], %[e], m0\n"
          "s_add_u32 %[ns], %[ns], 1\n"
          "s_add_u32 m0, m0, %[ol]\n"
          "s_and_b32 %[k], %[e], 511\n"
          "s_branch L_i1_%=\n"
          "L_i2_%=:\n"
          "s_cmp_ge_u32 %[k], 192\n"
          "s_cbranch_scc1 L_i3_%=\n"
          "v_readlane_b32 %[e], %[r2], %[k]\n"
          "s_bfe_u32 %[ol], %[e], 0x70009\n"
          "s_sub_u32 %[rem], %[rem], %[ol]\n"
          "s_cbranch_scc1 L_stop_%=\n"
          "v_writelane_b32 %[vr], %[e], m0\n"
          "s_add_u32 %[ns], %[ns], 1\n"
          "s_add_u32 m0, m0, %[ol]\n"
          "s_and_b32 %[k], %[e], 511\n"
          "s_branch L_i2_%=\n"
          "L_i3_%=:\n"
          "s_cmp_ge_u32 %[k], 256\n"
          "s_cbranch_scc1 L_out_%=\n"
          "v_readlane_b32 %[e], %[r3], %[k]\n"
          "s_bfe_u32 %[ol], %[e], 0x70009\n"
          "s_sub_u32 %[rem], %[rem], %[ol]\n"
          "s_cbranch_scc1 L_stop_%=\n"
          "v_writelane_b32 %[vr], %[e], m0\n"
          "s_add_u32 %[ns], %[ns], 1\n"
          "s_add_u32 m0, m0, %[ol]\n"
          "s_and_b32 %[k], %[e], 511\n"
          "s_branch L_i3_%=\n"
          "L_stop_%=:\n"
          "s_or_b32 %[olx], %[ol], 0x100\n"
          "L_out_%=:\n"
          "s_mov_b32 %[out], m0\n"
          "s_mov_b32 m0, %[m0s]\n"
          : [k] "=&s"(k), [out] "=&s"(out), [olx] "=&s"(olx), [ns] "=&s"(ns), [e] "=&s"(e),
            [ol] "=&s"(ol),
            [rem] "=&s"(rem), [m0s] "=&s"(m0_saved), [vr] "+v"(vrec)
          : [r0] "v"(rec[0]), [r1] "v"(rec[1]), [r2] "v"(rec[2]), [r3] "v"(rec[3]),
            [lim] "s"(lim)
          : "scc");
    }
    // stopped on a symbol (olx = 0x100 | its olen) rather than by running out of candidates:
    // the batch continues only when that symbol was cut by a full batch
    const uint32_t olxu = __builtin_amdgcn_readfirstlane(olx);
    const bool taken_all = olxu == 0 || (olxu != 0x17Fu && lim == 64u);
    // a long match (65..258 bytes) stopped the walk: its symbol at candidate k
    const bool long_next = olxu == 0x17Eu;
    auto long_match = [&]() __attribute__((always_inline)) -> bool {
      const uint32_t ku = __builtin_amdgcn_readfirstlane(k);
      const uint32_t jr = ku >> 6;
      const uint32_t rv = jr == 0 ? readlane(rec[0], ku) : jr == 1 ? readlane(rec[1], ku)
                          : jr == 2 ? readlane(rec[2], ku) : readlane(rec[3], ku);
      const uint32_t ml = jr == 0 ? readlane(mlv[0], ku) : jr == 1 ? readlane(mlv[1], ku)
                          : jr == 2 ? readlane(mlv[2], ku) : readlane(mlv[3], ku);
      if (s.op + ml > s.cap) return false;  // (the scalar path rejects it)
      match_copy(s, ring, ((rv >> 16) & 0x7FFFu) + 1u, ml);
      P += (rv & 511u) - ku;  // past the symbol and its extra bits
      moved = true;
      return true;
    };
    if (out == 0) {
      if (long_next && long_match()) continue;
      break;
    }
    // every output byte takes the payload of the latest symbol starting at or before it
    // (one symbol -- a batch cut short by a far match or a long code: its record for all)
    const uint32_t key = __builtin_amdgcn_readfirstlane(ns) == 1u
                             ? readlane(vrec, 0) >> 16
                             : wave_incl_max(vrec ? (lane << 24) | (vrec >> 16) : 0u);
    const uint32_t ostart = key >> 24;
    const uint32_t payload = key & 0xFFFFu;
    // (3) sources: the literal / ring history / an earlier lane of this batch
    const bool lit = (payload & 0x8000u) == 0;
    const uint32_t dist = (payload & 0x7FFFu) + 1u;
    const uint32_t r = lane - ostart;
    const float qf = floorf(((float)(r & 63u) + 0.5f) * __builtin_amdgcn_rcpf((float)(dist > 1u ? dist : 1u)));
    const uint32_t mm = dist <= r ? (r & 63u) - (uint32_t)qf * dist : r;
    const int32_t srel = (int32_t)(ostart + mm) - (int32_t)dist;  // vs op
    const uint32_t hist = kWin + ((base + s.op + (uint32_t)srel) & kRingMask);
    // bit31: alias (low bits: source lane); bit30: literal (low byte); bit29: far history
    // (low 16 bits: the output position, in HBM); else an LDS address
    const bool far = !lit && srel < -(int32_t)kNearOff;
    uint32_t st = lit ? (0x40000000u | (payload & 255u))
                      : srel >= 0 ? ((uint32_t)srel | 0x80000000u)
                      : far ? (0x20000000u | (s.op + (uint32_t)srel)) : hist;
    while (ballot((st & 0x80000000u) != 0u && lane < out)) {
      const uint32_t other = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((st & 63u) << 2), (int)st);
      st = (st & 0x80000000u) ? other : st;
    }
    lds_order();
    uint32_t v = (st & 0x40000000u) ? (st & 255u) : (uint32_t)win[st & 0x3FFFu];
    {
      // far history: already flushed (flushes keep out[.., op - 2112) in HBM and far sources
      // lie >= 3952 B back); fence once this wave's stores may not be visible to its loads
      const bool gfar = (st & 0x20000000u) != 0u && lane < out;
      const uint64_t farm = ballot(gfar);
      if (farm) {
        if (ballot((st & 0xFFFFu) >= s.fenced) & farm) {
          global_fence_wave();
          s.fenced = s.flushed;
        }
        if (gfar) v = s.dst[st & 0xFFFFu];
      }
    }
    if (lane < out) ring[(base + s.op + lane) & kRingMask] = (uint8_t)v;
    lds_order();
    s.op += out;
    P += k;
    moved = true;
    ++s.nbatch;
    if (long_next) {
      if (long_match()) continue;
      break;
    }
    if (!taken_all) break;  // stopped on a symbol the batch does not take
  }
  if (moved) seek(s, win, b, P);
}

__device__ __forceinline__ int inflate_codes(State& s, uint8_t* win, uint8_t* ring, Bits& b, Tables& t,
                             Lits& L) {
  RegTables rt;
  load_reg_tables(t, rt);
  for (;;) {
    if (!lits_flush(s, ring, L)) return -1;
    huff_batch(s, win, ring, b, t);
    bits_uniform(b);
    s.op = uniform(s.op);
    // one symbol on the scalar path
    const int ent = decode_lit_reg(s, win, b, rt.lit, t.lit_count, t.lit_sym);
    if (ent < 0) return -1;
    const uint32_t kind = (uint32_t)ent >> 13, pay = (uint32_t)ent & 511u;
    if (kind == 7u) {  // a literal
      if (lane_id() == L.n) L.v = pay;
      ++L.n;
      continue;
    }
    if (kind == 6u) return pay == 0 ? 0 : -1;  // end of block; symbols 286 / 287 are invalid
    uint32_t e;
    if (!take(s, win, b, kind, e)) return -1;
    const uint32_t len = pay + e;
    const int dsr = decode_reg(s, win, b, rt.dist, kDistFast, t.dist_count, t.dist_sym);
    if (dsr < 0) return -1;
    const uint32_t ds = (uint32_t)dsr & 31u;  // (a fast entry carries more above bit 4)
    if (ds >= 30) return -1;
    if (!take(s, win, b, dist_extra(ds), e)) return -1;
    const uint32_t d = dist_base(ds) + e;
    if (!lits_flush(s, ring, L)) return -1;
    if (d > s.op) return -1;
    if (s.op + len > s.cap) return -1;
    match_copy(s, ring, d, len);
  }
}

}  // namespace BITAR_INFL_NS

#ifndef BITAR_INFL_WAVES
#define BITAR_INFL_WAVES 0
#endif
#if BITAR_INFL_WAVES
#define BITAR_INFL_ATTR __attribute__((amdgpu_waves_per_eu(BITAR_INFL_WAVES)))
#else
#define BITAR_INFL_ATTR
#endif
__global__ __launch_bounds__(64) BITAR_INFL_ATTR void BITAR_INFL_KERNEL(
    const uint8_t* const* __restrict__ srcs, const uint8_t* __restrict__ slab,
    uint64_t slot_stride, const uint32_t* __restrict__ csizes, uint32_t nseg, uint32_t seg,
    uint8_t* __restrict__ out, uint32_t* __restrict__ produced, uint32_t* __restrict__ err,
    uint32_t defer_only, unsigned long long* __restrict__ stats, const uint32_t* __restrict__ order) {
  using namespace BITAR_INFL_NS;
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWin + kRing];
  __shared__ __attribute__((aligned(16))) Tables t;
  uint8_t* win = lds;
  uint8_t* ring = lds + kWin;
  if (blockIdx.x >= nseg) return;
  const uint32_t i = order ? order[blockIdx.x] : blockIdx.x;  // (cost-ordered dispatch)
  if (i >= nseg) return;
  // after inflate_lanes_kernel: only the segments it deferred (inflate_lanes.hip)
  if (defer_only && produced[i] != 0xFFFFFFFEu) return;
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
  s.nbatch = 0;

  Bits b;
  bits_reset(b, 0);
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
      const uint32_t drop = b.cnt & 7u;  // bits up to the next byte boundary
      uint32_t junk;
      if (drop && !take(s, win, b, drop, junk)) { ok = false; break; }
      const uint32_t p = (uint32_t)(used_bits(b) >> 3);
      if ((uint64_t)p + 4 > s.csize) { ok = false; break; }
      uint32_t w0;
      take(s, win, b, 32, w0);
      const uint32_t len = w0 & 0xFFFFu, nlen = w0 >> 16;
      if (len != (~nlen & 0xFFFFu)) { ok = false; break; }
      if ((uint64_t)p + 4 + len > s.csize) { ok = false; break; }
      if (!lits_flush(s, ring, L)) { ok = false; break; }
      if ((uint64_t)s.op + len > s.cap) { ok = false; break; }
      s.ip = p + 4;
      if (len >= kLongLit) literals_long(s, win, ring, len);
      else if (len) literals_short(s, win, ring, len);
      bits_reset(b, s.ip);  // restart the bit reader after the raw bytes
    } else if (type == 1 || type == 2) {
    uint32_t nlen = 288, ndist = 30;
    bool need_build = true;
    if (type == 1) {
      if (built_fixed) {
        need_build = false;
      } else {
        lds_order();
        for (uint32_t k = lane; k < 320; k += kWave)
          t.lens[k] = k < 144 ? 8 : k < 256 ? 9 : k < 280 ? 7 : k < 288 ? 8 : 5;
        lds_order();
      }
      built_fixed = 1;
    } else {
      built_fixed = 0;
      uint32_t hlit, hdist, hclen;
      if (!take(s, win, b, 5, hlit) || !take(s, win, b, 5, hdist) || !take(s, win, b, 4, hclen)) {
        ok = false;
        break;
      }
      nlen = hlit + 257;
      ndist = hdist + 1;
      const uint32_t ncode = hclen + 4;
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
      if (!build(t, t.lens, 19, t.cl_fast, kClFast, t.cl_count, t.cl_sym, 0u, true)) {
        ok = false;
        break;
      }
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
    }
    // literal/length then distance tables: one build site for fixed and dynamic blocks
    if (need_build) {
      for (uint32_t j = 0; j < 2 && ok; ++j) {
        const bool d = j == 1;
        ok = build(t, d ? t.lens + nlen : t.lens, d ? ndist : nlen, d ? t.dist_fast : t.lit_fast,
                   d ? kDistFast : kLitFast, d ? t.dist_count : t.lit_count,
                   d ? t.dist_sym : t.lit_sym, d ? 2u : 1u, type == 2);
      }
      if (!ok) break;
    }
    } else {
      ok = false;
      break;
    }
    // one call site for the Huffman-coded body of fixed and dynamic blocks
    if (type != 0 && inflate_codes(s, win, ring, b, t, L)) { ok = false; break; }
  } while (!last);
  // the stream must hold every bit the decode consumed (reads past its end returned zeros)
  if (ok && used_bits(b) > (uint64_t)s.csize * 8) ok = false;
  if (ok && !lits_flush(s, ring, L)) ok = false;
  if (ok) {
    flush(s, ring, s.op, true);
    if (lane == 0) produced[i] = s.op;
  } else if (lane == 0) {
    produced[i] = 0xFFFFFFFFu;
    atomicOr(err, 1u);
  }
  if (stats && lane == 0) {  // path counters (bitar_hip_path_counters)
    atomicAdd(stats + BITAR_HIP_PATH_INFLATE_WAVE, 1ull);
    if (!ok) atomicAdd(stats + BITAR_HIP_PATH_INFLATE_WAVE_REJECT, 1ull);
    if (s.nbatch) {
      atomicAdd(stats + BITAR_HIP_PATH_INFLATE_BATCH_SEGS, 1ull);
      atomicAdd(stats + BITAR_HIP_PATH_INFLATE_BATCHES, (unsigned long long)s.nbatch);
    }
  }
}

}  // namespace bitar_hip
