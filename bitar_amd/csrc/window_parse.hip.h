// window_parse.hip.h -- the window-scan parse shared by the segment compressors
// (compress.hip: LZ4 / fixed-Huffman DEFLATE; zstd_compress.hip: Zstandard), one wavefront
// per segment (gfx950).  Restated exactly by the oracle's bo_window_parse
// (oracle/bitar_oracle.c); every compressor must match the oracle's output byte for byte.
//
// Input staging.  The segment streams through a 4 KiB LDS input ring in 1 KiB rows (one
// aligned 16-B block per lane): each row is loaded into registers a whole row of windows
// before it is written into the ring, and the ring runs 576..1536 B ahead of the scan.
// Every byte a position, a candidate (matches are capped at 2560 B back) or a literal needs
// is then an LDS read.  One register block in a fixed register: a rotation between
// blocks would make the compiler wait for every load in flight.
//
// Per fixed window of 64 positions (one per lane):
//   1. hash the 4 bytes at every position (from the ring), look up a 1024-entry LDS table of
//      u16 positions, then insert every position with one ds_write_b16 (the largest position
//      wins a slot: the hardware keeps the highest lane's write, see BITAR_CMP_NOREDO);
//   2. lanes with a candidate verify + measure the match on 16 bytes from the ring, and
//      lanes still matching extend in parallel up to 32 bytes;
//   3. a scalar chain walk picks the greedy matches in lane order (one ctz per match,
//      cooperative extension only for matches reaching 32 bytes);
//   4. the codec's emitter (E::window) writes the window's output lane-parallel (or, the LZ4
//      emitter, records the matches and writes batches of them in E::between).
// Output is staged in LDS and flushed with aligned 16-B stores once per input row (E::drain),
// right before the next row's load is issued.
#pragma once

#include "wave.hip.h"

namespace bitar_hip {

namespace cmp {

// Build-time knobs for tuning experiments (scripts/build_variant.sh); the defaults are the
// shipped configuration and the one the oracle restates.
#ifndef BITAR_CMP_HASH_LOG
#define BITAR_CMP_HASH_LOG 10
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
// Match distance cap (all codecs): at window x the input ring holds positions
// [F - kIn, F) with F <= x + 1536, so every candidate (>= x - (kIn - 1536)) is in LDS; it
// is also inside the LZ4 decoder's 8 KiB history ring (reach 8048), so our streams decode
// from LDS.  4 KiB ring + 1024-entry table = 7.3 KiB of LDS per wave, 22 waves per CU
// (the VGPR limit is 24); an 8 KiB ring (cap 6656) measured 12-18 % slower for ~1 % ratio.
#ifndef BITAR_CMP_RING
#define BITAR_CMP_RING 4096
#endif
constexpr uint32_t kIn = BITAR_CMP_RING, kInMask = kIn - 1;  // LDS input ring
constexpr uint32_t kMaxDist = kIn - 1536;
constexpr uint32_t kInPad = 64;  // mirror of ring[0, 64) after its end: probes never wrap
constexpr uint32_t kRow = 1024;                   // prefetch row: one 16-B block per lane
// Same-slot inserts of one window (or probe) resolve by the hardware: lanes of ONE
// ds_write_b16 that hit the same address leave the highest lane's value, i.e. the largest
// position -- the oracle's ascending-insert rule -- so no read-back is needed (measured on
// gfx950: every segment of the 1 GiB LZ4 / LZ4_WIDE / DEFLATE / Zstd parity tests bit-exact
// without it, LZ4 compress 2.89 -> 2.74 ms/GiB).  BITAR_CMP_NOREDO=0 builds the read-back
// and re-write loop that enforces the rule independently of that ordering.  Either way only
// the candidate choice could differ, never the validity of a match (every candidate is
// verified against the input).
#ifndef BITAR_CMP_NOREDO
#define BITAR_CMP_NOREDO 1
#endif
#ifndef BITAR_CMP_PREEXT
#define BITAR_CMP_PREEXT 32
#endif
constexpr uint32_t kPreExt = BITAR_CMP_PREEXT;    // parallel per-lane match extension limit

template <uint32_t HLOG = kHashLog>
__device__ __forceinline__ uint32_t hash4(uint32_t v) { return (v * 2654435761u) >> (32 - HLOG); }

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
// v_ffbl_b32: index of the lowest set bit, ~0u for 0
__device__ __forceinline__ uint32_t ffbl(uint32_t d) {
  uint32_t r;
  __asm__("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(d));
  return r;
}
__device__ __forceinline__ uint32_t common16(uint4 a, uint4 b) {
  const uint32_t d0 = a.x ^ b.x, d1 = a.y ^ b.y, d2 = a.z ^ b.z, d3 = a.w ^ b.w;
  // first differing bit = min over dwords of (32 k + ffbl), ~0u (saturating add) for equal
  // dwords: 4 xor, 4 ffbl, 3 add, 2 min3, 1 shift
  const uint32_t c0 = ffbl(d0);
  const uint32_t c1 = __builtin_elementwise_add_sat(ffbl(d1), 32u);
  const uint32_t c2 = __builtin_elementwise_add_sat(ffbl(d2), 64u);
  const uint32_t c3 = __builtin_elementwise_add_sat(ffbl(d3), 96u);
  // (two v_min3: the 128 cap rides in the second's third operand)
  return min(min(min(min(c0, c1), c2), c3), 128u) >> 3;
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

// lowest set bit of a 64-bit mask (64 if none); highest set bit (mask nonzero)
__device__ __forceinline__ uint32_t lowbit(uint64_t m) { return m ? (uint32_t)__builtin_ctzll(m) : 64u; }
__device__ __forceinline__ uint32_t highbit(uint64_t m) { return 63u - (uint32_t)__builtin_clzll(m); }

// The LDS input ring: byte of segment position q lives at ring[(in_lo + q) & kInMask]
// (absolute-address indexing keeps aligned blocks aligned).
struct InRing {
  uint8_t* ring;
  uint32_t in_lo;  // low 32 bits of the segment's input address
  uint32_t lo;     // positions >= lo are in the ring (< the filled end)
  uint32_t mask;   // ring size - 1 (kIn - 1, or the wide LZ4 parse's 16 KiB ring)

  __device__ __forceinline__ uint32_t byte(uint32_t q) const {
    return ring[(in_lo + q) & mask];
  }
  // 4 / 16 bytes at position q (little-endian); the pad lets the dword reads run past the
  // ring's end without wrapping
  __device__ __forceinline__ uint32_t dword(uint32_t q) const {
    const uint32_t u = in_lo + q;
    const uint32_t* r32 = reinterpret_cast<const uint32_t*>(ring) + ((u & mask) >> 2);
    return funnel(r32[0], r32[1], u);  // (v_alignbyte_b32 reads the shift's low 2 bits)
  }
  __device__ __forceinline__ uint4 bytes16(uint32_t q) const {
    const uint32_t u = in_lo + q;
    const uint32_t* r32 = reinterpret_cast<const uint32_t*>(ring) + ((u & mask) >> 2);
    const uint32_t sh = u;  // (v_alignbyte_b32 reads the shift's low 2 bits only)
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
  uint32_t dm1;     // per lane: match distance - 1 (chain lanes)
  uint32_t byte;    // per lane: input byte at x + lane
  uint32_t pos_in;  // parse position at window start: [x, pos_in) is covered by a match
  uint32_t done;    // end of the positions earlier windows handed over (SKIP: positions in
                    // [done, x) lay in skipped probe windows and are all literals)
  __device__ __forceinline__ uint32_t off() const { return dm1 + 1u; }  // match distance
};

// ---- byte output staged in an LDS ring, flushed in aligned 16-B blocks ----------------
constexpr uint32_t kObuf = BITAR_CMP_OBUF, kObufMask = kObuf - 1;

// ZERO: flushed ring bytes are cleared as they go out, so every ring byte at or past op is
// zero (a bit writer ORs into them; the ring starts zeroed)
template <uint32_t OB = kObuf, bool ZERO = false>
struct ByteOutT {
  static constexpr uint32_t kSize = OB, kMask = OB - 1;
  uint8_t* ring;      // LDS, OB bytes + one trash byte per lane
  GMEM uint8_t* dst;  // slot
  uint64_t cap;
  uint32_t op, flushed;
  bool overflow;

  __device__ __forceinline__ uint32_t at(uint32_t k) const {
    return ((uint32_t)(uintptr_t)dst + k) & kMask;
  }
  __device__ __forceinline__ void flush(uint32_t upto, bool final) {
    const uint32_t lane = lane_id();
    const uintptr_t base = (uintptr_t)dst;
    uint32_t f = flushed;
    lds_order();
    uint32_t head = (uint32_t)((16u - ((base + f) & 15u)) & 15u);
    if (head > upto - f) head = upto - f;
    if (head) {
      if (lane < head) {
        dst[f + lane] = ring[at(f + lane)];
        if constexpr (ZERO) ring[at(f + lane)] = 0;
      }
      f += head;
    }
    const uint32_t nb = (upto - f) >> 4;
    for (uint32_t b = lane; b < nb; b += kWave) {
      const uint32_t k = f + 16u * b;
      *reinterpret_cast<GMEM uint4*>(dst + k) = *reinterpret_cast<const uint4*>(ring + at(k));
      if constexpr (ZERO) *reinterpret_cast<uint4*>(ring + at(k)) = make_uint4(0, 0, 0, 0);
    }
    f += nb << 4;
    if (final && f < upto) {
      if (lane < upto - f) {
        dst[f + lane] = ring[at(f + lane)];
        if constexpr (ZERO) ring[at(f + lane)] = 0;
      }
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
    if (op + n - flushed > OB - 64) flush(op, false);
    return true;
  }
  // lanes < n write byte `v` at op + lane
  __device__ __forceinline__ void put(uint32_t v, uint32_t n) {
    lds_order();
    if (lane_id() < n) ring[at(op + lane_id())] = (uint8_t)v;
    lds_order();
    op += n;
  }
};
using ByteOut = ByteOutT<>;

// The greedy chain's common step, written out (the parse is bound by scalar issue: the SQ
// issues one SALU per SIMD every 4 cycles): from the non-empty lane set m, take the first
// lane l; if l is in extm (its match may extend past kPreExt) return l with m unchanged;
// else add it to chain, set e = l + len[l], keep only lanes of m at or past e, and go on.
// Returns kWave (m = 0) when the chain leaves the window.  9 SALU + 1 VALU per match.
__device__ __forceinline__ uint32_t chain_fast(uint64_t& m, uint64_t extm, uint32_t len,
                                               uint64_t& chain, uint32_t& e) {
  uint32_t l, ml;
  uint64_t t;
  __asm__ volatile(
      "L_ch_%=:\n"
      "s_ff1_i32_b64 %[l], %[m]\n"
      "s_bitcmp1_b64 %[x], %[l]\n"
      "s_cbranch_scc1 L_out_%=\n"
      "v_readlane_b32 %[ml], %[len], %[l]\n"
      "s_bitset1_b64 %[ch], %[l]\n"
      "s_add_u32 %[e], %[l], %[ml]\n"
      "s_cmp_gt_u32 %[e], 63\n"
      "s_cbranch_scc1 L_end_%=\n"
      "s_lshl_b64 %[t], -1, %[e]\n"
      "s_and_b64 %[m], %[m], %[t]\n"
      "s_cbranch_scc1 L_ch_%=\n"
      "L_end_%=:\n"
      "s_mov_b64 %[m], 0\n"
      "s_mov_b32 %[l], 64\n"
      "L_out_%=:\n"
      : [l] "=&s"(l), [ml] "=&s"(ml), [t] "=&s"(t), [m] "+s"(m), [ch] "+s"(chain),
        [e] "+s"(e)
      : [x] "s"(extm), [len] "v"(len)
      : "scc");
  return l;
}

// Form 2 (BITAR_CMP_CHAIN == 2, the default; kind-2 LZ4 compress 6.25 -> 6.03 ms/GiB): lanes that need the cooperative extension carry a length
// of 128 (lenw, one v_cndmask per window), so the per-match "is it an extension lane" test
// folds into the chain-end compare and runs once per window: 7 SALU + 1 VALU per match.
// The lane's chain bit is set here (the caller sets it again after the extension).
#ifndef BITAR_CMP_CHAIN
#define BITAR_CMP_CHAIN 3
#endif
constexpr uint32_t kExtLen = 128;
__device__ __forceinline__ uint32_t chain_fast2(uint64_t& m, uint32_t lenw, uint64_t& chain,
                                                uint32_t& e) {
  uint32_t l, ml;
  uint64_t t;
  __asm__ volatile(
      "L_c2_%=:\n"
      "s_ff1_i32_b64 %[l], %[m]\n"
      "v_readlane_b32 %[ml], %[len], %[l]\n"
      "s_bitset1_b64 %[ch], %[l]\n"
      "s_add_u32 %[e], %[l], %[ml]\n"
      "s_cmp_gt_u32 %[e], 63\n"
      "s_cbranch_scc1 L_end_%=\n"
      "s_lshl_b64 %[t], -1, %[e]\n"
      "s_and_b64 %[m], %[m], %[t]\n"
      "s_cbranch_scc1 L_c2_%=\n"
      "s_mov_b32 %[l], 64\n"
      "s_branch L_out_%=\n"
      "L_end_%=:\n"
      "s_cmp_lt_u32 %[e], 128\n"
      "s_cbranch_scc0 L_out_%=\n"
      "s_mov_b64 %[m], 0\n"
      "s_mov_b32 %[l], 64\n"
      "L_out_%=:\n"
      : [l] "=&s"(l), [ml] "=&s"(ml), [t] "=&s"(t), [m] "+s"(m), [ch] "+s"(chain),
        [e] "+s"(e)
      : [len] "v"(lenw)
      : "scc");
  return l;
}

// Form 3 (BITAR_CMP_CHAIN == 3): the successor of every lane is computed once per window on
// the VALU -- nx[j] = the first valid lane at or past j + len[j] (64..127: the chain leaves
// the window; 128 + j: lane j needs the cooperative extension, whose length is not known yet) --
// so the scalar loop per match is one v_readlane (the next lane is the next lane select),
// one s_bitset1, one compare and one branch (unrolled twice).  Matches per window: 6.6 on
// kind 1, up to 8.6 on kind 5 (oracle counts), so the chain was ~half of the parse's scalar
// instructions.  Returns the lane that stopped the walk (64..127, or 128 + an extension lane),
// every chain lane before it set in `chain`.  (A VALU-written SGPR needs 4 wait states before
// it is a lane select: s_nop 1 + the compare + the branch + the bitset.)
__device__ __forceinline__ uint32_t chain_succ(uint32_t l, uint32_t nx, uint64_t& chain) {
  __asm__ volatile(
      "L_cs_%=:\n"
      "s_bitset1_b64 %[ch], %[l]\n"
      "v_readlane_b32 %[l], %[nx], %[l]\n"
      "s_nop 1\n"
      "s_cmp_gt_u32 %[l], 63\n"
      "s_cbranch_scc1 L_co_%=\n"
      "s_bitset1_b64 %[ch], %[l]\n"
      "v_readlane_b32 %[l], %[nx], %[l]\n"
      "s_nop 1\n"
      "s_cmp_lt_u32 %[l], 64\n"
      "s_cbranch_scc1 L_cs_%=\n"
      "L_co_%=:\n"
      : [l] "+s"(l), [ch] "+s"(chain)
      : [nx] "v"(nx)
      : "scc");
  return l;
}
// per lane: nx as above, from e = lane + lenw (lenw = 128 on extension lanes).  f = the first
// valid lane at or past e (64: none) is >= e whenever e < 64, so max(f, e) is f there and e
// for e >= 64 (f <= 64 then, whatever the masked shift made of it): a lane leaving the window
// returns e in [64, 128), an extension lane 128 + lane -- one v_max instead of two selects.
__device__ __forceinline__ uint32_t chain_next(uint64_t valid, uint32_t e) {
  const uint64_t t = ~0ull << (e & 63u);
  const uint32_t lo = (uint32_t)t & (uint32_t)valid, hi = (uint32_t)(t >> 32) & (uint32_t)(valid >> 32);
  const uint32_t f = min(min(ffbl(lo), __builtin_elementwise_add_sat(ffbl(hi), 32u)), 64u);
  return max(f, e);
}

// The window-scan parse over one segment; hands each window to E::window and the tail to
// E::sequence.
// Returns where the tail literals start (the emitter's pending_from).
// REP (the Zstd parse, oracle BO_PARSE_REP): a history h of the parse's 3 most recent distinct
// match distances (initially 1 4 8), fixed per window; every position first tries p - h0,
// p - h1, p - h2 (the first whose 4 bytes agree), then its hash candidate; a position with
// only a hash match does not start a match when one of the next kRepAhead positions holds a
// repeat match.
constexpr uint32_t kRepAhead = 3;
// SKIP (the LZ4 parse, oracle BO_PARSE_SKIP): with g = the gate (the parse position, or after
// a probe hit the end of the probed span, whichever is later), a window lying entirely inside
// the current match is skipped (no lookups, no inserts); a window starting >= kSkipProbe past g
// (two windows with no match start) is a PROBE of stride 2 (4 from kSkipWide past g): the 64
// positions x + s l look up their candidates; with no match among them they are inserted and
// the scan moves on to x + 64 s, else nothing is inserted, g moves to x + 64 (s - 1) - 127 and
// ordinary windows scan the region from x.  On incompressible stretches a window then covers
// 256 positions (liblz4's growing search step).  The common case -- an ordinary window close
// to the gate -- costs one scalar compare: both special cases lie outside (g - 64, g + 128).
constexpr uint32_t kSkipProbe = 128, kSkipWide = 640;
// RING / HLOG: the input ring's size and the hash table's log2 size (the defaults: 4 KiB and
// 1024 entries; the wide LZ4 parse: 16 KiB and 4096, max_dist = RING - 1536 either way).
template <class E, bool REP = false, bool SKIP = false, uint32_t RING = kIn,
          uint32_t HLOG = kHashLog>
__device__ __forceinline__ uint32_t parse(const GMEM uint8_t* in, uint32_t n, const GMEM uint8_t* in_end,
                                      uint16_t* table, uint8_t* inring, uint32_t max_dist,
                                      uint32_t max_mlen, E& em) {
  static_assert(RING >= kIn && (RING & (RING - 1)) == 0, "ring: a power of two >= 4 KiB");
  const uint32_t lane = lane_id();
  uint32_t anchor = 0, emitted = 0;
  uint32_t h0 = 1, h1 = 4, h2 = 8;  // REP: the distance history (uniform)
  InRing I;
  I.ring = inring;
  I.in_lo = (uint32_t)(uintptr_t)in;
  I.lo = 0xFFFFFFFFu;  // nothing staged: literal bytes come from HBM
  I.mask = RING - 1;
  if (n >= kMfLimit + 1) {
    // empty slot = candidate position 0 (the oracle's zeroed table)
    for (uint32_t k = lane; k < (1u << HLOG) / 8; k += kWave)
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
      const uint32_t blk = (rbase + (kRow / 16) * r + lane) & ((RING - 1) >> 4);
      ring16[blk] = v;
      if (blk < kInPad / 16) ring16[RING / 16 + blk] = v;  // the pad mirrors the ring's head
    };
    uint32_t pos = 0;
    uint32_t F = 0;  // the ring holds positions [F - RING, F)
    // one window of 64 positions at x; vp = the 16 bytes at x + lane, read during the
    // previous window (the ring already holds them then)
    uint4 vp = make_uint4(0, 0, 0, 0);
    // windows starting at or past x_edge hold a position past last_start, or one whose limit
    // (match_limit - p) does not exceed kPreExt
    const uint32_t int_end = min(last_start + 1u, match_limit > kPreExt ? match_limit - kPreExt : 0u);
    // (readfirstlane: kept in an SGPR, so the per-window test is a scalar compare)
    const uint32_t x_edge =
        __builtin_amdgcn_readfirstlane(int_end >= kWave ? int_end - (kWave - 1) : 0u);
    auto window = [&](uint32_t x) __attribute__((always_inline)) {
      const uint32_t p = x + lane;
      const bool act = p <= last_start;
#if !BITAR_CMP_NOREDO
      const uint64_t actm = ballot(p <= last_start);  // (a single compare: see the read-back)
#endif
      const uint4 v = vp;
      const uint32_t h = hash4<HLOG>(v.x);
      // Table and ring accesses are issued on all lanes (no exec-mask branches: the scalar
      // unit is the bottleneck).  Lanes past last_start exist only in the final window;
      // their table writes are never looked up again.
      uint32_t cand = table[h];
      bool isrep = false;
      if constexpr (REP) {
        // repeat candidates, read from the ring (h <= max_dist: every p - h >= x - kMaxDist is
        // staged); their 4 bytes against the position's
        const uint32_t r0 = I.dword(p - h0), r1 = I.dword(p - h1), r2 = I.dword(p - h2);
        const bool k0 = act && h0 <= p && r0 == v.x;
        const bool k1 = act && h1 <= p && r1 == v.x;
        const bool k2 = act && h2 <= p && r2 == v.x;
        isrep = k0 || k1 || k2;
        cand = k0 ? p - h0 : k1 ? p - h1 : k2 ? p - h2 : cand;
      }
      lds_order();
      table[h] = (uint16_t)p;
      lds_order();
      // read back now, settle same-slot writes at the end of the window
#if !BITAR_CMP_NOREDO
      const uint32_t back = table[h];
#endif
      vp = I.bytes16(p + kWave);  // next window's bytes
      // distance - 1: 1 <= p - cand <= max_dist is one unsigned compare (cand >= p wraps)
      const uint32_t dm1 = p + ~cand;
      const bool pre = dm1 < max_dist;
      // verify the 4 bytes and measure up to 16, from the input ring
      const uint32_t c16 = common16(v, I.bytes16(cand));
      uint32_t len = pre ? c16 : 0u;
      // lanes still matching after 16 bytes extend in parallel, up to kPreExt
      for (uint32_t k = 16; k < kPreExt; k += 16) {
        const bool go = len == k;  // (implies pre)
        if (!ballot(len == k)) break;
        const uint32_t l2 = k + common16(I.bytes16(p + k), I.bytes16(cand + k));
        len = go ? l2 : len;
      }
      // The segment's last windows: positions past last_start find nothing, matches stop at
      // match_limit (and max_mlen).  Elsewhere neither binds (every lane's limit exceeds
      // kPreExt), so those checks -- 6 VALU per window -- run only here, after the
      // pre-extension (clamping its result is the same as clamping each step).
      if (x >= x_edge) {
        __asm__ volatile("");  // (keeps this a branch: if-converted, every window paid it)
        const uint32_t l = match_limit - p;
        const uint32_t lim = act ? (l < max_mlen ? l : max_mlen) : 0u;
        len = len < lim ? len : lim;
      }
      // lanes at or past the parse position holding a match, and those of them whose match
      // reached kPreExt bytes and may go on (cooperative extension during the walk)
      const uint32_t pos_in = pos;
      // (pos > x ? pos - x : 0 as a uniform max: the compiler's saturating subtract is a VALU
      // clamp plus a readfirstlane)
      uint32_t start;
      __asm__("s_max_u32 %0, %1, %2" : "=s"(start) : "s"(pos), "s"(x));
      start -= x;
      // (len >= kMinMatch implies pre; ballots of single compares, see wave.hip.h)
      uint64_t valid = ballot(len >= kMinMatch) & (start < kWave ? ~0ull << start : 0ull);
      if constexpr (REP) {  // a hash-only match gives way to a repeat match just ahead
        const uint64_t repm = ballot(isrep);
        uint64_t ahead = 0;
#pragma unroll
        for (uint32_t k = 1; k <= kRepAhead; ++k) ahead |= repm >> k;
        valid &= ~(~repm & ahead);
      }
      // (a lane at its limit may be included: its cooperative extension stops at once)
      const uint64_t extm = valid & ballot(len == kPreExt);
      uint64_t chain = 0;
      uint32_t mlen_v = len;
      uint64_t m = valid;
      uint32_t e = 0;
#if BITAR_CMP_CHAIN == 3
      uint32_t lenw;
      __asm__("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(lenw) : "v"(len), "v"(kExtLen), "s"(extm));
      if (valid) {
        const uint32_t nx = chain_next(valid, lane + lenw);
        uint32_t l = lowbit(valid);
        for (;;) {
          l = chain_succ(l, nx, chain);
          if (l < 128u) break;
          l -= 128u;  // an extension lane (its chain bit is set): extend it cooperatively
          const uint32_t i = x + l;
          uint32_t li = match_limit - i;
          if (li > max_mlen) li = max_mlen;
          const uint32_t c = readlane(cand, l);
          const uint32_t lr = li < F - i ? li : F - i;
          uint32_t k = kPreExt;
          bool more = true;
          for (;;) {
            // every lane compares (ring reads stay in bounds by the mask; a lane at or past lr
            // stops the scan whatever it read), and the stop mask is two single-compare
            // ballots: no exec-mask branch, no bool re-materialised for the ballot
            const uint32_t kk = k + 4u * lane;
            const uint32_t cl = min(common4(I.dword(i + kk), I.dword(c + kk)), lr - kk);
            const uint64_t stop = ballot(kk >= lr) | ballot(cl < 4u);
            if (stop) {
              const uint32_t sl = (uint32_t)__builtin_ctzll(stop);
              const uint32_t ks = k + 4u * sl;
              k = ks >= lr ? lr : ks + readlane(cl, sl);
              more = k == lr && lr < li;
              break;
            }
            k += 4u * kWave;
          }
          while (more) {
            const uint32_t kk = k + 16u * lane;
            uint32_t cl = 16;
            if (kk < li) {  // (HBM: no load past the candidate's or the position's end)
              const uint4 a = ld16u(in + i + kk, in_end);
              const uint4 b = ld16u(in + c + kk, in_end);
              cl = common16(a, b);
              if (cl > li - kk) cl = li - kk;
            }
            const uint64_t stop = ballot(kk >= li) | ballot(cl < 16u);
            if (stop) {
              const uint32_t sl = (uint32_t)__builtin_ctzll(stop);
              const uint32_t ks = k + 16u * sl;
              k = ks >= li ? li : ks + readlane(cl, sl);
              break;
            }
            k += 16u * kWave;
          }
          if (lane == l) mlen_v = k;
          const uint32_t ee = l + k;
          const uint64_t rest = ee < kWave ? valid & (~0ull << ee) : 0ull;
          if (!rest) break;
          l = lowbit(rest);
        }
        const uint32_t last = highbit(chain);
        e = last + readlane(mlen_v, last);
      }
      if (false) {
#elif BITAR_CMP_CHAIN == 2
      uint32_t lenw;
      __asm__("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(lenw) : "v"(len), "v"(kExtLen), "s"(extm));
#endif
      while (m) {  // the greedy chain: the next match is the first valid lane past the end
        // matches that need no extension: the hand-scheduled scalar loop
#if BITAR_CMP_CHAIN == 2
        const uint32_t l = chain_fast2(m, lenw, chain, e);
#else
        const uint32_t l = chain_fast(m, extm, len, chain, e);
#endif
        if (l >= kWave) break;
        uint32_t mlen = readlane(len, l);
        {  // lane l's match reached kPreExt bytes: extend it cooperatively
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
#if BITAR_CMP_CHAIN == 3
      }
#endif
      if (chain) pos = x + e;
      if constexpr (REP) {
        // the history after this window's matches: the 3 most recently used distinct
        // distances (move-to-front) of [h2, h1, h0, the chain's distances in lane order],
        // found by ballots instead of a per-match scalar loop
        if (chain) {
          const uint32_t offv = dm1 + 1u;
          const uint32_t n0 = readlane(offv, highbit(chain));
          const uint64_t m1 = chain & ballot(offv != n0);
          const uint32_t o1 = h0 != n0 ? h0 : h1;  // first old distance unlike n0
          const uint32_t n1 = m1 ? readlane(offv, highbit(m1)) : o1;
          const uint64_t m2 = m1 & ballot(offv != n1);
          // first old distance unlike n0 and n1
          const uint32_t o2 = h0 != n0 && h0 != n1 ? h0 : h1 != n0 && h1 != n1 ? h1 : h2;
          const uint32_t n2 = m2 ? readlane(offv, highbit(m2)) : o2;
          h0 = n0;
          h1 = n1;
          h2 = n2;
        }
      }
      Window W;
      W.x = x;
      W.chain = chain;
      W.mlen = mlen_v;
      W.dm1 = dm1;
      W.byte = v.x & 0xFFu;
      W.pos_in = pos_in;
      W.done = emitted;
#ifndef BITAR_CMP_TIMING_NOEMIT  // (timing knob only: no output)
      em.window(in, I, W, anchor, n);
#endif
      if (chain) anchor = pos;
      emitted = pos > x + kWave ? pos : x + kWave;
      // same-slot writes of this window: re-write until the largest position holds the slot
      // (the empty asm pins the read-back's use, and so its wait, here)
#if !BITAR_CMP_NOREDO
      uint32_t bk = back;
      __asm__ volatile("" : "+v"(bk));
      if (ballot(bk < p) & actm) {  // rare: only on same-slot collisions
        bool redo = act && bk < p;
        while (ballot(redo)) {
          lds_order();
          if (redo) table[h] = (uint16_t)p;
          lds_order();
          redo = redo && table[h] < p;
        }
      }
#endif
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
    // Row k+1 is written when the scan reaches 1024 k + 512 (a probe may step past that
    // point by < 256 positions; the ring then still runs >= 497 B ahead of the scan and holds
    // every candidate: x - 2560 > 1024 k - 3072)
    uint32_t next_load = kRow / 2;
    uint32_t g = 0;  // SKIP: the gate, >= pos
    for (uint32_t x = 0; x <= last_start;) {
      if (x >= next_load) {
        const uint32_t k = next_load / kRow;
        lds_order();
        write_row(k + 1, nxt);
        F = kRow * (k + 2) - s0;
        I.lo = F > RING ? F - RING : 0u;
        em.drain();
        nxt = load_row(k + 2);
        next_load += kRow;
      }
      // the emitter's batched work, between windows (fewer live registers than inside one)
      em.between(in, I);
      if constexpr (SKIP) {
        if (x - g + (kWave - 1) >= kSkipProbe + kWave - 1) {  // g >= x + 64, or x >= g + 128
          if (pos >= x + kWave) {  // inside the current match
            // every window lying wholly inside it at once (skipped windows do nothing else),
            // but not past the next row load, which the loop's top must see
            const uint32_t xs = x + ((pos - x) & ~(kWave - 1));
            x = xs < next_load ? xs : next_load;
            lds_order();
            vp = I.bytes16(x + lane);
            continue;
          }
          if (x >= g + kSkipProbe) {  // a probe of stride st
            const uint32_t st = x >= g + kSkipWide ? 4u : 2u;
            lds_order();
            const uint32_t p = x + st * lane;
            const bool act = p <= last_start;
            const uint32_t v = I.dword(p);
            const uint32_t h = hash4<HLOG>(v);
            const uint32_t cand = table[h];
            const uint32_t cv = I.dword(cand);
            const bool hit = act & (cand < p) & (p - cand <= max_dist) & (cv == v);
            if (!ballot(hit)) {
              // no match among them: insert (ascending, the largest position wins the slot)
              lds_order();
              table[act ? h : (1u << HLOG)] = (uint16_t)p;
              lds_order();
#if !BITAR_CMP_NOREDO
              bool redo = act && table[h] < p;
              while (ballot(redo)) {
                lds_order();
                if (redo) table[h] = (uint16_t)p;
                lds_order();
                redo = redo && table[h] < p;
              }
#endif
              x += st * kWave;
              continue;
            }
            g = x + kWave * (st - 1) - 127u;  // ordinary windows over the probed span
          }
          lds_order();
          vp = I.bytes16(x + lane);  // (after skipped windows / probes)
        }
      }
      lds_order();
      window(x);
      if constexpr (SKIP) g = g > pos ? g : pos;
      x += kWave;
    }
  }
  const uint32_t t0 = em.pending_from(anchor, emitted);
  if (t0 < n) em.sequence(in, I, t0, n - t0, 0, 0);
  return t0;
}

}  // namespace cmp

}  // namespace bitar_hip
