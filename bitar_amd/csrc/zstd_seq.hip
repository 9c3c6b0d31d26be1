// zstd_seq.hip -- two-phase execution of the sequence sections that the wave Zstd decoder
// (zstd_decompress.hip) hands over (zstd_hand.hip.h), for segments of at most 64 KiB.
//
// Phase A, zstd_seqdec_kernel: ONE LANE PER SEGMENT runs the serial part -- the backward FSE
// bitstream, whose states chain from sequence to sequence -- and nothing else: every decoded
// sequence becomes one 8-byte record {literal length, match length, offset} (repeat offsets
// resolved), with all of the wave decoder's acceptance checks (oracle/bitar_zstd.c
// zs_sequences; the final frame checks too).  The three decode tables of a segment live in
// LDS as 16-bit cells (symbol | next-state number << 6; the state's bit count and baseline
// are recomputed from the number), 2.5 KiB per segment: 16 segments per wave, four waves per
// CU, so the 16384 chains of a GiB are all resident in one round and no cell lookup leaves
// the CU (the lane executor reads its 4-byte cells from L2 / the Infinity Cache).
//
// Phase B, zstd_exec_kernel: ONE WAVE PER SEGMENT executes the records 64 at a time.  The
// batch's output is produced 64 bytes per step, one byte per lane: the literal-run and match
// starts that fall in the step are scattered to their lanes through LDS, a prefix max gives
// every lane the run it lies in; a literal lane loads its byte, a match lane reads its source
// from the LDS history ring (or HBM when farther back), or -- source inside the same step --
// from another lane by pointer jumping; the step is stored into the ring, which is flushed to
// HBM in 16-B blocks (stream_ring.hip.h).  No per-lane wildcopies: every output byte is
// written once, by a coalesced store.
//
// Records: u64 = L | M << 22 | off << 44, L / M = literal-length / match-length code << 16 |
// its extra bits (the baseline is added by the executor), off a 20-bit offset: an absolute
// one <= 2^19 - 1 (saturated: a segment <= 64 KiB has offsets <= 65536), or -- blocks after
// the first of a multi-block hand-off, whose chains run before the history at their start is
// known -- a symbolic one, kSym | k << 17 | (2^17 - 1 - d) = "history slot k at the block's
// start, minus d" (the repeat offset r0 - 1 of RFC 8878 3.1.2.5 is then the same subtraction
// for both forms); zstd_exec_kernel resolves them block by block.
#include "lane_copy.hip.h"
#include "stream_ring.hip.h"
#include "zstd_hand.hip.h"
#include "order.hip.h"

namespace bitar_hip {

namespace zsq {

using namespace zhand;

constexpr uint32_t kTab = 1280;          // cells per segment: LL 512 | OF 256 | ML 512
constexpr uint32_t kSym = 0x80000u, kAbsMax = 0x7FFFFu;  // symbolic offsets, see above
__device__ __forceinline__ uint32_t sym_slot(uint32_t k) { return kSym | (k << 17) | 0x1FFFFu; }
// an offset field (record or history word) against the history r at the block's start:
// absolute, or slot k minus d; 0 (invalid) for slot 3 or a negative result
__device__ __forceinline__ uint32_t resolve_off(uint32_t v, uint32_t r0, uint32_t r1, uint32_t r2) {
  const uint32_t k = (v >> 17) & 3u, d = 0x1FFFFu - (v & 0x1FFFFu);
  const uint32_t base = k == 0 ? r0 : k == 1 ? r1 : k == 2 ? r2 : 0u;
  return (v & kSym) ? (base > d ? base - d : 0u) : v;
}
constexpr uint32_t kOfAt = 512, kMlAt = 768;

// Literal-length / match-length code -> baseline and extra-bit count (RFC 8878
// 3.1.1.3.2.1.1), computed: the codes in the middle of both tables share one shape.
__host__ __device__ constexpr uint32_t mid_t(uint32_t m) {
  return m < 4 ? m : (2u + (m & 1u)) << ((m >> 1) - 1u);
}
__host__ __device__ constexpr uint32_t mid_bits(uint32_t m) { return m < 4 ? 1u : m >> 1; }
__host__ __device__ constexpr uint32_t ll_bits(uint32_t c) {
  return c < 16 ? 0u : c < 25 ? mid_bits(c - 16) : c - 19;
}
__host__ __device__ constexpr uint32_t ll_base(uint32_t c) {
  return c < 16 ? c : c < 25 ? 16u + 2u * mid_t(c - 16) : 1u << (c - 19);
}
__host__ __device__ constexpr uint32_t ml_bits(uint32_t c) {
  return c < 32 ? 0u : c < 43 ? mid_bits(c - 32) : c - 36;
}
__host__ __device__ constexpr uint32_t ml_base(uint32_t c) {
  return c < 32 ? c + 3 : c < 43 ? 35u + 2u * mid_t(c - 32) : (1u << (c - 36)) + 3u;
}

// the RFC tables, to check the arithmetic at compile time
constexpr uint32_t kLLB[36] = {0,  1,  2,  3,  4,  5,  6,   7,   8,   9,    10,   11,
                               12, 13, 14, 15, 16, 18, 20,  22,  24,  28,   32,   40,
                               48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384,
                               32768, 65536};
constexpr uint32_t kLLX[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  1,  1,
                               1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
constexpr uint32_t kMLB[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13,   14,   15,   16,
                               17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27,   28,   29,   30,
                               31, 32, 33, 34, 35, 37, 39, 41, 43, 47, 51,   59,   67,   83,
                               99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771,
                               65539};
constexpr uint32_t kMLX[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                               0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                               2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
constexpr bool codes_ok() {
  for (uint32_t c = 0; c < 36; ++c)
    if (ll_base(c) != kLLB[c] || ll_bits(c) != kLLX[c]) return false;
  for (uint32_t c = 0; c < 53; ++c)
    if (ml_base(c) != kMLB[c] || ml_bits(c) != kMLX[c]) return false;
  return true;
}
static_assert(codes_ok(), "literal / match length code arithmetic");

// The same, branch-free for the decode loop: every shift amount masked to 5 bits, so each
// arm is well defined and the compiler selects instead of branching on the exec mask.
// (a ?: chain whose arms are not all trivial becomes exec-mask branches; `sel` is a select)
__device__ __forceinline__ uint32_t sel(bool c, uint32_t a, uint32_t b) {
  const uint32_t m = 0u - (uint32_t)c;
  return (a & m) | (b & ~m);
}
__device__ __forceinline__ uint32_t mid_t_d(uint32_t m) {
  return sel(m < 4, m, (2u + (m & 1u)) << (((m >> 1) - 1u) & 31u));
}
__device__ __forceinline__ uint32_t mid_bits_d(uint32_t m) { return sel(m < 4, 1u, m >> 1); }
__device__ __forceinline__ void ll_code(uint32_t c, uint32_t& base, uint32_t& bits) {
  const uint32_t m = c - 16, h = (c - 19) & 31u;
  base = sel(c < 16, c, sel(c < 25, 16u + 2u * mid_t_d(m), 1u << h));
  bits = sel(c < 16, 0u, sel(c < 25, mid_bits_d(m), h));
}
__device__ __forceinline__ void ml_code(uint32_t c, uint32_t& base, uint32_t& bits) {
  const uint32_t m = c - 32, h = (c - 36) & 31u;
  base = sel(c < 32, c + 3, sel(c < 43, 35u + 2u * mid_t_d(m), (1u << h) + 3u));
  bits = sel(c < 32, 0u, sel(c < 43, mid_bits_d(m), h));
}

// lane k of each quad, to all four (DPP quad_perm broadcast)
template <int K>
__device__ __forceinline__ uint32_t qbcast(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, K * 0x55, 0xF, 0xF, false);
}

// 4-byte scratch cell (sym | state bits << 8 | baseline << 16) -> 16-bit LDS cell
// (sym | next-state number << 6): number = (baseline + 2^al) >> bits, in [1, 1024)
__device__ __forceinline__ uint32_t cell16(uint32_t c, uint32_t al) {
  const uint32_t nb = (c >> 8) & 0xFFu, base = c >> 16;
  return (c & 63u) | (((base + (1u << al)) >> nb) << 6);
}

// a cell's state bit count and next-state baseline (FSE_buildDTable's rule)
struct Step {
  uint32_t nb, base;
};
__device__ __forceinline__ Step step_of(uint32_t cell, uint32_t al) {
  const uint32_t ns = cell >> 6;
  const uint32_t nb = al - (31u - (uint32_t)__builtin_clz(ns));
  return {nb, (ns << nb) - (1u << al)};
}

}  // namespace zsq

// ---- phase A -----------------------------------------------------------------------------
// L segments per wave (lane l < L owns segment blockIdx.x * L + l), B chains (blocks) per
// segment: B = 1 takes the frames that handed their last block only (kNb == 1), B = 4 the
// multi-block hand-offs (kNb >= 2), whose blocks' chains run side by side -- by units of 4
// blocks (zstd_hand.hip.h kUnitBlocks: slot l owns unit blockIdx.x * L + l, blocks 4 g ..
// 4 g + 3 of segment unit >> 1, g = unit & 1; 2 nseg units).  A segment is
// taken when the wave decoder handed it over (produced == kHanded) and it has at most `rcap`
// sequences; on success (every chain's bitstream consumed exactly) produced = kRecs, else
// SEGMENT_ERROR and the stream's error word; the sequence rules are checked by
// zstd_exec_kernel.  Single-block segments beyond rcap stay kHanded for zstd_handoff_kernel
// (a multi-block one beyond rcap cannot be valid: rejected here).
template <uint32_t L, uint32_t B = 1>
__global__ __launch_bounds__(64) void zstd_seqdec_kernel(
    const uint8_t* const* __restrict__ srcs, const uint8_t* __restrict__ slab,
    uint64_t slot_stride, const uint32_t* __restrict__ csizes, uint32_t nseg, uint32_t seg,
    uint32_t* __restrict__ produced, uint8_t* __restrict__ hscr, uint64_t* __restrict__ recs,
    uint32_t rcap, uint32_t* __restrict__ err, unsigned long long* __restrict__ stats,
    const uint32_t* __restrict__ order) {
  using namespace zsq;
  using lanes::ld8;
  static_assert(L * B * 4 <= kWave, "a quad per chain");
  __shared__ __attribute__((aligned(16))) uint16_t cel[L * kTab];
  const uint32_t lane = lane_id();
  // stage the decode tables of the wave's segments, 4 cells per lane per step.  The headers
  // are loaded one lane per segment, together, and a segment's table loads are all issued
  // before the first is used: at about one wave per SIMD every serial load is exposed.
  // (order: the segments by sequence count, most first, hand_key_kernel: slot x takes
  // segment order[x], so a wave's chains are of similar length and the longest start first)
  static_assert(B == 1 || B == kUnitBlocks, "whole units");
  const uint32_t nun = B > 1 ? 2 * nseg : nseg;  // units
  uint32_t p0 = 0, nq0 = 0, als0 = 0, nb0 = 0, il0 = 0, g0 = 0;
  {
    const uint32_t bl = blockIdx.x * L + lane;
    const uint32_t u = bl < nun ? (order ? order[bl] : bl) : bl;
    const uint32_t il = B > 1 ? u >> 1 : u;
    il0 = il;
    g0 = B > 1 ? u & 1u : 0u;
    if (lane < L && bl < nun && il < nseg) {
      const GMEM uint32_t* h = global_ptr(reinterpret_cast<const uint32_t*>(hscr + (uint64_t)il * kStride));
      p0 = produced[il];
      nq0 = h[kNseqAll];
      als0 = h[kAls];
      nb0 = h[kNb];
    }
  }
  // (B > 1: the other unit of an 8-block frame may already have finished and moved the
  // segment to kRecs -- its units can sit in different workgroups under the cost order -- so
  // kRecs is taken too; exec runs after this whole launch, and a failure's 0xFFFFFFFF, which
  // is never overwritten, still excludes the segment)
  const bool handed = p0 == kHanded || (B > 1 && p0 == kRecs);
  const bool mine = handed && (B == 1 ? nb0 == 1u : nb0 >= 2u && B * g0 < nb0);
  if (B > 1 && lane < L && mine && nq0 > rcap) {  // (more sequences than a valid frame has)
    produced[il0] = 0xFFFFFFFFu;
    atomicOr(err, 1u);
  }
  const uint64_t tm = ballot(mine && nq0 <= rcap);
  for (uint64_t mm = tm; mm; mm &= mm - 1) {
    const uint32_t l = (uint32_t)__builtin_ctzll(mm);
    const uint32_t il = readlane(il0, l);
    const GMEM uint32_t* h = global_ptr(reinterpret_cast<const uint32_t*>(hscr + (uint64_t)il * kStride));
    const uint32_t als = readlane(als0, l);
    constexpr uint32_t kPer = (kCells / 4 + kWave - 1) / kWave;  // uint4 loads per lane per table
    uint4 cv[3][kPer];
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) {
      const uint32_t al = (als >> (8 * k)) & 0xFFu;
      const uint32_t n4 = al >= 2 ? (1u << al) / 4 : 1u;
      const GMEM uint4* t = reinterpret_cast<const GMEM uint4*>(h + kCellsAt + k * kCells);
#pragma unroll
      for (uint32_t e = 0; e < kPer; ++e) {
        const uint32_t u = lane + e * kWave;
        cv[k][e] = t[u < n4 ? u : 0u];
      }
    }
#pragma unroll
    for (uint32_t k = 0; k < 3; ++k) {
      const uint32_t al = (als >> (8 * k)) & 0xFFu;
      const uint32_t n4 = al >= 2 ? (1u << al) / 4 : 1u;
      uint16_t* d = cel + l * kTab + (k == 0 ? 0u : k == 1 ? kOfAt : kMlAt);
#pragma unroll
      for (uint32_t e = 0; e < kPer; ++e) {
        const uint32_t u = lane + e * kWave;
        if (u < n4) {
          const uint4 c = cv[k][e];
          const uint32_t lo = cell16(c.x, al) | (cell16(c.y, al) << 16);
          const uint32_t hi = cell16(c.z, al) | (cell16(c.w, al) << 16);
          *reinterpret_cast<uint2*>(d + 4 * u) = make_uint2(lo, hi);
        }
      }
    }
  }
  lds_order();
  // Four lanes per segment (lane 4 l + j): j = 0 the literal-length table, 1 match lengths,
  // 2 offsets, 3 a copy of lane 0.  Each lane looks up its own table, works out its code's
  // baseline and extra bits and its state's bit count, the quad exchanges the widths (DPP
  // quad broadcasts) so every lane knows where its fields lie in the bitstream, each lane
  // extracts its two fields, and the quad exchanges the three values; the bit reader,
  // repeat offsets and records are replicated over the quad.  One wave instruction thus
  // advances all three FSE chains of 16 segments.
  const uint32_t l = lane / (4 * B), j = lane & 3u;
  // (fetched while every lane is active: a disabled source lane reads as 0)
  const uint32_t i = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((l < L ? l : 0u) << 2), (int)il0);
  const uint32_t g = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((l < L ? l : 0u) << 2), (int)g0);
  const uint32_t bk = B * g + (lane >> 2) % B;  // the block
  if (l >= L || blockIdx.x * L + l >= nun || !((tm >> l) & 1u)) return;  // quad-uniform
  GMEM uint32_t* h0 = global_ptr(reinterpret_cast<uint32_t*>(hscr + (uint64_t)i * kStride));
  if (bk >= h0[kNb]) return;
  const GMEM uint32_t* h = h0 + blk_at(bk);
  const uint32_t nseq = h[kNseq];
  const GMEM uint8_t* src = global_ptr(srcs ? srcs[i] : slab + (uint64_t)i * slot_stride);
  GMEM uint64_t* rec = global_ptr(recs + (uint64_t)i * rcap + h0[kX0 + kXW * bk + kXRec]);
  const uint32_t cs = csizes[i];
  const uint32_t q = h[kQ], end = h[kEnd], w3 = h[kAls];
  // the history at the block's start: known for the first, symbolic for the others
  uint32_t r0 = bk ? sym_slot(0) : h0[kRep0], r1 = bk ? sym_slot(1) : h0[kRep1],
           r2 = bk ? sym_slot(2) : h0[kRep2];
  const uint32_t al0 = w3 & 0xFFu, al1 = (w3 >> 8) & 0xFFu;
  const uint32_t t = j == 1 ? 2u : j == 2 ? 1u : 0u;  // table in the frame's LL, OF, ML order
  const uint32_t al = (w3 >> (8 * t)) & 0xFFu;
  const uint16_t* tab = cel + l * kTab + (t == 0 ? 0u : t == 1 ? kOfAt : kMlAt);
  // code -> extra-bit count: ll_code / ml_code's bits as one formula with per-table
  // constants (an offset code c is the formula's top range: c extra bits)
  const uint32_t c_lo = t == 0 ? 16u : t == 2 ? 32u : 0u, c_mid = t == 0 ? 25u : t == 2 ? 43u : 0u;
  const uint32_t c_hs = t == 0 ? 19u : t == 2 ? 36u : 0u;
  // Backward bit reader (replicated over the quad): C = the 8 stream bytes at [ptr, ptr+8),
  // `used` bits consumed from its top; N1, N2 = the 16 bytes below.  Two reloads per
  // sequence, unconditional and branch-free (a load under a condition is a phi the compiler
  // settles with vmcnt(0) on the spot).  Between two reloads at most 47 bits are consumed,
  // so a reload shifts by 0..6 bytes.  Bytes below q are not masked: a stream that reads
  // them is rejected by the final count whatever they hold, a valid one never uses them.
  const int32_t lo = (int32_t)q - 8;  // q >= 12 inside the frame
  // (the clamped position is >= 4: zero-extended, one 64-bit add forms the address)
  auto at = [&](int32_t a) __attribute__((always_inline)) {
    return ld8(src + (uint32_t)(a < lo ? lo : a));
  };
  int32_t ptr = (int32_t)end - 8;
  uint64_t C = at(ptr), N1 = at(ptr - 8), N2 = at(ptr - 16);
  uint32_t used = 0;
  auto reload = [&]() __attribute__((always_inline)) {
    const uint32_t sh = used & ~7u;
    C = (C << sh) | ((N1 >> (63u - sh)) >> 1);  // (two shifts: sh = 0 shifts N1 out)
    N1 = (N1 << sh) | ((N2 >> (63u - sh)) >> 1);
    used &= 7u;
    ptr -= (int32_t)(sh >> 3);
    N2 = at(ptr - 16);
  };
  auto peek = [&](uint32_t p, uint32_t n) __attribute__((always_inline)) {
    return (uint32_t)(C >> ((64u - p - n) & 63u)) & ((1u << n) - 1u);
  };
  const uint32_t lastb = (uint32_t)(C >> 56);
  // (a multi-block hand-off ends at the frame's end: zstd_decompress_kernel checked it)
  bool ok = (lastb != 0 || nseq == 0) && (B > 1 || end == cs);
  if (nseq == 0) {
    ok = ok && q == end;  // no sequences: no bitstream
  } else if (ok) {
    used = 8 - (31u - (uint32_t)__builtin_clz(lastb));
    // initial states, in the order LL, OF, ML
    uint32_t cell = tab[peek(used + (t == 0 ? 0u : t == 1 ? al0 : al0 + al1), al)];
    used += (w3 & 0xFFu) + ((w3 >> 8) & 0xFFu) + ((w3 >> 16) & 0xFFu);
    auto step = [&](bool more) __attribute__((always_inline)) {
      reload();
      const uint32_t sym = cell & 63u, ns = cell >> 6;
      const uint32_t m = sym - c_lo, hh = (sym - c_hs) & 31u;
      const uint32_t x = sel(sym < c_lo, 0u, sel(sym < c_mid, mid_bits_d(m), hh));
      const uint32_t nb0 = al - (31u - (uint32_t)__builtin_clz(ns));
      const uint32_t nbase = (ns << nb0) - (1u << al);
      const uint32_t nb = more ? nb0 : 0u;  // no state update after the last sequence
      const uint32_t w = x | (nb << 8);
      const uint32_t wl = qbcast<0>(w), wm = qbcast<1>(w), wo = qbcast<2>(w);
      const uint32_t xl = wl & 0xFFu, xm = wm & 0xFFu, xo = wo & 0xFFu;
      const uint32_t nbl = wl >> 8, nbm = wm >> 8, nbo = wo >> 8;
      // bits: offset extra, match extra | literal extra, LL state, ML state, OF state
      const uint32_t e1 = peek(used + sel(t == 2, xo, 0u), x);
      used += xo + xm;
      reload();
      const uint32_t e2 = peek(used, x);
      const uint32_t sof = xl + sel(t == 0, 0u, sel(t == 2, nbl, nbl + nbm));
      const uint32_t sbits = peek(used + sof, nb);
      used += xl + nbl + nbm + nbo;
      // the literal-length and match-length lanes send code << 16 | extra bits (the
      // baselines are added by zstd_exec_kernel, 64 records per instruction there against 16
      // segments per instruction here), the offset lane the offset value 2^code + extra
      const uint32_t e = sel(t == 0, e2, e1);
      const uint32_t val = sel(t == 1, (1u << (sym & 31u)) + e, (sym << 16) | e);
      cell = tab[nbase + sbits];
      const uint32_t lf = qbcast<0>(val), mf = qbcast<1>(val), ofv = qbcast<2>(val);
      // repeat offsets in select form (no exec-mask branches); literal length 0 = LL code 0
      // (which has no extra bits)
      const uint32_t idx = ofv + (lf == 0 ? 1u : 0u);
      // (a new offset saturates below kSym: a valid one is <= 65536)
      const uint32_t onew = ofv - 3 < kAbsMax ? ofv - 3 : kAbsMax;
      const uint32_t off =
          sel(ofv > 3, onew, sel(idx == 1, r0, sel(idx == 2, r1, sel(idx == 3, r2, r0 - 1))));
      const bool shift2 = ofv > 3 || idx >= 3, shift1 = ofv > 3 || idx >= 2;
      const uint32_t c0 = r0, c1 = r1, c2 = r2;
      r2 = sel(shift2, c1, c2);
      r1 = sel(shift1, c0, c1);
      r0 = off;
      // (r0 - 1 of an absolute 0 wraps: its low 20 bits read as slot 3, which resolves to 0)
      return (uint64_t)lf | ((uint64_t)mf << 22) | ((uint64_t)(off & 0xFFFFFu) << 44);
    };
    // Groups of kG sequences: the records stay in registers and lane 0 of the quad stores
    // them at the group's end (the compiler waits for every outstanding store at the next
    // load use -- it does not let loads overtake stores -- so one store burst per group)
    // (the last sequence, which updates no state, is peeled off: the loops pass `more` as
    // a constant)
    constexpr uint32_t kG = 8;
    uint32_t k = 0;
    for (; k + kG < nseq; k += kG) {
      uint64_t rb[kG];
#pragma unroll
      for (uint32_t g = 0; g < kG; ++g) rb[g] = step(true);
      if (j == 0) {
#pragma unroll
        for (uint32_t g = 0; g < kG; ++g) rec[k + g] = rb[g];
      }
    }
    for (; k + 1 < nseq; ++k) {
      const uint64_t r = step(true);
      if (j == 0) rec[k] = r;
    }
    {
      const uint64_t r = step(false);
      if (j == 0) rec[k] = r;
    }
    ok = 8 * (ptr - (int32_t)q) + 64 - (int32_t)used == 0;  // the stream consumed exactly
  }
  if (j == 0) {
    if (ok) {
      // the history after the block (zstd_exec_kernel resolves the next block's offsets)
      h0[kX0 + kXW * bk + kXFin0] = r0 & 0xFFFFFu;
      h0[kX0 + kXW * bk + kXFin1] = r1 & 0xFFFFFu;
      h0[kX0 + kXW * bk + kXFin2] = r2 & 0xFFFFFu;
      // (zstd_hlit_kernel, or the segment's other chains, may mark the segment failed first:
      // a failure overwrites kRecs and is never overwritten)
      atomicCAS(&produced[i], kHanded, kRecs);
    }
    uint32_t was = 0xFFFFFFFFu;
    if (!ok) {
      was = atomicExch(&produced[i], 0xFFFFFFFFu);
      atomicOr(err, 1u);
    }
    if (stats) {  // (per segment: its first block's chain counts it, its first failure rejects it)
      if (bk == 0) atomicAdd(stats + BITAR_HIP_PATH_ZSTD_SEQDEC, 1ull);
      if (!ok && was != 0xFFFFFFFFu) atomicAdd(stats + BITAR_HIP_PATH_ZSTD_SEQDEC_REJECT, 1ull);
    }
  }
}

// ---- phase B -----------------------------------------------------------------------------
// One wave per segment with produced == kRecs: out[kOp, ..) from the records, the literals
// (raw: the frame; RLE: one byte; Huffman: the slot tail, decoded there by zstd_hlit_kernel)
// and the history.  Each batch of 64 records is checked before it runs -- the wave
// decoder's per-sequence rules (literals left, output room for the match and the unread
// literals, 1 <= offset <= output so far) from the batch's prefix sums -- and the frame's
// content size at the end; a failure sets SEGMENT_ERROR and the error word.  The literal
// tail is read ahead of every store: room for the unread literals was checked.
// A block's literals (raw or Huffman) stream through an LDS ring of two 512-B rows, one
// aligned 16-B block per lane of the first 32, the next row held in registers a row of
// literals ahead: a step reads its literal bytes from LDS instead of waiting on HBM (the
// prefetched rows lie at or past the next literal, which no output store has reached: the
// room rule).  1 GiB decode against literal loads from HBM: kind 1 4.08 -> 3.96 ms, kinds
// 2 / 5 equal; 1 KiB rows cost occupancy (6.7 KiB of LDS: 23 waves per CU) and were slower.
#ifndef BITAR_EXEC_LRING
#define BITAR_EXEC_LRING 1
#endif
#ifndef BITAR_EXEC_LROW
#define BITAR_EXEC_LROW 512
#endif
constexpr uint32_t kLRow = BITAR_EXEC_LROW, kLRing = 2 * kLRow;
#ifndef BITAR_EXEC_MARKS
#define BITAR_EXEC_MARKS 1
#endif
__global__ __launch_bounds__(64) void zstd_exec_kernel(
    const uint8_t* const* __restrict__ srcs, const uint8_t* __restrict__ slab,
    uint64_t slot_stride, uint32_t nseg, uint32_t seg, uint8_t* __restrict__ out,
    uint32_t* __restrict__ produced, const uint8_t* __restrict__ hscr,
    const uint64_t* __restrict__ recs, uint32_t rcap, uint32_t* __restrict__ err,
    unsigned long long* __restrict__ stats, const uint32_t* __restrict__ order) {
  using namespace zsq;
  using namespace sr;
  // (a trash byte / word per lane after the ring and the event array: lanes with nothing to
  // store write there instead of branching -- exec-mask changes are scalar instructions, and
  // the scalar unit, shared by the CU's waves, bounds this kernel)
  __shared__ __attribute__((aligned(16))) uint8_t ring[kRing + kWave];
  __shared__ uint32_t ev[2 * kWave];
  __shared__ __attribute__((aligned(16))) uint8_t lring[BITAR_EXEC_LRING ? kLRing : 16];
  if (blockIdx.x >= nseg) return;
  const uint32_t i = order ? order[blockIdx.x] : blockIdx.x;  // (cost-ordered dispatch)
  if (i >= nseg || uniform(produced[i]) != kRecs) return;
  const uint32_t lane = lane_id();
  if (BITAR_EXEC_MARKS) {  // the sequence marks: zero between steps
    ev[lane] = 0u;
    lds_order();
  }
  const GMEM uint32_t* h = global_ptr(reinterpret_cast<const uint32_t*>(hscr + (uint64_t)i * kStride));
  const uint32_t nbk = uniform(h[kNb]), lall = uniform(h[kLitAll]), op0 = uniform(h[kOp]);
  const uint32_t fsz = uniform(h[kFsz]), fcs = uniform(h[kFcs]);
  const uint32_t cap = seg;
  State s;
  s.dst = global_ptr(out + (uint64_t)i * seg);
  s.cap = cap;
  s.op = op0;
  s.flushed = op0;
  s.fenced = op0;  // out[0, op0) was written by an earlier launch
  const GMEM uint8_t* src = global_ptr(srcs ? srcs[i] : slab + (uint64_t)i * slot_stride);
  // Huffman literals: the slot tail [cap - lall, cap), block b's at its kXLit
  const GMEM uint8_t* tail = s.dst + (cap - lall);
  const uintptr_t base = (uintptr_t)s.dst;
  // the history at the current block's start (block 0: the wave decoder's)
  uint32_t R0 = uniform(h[kRep0]), R1 = uniform(h[kRep1]), R2 = uniform(h[kRep2]);
  uint32_t lbase = 0;  // literals of the earlier blocks (for the room check)
  bool ok = true;
  // per block: literal index j -> byte: lsrc[j] (raw / Huffman) or the RLE byte
  uint32_t lt = 0, lbyte = 0;
  // the literal ring: literal index j of the block at lring[(la + j) & (kLRing - 1)] (absolute
  // addressing: an aligned HBM block is an aligned ring block); indices [lF - kLRing, lF) are
  // staged, lnx holds row lrow; lnext = the next literal index a step takes
  uint64_t la = 0, lend = 0;
  const GMEM uint8_t* lsafe = s.dst;  // (BITAR_EXEC_LRING 0: literals read from HBM)
  uint32_t lF = 0, lrow = 0, lnext = 0;
  uint4 lnx = make_uint4(0, 0, 0, 0);
  auto lrow_load = [&](uint32_t r) __attribute__((always_inline)) -> uint4 {
    const uint64_t a = (la & ~15ull) + (uint64_t)kLRow * r + 16u * lane;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (16u * lane < kLRow && a < lend) v = *reinterpret_cast<const GMEM uint4*>(a);
    return v;
  };
  auto lrow_write = [&](uint32_t r, const uint4& v) __attribute__((always_inline)) {
    const uint32_t a = (uint32_t)(la & ~15ull) + kLRow * r + 16u * lane;
    if (16u * lane < kLRow) *reinterpret_cast<uint4*>(lring + (a & (kLRing - 1))) = v;
  };
  // one 64-byte step at output [xa, xa + 64) ∩ [.., xa + act): e = the run each lane lies in
  // (key << 24 | payload: odd key = literals, payload = output pos - literal index; even key
  // = match, payload = offset)
  // (ism: a match byte, from = its source position; else a literal, from = its index)
  auto chunk = [&](uint32_t xa, uint32_t nact, bool ism, uint32_t from) __attribute__((always_inline)) {
    const uint32_t x = xa + lane;
    const bool act = lane < nact;
    // far history (before the ring's reach, or written by the wave decoder): HBM, after a
    // fence over what this wave flushed
    const bool far = act && ism && from < xa && (from < op0 || from + kNearOff < x);
    if (ballot(far && from >= s.fenced)) {
      flush(s, ring, xa, true);
      global_fence_wave();
      s.fenced = s.flushed;
    }
    // every lane loads both candidates (branch-free): its literal byte (index 0 for the
    // others) and its ring byte
    const bool lit = act && !ism;
    if (BITAR_EXEC_LRING && lt != 1 && lnext + kWave > lF) {  // stage the next row (it overwrites row lrow - 2)
      lds_order();
      lrow_write(lrow, lnx);
      lF += kLRow;
      ++lrow;
      lnx = lrow_load(lrow);
    }
    lds_order();
    uint32_t vl;
    if constexpr (BITAR_EXEC_LRING != 0) {
      vl = lt == 1 ? lbyte : (uint32_t)lring[((uint32_t)la + from) & (kLRing - 1)];
      lnext += (uint32_t)__builtin_popcountll(ballot(lit));
    } else {
      vl = lt == 1 ? lbyte : (uint32_t)lsafe[lit ? from : 0u];
    }
    const uint32_t vr = ring[(base + from) & kRingMask];
    uint32_t v = lit ? vl : vr;
    if (ballot(far)) {  // (rare)
      if (far) v = s.dst[from];
    }
    // the pending flag kept as data (0x100 / 0), not as a loop-carried lane mask: a bool
    // updated in a divergent loop costs ~8 scalar mask merges per round
    const bool pend0 = act && ism && from >= xa;
    uint32_t pv = pend0 ? 0x100u : 0u;
    uint32_t ptr = pend0 ? from - xa : lane;
    // sources inside this step: pointer jumping (each round halves the chains)
    while (ballot(pv != 0)) {
      const uint32_t w = v | pv | (ptr << 9);
      const uint32_t t = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(ptr << 2), (int)w);
      const uint32_t still = pv & t;
      v = (pv ^ still) ? t & 0xFFu : v;  // resolved this round
      ptr = still ? t >> 9 : ptr;
      pv = still;
    }
    lds_order();
    ring[act ? (uint32_t)((base + x) & kRingMask) : kRing + lane] = (uint8_t)v;
    lds_order();
  };
  for (uint32_t bk = 0; bk < nbk && ok; ++bk) {
    const GMEM uint32_t* hb = h + blk_at(bk);
    const uint32_t nseq = uniform(hb[kNseq]), w3 = uniform(hb[kAls]), litv = uniform(hb[kLitV]);
    const uint32_t regen = uniform(hb[kRegen]);
    const uint32_t xrec = uniform(h[kX0 + kXW * bk + kXRec]), xlit = uniform(h[kX0 + kXW * bk + kXLit]);
    lt = w3 >> 24;
    lbyte = litv & 0xFFu;
    const GMEM uint8_t* lsrc = lt == 0 ? src + litv : tail + xlit;
    lnext = 0;
    lsafe = regen ? lsrc : s.dst;  // (a literal-less block's lsrc may lie past the buffer)
    if (BITAR_EXEC_LRING && lt != 1) {  // prime the ring with rows 0 and 1, row 2 in registers
      la = (uint64_t)(uintptr_t)lsrc;
      lend = la + regen;  // (no literals: nothing is loaded)
      const uint4 v0 = lrow_load(0), v1 = lrow_load(1);
      lnx = lrow_load(2);
      lds_order();
      lrow_write(0, v0);
      lrow_write(1, v1);
      lrow = 2;
      lF = kLRing - (uint32_t)(la & 15u);
    }
    const GMEM uint64_t* rec = global_ptr(recs + (uint64_t)i * rcap + xrec);
    uint32_t lp = 0;
    // the records of the next 64 sequences are loaded while this batch runs
    uint64_t rn = 0;
    if (nseq) rn = rec[lane < nseq ? lane : nseq - 1];
    for (uint32_t kb = 0; kb < nseq; kb += kWave) {
      const uint32_t n = nseq - kb < kWave ? nseq - kb : kWave;
      const uint64_t r0 = rn;
      if (kb + kWave < nseq) {
        const uint32_t kn = kb + kWave + lane;
        rn = rec[kn < nseq ? kn : nseq - 1];
      }
      const uint64_t r = lane < n ? r0 : 0ull;
      const uint32_t lf = (uint32_t)r & 0x3FFFFFu, mf = (uint32_t)(r >> 22) & 0x3FFFFFu;
      uint32_t lb, lx, mb, mx;
      ll_code(lf >> 16, lb, lx);
      ml_code(mf >> 16, mb, mx);
      const uint32_t ll = lb + (lf & 0xFFFFu), ml = lane < n ? mb + (mf & 0xFFFFu) : 0u;
      // (blocks after the first: offsets relative to the history at the block's start)
      const uint32_t off = resolve_off((uint32_t)(r >> 44), R0, R1, R2);
      const uint32_t inc = wave_incl_sum(ll + ml), ex = inc - (ll + ml);
      const uint32_t linc = wave_incl_sum(ll), lex = linc - ll;
      const uint32_t T = readlane(inc, kWave - 1), LT = readlane(linc, kWave - 1);
      {
        const uint32_t lpk = lp + lex, opk = s.op + ex;  // before sequence k
        // (room: the output of the match and every unread literal of this and later blocks,
        // which the slot tail holds)
        const bool bad = (lpk + ll > regen) | (opk + ml + (lall - lbase - lpk) > cap) |
                         (off == 0) | (off > opk + ll);
        if (ballot(lane < n && bad)) {
          ok = false;
          break;
        }
      }
#if BITAR_EXEC_MARKS
      // Each output byte finds its sequence as the compressors' gathers do: every sequence
      // (>= 3 bytes: its first byte is its own) stores its u (batch byte index + 1) into the
      // mark of its first byte, the byte's lane reads and clears its mark, one compare gives
      // the step's start mask, the sequence is a scalar base + v_mbcnt, and three ds_bpermute
      // fetch its first match byte, literal-index delta and offset.  (Was: the starts of its
      // literal run and its match scattered to LDS events, a DPP prefix max, a carry.)
      const bool live = lane < n;
      const uint32_t a4 = live ? ex << 2 : 0x7FFFFF00u;  // mark slot x4 (others: the trash)
      const uint32_t mark = ex + 1u;
      const uint32_t T1 = ex + ll;                         // first match byte (batch index)
      const uint32_t D = (lp + lex) - ex;                  // literal index = batch index + D
      const uint32_t zero = 0;
      uint32_t before = 0xFFFFFFFFu;  // sequences started before the step, less one
      for (uint32_t cb = 0; cb < T; cb += kWave) {
        const uint32_t xa = s.op + cb;
        if (xa + kWave - s.flushed > kFlushAt) flush(s, ring, xa, false);
        lds_order();
        const uint32_t slot = min(a4 - (cb << 2), (uint32_t)kWave << 2);
        *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(ev) + slot) = mark;
        lds_order();
        const uint32_t b = cb + lane;  // batch byte index
        const uint32_t mk = ev[lane];
        ev[lane] = zero;
        const uint64_t S = ballot(mk == b + 1u);
        const uint32_t base = before + (uint32_t)(S & 1u);
        const uint64_t S1 = S >> 1;
        const uint32_t k = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(S1 >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)S1, 0u));
        before += (uint32_t)__builtin_popcountll(S);
        const int src4 = (int)(k << 2);
        const uint32_t qT1 = (uint32_t)__builtin_amdgcn_ds_bpermute(src4, (int)T1);
        const uint32_t qD = (uint32_t)__builtin_amdgcn_ds_bpermute(src4, (int)D);
        const uint32_t qoff = (uint32_t)__builtin_amdgcn_ds_bpermute(src4, (int)off);
        const bool ism = b >= qT1;
        chunk(xa, T - cb < kWave ? T - cb : kWave, ism, ism ? xa + lane - qoff : b + qD);
      }
#else
      const uint32_t e_lit = ((2u * lane + 1u) << 24) | ((s.op + ex) - (lp + lex));
      const uint32_t e_mat = ((2u * lane + 2u) << 24) | off;
      uint32_t carry = 0;
      for (uint32_t cb = 0; cb < T; cb += kWave) {
        const uint32_t xa = s.op + cb;
        if (xa + kWave - s.flushed > kFlushAt) flush(s, ring, xa, false);
        lds_order();
        ev[lane] = 0u;
        lds_order();
        const uint32_t p1 = ex - cb, p2 = ex + ll - cb;
        ev[lane < n && ll && p1 < kWave ? p1 : kWave + lane] = e_lit;
        ev[lane < n && p2 < kWave ? p2 : kWave + lane] = e_mat;
        lds_order();
        uint32_t e = ev[lane];
        e = wave_incl_max(e > carry ? e : carry);
        carry = readlane(e, kWave - 1);
        chunk(xa, T - cb < kWave ? T - cb : kWave, ((e >> 24) & 1u) == 0, xa + lane - (e & 0xFFFFFFu));
      }
#endif
      s.op += T;
      lp += LT;
    }
    // the literals after the block's last sequence
    const uint32_t rest = ok ? regen - lp : 0u;
    if (ok && (uint64_t)s.op + (lall - lbase - lp) > cap) ok = false;
    for (uint32_t cb = 0; ok && cb < rest; cb += kWave) {
      const uint32_t xa = s.op + cb;
      if (xa + kWave - s.flushed > kFlushAt) flush(s, ring, xa, false);
      chunk(xa, rest - cb < kWave ? rest - cb : kWave, false, xa + lane - (s.op - lp));
    }
    if (ok) s.op += rest;
    lbase += regen;
    // the history at the next block's start
    const uint32_t f0 = uniform(h[kX0 + kXW * bk + kXFin0]), f1 = uniform(h[kX0 + kXW * bk + kXFin1]),
                   f2 = uniform(h[kX0 + kXW * bk + kXFin2]);
    const uint32_t n0 = resolve_off(f0, R0, R1, R2), n1 = resolve_off(f1, R0, R1, R2),
                   n2 = resolve_off(f2, R0, R1, R2);
    R0 = n0;
    R1 = n1;
    R2 = n2;
  }
  flush(s, ring, s.op, true);
  ok = ok && (!fsz || fcs == s.op);
  if (lane == 0) {
    if (ok) {
      produced[i] = s.op;
    } else {
      produced[i] = 0xFFFFFFFFu;
      atomicOr(err, 1u);
    }
    if (stats) {
      atomicAdd(stats + BITAR_HIP_PATH_ZSTD_EXEC, 1ull);
      if (!ok) atomicAdd(stats + BITAR_HIP_PATH_ZSTD_EXEC_REJECT, 1ull);
    }
  }
}

// Dispatch keys of the multi-block lane kernels (order.hip.h: lower keys first): which = 0
// the segment's sequences (zstd_seqdec_kernel<4, 4>'s chains), 1 its literals
// (zstd_hlit_kernel<4, 4>'s streams); segments they do not take sort last.
__global__ __launch_bounds__(64) void hand_key_kernel(const uint32_t* __restrict__ produced,
                                                      const uint8_t* __restrict__ hscr,
                                                      uint32_t nseg, uint32_t which,
                                                      uint32_t* __restrict__ keys) {
  using namespace zhand;
  // (keys of the 2 nseg units: unit u = blocks 4 (u & 1) .. of segment u >> 1, each unit of
  // an 8-block frame about half of the frame's work)
  const uint32_t u = blockIdx.x * kWave + lane_id(), i = u >> 1;
  if (u >= 2 * nseg) return;
  uint32_t c = 0;
  if (produced[i] == kHanded) {
    const GMEM uint32_t* h = global_ptr(reinterpret_cast<const uint32_t*>(hscr + (uint64_t)i * kStride));
    const uint32_t nb = h[kNb], sh = nb > kUnitBlocks ? 1u : 0u;
    if (nb >= 2u && kUnitBlocks * (u & 1u) < nb)
      c = 1u + ((which ? h[kLitAll] >> 8 : h[kNseqAll] >> 7) >> sh);
  }
  keys[u] = kOrderBins - 1u - (c < kOrderBins - 1u ? c : kOrderBins - 1u);
}

#define BITAR_SEQDEC_INST(L, B)                                                              \
  template __global__ void zstd_seqdec_kernel<L, B>(const uint8_t* const*, const uint8_t*,     \
                                                    uint64_t, const uint32_t*, uint32_t,       \
                                                    uint32_t, uint32_t*, uint8_t*, uint64_t*,  \
                                                    uint32_t, uint32_t*, unsigned long long*,  \
                                                    const uint32_t*);
BITAR_SEQDEC_INST(16, 1)
BITAR_SEQDEC_INST(8, 1)
BITAR_SEQDEC_INST(4, 1)
BITAR_SEQDEC_INST(4, 4)
#undef BITAR_SEQDEC_INST

}  // namespace bitar_hip
