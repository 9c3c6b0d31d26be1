// deflate_dyn.hip -- raw DEFLATE with DYNAMIC Huffman codes per segment (gfx950): the
// reference's default frame (RTE_COMP_HUFFMAN_DYNAMIC, reference src/include/config.h:151;
// accepted by the BlueField device, src/device.cc:566-574).  Restated exactly by the oracle's
// bo_deflate_dynamic_block (oracle/bitar_deflate_dyn.c); the GPU output must match it byte for
// byte.
//
// Two launches, one wavefront per segment each, through a scratch area of
// kPlanBytes + slot_stride bytes per segment:
//   deflate_dyn_parse_kernel  the window-scan parse of window_parse.hip.h with a "record"
//                             emitter: per window of 64 positions, the 8-byte chain mask of
//                             selected matches + one u32 (length | distance << 16) per match,
//                             staged in LDS and flushed with 16-B stores; literal/length and
//                             distance histograms counted with LDS atomics.
//   deflate_dyn_emit_kernel   builds the codes from the histograms (length-limited Huffman,
//                             code-length RLE, code-length code), sizes the dynamic / fixed /
//                             stored alternatives and writes the smallest: per window every
//                             lane places its literal code or whole match symbol (up to 45 bits)
//                             by a prefix sum of bit lengths into an LDS bit ring, from the
//                             records and the input bytes.
// The parse (the expensive part, ~250 instructions per window) runs once; the emit pass is
// a streaming read of records + input and write of the stream.
#include "huffman.hip.h"
#include "window_parse.hip.h"

namespace bitar_hip {

namespace dyn {

using namespace cmp;

#ifndef BITAR_DYN_VARIANT
#define BITAR_DYN_VARIANT 0  // timing experiments only (scripts/build_variant.sh)
#endif

constexpr uint32_t kPlanBytes = 2048;  // per segment: histograms + record count
constexpr uint32_t kNLit = 286, kNDist = 30, kNCl = 19;
constexpr uint32_t kPlanRecBytes = kNLit + kNDist;  // word index of the record byte count

__device__ __forceinline__ uint32_t len_sym(uint32_t mlen, uint32_t& nx, uint32_t& xv) {
  // RFC 1951 3.2.5, branch-free (mlen in [3, 258])
  const uint32_t v = mlen - 3;
  const uint32_t lev = 29u - __builtin_clz(v | 8u);  // floor(log2 v) - 2 for v >= 8
  nx = mlen == 258 || v < 8 ? 0u : lev;
  xv = v & ((1u << nx) - 1);
  return mlen == 258 ? 28u : v < 8 ? v : 4 * lev + 4 + ((v >> lev) & 3u);
}
__device__ __forceinline__ uint32_t dist_sym(uint32_t off, uint32_t& nx, uint32_t& xv) {
  const uint32_t d = off - 1;
  const uint32_t dev = 30u - __builtin_clz(d | 4u);  // floor(log2 d) - 1 for d >= 4
  nx = d < 4 ? 0u : dev;
  xv = d & ((1u << nx) - 1);
  return d < 4 ? d : 2 * dev + 2 + ((d >> dev) & 1u);
}
__device__ __forceinline__ uint32_t len_extra_bits(uint32_t ls) {  // kLenExtra[ls]
  return ls < 8 || ls == 28 ? 0u : (ls - 4) >> 2;
}
__device__ __forceinline__ uint32_t dist_extra_bits(uint32_t ds) {  // kDistExtra[ds]
  return ds < 4 ? 0u : (ds - 2) >> 1;
}
// transmission order of the code-length code's lengths (RFC 1951 3.2.7)
__constant__ uint8_t kClo[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

__device__ __forceinline__ uint32_t fixed_len(uint32_t s) {
  return s < 144 ? 8u : s < 256 ? 9u : s < 280 ? 7u : 8u;
}

// ---- pass 1: records + histograms ---------------------------------------------------------
// Scratch per segment: [plan kPlanBytes][window masks kMaskBytes][match records ...].
// Window w: 16 B = the lanes that start a selected match (u64) + the lanes that emit a
// literal (u64); match k of the segment: one u32 = length symbol - 257 (5 bits) | its extra
// bits (5) | distance symbol (5) | its extra bits (<= 10) -- the emit pass needs neither the
// parse's coverage rule nor the symbol arithmetic again.
[[maybe_unused]] constexpr uint32_t kMaskBytes = 16384;  // <= 1024 windows (n <= 65536)
constexpr uint32_t kPlanWindows = kPlanRecBytes + 1;  // word index of the window count
constexpr uint32_t kPlanTail = kPlanRecBytes + 2;     // word index of the tail start

// (a 512-B byte ring and a 32-window mask ring: 8.4 KiB of LDS, 19 waves per CU instead of
// 17 -- the parse is latency-bound; a row of input adds <= 16 windows between drains)
constexpr uint32_t kRecBuf = 512, kMaskRing = 32;
struct RecOut : ByteOutT<kRecBuf> {  // the byte ring carries the match records
  uint32_t* lh;          // LDS literal/length histogram (286)
  uint32_t* dh;          // LDS distance histogram (30)
  uint4* cst;            // LDS ring of kMaskRing window mask pairs
  GMEM uint4* cdst;      // mask area
  uint32_t nwin, cflushed;

  __device__ __forceinline__ void window(const GMEM uint8_t*, const InRing&, const Window& W,
                                         uint32_t, uint32_t n) {
    const uint32_t lane = lane_id();
    const uint32_t q = W.x + lane;
    const bool cl = (W.chain >> lane) & 1;
    const uint32_t pend = wave_incl_max(cl ? q + W.mlen : 0u);
    const bool covered = q < W.pos_in || (!cl && q < pend);
    const bool lit = !cl && !covered && q < n;
    const uint64_t litm = ballot(lit);
    uint32_t lnx, lxv, dnx, dxv;
    const uint32_t ls = len_sym(cl ? W.mlen : 3u, lnx, lxv);
    const uint32_t ds = dist_sym(cl ? W.off() : 1u, dnx, dxv);
    lds_order();
    if (lit) atomicAdd(&lh[W.byte], 1u);
    if (cl) {
      atomicAdd(&lh[257 + ls], 1u);
      atomicAdd(&dh[ds], 1u);
    }
    if (lane == 0)
      cst[nwin & (kMaskRing - 1)] = make_uint4((uint32_t)W.chain, (uint32_t)(W.chain >> 32), (uint32_t)litm,
                                   (uint32_t)(litm >> 32));
    lds_order();
    ++nwin;
    if (overflow || !W.chain) return;
    const uint32_t nm = (uint32_t)__builtin_popcountll(W.chain);
    if (!room(4 * nm)) return;
    const uint32_t rank = (uint32_t)__builtin_popcountll(W.chain & ((1ull << lane) - 1));
    uint32_t* r32 = reinterpret_cast<uint32_t*>(ring);
    lds_order();
    if (cl) r32[at(op + 4 * rank) >> 2] = ls | (lxv << 5) | (ds << 10) | (dxv << 15);
    lds_order();
    op += 4 * nm;
  }
  // window masks [cflushed, upto) to HBM, one window (16 B) per lane
  __device__ __forceinline__ void flush_masks(uint32_t upto) {
    const uint32_t lane = lane_id();
    lds_order();
    for (uint32_t w = cflushed + lane; w < upto; w += kWave) cdst[w] = cst[w & (kMaskRing - 1)];
    cflushed = upto;
  }
  __device__ __forceinline__ void drain() {
    ByteOutT<kRecBuf>::drain();
    flush_masks(nwin);
  }
  // the tail literals [s, s + n)
  __device__ __forceinline__ void sequence(const GMEM uint8_t* in, const InRing& I, uint32_t s,
                                           uint32_t n, uint32_t, uint32_t) {
    const uint32_t lane = lane_id();
    const bool ring_ok = s >= I.lo;
    for (uint32_t k = 0; k < n; k += kWave) {
      const uint32_t step = n - k < kWave ? n - k : kWave;
      const uint32_t q = s + k + (lane < step ? lane : 0);
      lds_order();
      const uint32_t b = ring_ok ? I.byte(q) : (uint32_t)in[q];
      if (lane < step) atomicAdd(&lh[b], 1u);
      lds_order();
    }
  }
  __device__ __forceinline__ void between(const GMEM uint8_t*, const InRing&) {}
  __device__ __forceinline__ uint32_t pending_from(uint32_t, uint32_t emitted) const { return emitted; }
};

#ifndef BITAR_DYN_BULK
#define BITAR_DYN_BULK 1
#endif
#if BITAR_DYN_BULK
// Batched pass 1 (as the LZ4 / Zstd collectors): a window only appends its matches {start |
// distance - 1 << 16, length} to an LDS list (~6 VALU instead of the per-window symbol
// arithmetic, prefix max and mask pair); every <= 48 records -- and whenever the oldest pending
// literal is 1 KiB behind the scan, so literal runs stay in the input ring -- one flush writes
// the records to the record area with one coalesced store, counts their length and distance
// symbols (one lane per record), and gathers their literal runs 64 bytes per step (the LZ4
// gather: start marks, one compare, v_mbcnt) into the literal histogram AND the literal area,
// in position order.  Pass 2 then reads records and a contiguous literal stream, never the
// input.  Scratch per segment: [plan kPlanBytes][literals: lit_cap(seg)][records: 8 B each].
constexpr uint32_t kDynCap = 64;     // records per flush (a window adds <= 16)
#ifndef BITAR_DYN_OBUF
#define BITAR_DYN_OBUF 512
#endif
constexpr uint32_t kDynObuf = BITAR_DYN_OBUF;   // literal staging ring
constexpr uint32_t kDynGap = 1024;   // flush once the oldest pending literal is this far behind
__host__ __device__ constexpr uint32_t lit_cap(uint32_t seg) { return (seg + 15u) & ~15u; }
struct DynLds {
  uint8_t ring[kDynObuf];
  uint2 recs[kDynCap + 1];     // + a trash record
  uint32_t marks[kWave + 1];   // zero between steps; + trash
};
struct DynCollect : ByteOutT<kDynObuf> {
  DynLds* L;
  uint32_t* lh;          // LDS literal/length histogram (286)
  uint32_t* dh;          // LDS distance histogram (30)
  GMEM uint2* seqs;      // record area
  uint32_t nseq, rec_cap, npend;
  uint32_t last_end;     // literals before it are in the literal area
  uint32_t x_seen;       // positions below it are decided (literal or inside a match)

  // literal bytes [s, s + len): counted and appended, 64 per step (from the input ring when
  // it holds them, else from HBM)
  __device__ __forceinline__ void lit_run(const GMEM uint8_t* in, const InRing& I, uint32_t s,
                                          uint32_t len) {
    const uint32_t lane = lane_id();
    for (uint32_t k = 0; k < len && !overflow; k += kWave) {
      const uint32_t step = len - k < kWave ? len - k : kWave;
      if (!room(step)) return;
      const uint32_t q = s + k + (lane < step ? lane : 0u);
      lds_order();
      const uint32_t b = s + k >= I.lo ? I.byte(q) : (uint32_t)in[q];
      if (lane < step) atomicAdd(&lh[b], 1u);
      put(b, step);
    }
  }
  // the literal runs of record lanes [lo, hi) (all in the input ring), 64 bytes per step
  __device__ __forceinline__ void gather(const InRing& I, uint32_t lo, uint32_t hi,
                                         uint32_t lit_start, uint32_t ll) {
    const uint32_t lane = lane_id();
    const bool ne = (lane >= lo) & (lane < hi) & (ll != 0u);
    const uint32_t e = ne ? ll : 0u;
    const uint32_t incl = wave_incl_sum(e);
    const uint32_t total = readlane(incl, kWave - 1);
    if (!total) return;
    if ((uint64_t)op + total > cap) { overflow = true; return; }
    const uint32_t a = incl - e;  // the run's first literal, in the batch's literals
    // the non-empty runs' ring offsets (ring index of a literal = D + u), compacted by rank
    const uint64_t nem = ballot(ne);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(nem >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)nem, 0u));
    const uint32_t D = I.in_lo + lit_start - a - 1u;
    lds_order();
    uint32_t* tmp = reinterpret_cast<uint32_t*>(L->recs);  // (the records are in registers)
    tmp[ne ? rank : kWave] = D;
    lds_order();
    const uint32_t Dc = tmp[lane];
    const uint32_t a4 = ne ? a << 2 : 0x7FFFFF00u;  // mark slot x4 (others: the trash slot)
    const uint32_t mark = a + 1u;
    const uint32_t zero = 0;
    const uint32_t rbase = (uint32_t)(uintptr_t)dst + op - 1u;  // ring index = rbase + u
    uint32_t u = lane + 1u;
    uint32_t before = 0;  // non-empty runs starting before the step
    lds_order();
    for (uint32_t R = 0; R < total; R += kWave) {
      if (op + kWave - flushed > kDynObuf - 64) flush(op, false);
      lds_order();
      const uint32_t slot = min(a4 - (R << 2), (uint32_t)kWave << 2);
      *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(L->marks) + slot) = mark;
      lds_order();
      const uint32_t mk = L->marks[lane];
      L->marks[lane] = zero;
      const uint64_t S = ballot(mk == u);
      const uint32_t base = before - 1u + (uint32_t)(S & 1u);
      const uint64_t S1 = S >> 1;
      const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(S1 >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)S1, 0u));
      before += (uint32_t)__builtin_popcountll(S);
      const uint32_t d = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((k << 2) + (base << 2)),
                                                                (int)Dc);
      const uint32_t b = I.ring[(d + u) & I.mask];
      const uint32_t nb = total - R < kWave ? total - R : kWave;
      if (lane < nb) atomicAdd(&lh[b], 1u);
      // all 64 bytes are written: those past nb lie at or past the new op, inside the room
      // just made, and are rewritten before they are flushed
      ring[(rbase + u) & kMask] = (uint8_t)b;
      lds_order();
      op += nb;
      u += kWave;
    }
  }
  // every pending record: to the record area, its symbols counted, its literal run gathered;
  // then the literals up to x_seen
  __device__ __forceinline__ void flush_seqs(const GMEM uint8_t* in, const InRing& I) {
    const uint32_t cnt = npend;
    npend = 0;
    if (overflow) return;
    const uint32_t lane = lane_id();
    if (cnt) {
      lds_order();
      const uint2 rec = L->recs[lane < cnt ? lane : kDynCap];
      const uint32_t q = rec.x & 0xFFFFu, off = (rec.x >> 16) + 1u, mlen = rec.y;
      const uint32_t end = q + mlen;
      const uint32_t prev = wave_shr1(end);
      const uint32_t lit_start = lane == 0 ? last_end : prev;
      const uint32_t ll = q - lit_start;
      last_end = readlane(end, cnt - 1);
      if (nseq + cnt > rec_cap) { overflow = true; return; }
      if (lane < cnt) seqs[nseq + lane] = rec;
      nseq += cnt;
      uint32_t lnx, lxv, dnx, dxv;
      const uint32_t ls = len_sym(lane < cnt ? mlen : 3u, lnx, lxv);
      const uint32_t ds = dist_sym(lane < cnt ? off : 1u, dnx, dxv);
      lds_order();
      if (lane < cnt) {
        atomicAdd(&lh[257 + ls], 1u);
        atomicAdd(&dh[ds], 1u);
      }
      lds_order();
      const uint64_t live = cnt < kWave ? (1ull << cnt) - 1 : ~0ull;
      uint64_t special = ballot(lit_start < I.lo) & ballot(ll != 0u) & live;
      uint32_t lo = 0;
      for (;;) {
        const uint32_t k = special ? (uint32_t)__builtin_ctzll(special) : cnt;
        if (k > lo) gather(I, lo, k, lit_start, ll);
        if (k >= cnt || overflow) break;
        lit_run(in, I, readlane(lit_start, k), readlane(ll, k));
        special &= special - 1;
        lo = k + 1;
      }
    }
    if (x_seen > last_end && !overflow) {
      lit_run(in, I, last_end, x_seen - last_end);
      last_end = x_seen;
    }
  }
  __device__ __forceinline__ void between(const GMEM uint8_t* in, const InRing& I) {
    if (npend > kDynCap - 16 || x_seen > last_end + kDynGap) flush_seqs(in, I);
  }
  // the tail: everything pending, then the literals to the segment's end (matches end >= 5
  // bytes before it, so this always runs)
  __device__ __forceinline__ void sequence(const GMEM uint8_t* in, const InRing& I, uint32_t s,
                                           uint32_t len, uint32_t, uint32_t) {
    x_seen = s + len;  // (the segment's end)
    flush_seqs(in, I);
  }
  __device__ __forceinline__ uint32_t pending_from(uint32_t anchor, uint32_t) const { return anchor; }
  __device__ __forceinline__ void window(const GMEM uint8_t*, const InRing&, const Window& W,
                                         uint32_t, uint32_t n) {
    x_seen = W.x + kWave < n ? W.x + kWave : n;
    if (!W.chain) return;
    const uint64_t chain = W.chain;
    const uint32_t lane = lane_id();
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(chain >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)chain, 0u));
    lds_order();
    L->recs[(chain >> lane) & 1u ? npend + rank : kDynCap] =
        make_uint2((W.x + lane) | (W.dm1 << 16), W.mlen);
    lds_order();
    npend += (uint32_t)__builtin_popcountll(chain);
  }
};
#endif

// ---- code construction (restated by oracle/bitar_deflate_dyn.c) --------------------------
using huf::TreeLds;
using huf::huff_lengths;

// canonical codes (RFC 1951 3.2.2), bit-reversed: tab[s] = code | len << 16.  Lane-parallel:
// a symbol's code = first code of its length + the number of earlier symbols of that length
// (ballots per 64-symbol chunk, counts carried per length).
__device__ void canon_codes(const uint8_t* lens, uint32_t n, uint32_t* tab) {
  const uint32_t lane = lane_id();
  const uint64_t lt = (1ull << lane) - 1;
  uint32_t cnt[16];  // per length: symbols so far (uniform)
#pragma unroll
  for (int b = 0; b < 16; ++b) cnt[b] = 0;
  lds_order();
  for (uint32_t s0 = 0; s0 < n; s0 += kWave) {
    const uint32_t s = s0 + lane;
    const uint32_t l = s < n ? lens[s] : 0u;
#pragma unroll
    for (int b = 1; b < 16; ++b) cnt[b] += (uint32_t)__builtin_popcountll(ballot(l == (uint32_t)b));
  }
  uint32_t first[16];
  uint32_t code = 0;
  first[0] = 0;
#pragma unroll
  for (int b = 1; b < 16; ++b) {
    code = (code + (b > 1 ? cnt[b - 1] : 0u)) << 1;
    first[b] = code;
    cnt[b - 1] = 0;
  }
  cnt[15] = 0;
  for (uint32_t s0 = 0; s0 < n; s0 += kWave) {
    const uint32_t s = s0 + lane;
    const uint32_t l = s < n ? lens[s] : 0u;
    uint32_t c = 0;
#pragma unroll
    for (int b = 1; b < 16; ++b) {
      const uint64_t m = ballot(l == (uint32_t)b);
      c = l == (uint32_t)b ? first[b] + cnt[b] + (uint32_t)__builtin_popcountll(m & lt) : c;
      cnt[b] += (uint32_t)__builtin_popcountll(m);
    }
    if (s < n) tab[s] = (l ? __builtin_bitreverse32(c) >> (32 - l) : 0u) | (l << 16);
  }
  lds_order();
}

// zlib send_tree: RLE of lens[0..n) into (symbol | extra << 8); returns the count
__device__ uint32_t rle_lens(const uint8_t* lens, uint32_t n, uint16_t* out) {
  uint32_t k = 0;
  int prevlen = -1, count = 0, max_count = 7, min_count = 4;
  int nextlen = lens[0];
  if (nextlen == 0) { max_count = 138; min_count = 3; }
  for (uint32_t i = 0; i < n; ++i) {
    const int curlen = nextlen;
    nextlen = i + 1 < n ? (int)lens[i + 1] : 0xFFFF;
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

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) { return readlane(wave_incl_sum(v), 63); }

// ---- pass 2 output: LDS bit ring of 64-bit lane contributions -----------------------------
constexpr uint32_t kB = 4;  // windows per emit step
constexpr uint32_t kStageWords = 512, kStageMask = kStageWords - 1;
// one window adds <= 64 lanes x 45 bits = 90 words (+2 for the spill)
constexpr uint32_t kFlushMargin = kB * 92 + 8;

struct BitOut {
  uint32_t* stage;     // LDS, zero outside the pending range
  GMEM uint32_t* dst;  // slot (16-B aligned)
  uint64_t cap;        // bytes
  uint64_t bits;
  uint32_t wflushed;
  bool overflow;

  __device__ __forceinline__ void flush_words(uint32_t upto) {
    const uint32_t lane = lane_id();
    lds_order();
    for (uint32_t w = wflushed + lane; w < upto; w += kWave) {
      dst[w] = stage[w & kStageMask];
      stage[w & kStageMask] = 0;
    }
    lds_order();
    wflushed = upto;
  }
  __device__ __forceinline__ void or3(uint64_t bp, uint64_t val, uint32_t nb) {
    const uint32_t w = (uint32_t)(bp >> 5), sh = (uint32_t)(bp & 31);
    const uint64_t lo = val << sh;
    const uint32_t w2 = sh && sh + nb > 64 ? (uint32_t)(val >> (64 - sh)) : 0u;
    // only the lanes with bits for a word take part in its atomic: the lanes of one word
    // serialize on its LDS address, zero contributions included (PMC: LDS bank-conflict
    // cycles of the emit kernel 1.18 G -> 0.08 G per GiB; compress 12.2 -> 9.1 ms, kind 1)
    if (nb) atomicOr(&stage[w & kStageMask], (uint32_t)lo);
    if (sh + nb > 32) atomicOr(&stage[(w + 1) & kStageMask], (uint32_t)(lo >> 32));
    if (sh + nb > 64) atomicOr(&stage[(w + 2) & kStageMask], w2);
  }
  // append each lane's (val, nb) in lane order, nb <= 64
  __device__ __forceinline__ void put(uint64_t val, uint32_t nb) {
    if (overflow) return;
    const uint32_t incl = wave_incl_sum(nb);
    const uint32_t total = readlane(incl, 63);
    if ((bits + total + 7) / 8 > cap) { overflow = true; return; }
    lds_order();
    or3(bits + incl - nb, val, nb);
    lds_order();
    bits += total;
    const uint32_t full = (uint32_t)(bits >> 5);
    if (full - wflushed >= kStageWords - kFlushMargin) flush_words(full);
  }
  // kB windows at once: window k's lanes follow window k-1's (independent prefix sums)
  __device__ __forceinline__ void put_multi(const uint64_t* val, const uint32_t* nb) {
    if (overflow) return;
    uint32_t incl[kB], total = 0;
#pragma unroll
    for (uint32_t k = 0; k < kB; ++k) incl[k] = wave_incl_sum(nb[k]);
    uint64_t base[kB];
#pragma unroll
    for (uint32_t k = 0; k < kB; ++k) {
      base[k] = bits + total;
      total += readlane(incl[k], 63);
    }
    if ((bits + total + 7) / 8 > cap) { overflow = true; return; }
    lds_order();
#pragma unroll
    for (uint32_t k = 0; k < kB; ++k) or3(base[k] + incl[k] - nb[k], val[k], nb[k]);
    lds_order();
    bits += total;
    const uint32_t full = (uint32_t)(bits >> 5);
    if (full - wflushed >= kStageWords - kFlushMargin) flush_words(full);
  }
};

// A global byte range streamed through an LDS ring of two rows of RB bytes (RB = 1024: 16 B
// per lane, 512: 8 B), the next row prefetched into registers a whole row ahead: the emit
// pass's per-window reads are LDS reads, never a dependent HBM round trip.  Byte k of the
// range (relative to its 16-B aligned base) lives at ring[k & (2 RB - 1)] once ensure(k + 1)
// has run.
template <uint32_t RB>
struct RowRing {
  using V = typename std::conditional<RB == 1024, uint4, uint2>::type;
  static constexpr uint32_t kPer = RB / 64, kMask = 2 * RB - 1;
  const GMEM V* srcv;  // the range's aligned base
  uint32_t limit;      // bytes readable from it (blocks at or past it are not loaded)
  uint8_t* ring;       // 2 RB bytes of LDS
  uint32_t loaded;     // [0, loaded) committed; the ring holds [loaded - 2 RB, loaded)
  V nxt;               // the next row, in flight

  __device__ __forceinline__ V load_row(uint32_t r) const {
    const uint32_t o = RB * r + kPer * lane_id();
    V v{};
    if (o < limit) v = srcv[o / kPer];
    return v;
  }
  __device__ __forceinline__ void init(const GMEM uint4* base, uint32_t lim, uint8_t* lds) {
    srcv = reinterpret_cast<const GMEM V*>(base);
    limit = lim;
    ring = lds;
    loaded = 0;
    nxt = load_row(0);
  }
  __device__ __forceinline__ void ensure(uint32_t end) {
    while (loaded < end) {
      const uint32_t r = loaded / RB;
      lds_order();
      reinterpret_cast<V*>(ring)[((r & 1u) << 6) + lane_id()] = nxt;
      lds_order();
      loaded += RB;
      nxt = load_row(r + 1);
    }
  }
  __device__ __forceinline__ uint32_t byte(uint32_t k) const { return ring[k & kMask]; }
  __device__ __forceinline__ uint32_t word(uint32_t k) const {  // k 4-aligned
    return reinterpret_cast<const uint32_t*>(ring)[(k & kMask) >> 2];
  }
};

}  // namespace dyn

__global__ __launch_bounds__(64) void deflate_dyn_parse_kernel(
    const uint8_t* __restrict__ input, uint64_t n_total, uint32_t seg,
    uint8_t* __restrict__ scratch, uint64_t scr_stride, uint32_t* __restrict__ err, const uint32_t* __restrict__ order) {
  using namespace dyn;
  __shared__ __attribute__((aligned(16))) uint16_t table[1u << kHashLog];
  __shared__ __attribute__((aligned(16))) uint8_t inring[kIn + kInPad];
  __shared__ uint32_t hist[kNLit + kNDist];
#if BITAR_DYN_BULK
  __shared__ __attribute__((aligned(16))) DynLds dl;
#else
  __shared__ __attribute__((aligned(16))) uint8_t obuf[kRecBuf + kWave];
  __shared__ __attribute__((aligned(16))) uint4 cst[kMaskRing];
#endif
  const uint32_t i_seg = order ? order[blockIdx.x] : blockIdx.x;  // (cost-ordered dispatch)
  const uint64_t seg_off = (uint64_t)i_seg * seg;
  if (seg_off >= n_total) return;
  const uint32_t n = (uint32_t)((n_total - seg_off) < seg ? (n_total - seg_off) : seg);
  for (uint32_t k = lane_id(); k < kNLit + kNDist; k += kWave) hist[k] = 0;
  GMEM uint8_t* scr = global_ptr(scratch + (uint64_t)i_seg * scr_stride);
#if BITAR_DYN_BULK
  DynCollect o;
  o.L = &dl;
  o.ring = dl.ring;
  o.dst = scr + kPlanBytes;
  o.cap = lit_cap(seg);
  o.op = 0;
  o.flushed = 0;
  o.overflow = false;
  o.lh = hist;
  o.dh = hist + kNLit;
  o.seqs = reinterpret_cast<GMEM uint2*>(scr + kPlanBytes + lit_cap(seg));
  o.rec_cap = (uint32_t)((scr_stride - kPlanBytes - lit_cap(seg)) / 8u);
  o.nseq = 0;
  o.npend = 0;
  o.last_end = 0;
  o.x_seen = 0;
  dl.marks[lane_id()] = 0;
  lds_order();
  parse(global_ptr(input + seg_off), n, global_ptr(input + n_total), table, inring, kMaxDist,
        258u, o);
  o.flush(o.op, true);
  lds_order();
  GMEM uint32_t* plan = reinterpret_cast<GMEM uint32_t*>(scr);
  for (uint32_t k = lane_id(); k < kNLit + kNDist; k += kWave) plan[k] = hist[k];
  if (lane_id() == 0) {
    plan[kPlanRecBytes] = o.overflow ? 0xFFFFFFFFu : o.nseq;  // (bulk: the record count)
    plan[kPlanWindows] = o.op;                                  // (bulk: the literal count)
    plan[kPlanTail] = o.last_end;
  }
  if (o.overflow && lane_id() == 0) atomicOr(err, 2u);
#else
  RecOut o;
  o.ring = obuf;
  o.dst = scr + kPlanBytes + kMaskBytes;
  o.cap = scr_stride - kPlanBytes - kMaskBytes;
  o.op = 0;
  o.flushed = 0;
  o.overflow = false;
  o.lh = hist;
  o.dh = hist + kNLit;
  o.cst = cst;
  o.cdst = reinterpret_cast<GMEM uint4*>(scr + kPlanBytes);
  o.nwin = 0;
  o.cflushed = 0;
  const uint32_t tail = parse(global_ptr(input + seg_off), n, global_ptr(input + n_total), table,
                             inring, kMaxDist, 258u, o);
  o.flush(o.op, true);
  o.flush_masks(o.nwin);
  lds_order();
  GMEM uint32_t* plan = reinterpret_cast<GMEM uint32_t*>(scr);
  for (uint32_t k = lane_id(); k < kNLit + kNDist; k += kWave) plan[k] = hist[k];
  if (lane_id() == 0) {
    plan[kPlanRecBytes] = o.overflow ? 0xFFFFFFFFu : o.op;
    plan[kPlanWindows] = o.nwin;
    plan[kPlanTail] = tail;
  }
  if (o.overflow && lane_id() == 0) atomicOr(err, 2u);
#endif
}

__global__ __launch_bounds__(64) void deflate_dyn_emit_kernel(
    const uint8_t* __restrict__ input, uint64_t n_total, uint32_t seg,
    const uint8_t* __restrict__ scratch, uint64_t scr_stride, uint8_t* __restrict__ slab,
    uint64_t slot_stride, uint8_t* const* __restrict__ dsts, uint32_t* __restrict__ sizes,
    uint32_t* __restrict__ err, const uint32_t* __restrict__ order) {
  using namespace dyn;
  __shared__ uint32_t hist[kNLit + kNDist];
  __shared__ uint32_t ltab[288];
  __shared__ uint32_t dtab[kNDist];
  __shared__ uint32_t ctab[kNCl];
  __shared__ uint8_t lens[kNLit + kNDist + kNCl + 1];
  __shared__ uint16_t cls[kNLit + kNDist + 4];
  __shared__ uint32_t clf[kNCl];
  // the tree scratch and the output bit ring share LDS: codes are built before any output
  // (codes first; then the 2-KiB bit ring + the window-mask and input rings, 1 KiB each,
  // and the record ring, 2 KiB: a step may read 1 KiB of records).  6 KiB instead of 10:
  // 16 workgroups per CU instead of 11 (the pass is latency-bound: 8 cost it 10 %)
#if BITAR_DYN_BULK
  // (batched: the bit ring, the literal stream's 2-KiB ring and the marks -- the pool is then
  // the tree scratch's size: 16 -> 18 workgroups per CU)
  constexpr uint32_t kEmitLds = kStageWords * 4 + 2048 + 4 * (kWave + 4);
#else
  constexpr uint32_t kEmitLds = kStageWords * 4 + 1024 + 2048 + 1024;
#endif
  __shared__ __attribute__((aligned(16))) uint8_t pool[sizeof(TreeLds) > kEmitLds
                                                           ? sizeof(TreeLds) : kEmitLds];
  TreeLds& T = *reinterpret_cast<TreeLds*>(pool);
  const uint32_t lane = lane_id();
  const uint32_t i_seg = order ? order[blockIdx.x] : blockIdx.x;  // (cost-ordered dispatch)
  const uint64_t seg_off = (uint64_t)i_seg * seg;
  if (seg_off >= n_total) return;
  const uint32_t n = (uint32_t)((n_total - seg_off) < seg ? (n_total - seg_off) : seg);
  const GMEM uint8_t* in = global_ptr(input + seg_off);
  const GMEM uint8_t* scr = global_ptr(scratch + (uint64_t)i_seg * scr_stride);
  const GMEM uint32_t* plan = reinterpret_cast<const GMEM uint32_t*>(scr);
  GMEM uint8_t* dst = global_ptr(dsts ? dsts[i_seg] : slab + (uint64_t)i_seg * slot_stride);
  if (plan[kPlanRecBytes] == 0xFFFFFFFFu) {  // pass 1 overflowed its record area
    if (lane == 0) sizes[i_seg] = 0xFFFFFFFFu;
    return;
  }
  for (uint32_t k = lane; k < kNLit + kNDist; k += kWave) hist[k] = plan[k];
  lds_order();
  if (lane == 0) hist[256] = 1;  // end of block
  lds_order();
  uint8_t* ll = lens;
  uint8_t* dl = lens + kNLit;
  uint8_t* cll = lens + kNLit + kNDist;
#if BITAR_DYN_VARIANT == 2  // timing experiment: no code construction (fixed codes)
  for (uint32_t s = lane; s < kNLit + kNDist + kNCl; s += kWave) lens[s] = 8;
  if (lane == 0) hist[0] = 0x7FFFFFFF;
#else
  huff_lengths(hist, kNLit, 15, ll, T);
  huff_lengths(hist + kNLit, kNDist, 15, dl, T);
#endif
  // HLIT / HDIST: trailing zero lengths trimmed
  uint32_t hlit = 257, hdist = 1;
  for (uint32_t s = lane; s < kNLit; s += kWave)
    if (ll[s]) hlit = max(hlit, s + 1);
  for (uint32_t s = lane; s < kNDist; s += kWave)
    if (dl[s]) hdist = max(hdist, s + 1);
  for (uint32_t d = 1; d < 64; d <<= 1) {
    hlit = max(hlit, (uint32_t)__shfl_xor((int)hlit, (int)d, 64));
    hdist = max(hdist, (uint32_t)__shfl_xor((int)hdist, (int)d, 64));
  }
  uint32_t ncl = 0;
  if (lane == 0) {
    ncl = rle_lens(ll, hlit, cls);
    ncl += rle_lens(dl, hdist, cls + ncl);
  }
  ncl = readlane(ncl, 0);
  lds_order();
  if (lane < kNCl) clf[lane] = 0;
  lds_order();
  for (uint32_t k = lane; k < ncl; k += kWave) atomicAdd(&clf[cls[k] & 31u], 1u);
  lds_order();
#if BITAR_DYN_VARIANT != 2
  huff_lengths(clf, kNCl, 7, cll, T);
#endif
  // the code-length code's lengths in transmission order, trailing zeros trimmed
  uint32_t hclen = 4;
  if (lane < kNCl && cll[kClo[lane]]) hclen = lane + 1;
  for (uint32_t d = 1; d < 64; d <<= 1) hclen = max(hclen, (uint32_t)__shfl_xor((int)hclen, (int)d, 64));
  // sizes of the three alternatives (bits; stored in bytes)
  uint32_t dyn_p = 0, fix_p = 0;
  for (uint32_t s = lane; s < kNLit; s += kWave) {
    const uint32_t f = hist[s];
    const uint32_t x = s > 256 ? len_extra_bits(s - 257) : 0u;
    dyn_p += f * (ll[s] + x);
    fix_p += f * (fixed_len(s) + x);
  }
  if (lane < kNDist) {
    const uint32_t f = hist[kNLit + lane];
    dyn_p += f * (dl[lane] + dist_extra_bits(lane));
    fix_p += f * (5u + dist_extra_bits(lane));
  }
  if (lane < kNCl) {
    const uint32_t f = clf[lane];
    dyn_p += f * (cll[lane] + (lane == 16 ? 2u : lane == 17 ? 3u : lane == 18 ? 7u : 0u));
  }
  const uint64_t dyn_bits = 3 + 14 + 3 * (uint64_t)hclen + wave_sum(dyn_p);
  const uint64_t fix_bits = 3 + (uint64_t)wave_sum(fix_p);
  const uint64_t nblk = (n + 65534u) / 65535u;
  const uint64_t stored = nblk * 5 + n;
  uint32_t mode = dyn_bits < fix_bits ? 2u : 1u;
  const uint64_t best = ((mode == 2 ? dyn_bits : fix_bits) + 7) / 8;
  if (stored < best + (n >> 4)) mode = 0;  // unless coding saves n / 16 (oracle BO_STORE_MARGIN)

  if (mode == 0) {  // stored blocks of <= 65535 bytes
    if (stored > slot_stride) {
      if (lane == 0) { sizes[i_seg] = 0xFFFFFFFFu; atomicOr(err, 2u); }
      return;
    }
    uint32_t p = 0, o = 0;
    for (uint64_t b = 0; b < nblk; ++b) {
      const uint32_t len = n - p < 65535u ? n - p : 65535u;
      const uint32_t hdr[5] = {(uint32_t)(b + 1 == nblk), len & 0xFFu, len >> 8,
                               ~len & 0xFFu, (~len >> 8) & 0xFFu};
      if (lane < 5) dst[o + lane] = (uint8_t)(lane == 0 ? hdr[0] : lane == 1 ? hdr[1] : lane == 2 ? hdr[2] : lane == 3 ? hdr[3] : hdr[4]);
      wave_copy_global(dst + o + 5, in + p, len);
      o += 5 + len;
      p += len;
    }
    if (lane == 0) sizes[i_seg] = o;
    return;
  }
  // codes
  if (mode == 2) {
    canon_codes(ll, kNLit, ltab);
    canon_codes(dl, kNDist, dtab);
    canon_codes(cll, kNCl, ctab);
  } else {
    uint8_t* fl = reinterpret_cast<uint8_t*>(T.w);  // 288 fixed lengths
    for (uint32_t s = lane; s < 288; s += kWave) fl[s] = (uint8_t)fixed_len(s);
    if (lane < kNDist) lens[kNLit + lane] = 5;
    lds_order();
    canon_codes(fl, 288, ltab);
    canon_codes(dl, kNDist, dtab);  // dl = 5 everywhere now
  }
  // the bit ring (over the tree scratch): zero, then the block header
  uint32_t* stage = reinterpret_cast<uint32_t*>(pool);
  lds_order();
  for (uint32_t k = lane; k < kStageWords; k += kWave) stage[k] = 0;
  lds_order();
  BitOut o;
  o.stage = stage;
  o.dst = reinterpret_cast<GMEM uint32_t*>(dst);
  o.cap = slot_stride;
  o.bits = 0;
  o.wflushed = 0;
  o.overflow = false;
  uint32_t hbits = 0;
  if (lane == 0) {
    uint64_t bp = 0;
    auto putb = [&](uint32_t v, uint32_t nb) {
      const uint32_t w = (uint32_t)(bp >> 5), sh = (uint32_t)(bp & 31);
      stage[w] |= v << sh;
      if (sh + nb > 32) stage[w + 1] |= v >> (32 - sh);
      bp += nb;
    };
    putb(1u | (mode << 1), 3);  // BFINAL = 1, BTYPE = 01 fixed / 10 dynamic
    if (mode == 2) {
      putb(hlit - 257, 5);
      putb(hdist - 1, 5);
      putb(hclen - 4, 4);
      for (uint32_t k = 0; k < hclen; ++k) putb(cll[kClo[k]], 3);
      for (uint32_t k = 0; k < ncl; ++k) {
        const uint32_t c = cls[k], s = c & 31u, x = c >> 8;
        const uint32_t t = ctab[s];
        putb(t & 0xFFFFu, t >> 16);
        if (s == 16) putb(x, 2);
        else if (s == 17) putb(x, 3);
        else if (s == 18) putb(x, 7);
      }
    }
    hbits = (uint32_t)bp;
  }
  lds_order();
  o.bits = readlane(hbits, 0);  // < kStageWords * 32 - the flush margin: no flush needed yet

#if BITAR_DYN_BULK
  // Symbols from the records and the literal stream, 64 per step.  Per chunk of 64 records
  // (one 8-B load per lane, the next chunk's issued a chunk ahead): each record's literal run
  // [previous match end, start) and its match symbol (codes + extra bits, <= 45 bits, built
  // once per record); then the chunk's symbols 64 per step -- every run marks its first
  // symbol, one compare gives the step's start mask, v_mbcnt the run k, two ds_bpermute the
  // match code and one its position | length; a literal symbol u of run k is literal number
  // lit_base + u - 1 - k of the stream, read from an LDS ring the stream flows through.
  {
    const uint32_t nrec = plan[kPlanRecBytes], nlit = plan[kPlanWindows];
    uint8_t* rings = pool + kStageWords * 4;
    RowRing<1024> Lr;
    Lr.init(reinterpret_cast<const GMEM uint4*>(scr + kPlanBytes), (nlit + 15u) & ~15u, rings);
    uint32_t* marks = reinterpret_cast<uint32_t*>(rings + 2048);  // kWave + 1
    marks[lane] = 0;
    const GMEM uint2* recs = reinterpret_cast<const GMEM uint2*>(scr + kPlanBytes + lit_cap(seg));
    uint2 nxt = make_uint2(0, 0);
    if (lane < nrec) nxt = recs[lane];
    uint32_t last_end = 0, lit_base = 0;
    for (uint32_t c0 = 0; c0 < nrec && !o.overflow; c0 += kWave) {
      const uint2 rec = nxt;
      nxt = make_uint2(0, 0);
      if (c0 + kWave + lane < nrec) nxt = recs[c0 + kWave + lane];
      const uint32_t cnt = nrec - c0 < kWave ? nrec - c0 : kWave;
      const bool live = lane < cnt;
      const uint32_t q = rec.x & 0xFFFFu, off = (rec.x >> 16) + 1u, mlen = rec.y;
      const uint32_t end = q + mlen;
      const uint32_t prev = wave_shr1(end);
      const uint32_t ll = q - (lane == 0 ? last_end : prev);
      last_end = readlane(end, cnt - 1);
      uint32_t lnx, lxv, dnx, dxv;
      const uint32_t ls = len_sym(live ? mlen : 3u, lnx, lxv);
      const uint32_t ds = dist_sym(live ? off : 1u, dnx, dxv);
      lds_order();
      const uint32_t lt_ = ltab[257 + ls];
      const uint32_t dt = dtab[ds];
      const uint32_t ln = lt_ >> 16, dn = dt >> 16;
      const uint32_t lo = (lt_ & 0xFFFFu) | (lxv << ln);  // <= 20 bits
      const uint64_t mv = (uint64_t)lo | ((uint64_t)((dt & 0xFFFFu) | (dxv << dn)) << (ln + lnx));
      const uint32_t mb = ln + lnx + dn + dnx;
      const uint32_t e = live ? ll + 1u : 0u;
      const uint32_t incl = wave_incl_sum(e);
      const uint32_t total = readlane(incl, kWave - 1);
      const uint32_t a = incl - e;                    // the run's first symbol
      const uint32_t pX = ((a + ll + 1u) << 8) | mb;  // u of the match symbol | its bit count
      const uint32_t mlo = (uint32_t)mv, mhi = (uint32_t)(mv >> 32);
      const uint32_t a4 = live ? a << 2 : 0x7FFFFF00u;
      const uint32_t mark = a + 1u;
      const uint32_t zero = 0;
      uint32_t u = lane + 1u;
      uint32_t before = 0xFFFFFFFFu;  // runs started before the step, less one
      for (uint32_t R = 0; R < total && !o.overflow; R += kWave) {
        Lr.ensure(lit_base + R + kWave);
        lds_order();
        const uint32_t slot = min(a4 - (R << 2), (uint32_t)kWave << 2);
        *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(marks) + slot) = mark;
        lds_order();
        const uint32_t mk = marks[lane];
        marks[lane] = zero;
        const uint64_t S = ballot(mk == u);
        const uint32_t base = before + (uint32_t)(S & 1u);
        const uint64_t S1 = S >> 1;
        const uint32_t k = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(S1 >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)S1, 0u));
        before += (uint32_t)__builtin_popcountll(S);
        const int src = (int)(k << 2);
        const uint32_t qX = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)pX);
        const uint32_t qlo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)mlo);
        const uint32_t qhi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)mhi);
        const uint32_t b = Lr.byte(lit_base + u - 1u - k);
        const uint32_t lt = ltab[b];
        const bool ism = u == (qX >> 8);
        const bool act = u <= total;
        const uint64_t val = ism ? ((uint64_t)qhi << 32 | qlo) : (uint64_t)(lt & 0xFFFFu);
        o.put(act ? val : 0ull, act ? (ism ? (qX & 0xFFu) : (lt >> 16)) : 0u);
        u += kWave;
      }
      lit_base += total - cnt;
    }
    // the tail literals (after the last match): the rest of the stream
    for (uint32_t k = lit_base; k < nlit && !o.overflow; k += kWave) {
      const bool act = k + lane < nlit;
      Lr.ensure(k + kWave);
      lds_order();
      const uint32_t b = act ? Lr.byte(k + lane) : 0u;
      lds_order();
      const uint32_t lt = ltab[b];
      o.put(act ? (uint64_t)(lt & 0xFFFFu) : 0ull, act ? (lt >> 16) : 0u);
    }
  }
#else
  // symbols, kB windows per step (independent LDS reads and prefix sums across the
  // windows of a step); window masks, match records and input bytes stream through LDS rings
  RowRing<512> C, I;
  RowRing<1024> R;
  const uint32_t s0 = (uint32_t)((uintptr_t)in & 15u);
  const uint32_t nwin = plan[kPlanWindows];
  uint32_t emitted = plan[kPlanTail];
  {
    uint8_t* rings = pool + kStageWords * 4;
    C.init(reinterpret_cast<const GMEM uint4*>(scr + kPlanBytes), 16 * nwin, rings);
    R.init(reinterpret_cast<const GMEM uint4*>(scr + kPlanBytes + kMaskBytes),
           (plan[kPlanRecBytes] + 15u) & ~15u, rings + 1024);
    const uint64_t span = (uint64_t)(global_ptr(input + n_total) - (in - s0));
    I.init(reinterpret_cast<const GMEM uint4*>(in - s0),
           (uint32_t)(span < (uint64_t)n + s0 ? span : (uint64_t)n + s0), rings + 3072);
  }
  if (BITAR_DYN_VARIANT == 1) emitted = n;  // timing experiment: no symbol emission
  if (BITAR_DYN_VARIANT != 1) {
    const uint64_t lt = (1ull << lane) - 1;
    uint32_t rp = 0;  // record byte offset
    for (uint32_t w0 = 0; w0 < nwin; w0 += kB) {
      C.ensure(16 * (w0 + kB));
      R.ensure(rp + 4 * kWave * kB);
      I.ensure(s0 + kWave * (w0 + kB));
      lds_order();
      uint64_t val[kB];
      uint32_t nb[kB];
      uint32_t rb = rp;
#pragma unroll
      for (uint32_t k = 0; k < kB; ++k) {
        const uint32_t w = w0 + k;
        const bool valid = w < nwin;
        const uint64_t chain = valid ? (uint64_t)C.word(16 * w) | ((uint64_t)C.word(16 * w + 4) << 32) : 0ull;
        const uint64_t litm = valid ? (uint64_t)C.word(16 * w + 8) | ((uint64_t)C.word(16 * w + 12) << 32) : 0ull;
        const bool cl = (chain >> lane) & 1, lit = (litm >> lane) & 1;
        const uint32_t r = R.word(rb + 4 * (uint32_t)__builtin_popcountll(chain & lt));
        rb += 4 * (uint32_t)__builtin_popcountll(chain);
        const uint32_t byte = I.byte(s0 + kWave * w + lane);
        const uint32_t ls = r & 31u, lxv = (r >> 5) & 31u, ds = (r >> 10) & 31u, dxv = r >> 15;
        const uint32_t lt_ = ltab[cl ? 257 + ls : byte];
        const uint32_t dt = dtab[ds];
        const uint32_t ln = lt_ >> 16, dn = dt >> 16;
        const uint32_t lnx = len_extra_bits(ls), dnx = dist_extra_bits(ds);
        const uint32_t lo = (lt_ & 0xFFFFu) | (lxv << ln);  // <= 20 bits
        const uint64_t mv = (uint64_t)lo | ((uint64_t)((dt & 0xFFFFu) | (dxv << dn)) << (ln + lnx));
        val[k] = cl ? mv : lit ? (uint64_t)(lt_ & 0xFFFFu) : 0ull;
        nb[k] = cl ? ln + lnx + dn + dnx : lit ? ln : 0u;
      }
      rp = rb;
      o.put_multi(val, nb);
    }
  }
  // tail literals
  for (uint32_t k = emitted; k < n; k += kWave) {
    const uint32_t q = k + lane;
    const bool act = q < n;
    I.ensure(s0 + k + kWave);
    lds_order();
    const uint32_t b = act ? I.byte(s0 + q) : 0u;
    lds_order();
    const uint32_t lt = ltab[b];
    o.put(act ? (uint64_t)(lt & 0xFFFFu) : 0ull, act ? (lt >> 16) : 0u);
  }
#endif
  {
    lds_order();
    const uint32_t eob = ltab[256];
    o.put(lane == 0 ? (uint64_t)(eob & 0xFFFFu) : 0ull, lane == 0 ? (eob >> 16) : 0u);
  }
  o.flush_words((uint32_t)((o.bits + 31) >> 5));
  if (lane == 0) {
    sizes[i_seg] = o.overflow ? 0xFFFFFFFFu : (uint32_t)((o.bits + 7) >> 3);
    if (o.overflow) atomicOr(err, 2u);
  }
}

}  // namespace bitar_hip
