// zstd_compress.hip -- Zstandard (RFC 8878) frame per segment, level-1 class (gfx950):
// BASELINE configs[4] / [5].  The frame is exactly the one the oracle's bo_zstd_compress_block
// (oracle/bitar_zstd.c) writes: single-segment header with the content size, ONE block
// (compressed, or raw when that is not smaller), Huffman literals (1 or 4 streams, direct or
// FSE-compressed weights) or raw / RLE ones, repeat offsets, and per-table RLE /
// FSE_Compressed / predefined sequence codes chosen by integer cost estimates.
//
// Two launches, one wavefront per segment each, through a scratch area per segment
// (kLitCap literal bytes, then 8-byte sequence records):
//   zstd_parse_kernel    the window-scan parse (window_parse.hip.h) in its repeat-offset
//                        form (REP): literal bytes staged in LDS and flushed to the literal
//                        area, one {literal length | distance << 17, match length} record
//                        per match; per segment {nlit, nseq} in the meta array.
//   zstd_entropy_kernel  literal histograms per stream quarter, code lengths
//                        (huffman.hip.h), weights, stream sizes; repeat-offset codes by a
//                        scalar scan of the records; sequence code histograms, table
//                        choice and FSE tables (one lane); then the literal streams and the
//                        sequence bitstream, each lane placing its bit field by a prefix
//                        sum into the LDS output ring.
#include "huffman.hip.h"
#include "zstd_layout.hip.h"
#include "window_parse.hip.h"

namespace bitar_hip {

namespace zse {

using namespace cmp;

#ifndef BITAR_ZSTD_STOP
#define BITAR_ZSTD_STOP 0  // timing experiments only: end the entropy kernel after phase k
#endif
#define ZSE_PHASE(k)                             \
  if constexpr (BITAR_ZSTD_STOP == (k)) {        \
    if (lane == 0) wrec[zse::kWHanded] = 0u;     \
    return;                                      \
  }

// ---- code tables (RFC 8878 3.1.1.3.2.1-2) ----------------------------------------------------
constexpr uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,   7,   8,   9,    10,   11,
                                  12, 13, 14, 15, 16, 18, 20,  22,  24,  28,   32,   40,
                                  48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384,
                                  32768, 65536};
constexpr uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  1,  1,
                                 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
constexpr uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13,   14,   15,   16,
                                  17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27,   28,   29,   30,
                                  31, 32, 33, 34, 35, 37, 39, 41, 43, 47, 51,   59,   67,   83,
                                  99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771,
                                  65539};
constexpr uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                                 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
// predefined distributions (accuracy logs 6 / 5 / 6)
constexpr int16_t kLLNorm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
constexpr int16_t kMLNorm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
constexpr int16_t kOFNorm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
// 256 * log2(1 + i / 64), rounded (oracle kLog2Frac)
constexpr uint8_t kLog2Frac[64] = {
    0,   6,   11,  17,  22,  28,  33,  38,  44,  49,  54,  59,  63,  68,  73,  78,
    82,  87,  92,  96,  100, 105, 109, 113, 118, 122, 126, 130, 134, 138, 142, 146,
    150, 154, 157, 161, 165, 169, 172, 176, 179, 183, 186, 190, 193, 197, 200, 203,
    207, 210, 213, 216, 220, 223, 226, 229, 232, 235, 238, 241, 244, 247, 250, 253};

struct Tabs {
  uint8_t ll_bits[36], ml_bits[53];
  uint8_t ll_code[64], ml_code[128];  // ZSTD_LLcode below 64 / ZSTD_MLcode of ml - 3 below 128
  int16_t ll_norm[36], ml_norm[53], of_norm[29];
  uint8_t log2frac[64];
};
constexpr Tabs build_tabs() {
  Tabs t{};
  for (uint32_t i = 0; i < 36; ++i) {
    t.ll_bits[i] = kLLBits[i];
    t.ll_norm[i] = kLLNorm[i];
  }
  for (uint32_t i = 0; i < 53; ++i) {
    t.ml_bits[i] = kMLBits[i];
    t.ml_norm[i] = kMLNorm[i];
  }
  for (uint32_t i = 0; i < 29; ++i) t.of_norm[i] = kOFNorm[i];
  for (uint32_t i = 0; i < 64; ++i) t.log2frac[i] = kLog2Frac[i];
  for (uint32_t v = 0; v < 64; ++v) {
    uint32_t c = 35;
    while (kLLBase[c] > v) --c;
    t.ll_code[v] = (uint8_t)c;
  }
  for (uint32_t v = 0; v < 128; ++v) {
    uint32_t c = 52;
    while (kMLBase[c] > v + 3) --c;
    t.ml_code[v] = (uint8_t)c;
  }
  return t;
}
__constant__ Tabs kT = build_tabs();
// the entropy kernel's copy in LDS: a __constant__ read compiles to a global load whose
// latency would sit on every dependent step
__shared__ __attribute__((aligned(16))) Tabs sT;

__device__ __forceinline__ uint32_t hb32(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }
__device__ __forceinline__ uint32_t ll_code(uint32_t ll) { return ll < 64 ? sT.ll_code[ll] : hb32(ll) + 19u; }
__device__ __forceinline__ uint32_t ml_code(uint32_t ml) {  // ml >= 3
  const uint32_t b = ml - 3;
  return b < 128 ? sT.ml_code[b] : hb32(b) + 36u;
}

// ---- scratch layout: zstd_layout.hip.h ------------------------------------------------------

// ---- pass 1: the parse, literals + sequence records ---------------------------------------
#ifndef BITAR_ZSTD_BULK
#define BITAR_ZSTD_BULK 1
#endif
#if BITAR_ZSTD_BULK
// Batched (as the LZ4 emitter, compress.hip): each window only appends its matches {start |
// distance << 16, length} to an LDS list; every <= 48 records (and before the tail) one flush
// writes their 8-byte records with one coalesced store and gathers their literal runs
// [previous match end, match start) into the literal area, 64 literal bytes per step: every
// non-empty run marks its first byte (its u = offset + 1 in the batch's literals), one compare
// gives the step's start mask, a v_mbcnt pair the run (counted over the non-empty runs, whose
// ring offsets are compacted to their rank once per batch), one ds_bpermute its offset, one
// LDS read the byte.  Runs that start before the input ring's low end (probe-skipped stretches,
// long random runs) take the per-run path (HBM -> HBM beyond 256 bytes).
constexpr uint32_t kZsCap = 64;      // records per flush (a window adds <= 16)
constexpr uint32_t kZsObuf = 512;    // literal staging ring
struct ZsLds {
  uint8_t ring[kZsObuf];
  uint2 recs[kZsCap + 1];            // + a trash record
  uint32_t marks[kWave + 1];         // zero between steps; + trash
};
struct SeqCollect : ByteOutT<kZsObuf> {
  ZsLds* L;
  GMEM uint2* seqs;
  uint32_t nseq;      // records written
  uint32_t npend;     // records pending in L->recs
  uint32_t last_end;  // end of the last match (the next literal run's start)

  // literal bytes [s, s + len) of the input, appended to the literal area
  __device__ __forceinline__ void literals(const GMEM uint8_t* in, const InRing& I, uint32_t s,
                                           uint32_t len) {
    if (!len) return;
    const uint32_t lane = lane_id();
    if (len <= 256 && s >= I.lo) {
      for (uint32_t k = 0; k < len; k += kWave) {
        const uint32_t step = len - k < kWave ? len - k : kWave;
        room(step);
        lds_order();
        const uint32_t b = I.byte(s + k + (lane < step ? lane : 0u));
        put(b, step);
      }
    } else {  // long run (or not in the input ring): drain the ring, then HBM -> HBM
      flush(op, true);
      wave_copy_global(dst + op, in + s, len);
      op += len;
      flushed = op;
    }
  }
  // the literal runs of lanes [lo, hi) (all in the input ring), gathered 64 bytes per step
  __device__ __forceinline__ void gather(const InRing& I, uint32_t lo, uint32_t hi,
                                         uint32_t lit_start, uint32_t ll) {
    const uint32_t lane = lane_id();
    const bool ne = (lane >= lo) & (lane < hi) & (ll != 0u);
    const uint32_t e = ne ? ll : 0u;
    const uint32_t incl = wave_incl_sum(e);
    const uint32_t total = readlane(incl, kWave - 1);
    if (!total) return;
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
      if (op + kWave - flushed > kZsObuf - 64) flush(op, false);
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
      // all 64 bytes are written: those past nb lie at or past the new op, inside the room
      // just made, and are rewritten before they are flushed
      ring[(rbase + u) & kMask] = (uint8_t)b;
      lds_order();
      op += nb;
      u += kWave;
    }
  }
  // every pending record: to HBM, and its literal run to the literal area
  __device__ __forceinline__ void flush_seqs(const GMEM uint8_t* in, const InRing& I) {
    const uint32_t cnt = npend;
    npend = 0;
    if (!cnt) return;
    const uint32_t lane = lane_id();
    lds_order();
    const uint2 rec = L->recs[lane < cnt ? lane : kZsCap];
    const uint32_t q = rec.x & 0xFFFFu, off = (rec.x >> 16) + 1u, mlen = rec.y;
    const uint32_t end = q + mlen;
    const uint32_t prev = wave_shr1(end);
    const uint32_t lit_start = lane == 0 ? last_end : prev;
    const uint32_t ll = q - lit_start;
    last_end = readlane(end, cnt - 1);
    if (lane < cnt) seqs[nseq + lane] = make_uint2(ll | (off << 17), mlen);
    nseq += cnt;
    const uint64_t live = cnt < kWave ? (1ull << cnt) - 1 : ~0ull;
    uint64_t special = ballot(lit_start < I.lo) & ballot(ll != 0u) & live;
    uint32_t lo = 0;
    for (;;) {
      const uint32_t k = special ? (uint32_t)__builtin_ctzll(special) : cnt;
      if (k > lo) gather(I, lo, k, lit_start, ll);
      if (k >= cnt) break;
      literals(in, I, readlane(lit_start, k), readlane(ll, k));
      special &= special - 1;
      lo = k + 1;
    }
  }
  // the tail literals (after whatever is pending)
  __device__ __forceinline__ void sequence(const GMEM uint8_t* in, const InRing& I, uint32_t s,
                                           uint32_t len, uint32_t, uint32_t) {
    flush_seqs(in, I);
    literals(in, I, s, len);
  }
  __device__ __forceinline__ void between(const GMEM uint8_t* in, const InRing& I) {
    if (npend > kZsCap - 16) flush_seqs(in, I);
  }
  // the tail starts at the last match's end
  __device__ __forceinline__ uint32_t pending_from(uint32_t anchor, uint32_t) const {
    return anchor;
  }
  __device__ __forceinline__ void window(const GMEM uint8_t*, const InRing&, const Window& W,
                                         uint32_t, uint32_t) {
    if (!W.chain) return;
    const uint64_t chain = W.chain;
    // (the record index: v_mbcnt adds its second operand, so no separate add)
    const uint32_t idx = __builtin_amdgcn_mbcnt_hi((uint32_t)(chain >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)chain, npend));
    const uint32_t lane = lane_id();
    lds_order();
    L->recs[(chain >> lane) & 1u ? idx : kZsCap] =
        make_uint2((W.x + lane) | (W.dm1 << 16), W.mlen);
    lds_order();
    npend += (uint32_t)__builtin_popcountll(chain);
  }
};
#else
struct SeqCollect : ByteOut {  // the byte ring carries literal bytes to the literal area
  GMEM uint2* seqs;
  uint32_t nseq;

  // literal bytes [s, s + len) of the input, appended to the literal area
  __device__ __forceinline__ void literals(const GMEM uint8_t* in, const InRing& I, uint32_t s,
                                           uint32_t len) {
    if (!len) return;
    const uint32_t lane = lane_id();
    if (len <= 256 && s >= I.lo) {
      for (uint32_t k = 0; k < len; k += kWave) {
        const uint32_t step = len - k < kWave ? len - k : kWave;
        room(step);
        lds_order();
        const uint32_t b = I.byte(s + k + (lane < step ? lane : 0u));
        put(b, step);
      }
    } else {  // long run (or not in the input ring): drain the ring, then HBM -> HBM
      flush(op, true);
      wave_copy_global(dst + op, in + s, len);
      op += len;
      flushed = op;
    }
  }
  __device__ __forceinline__ void sequence(const GMEM uint8_t* in, const InRing& I, uint32_t s,
                                           uint32_t len, uint32_t, uint32_t) {
    literals(in, I, s, len);
  }
  __device__ __forceinline__ void between(const GMEM uint8_t*, const InRing&) {}
  __device__ __forceinline__ uint32_t pending_from(uint32_t, uint32_t emitted) const {
    return emitted;
  }
  __device__ __forceinline__ void window(const GMEM uint8_t* in, const InRing& I,
                                         const Window& W, uint32_t anchor, uint32_t n) {
    // SKIP: the positions of probe windows that found nothing were never handed over; they
    // are literals and come first (the oracle's emit takes each sequence's literal run whole)
    if (W.done < W.x) literals(in, I, W.done, W.x - W.done);
    const uint32_t lane = lane_id();
    const uint32_t q = W.x + lane;
    const bool cl = (W.chain >> lane) & 1;
    // match ends increase along the chain: "end of the previous match" is a prefix max
    const uint32_t end_incl = wave_incl_max(cl ? q + W.mlen : 0u);
    const uint32_t end_excl = wave_shr1(end_incl);
    const uint32_t lit_start = max(anchor, cl ? end_excl : end_incl);
    const uint32_t ll = q - lit_start;  // chain lanes: their literal length
    const bool lit = !cl && q >= W.pos_in && q >= end_incl && q < n;
    const uint64_t litm = ballot(lit);
    const uint32_t nl = (uint32_t)__builtin_popcountll(litm);
    if (nl) {
      room(nl);
      const uint32_t li = __builtin_amdgcn_mbcnt_hi((uint32_t)(litm >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)litm, 0u));
      lds_order();
      ring[lit ? at(op + li) : kObuf + lane] = (uint8_t)W.byte;
      lds_order();
      op += nl;
    }
    if (W.chain) {
      const uint32_t si = __builtin_amdgcn_mbcnt_hi((uint32_t)(W.chain >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)W.chain, 0u));
      if (cl) seqs[nseq + si] = make_uint2(ll | (W.off() << 17), W.mlen);
      nseq += (uint32_t)__builtin_popcountll(W.chain);
    }
  }
};
#endif

// ---- repeat offsets (RFC 8878 3.1.2.5), 64 sequences per step ------------------------------
// The offset value of each lane's sequence (distance o, literal length ll) from the history
// {c0, c1, c2} before the step; the history after the step replaces c0..c2 (cnt = the
// step's sequences).  Scanned lane-parallel: after sequence i, r0 = o_i; r1 = o_{j-1} for the
// last j <= i that is not a plain repeat of r0 (ll_j > 0 && o_j == o_{j-1}); r2 = r1 before the
// last k <= i that is neither such a repeat nor a repeat of r1 (prefix maxima + bpermute).
// Every cross-lane op runs on all 64 lanes (a DPP or bpermute source lane that is off in
// EXEC reads as 0).  zstd_entropy_kernel keeps each sequence's offset value beside its codes
// (the walk scratch's code word), so zstd_emit_kernel reads it instead of scanning again.
__device__ __forceinline__ uint32_t rep_scan(uint32_t ll, uint32_t o, bool act, uint32_t cnt,
                                             uint32_t& c0r, uint32_t& c1r, uint32_t& c2r) {
  const uint32_t lane = lane_id();
  const uint32_t so = wave_shr1(o);
  const uint32_t oprev = lane == 0 ? c0r : so;                      // r0 before
  const bool same = !act || (ll != 0 && o == oprev);
  const uint32_t mj = wave_incl_max(same ? 0u : lane + 1);
  const uint32_t p1 = bpermute(oprev, mj ? mj - 1 : 0u);
  const uint32_t r1a = mj ? p1 : c1r;                               // r1 after
  const uint32_t s1 = wave_shr1(r1a);
  const uint32_t r1b = lane == 0 ? c1r : s1;                        // r1 before
  const bool ev = !same && o != r1b;
  const uint32_t mk = wave_incl_max(ev ? lane + 1 : 0u);
  const uint32_t p2 = bpermute(r1b, mk ? mk - 1 : 0u);
  const uint32_t r2a = mk ? p2 : c2r;                               // r2 after
  const uint32_t s2 = wave_shr1(r2a);
  const uint32_t r2b = lane == 0 ? c2r : s2;                        // r2 before
  uint32_t ov;
  if (ll) ov = o == oprev ? 1u : o == r1b ? 2u : o == r2b ? 3u : o + 3u;
  else ov = o == r1b ? 1u : o == r2b ? 2u : o == oprev - 1u ? 3u : o + 3u;
  c0r = readlane(o, cnt - 1);
  c1r = readlane(r1a, cnt - 1);
  c2r = readlane(r2a, cnt - 1);
  return ov;
}

// ---- pass 2: entropy coding ------------------------------------------------------------------
// FSE state tables in LDS: literal lengths at 0 (<= 512 states), offsets at 512 (<= 256),
// match lengths at 768 (<= 512); entry kTabDummy = 0 serves the idle lanes of the chain walk.
constexpr uint32_t kTabLL = 0, kTabOF = 512, kTabML = 768, kTabDummy = 1280;

struct EntLds {
  uint32_t hist[256];      // literal histogram
  uint8_t len[256];        // code lengths
  uint8_t w[256];          // weights
  uint8_t desc[192];       // Huffman tree description; then modes + table descriptions
  uint8_t tmp[256];        // serial bit writer output (weights FSE form, table descriptions)
  int16_t norm[64];
  uint32_t u[16];          // lane-0 results: sizes, modes, accuracy logs
  uint32_t wk[32];         // lane-0 work: weight counts, code ranges
  uint32_t sh[3][64];      // sequence code histograms: LL, OF, ML
  union {                  // by phase (8.9 KiB of LDS in all: 17 waves per CU, was 13)
    huf::TreeLds T;        // the literal code lengths (huff_lengths), dead once L.len is set
    struct {               // then the FSE tables: the weights' (weights_fse), the sequences'
      uint16_t tabs[kTabDummy + 1];
      uint32_t tr[3][64];  // per symbol: deltaNbBits | deltaFindState << 20 (12-bit signed)
      uint8_t sym_at[512];
      uint16_t nxt[64];
    };
  };
};
// 256 * log2(x), x >= 1
__device__ __forceinline__ uint32_t log2fix(uint32_t x) {
  const uint32_t hb = hb32(x);
  const uint32_t f = (hb >= 6 ? x >> (hb - 6) : x << (6 - hb)) & 63u;
  return (hb << 8) + sT.log2frac[f];
}

// oracle zs_table_log (total >= 2, max_sym >= 1)
__device__ uint32_t table_log(uint32_t max_log, uint32_t total, uint32_t max_sym) {
  int tl = (int)max_log;
  const int src_bits = (int)hb32(total - 1) - 2;
  if (src_bits < tl) tl = src_bits;
  const int a = (int)hb32(total) + 1, b = (int)hb32(max_sym) + 2;
  const int mb = a < b ? a : b;
  if (mb > tl) tl = mb;
  if (tl < 5) tl = 5;
  if (tl > (int)max_log) tl = (int)max_log;
  return (uint32_t)tl;
}

// oracle zs_normalize (lane-serial)
__device__ void normalize(const uint32_t* cnt, uint32_t max_sym, uint32_t total, uint32_t tl,
                          int16_t* norm) {
  const uint32_t size = 1u << tl;
  int32_t sum = 0;
  for (uint32_t s = 0; s <= max_sym; ++s) {
    uint32_t v = 0;
    if (cnt[s]) {
      v = (cnt[s] * size + total / 2) / total;
      if (v == 0) v = 1;
    }
    norm[s] = (int16_t)v;
    sum += (int32_t)v;
  }
  int32_t delta = (int32_t)size - sum;
  if (delta > 0) {
    uint32_t best = 0;
    for (uint32_t s = 1; s <= max_sym; ++s) if (cnt[s] > cnt[best]) best = s;
    norm[best] = (int16_t)(norm[best] + delta);
  }
  while (delta < 0) {
    uint32_t best = 0;
    for (uint32_t s = 1; s <= max_sym; ++s) if (norm[s] > norm[best]) best = s;
    int32_t take = norm[best] - 1;
    if (take > -delta) take = -delta;
    norm[best] = (int16_t)(norm[best] - take);
    delta += take;
  }
}

// lane-serial forward bit writer into LDS bytes (BIT_CStream)
struct SBits {
  uint8_t* out;
  uint32_t pos;
  uint64_t acc;
  uint32_t nb;
  // (a constructor, not an aggregate: {LDS address, 0, ...} may become a constant global
  // initialised with that address, which a gfx950 code object cannot hold)
  __device__ explicit SBits(uint8_t* o) : out(o), pos(0), acc(0), nb(0) {}
  __device__ __forceinline__ void add(uint64_t v, uint32_t n) {
    if (!n) return;
    acc |= (v & ((1ull << n) - 1)) << nb;
    nb += n;
    while (nb >= 8) {
      out[pos++] = (uint8_t)acc;
      acc >>= 8;
      nb -= 8;
    }
  }
  __device__ __forceinline__ void pad() {
    if (nb) {
      out[pos++] = (uint8_t)acc;
      acc = 0;
      nb = 0;
    }
  }
};

// oracle zs_write_ncount
__device__ uint32_t write_ncount(SBits& w, const int16_t* norm, uint32_t max_sym, uint32_t tl) {
  const uint32_t p0 = w.pos;
  w.add(tl - 5, 4);
  int remaining = (1 << tl) + 1, threshold = 1 << tl;
  uint32_t nbits = tl + 1, s = 0;
  bool prev0 = false;
  while (s <= max_sym && remaining > 1) {
    if (prev0) {
      uint32_t start = s;
      while (norm[s] == 0) ++s;
      while (s >= start + 3) {
        w.add(3, 2);
        start += 3;
      }
      w.add(s - start, 2);
    }
    int count = norm[s++];
    const int mx = (2 * threshold - 1) - remaining;
    remaining -= count < 0 ? -count : count;
    ++count;
    if (count >= threshold) count += mx;
    w.add((uint32_t)count, nbits - (count < mx ? 1u : 0u));
    prev0 = count == 1;
    while (remaining < threshold) {
      --nbits;
      threshold >>= 1;
    }
  }
  w.pad();
  return w.pos - p0;
}

// oracle zs_build_ctable (lane-serial): state table at st, per-symbol transforms at tr
__device__ void build_ctable(const int16_t* norm, uint32_t max_sym, uint32_t al, uint16_t* st,
                             uint32_t* tr, uint8_t* sym_at, uint16_t* cumul) {
  const uint32_t size = 1u << al, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
  uint32_t high = size - 1;
  cumul[0] = 0;
  for (uint32_t s = 1; s <= max_sym + 1; ++s) {
    if (norm[s - 1] == -1) {
      cumul[s] = (uint16_t)(cumul[s - 1] + 1);
      sym_at[high--] = (uint8_t)(s - 1);
    } else {
      cumul[s] = (uint16_t)(cumul[s - 1] + norm[s - 1]);
    }
  }
  uint32_t pos = 0;
  for (uint32_t s = 0; s <= max_sym; ++s)
    for (int i = 0; i < norm[s]; ++i) {
      sym_at[pos] = (uint8_t)s;
      do {
        pos = (pos + step) & mask;
      } while (pos > high);
    }
  for (uint32_t u = 0; u < size; ++u) st[cumul[sym_at[u]]++] = (uint16_t)(size + u);
  int32_t total = 0;
  for (uint32_t s = 0; s <= max_sym; ++s) {
    int32_t dnb, dfs = 0;
    if (norm[s] == 0) {
      dnb = (int32_t)(((al + 1) << 16) - size);
    } else if (norm[s] == -1 || norm[s] == 1) {
      dnb = (int32_t)((al << 16) - size);
      dfs = total - 1;
      total += 1;
    } else {
      const uint32_t mbo = al - hb32((uint32_t)norm[s] - 1);
      const uint32_t msp = (uint32_t)norm[s] << mbo;
      dnb = (int32_t)((mbo << 16) - msp);
      dfs = total - norm[s];
      total += norm[s];
    }
    tr[s] = (uint32_t)dnb | ((uint32_t)dfs << 20);
  }
}

// build_ctable, all lanes (symbols <= 63: one per lane).  The spread visits the positions
// k * step & mask for k = 0, 1, ...; the c-th of them not in the high region (the "less than
// 1" symbols' cells) takes the symbol whose run [cumN, cumN + norm) holds c.  Then each
// symbol's cells, in position order, take its consecutive state slots from cumul: ranks
// within a 64-cell chunk by one ballot per distinct symbol there, across chunks by a
// per-symbol running count (lane s).  Same tables as the serial build, bit for bit.
__device__ void build_ctable_par(const int16_t* norm, uint32_t max_sym, uint32_t al, uint16_t* st,
                                 uint32_t* tr, uint8_t* sym_at) {
  const uint32_t lane = lane_id();
  const uint32_t size = 1u << al, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
  const int32_t nv = lane <= max_sym ? (int32_t)norm[lane] : 0;
  const uint32_t low = nv == -1 ? 1u : 0u, pos = nv > 0 ? (uint32_t)nv : 0u;
  const uint32_t cumul = wave_incl_sum(low + pos) - (low + pos);  // state slots before s
  const uint32_t lowi = wave_incl_sum(low);
  const uint32_t high = size - 1 - readlane(lowi, kWave - 1);
  const uint32_t cum_n = wave_incl_sum(pos) - pos;                  // spread cells before s
  if (low) sym_at[size - lowi] = (uint8_t)lane;                     // (high, downwards)
  uint32_t c0 = 0;
  for (uint32_t k0 = 0; k0 < size; k0 += kWave) {
    const uint32_t k = k0 + lane;
    const uint32_t v = (k * step) & mask;
    const bool ok = k < size && v <= high;
    const uint64_t bm = ballot(ok);
    const uint32_t c = c0 + __builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
    c0 += (uint32_t)__builtin_popcountll(bm);
    // the last symbol whose run starts at or before c (cum_n is non-decreasing over lanes)
    uint32_t sl = 0;
#pragma unroll
    for (uint32_t d = 32; d != 0; d >>= 1) {
      const uint32_t x = bpermute(cum_n, sl + d);
      sl = x <= c ? sl + d : sl;
    }
    if (ok) sym_at[v] = (uint8_t)sl;
  }
  lds_order();
  uint32_t run = 0;  // lane s: cells of symbol s placed so far
  for (uint32_t u0 = 0; u0 < size; u0 += kWave) {
    const uint32_t u = u0 + lane;
    const bool in = u < size;
    const uint32_t sy = in ? sym_at[u] : 0u;
    uint64_t todo = ballot(in);
    uint32_t rank = 0;
    while (todo) {
      const uint32_t y = readlane(sy, (uint32_t)__builtin_ctzll(todo));
      const uint64_t mm = ballot(in && sy == y);
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
      rank = in && sy == y ? readlane(run, y) + below : rank;
      run += lane == y ? (uint32_t)__builtin_popcountll(mm) : 0u;
      todo &= ~mm;
    }
    const uint32_t slot = bpermute(cumul, sy) + rank;
    if (in) st[slot] = (uint16_t)(size + u);
  }
  if (lane <= max_sym) {
    int32_t dnb, dfs = 0;
    if (nv == 0) {
      dnb = (int32_t)(((al + 1) << 16) - size);
    } else if (nv == -1 || nv == 1) {
      dnb = (int32_t)((al << 16) - size);
      dfs = (int32_t)cumul - 1;
    } else {
      const uint32_t mbo = al - hb32((uint32_t)nv - 1);
      const uint32_t msp = (uint32_t)nv << mbo;
      dnb = (int32_t)((mbo << 16) - msp);
      dfs = (int32_t)cumul - nv;
    }
    tr[lane] = (uint32_t)dnb | ((uint32_t)dfs << 20);
  }
  lds_order();
}

__device__ __forceinline__ uint32_t tr_d(uint32_t e) { return e & 0xFFFFFu; }
__device__ __forceinline__ int32_t tr_f(uint32_t e) { return (int32_t)e >> 20; }

// FSE_initCState2 / FSE_encodeSymbol over an LDS table (lane-serial)
__device__ __forceinline__ uint32_t enc_init(const uint16_t* st, const uint32_t* tr, uint32_t s) {
  const uint32_t d = tr_d(tr[s]);
  const uint32_t nbo = (d + (1u << 15)) >> 16;
  const uint32_t val = (nbo << 16) - d;
  return st[(int32_t)(val >> nbo) + tr_f(tr[s])];
}
__device__ __forceinline__ uint32_t enc_sym(SBits& w, const uint16_t* st, const uint32_t* tr,
                                            uint32_t state, uint32_t s) {
  const uint32_t nbo = (state + tr_d(tr[s])) >> 16;
  w.add(state, nbo);
  return st[(int32_t)(state >> nbo) + tr_f(tr[s])];
}

// Huffman weights in FSE form into L.tmp (oracle zs_weights_fse); 0 if not codable.  All
// lanes: the weight counts by ballots, the table by build_ctable_par; one lane normalizes
// and writes the header (<= 13 symbols).  The two interleaved state chains then run as
// uniform scalar code: the weights, the state table (<= 64 cells) and the transforms (<= 13)
// sit in VGPRs, one per lane, read with v_readlane; bits collect in a 64-bit accumulator
// written out 4 bytes at a time (the serial writer's bytes, in its order).
__device__ uint32_t weights_fse(EntLds& L, uint32_t nw) {
  const uint32_t lane = lane_id();
  if (nw < 2) return 0;
  uint32_t wv[4];
#pragma unroll
  for (uint32_t c = 0; c < 4; ++c) wv[c] = 64 * c + lane < nw ? L.w[64 * c + lane] : 0xFFu;
  uint32_t max_w = 0, distinct = 0;
  for (uint32_t x = 0; x <= 12; ++x) {
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t c = 0; c < 4; ++c) cnt += (uint32_t)__builtin_popcountll(ballot(wv[c] == x));
    if (lane == 0) L.wk[x] = cnt;
    distinct += cnt ? 1u : 0u;
    max_w = cnt ? x : max_w;
  }
  if (distinct < 2) return 0;
  const uint32_t tl = table_log(6, nw, max_w);
  uint32_t hdr = 0;
  lds_order();
  if (lane == 0) {
    normalize(L.wk, max_w, nw, tl, L.norm);
    SBits hw(L.tmp + 1);
    hdr = write_ncount(hw, L.norm, max_w, tl);  // (padded to a byte)
  }
  lds_order();
  hdr = readlane(hdr, 0);
  build_ctable_par(L.norm, max_w, tl, L.tabs, L.tr[0], L.sym_at);
  const uint32_t stv = lane < (1u << tl) ? L.tabs[lane] : 0u;
  const uint32_t trv = lane <= max_w ? L.tr[0][lane] : 0u;
  // the serial writer's state, as uniform values: out byte pos, accumulator, its bit count
  uint32_t pos = 1 + hdr, nb = 0;
  uint64_t acc = 0;
  auto put = [&](uint32_t v, uint32_t n) __attribute__((always_inline)) {
    acc |= (uint64_t)(v & ((1u << n) - 1u)) << nb;  // (n <= 6 here; n == 0 adds nothing)
    nb += n;
    if (nb >= 32) {
      const uint32_t word = (uint32_t)acc;
      if (lane < 4) L.tmp[pos + lane] = (uint8_t)(word >> (8 * lane));
      pos += 4;
      acc >>= 32;
      nb -= 32;
    }
  };
  auto wat = [&](uint32_t i) __attribute__((always_inline)) {
    const uint32_t c = i >> 6, l = i & 63u;
    return readlane(c == 0 ? wv[0] : c == 1 ? wv[1] : c == 2 ? wv[2] : wv[3], l);
  };
  auto init = [&](uint32_t sy) __attribute__((always_inline)) {
    const uint32_t e = readlane(trv, sy);
    const uint32_t d = tr_d(e);
    const uint32_t nbo = (d + (1u << 15)) >> 16;
    const uint32_t val = (nbo << 16) - d;
    return readlane(stv, (uint32_t)((int32_t)(val >> nbo) + tr_f(e)));
  };
  auto enc = [&](uint32_t state, uint32_t sy) __attribute__((always_inline)) {
    const uint32_t e = readlane(trv, sy);
    const uint32_t nbo = (state + tr_d(e)) >> 16;
    put(state, nbo);
    return readlane(stv, (uint32_t)((int32_t)(state >> nbo) + tr_f(e)));
  };
  uint32_t s1, s2;
  int32_t i = (int32_t)nw;
  if (nw & 1) {
    s1 = init(wat((uint32_t)--i));
    s2 = init(wat((uint32_t)--i));
    s1 = enc(s1, wat((uint32_t)--i));
  } else {
    s2 = init(wat((uint32_t)--i));
    s1 = init(wat((uint32_t)--i));
  }
  while (i > 0) {
    s2 = enc(s2, wat((uint32_t)--i));
    s1 = enc(s1, wat((uint32_t)--i));
    if (pos - 1 + (nb >> 3) > 200) return 0;  // far past the 128-byte limit: give up early
  }
  put(s2, tl);
  put(s1, tl);
  put(1, 1);
  // the rest of the accumulator, then the final partial byte
  const uint32_t nbytes = (nb + 7) >> 3;
  if (lane < nbytes) L.tmp[pos + lane] = (uint8_t)(acc >> (8 * lane));
  const uint32_t size = pos + nbytes - 1;  // (L.tmp[0] is the size byte)
  if (size >= 128) return 0;
  if (lane == 0) L.tmp[0] = (uint8_t)size;
  lds_order();
  return size + 1;
}

// one sequence table's choice (oracle zs_choose), lane-serial; t: 0 LL, 1 OF, 2 ML.  Appends
// its description to w, returns mode | al << 8 | max_sym << 16 (RLE: its state table and
// transform written here, al 0); the caller builds the FSE tables of modes 0 and 2 from
// L.norm (2) or the predefined distribution (0) with all lanes.
__device__ uint32_t choose_table(EntLds& L, uint32_t t, uint32_t nseq, SBits& w) {
  const uint32_t* cnt = L.sh[t];
  const uint32_t nsym = t == 0 ? 36u : t == 1 ? 32u : 53u;
  uint32_t max_sym = 0, distinct = 0;
  for (uint32_t s = 0; s < nsym; ++s)
    if (cnt[s]) {
      ++distinct;
      max_sym = s;
    }
  uint16_t* st = L.tabs + (t == 0 ? kTabLL : t == 1 ? kTabOF : kTabML);
  uint32_t* tr = L.tr[t];
  if (distinct == 1) {  // RLE: no state, no bits
    w.add(max_sym, 8);
    tr[max_sym] = 0;
    st[0] = 0;
    return 1u;
  }
  const int16_t* def = t == 0 ? sT.ll_norm : t == 1 ? sT.of_norm : sT.ml_norm;
  const uint32_t def_al = t == 1 ? 5u : 6u, def_max = t == 0 ? 35u : t == 1 ? 28u : 52u;
  uint32_t cost_pre = 0;
  for (uint32_t s = 0; s <= max_sym; ++s) {
    if (!cnt[s]) continue;
    const uint32_t nd = def[s] == -1 ? 1u : (uint32_t)def[s];
    cost_pre += cnt[s] * ((def_al << 8) - log2fix(nd));
  }
  const uint32_t tl = table_log(t == 1 ? 8u : 9u, nseq, max_sym);
  int16_t* norm = L.norm;
  normalize(cnt, max_sym, nseq, tl, norm);
  uint32_t cost_fse = 0;
  for (uint32_t s = 0; s <= max_sym; ++s)
    if (cnt[s]) cost_fse += cnt[s] * ((tl << 8) - log2fix((uint32_t)norm[s]));
  SBits tw(L.tmp);
  const uint32_t nb = write_ncount(tw, norm, max_sym, tl);
  cost_fse += nb * 8u * 256u;
  if (cost_fse < cost_pre) {
    for (uint32_t k = 0; k < nb; ++k) w.add(L.tmp[k], 8);
    return 2u | (tl << 8) | (max_sym << 16);  // (tables: build_ctable_par over L.norm)
  }
  // predefined: its distribution (with "less than 1" symbols)
  return 0u | (def_al << 8) | (def_max << 16);
}

struct EntOut : ByteOutT<kObuf, true> {
  // OR the lanes' bit fields (v0 of n0 bits, then v1 of n1 bits; n0 + n1 <= 96), in
  // DESCENDING lane order, into the bitstream that starts at output byte p0; bits = bits
  // written so far (zeroed: unused, the ring is cleared as it is flushed)
  __device__ __forceinline__ void put_bits(uint64_t v0, uint32_t n0, uint64_t v1, uint32_t n1,
                                           uint32_t p0, uint32_t& bits, uint32_t& zeroed) {
    const uint32_t nb = n0 + n1;
    const uint32_t incl = wave_incl_sum(nb);
    const uint32_t total = readlane(incl, 63);
    op = p0 + (bits >> 3);
    if (!room((total >> 3) + 16)) return;
    (void)zeroed;  // (the ring bytes at and past op are zero: cleared as they are flushed)
    const uint32_t pos = bits + total - incl;  // lanes above come first
    const uint32_t base = (((uint32_t)(uintptr_t)dst + p0) & kObufMask) << 3;
    const uint32_t wmask = kObufMask >> 2;
    uint32_t* r32 = reinterpret_cast<uint32_t*>(ring);
    auto place = [&](uint64_t v, uint32_t a) {
      const uint32_t wi = (a >> 5) & wmask, sh = a & 31u;
      const uint32_t x0 = (uint32_t)(v << sh);
      const uint32_t x1 = (uint32_t)((v << sh) >> 32);
      const uint32_t x2 = sh ? (uint32_t)(v >> (64 - sh)) : 0u;
      if (x0) atomicOr(&r32[wi], x0);
      if (x1) atomicOr(&r32[(wi + 1) & wmask], x1);
      if (x2) atomicOr(&r32[(wi + 2) & wmask], x2);
    };
    lds_order();
    if (n0) place(v0 & (n0 >= 64 ? ~0ull : (1ull << n0) - 1), base + pos);
    if (n1) place(v1 & (n1 >= 64 ? ~0ull : (1ull << n1) - 1), base + pos + n0);
    lds_order();
    bits += total;
    op = p0 + (bits >> 3);
  }

  // bytes from LDS (lane-parallel), n <= 256
  __device__ __forceinline__ void put_lds(const uint8_t* src, uint32_t n) {
    for (uint32_t k = 0; k < n; k += kWave) {
      const uint32_t step = n - k < kWave ? n - k : kWave;
      if (!room(step)) return;
      lds_order();
      const uint32_t b = src[k + (lane_id() < step ? lane_id() : 0u)];
      put(b, step);
    }
  }
};

}  // namespace zse

// The Zstd parse is the repeat-offset form with window skipping (oracle BO_PARSE_REP |
// BO_PARSE_SKIP); BITAR_ZSTD_SKIP=0 builds the plain repeat-offset scan, BITAR_ZSTD_REP=0 the
// parse without repeat candidates (timing knobs only: not the oracle's output).
#ifndef BITAR_ZSTD_SKIP
#define BITAR_ZSTD_SKIP 1
#endif
#ifndef BITAR_ZSTD_REP
#define BITAR_ZSTD_REP 1
#endif
__global__ __launch_bounds__(64) void zstd_parse_kernel(const uint8_t* __restrict__ input,
                                                        uint64_t n_total, uint32_t seg,
                                                        uint8_t* __restrict__ scratch,
                                                        uint64_t sstride,
                                                        uint2* __restrict__ meta, const uint32_t* __restrict__ order) {
  using namespace cmp;
  // (+ one trash entry: probe lanes past the segment insert there, see parse)
  __shared__ __attribute__((aligned(16))) uint16_t table[(1u << kHashLog) + 8];
  __shared__ __attribute__((aligned(16))) uint8_t inring[kIn + kInPad];
#if BITAR_ZSTD_BULK
  __shared__ __attribute__((aligned(16))) zse::ZsLds zl;
#else
  __shared__ __attribute__((aligned(16))) uint8_t obuf[kObuf + kWave];  // + trash bytes
#endif
  const uint32_t i_seg = order ? order[blockIdx.x] : blockIdx.x;  // (cost-ordered dispatch)
  const uint64_t seg_off = (uint64_t)i_seg * seg;
  if (seg_off >= n_total) return;
  const uint32_t n = (uint32_t)((n_total - seg_off) < seg ? (n_total - seg_off) : seg);
  zse::SeqCollect o;
#if BITAR_ZSTD_BULK
  o.L = &zl;
  o.ring = zl.ring;
  o.npend = 0;
  o.last_end = 0;
  zl.marks[lane_id()] = 0;
  lds_order();
#else
  o.ring = obuf;
#endif
  o.dst = global_ptr(scratch + (uint64_t)i_seg * sstride);
  o.cap = zse::lit_cap(seg);
  o.op = 0;
  o.flushed = 0;
  o.overflow = false;
  o.seqs = reinterpret_cast<GMEM uint2*>(o.dst + zse::lit_cap(seg));
  o.nseq = 0;
  const GMEM uint8_t* in = global_ptr(input + seg_off);
  parse<zse::SeqCollect, BITAR_ZSTD_REP != 0, BITAR_ZSTD_SKIP != 0>(in, n, global_ptr(input + n_total), table, inring, kMaxDist,
                               0xFFFFFFFFu, o);
  o.flush(o.op, true);
  if (lane_id() == 0) meta[i_seg] = make_uint2(o.op, o.nseq);
}

// first sequence of block b of nb (block nb: nseq), oracle zs_nblocks' split
__device__ __forceinline__ uint32_t blk_start_of(uint32_t b, uint32_t nseq, uint32_t nb) {
  return b >= nb ? nseq : (uint32_t)((uint64_t)b * nseq / nb);
}

#ifndef BITAR_ZSE_RUNS
#define BITAR_ZSE_RUNS 1
#endif
// h[c] += 1 for each active lane's code c, as one LDS atomic per run of equal codes (lanes
// [0, cnt) active): a run starts where the code differs from the previous lane's, and its
// first lane adds the distance to the next run's start
__device__ __forceinline__ void run_add(uint32_t* h, uint32_t c, bool act, uint32_t cnt) {
  const uint32_t lane = lane_id();
  const uint32_t prev = wave_shr1(c);
  const uint64_t heads = ballot(act & ((lane == 0) | (c != prev)));
  const uint64_t after = (heads >> lane) >> 1;
  const uint32_t nxt = after ? lane + 1u + (uint32_t)__builtin_ctzll(after) : cnt;
  if ((heads >> lane) & 1u) atomicAdd(&h[c], nxt - lane);
}

__global__ __launch_bounds__(64) void zstd_entropy_kernel(
    const uint8_t* __restrict__ input, uint64_t n_total, uint32_t seg,
    uint8_t* __restrict__ scratch, uint64_t sstride, const uint2* __restrict__ meta,
    uint8_t* __restrict__ wscr, uint64_t wstride, const uint32_t* __restrict__ order) {
  using namespace cmp;
  using namespace zse;
  __shared__ __attribute__((aligned(16))) EntLds L;
  const uint32_t i_seg = order ? order[blockIdx.x] : blockIdx.x;  // (cost-ordered dispatch)
  const uint64_t seg_off = (uint64_t)i_seg * seg;
  if (seg_off >= n_total) return;
  const uint32_t n = (uint32_t)((n_total - seg_off) < seg ? (n_total - seg_off) : seg);
  const uint32_t lane = lane_id();
  GMEM uint8_t* lits = global_ptr(scratch + (uint64_t)i_seg * sstride);
  GMEM uint2* seqs = reinterpret_cast<GMEM uint2*>(lits + lit_cap(seg));
  GMEM uint32_t* wrec = global_ptr(reinterpret_cast<uint32_t*>(wscr + (uint64_t)i_seg * wstride));
  GMEM uint8_t* wbytes = reinterpret_cast<GMEM uint8_t*>(wrec);
  for (uint32_t k = lane; k < sizeof(Tabs); k += kWave)
    reinterpret_cast<uint8_t*>(&sT)[k] = reinterpret_cast<const uint8_t*>(&kT)[k];
  lds_order();
  const uint2 mt = meta[i_seg];
  const uint32_t nlit = mt.x, nseq = mt.y;

  // ---- the literal code (shared by the frame's blocks): histogram, code lengths, codes,
  // tree description.  Which blocks use it, and the literal sections themselves, are
  // zstd_emit_kernel's (oracle zs_littab_build / zs_literals_block). ----
  for (uint32_t k = lane; k < 256; k += kWave) L.hist[k] = 0;
  lds_order();
  // (the next 1 KiB is loaded before this one's 16 LDS atomics per lane: at one load per
  // step the wave waited on every one of them)
  uint4 vn = make_uint4(0, 0, 0, 0);
  if (16u * lane < nlit) vn = *reinterpret_cast<const GMEM uint4*>(lits + 16u * lane);
  for (uint32_t b0 = 0; b0 < nlit; b0 += 16u * kWave) {
    const uint32_t at = b0 + 16u * lane;
    const uint4 v = vn;
    const uint32_t an = at + 16u * kWave;
    if (an < nlit) vn = *reinterpret_cast<const GMEM uint4*>(lits + an);
    const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j)
      if (at + j < nlit) atomicAdd(&L.hist[(wv[j >> 2] >> (8 * (j & 3))) & 0xFFu], 1u);
  }
  lds_order();
  uint32_t distinct = 0;
  for (uint32_t s0 = 0; s0 < 256; s0 += kWave)
    distinct += (uint32_t)__builtin_popcountll(ballot(L.hist[s0 + lane] != 0));
  lds_order();
  ZSE_PHASE(1)
  uint32_t lmode = 0, lrle = 0, dsz = 0, tbits = 0;
  if (nlit > 0 && distinct == 1) {
    lmode = 1;
    lrle = lits[0];
  } else if (nlit > 0) {
    huf::huff_lengths(L.hist, 256, 11, L.len, L.T);
    ZSE_PHASE(6)
    // max length, highest used symbol, weights
    uint32_t lmax = 0, msym = 0;
    for (uint32_t s0 = 0; s0 < 256; s0 += kWave) {
      const uint32_t l = L.len[s0 + lane];
      lmax = max(lmax, l);
      const uint64_t used = ballot(l != 0);
      if (used) msym = s0 + 63u - (uint32_t)__builtin_clzll(used);
    }
    for (uint32_t d = 1; d < 64; d <<= 1) lmax = max(lmax, (uint32_t)__shfl_xor((int)lmax, (int)d, 64));
    lmax = readlane(lmax, 0);
    for (uint32_t s0 = 0; s0 < 256; s0 += kWave) {
      const uint32_t l = L.len[s0 + lane];
      L.w[s0 + lane] = (uint8_t)(l ? lmax + 1 - l : 0u);
    }
    lds_order();
    {
      // codes: table ranges by increasing weight, then symbol (HUF_readDTableX1): a symbol
      // of weight wt takes start[wt] >> (wt - 1) plus its rank among the weight's symbols
      // (ballots per weight, all lanes)
      uint32_t wv[4], rk[4];
#pragma unroll
      for (uint32_t c = 0; c < 4; ++c) {
        wv[c] = L.len[64 * c + lane] ? L.w[64 * c + lane] : 0u;
        rk[c] = 0;
      }
      uint32_t next = 0;
      for (uint32_t wt = 1; wt <= lmax; ++wt) {
        uint32_t tot = 0;
#pragma unroll
        for (uint32_t c = 0; c < 4; ++c) {
          const uint64_t mw = ballot(wv[c] == wt);
          const uint32_t below = __builtin_amdgcn_mbcnt_hi(
              (uint32_t)(mw >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mw, 0u));
          rk[c] = wv[c] == wt ? tot + below : rk[c];
          tot += (uint32_t)__builtin_popcountll(mw);
        }
        if (lane == 0) L.wk[wt] = next >> (wt - 1);
        next += tot << (wt - 1);
      }
      lds_order();
#pragma unroll
      for (uint32_t c = 0; c < 4; ++c) {
        const uint32_t s = 64 * c + lane, l = L.len[s];
        wrec[kWCodeAt + s] = l ? (L.wk[wv[c]] + rk[c]) | (l << 16) : 0u;
      }
      lds_order();
    }
    const uint32_t fsz = BITAR_ZSTD_STOP == 7 ? 0u : weights_fse(L, msym);  // (all lanes)
    if (lane == 0) {
      // tree description: direct when possible and not larger than the FSE form
      const uint32_t nw = msym;
      const uint32_t direct = nw <= 128 ? 1 + (nw + 1) / 2 : 0u;
      uint32_t d = 0;
      if (direct && (!fsz || direct <= fsz)) {
        L.desc[0] = (uint8_t)(127 + nw);
        for (uint32_t i = 0; i < nw; i += 2)
          L.desc[1 + i / 2] = (uint8_t)((L.w[i] << 4) | (i + 1 < nw ? L.w[i + 1] : 0u));
        d = direct;
      } else if (fsz) {
        for (uint32_t k = 0; k < fsz; ++k) L.desc[k] = L.tmp[k];
        d = fsz;
      }
      L.u[0] = d;
    }
    lds_order();
    dsz = L.u[0];
    for (uint32_t k = lane; k < dsz; k += kWave) wbytes[4 * kWTreeAt + k] = L.desc[k];
    if (dsz) lmode = 2;
    uint32_t tbl = 0;
#pragma unroll
    for (uint32_t c = 0; c < 4; ++c) tbl += (uint32_t)L.len[64 * c + lane] * L.hist[64 * c + lane];
    tbits = readlane(wave_incl_sum(tbl), kWave - 1);
  }
  ZSE_PHASE(2)

  // ---- sequences: the blocks (equal sequence counts), repeat offsets (rep_scan), codes,
  // histograms, 64 sequences per step from each block's first; the history before each step
  // goes to the walk scratch (the records stay as the parse wrote them) ----
  const uint32_t nb = frame_blocks(nseq, nlit);
  uint32_t tdesc = 0;
  if (nseq) {
    for (uint32_t k = lane; k < 3 * 64; k += kWave) (&L.sh[0][0])[k] = 0;
    lds_order();
    uint32_t c0r = 1, c1r = 4, c2r = 8;  // the history before the step (uniform)
    GMEM uint32_t* wcodes = reinterpret_cast<GMEM uint32_t*>(wbytes + kWWords);
    uint32_t st = 0, lacc = 0;  // literal bytes before the step, per lane (summed per block)
    uint2 nrec = lane < nseq ? seqs[lane] : make_uint2(0, 3);
    uint32_t s0 = 0, s1 = blk_start_of(1u, nseq, nb);
    for (uint32_t b = 0; b < nb; ++b) {
      const uint32_t lsum = b ? readlane(wave_incl_sum(lacc), kWave - 1) : 0u;
      wrec[lane == 0 ? kWSb + b : kWTrash] = s0;
      wrec[lane == 0 ? kWLb + b : kWTrash] = lsum;
      for (uint32_t c0 = s0; c0 < s1; c0 += kWave, ++st) {
        const uint32_t j = c0 + lane;
        const uint32_t cnt = s1 - c0 < kWave ? s1 - c0 : kWave;
        const bool act = lane < cnt;
        const uint2 rec = nrec;
        // prefetch the next step (it starts right after this one's last sequence).  The
        // step's load and stores are issued on every lane (past the end: the last record, the
        // record's trash word): their number per step is fixed, so the wait for this load
        // does not have to wait for the stores issued after it.
        const uint32_t jn = c0 + cnt + lane;
        nrec = seqs[jn < nseq ? jn : nseq - 1u];
        const uint32_t ll = act ? rec.x & 0x1FFFFu : 0u, o = rec.x >> 17, ml = rec.y;
        const uint32_t ov = rep_scan(ll, o, act, cnt, c0r, c1r, c2r);
        const uint32_t llc = ll_code(ll), ofc = hb32(ov), mlc = ml_code(ml);
#if BITAR_ZSE_RUNS
        // histograms: LDS atomics cost about a cycle per lane, and a step holds few distinct
        // codes in runs of equal ones (kind 2: ~30 runs of 64), so one lane per run adds the
        // run's length
        run_add(L.sh[0], llc, act, cnt);
        run_add(L.sh[1], ofc, act, cnt);
        run_add(L.sh[2], mlc, act, cnt);
#else
        if (act) {
          atomicAdd(&L.sh[0][llc], 1u);
          atomicAdd(&L.sh[1][ofc], 1u);
          atomicAdd(&L.sh[2][mlc], 1u);
        }
#endif
        // for zstd_walk_kernel (the codes) and zstd_emit_kernel (the codes, the offset value:
        // <= kMaxDist + 3, 15 bits)
        static_assert(cmp::kMaxDist + 3u < (1u << 15), "offset values in the code word");
        *(act ? wcodes + j : wrec + kWTrash) = llc | (ofc << 6) | (mlc << 11) | (ov << 17);
        lacc += ll;
      }
      s0 = s1;
      s1 = blk_start_of(b + 2u, nseq, nb);
    }
    lds_order();
    ZSE_PHASE(4)
    // tables (one lane): modes byte + descriptions in L.desc, states / transforms
    SBits w(L.desc + 1);  // (lane 0's)
    uint32_t md[3];
#pragma unroll
    for (uint32_t t = 0; t < 3; ++t) {
      uint32_t mo = 0;
      if (lane == 0) mo = choose_table(L, t, nseq, w);
      lds_order();
      mo = readlane(mo, 0);
      md[t] = mo;
      if ((mo & 3u) != 1u) {  // FSE_Compressed (from L.norm) or predefined
        const int16_t* nrm = (mo & 3u) == 2u ? L.norm : t == 0 ? sT.ll_norm : t == 1 ? sT.of_norm : sT.ml_norm;
        build_ctable_par(nrm, mo >> 16, (mo >> 8) & 0xFFu,
                         L.tabs + (t == 0 ? kTabLL : t == 1 ? kTabOF : kTabML), L.tr[t], L.sym_at);
      }
    }
    if (lane == 0) {
      L.desc[0] = (uint8_t)(((md[0] & 3u) << 6) | ((md[1] & 3u) << 4) | ((md[2] & 3u) << 2));
      L.u[1] = w.pos + 1;
      L.u[2] = (md[0] >> 8) & 0xFFu;
      L.u[3] = (md[1] >> 8) & 0xFFu;
      L.u[4] = (md[2] >> 8) & 0xFFu;
      L.tabs[kTabDummy] = 0;
    }
    lds_order();
    ZSE_PHASE(5)
    tdesc = L.u[1];
    for (uint32_t k = lane; k < tdesc; k += kWave) wbytes[4 * kWDescAt + k] = L.desc[k];
    // the state tables and transforms for zstd_walk_kernel
    for (uint32_t k = lane; k < (kTabDummy + 1 + 1) / 2; k += kWave)
      wrec[kWTabs / 4 + k] = reinterpret_cast<const uint32_t*>(L.tabs)[k];
    for (uint32_t k = lane; k < 3 * 64; k += kWave) wrec[kWTr / 4 + k] = (&L.tr[0][0])[k];
  } else if (lane == 0) {
    wrec[kWSb] = 0;
    wrec[kWLb] = 0;
  }
  // the record: everything zstd_emit_kernel needs to write the frame
  if (lane == 0) {
    wrec[kWN] = n;
    wrec[kWNseq] = nseq;
    wrec[kWAls] = nseq ? L.u[2] | (L.u[3] << 8) | (L.u[4] << 16) : 0u;
    wrec[kWNb] = nb;
    wrec[kWLit] = lmode | (lrle << 8) | (dsz << 16);
    wrec[kWNlit] = nlit;
    wrec[kWTdesc] = tdesc;
    wrec[kWTb] = tbits;
    wrec[kWSb + nb] = nseq;
    wrec[kWLb + nb] = nlit;
    wrec[kWHanded] = 1u;
  }
}

template <int K>
__device__ __forceinline__ uint32_t zsq_qbcast(uint32_t v) {  // lane K of each quad, to all four
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, K * 0x55, 0xF, 0xF, false);
}

// ---- pass 3: the FSE state chains, four lanes per chain set --------------------------------
// Lane 16 l + 4 b + j of the wave walks chain j (0 offsets, 1 match lengths, 2 literal
// lengths; 3 repeats 0) of block b (then b + 4) of segment blockIdx.x * 4 + l, the block's last sequence
// first, with the segment's state table and transforms in LDS: the chains of a block are
// independent of each other and of the other blocks' (each block's states start from its own
// last sequence), so each is a lane's own loop.  Per sequence the lane stores its chain's
// state bits | count << 12 (u16), 8 at a time; each block's final states go to the segment's
// record.  Same arithmetic as the oracle's per-block walk (bo_zstd_compress_block), bit for
// bit.
constexpr uint32_t kWalkSegs = 4;
__global__ __launch_bounds__(64) void zstd_walk_kernel(const uint8_t* __restrict__ scratch,
                                                        uint64_t sstride, uint32_t seg,
                                                        uint32_t nseg, uint8_t* __restrict__ wscr,
                                                        uint64_t wstride,
                                                        const uint32_t* __restrict__ order) {
  using namespace cmp;
  using namespace zse;
  static_assert(kWalkSegs * 4 * 4 == kWave && kBlocks <= 8, "a lane per chain of 4 blocks");
  __shared__ __attribute__((aligned(16))) uint16_t tabs[kWalkSegs][1284];
  __shared__ uint32_t trs[kWalkSegs][3][64];
  const uint32_t lane = lane_id();
  // (order: the segments by sequence count, walk_key_kernel; slot b walks segment order[b])
  // The wave's segments are looked up one lane each, together, and each segment's table loads
  // are issued before the first is stored.
  uint32_t il0 = 0, hd0 = 0;
  {
    const uint32_t bl = blockIdx.x * kWalkSegs + lane;
    if (lane < kWalkSegs && bl < nseg) {
      il0 = order ? order[bl] : bl;
      const GMEM uint32_t* w0 = global_ptr(reinterpret_cast<const uint32_t*>(wscr + (uint64_t)il0 * wstride));
      hd0 = w0[kWHanded] == 1u && w0[kWNseq] != 0u;
    }
  }
  const uint64_t hm = ballot(hd0 != 0u);
  for (uint64_t m = hm; m; m &= m - 1) {
    const uint32_t l = (uint32_t)__builtin_ctzll(m);
    const uint32_t il = readlane(il0, l);
    const GMEM uint32_t* w = global_ptr(reinterpret_cast<const uint32_t*>(wscr + (uint64_t)il * wstride));
    constexpr uint32_t kTw = 1284 / 2, kTn = (kTw + kWave - 1) / kWave;
    uint32_t tv[kTn], rv[3];
#pragma unroll
    for (uint32_t e = 0; e < kTn; ++e) {
      const uint32_t k = lane + e * kWave;
      tv[e] = w[kWTabs / 4 + (k < kTw ? k : 0u)];
    }
#pragma unroll
    for (uint32_t e = 0; e < 3; ++e) rv[e] = w[kWTr / 4 + lane + e * kWave];
#pragma unroll
    for (uint32_t e = 0; e < kTn; ++e) {
      const uint32_t k = lane + e * kWave;
      if (k < kTw) reinterpret_cast<uint32_t*>(tabs[l])[k] = tv[e];
    }
#pragma unroll
    for (uint32_t e = 0; e < 3; ++e) (&trs[l][0][0])[lane + e * kWave] = rv[e];
  }
  lds_order();
  const uint32_t l = lane >> 4, j = lane & 3u;
  const uint32_t b = blockIdx.x * kWalkSegs + l;
  // (fetched while every lane is active: a disabled source lane reads as 0)
  const uint32_t i = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(l << 2), (int)il0);
  if (b >= nseg || !((hm >> l) & 1u)) return;  // uniform over the segment's 16 lanes
  GMEM uint32_t* w = global_ptr(reinterpret_cast<uint32_t*>(wscr + (uint64_t)i * wstride));
  const uint32_t nbk = w[kWNb];
  const GMEM uint32_t* codes = w + kWWords / 4;
  const uint32_t c = j == 3 ? 0u : j;  // chain
  // (walk_state_at: the quad's three chains store 48 contiguous bytes per group of 8)
  GMEM uint16_t* outs =
      reinterpret_cast<GMEM uint16_t*>(reinterpret_cast<GMEM uint8_t*>(w) + walk_state_bytes(seg)) +
      c * 8u;
  auto at = [](uint32_t k) __attribute__((always_inline)) { return (k >> 3) * 24u + (k & 7u); };
  const uint16_t* tb = tabs[l] + (c == 0 ? kTabOF : c == 1 ? kTabML : kTabLL);
  const uint32_t* tr = trs[l][c == 0 ? 1 : c == 1 ? 2 : 0];
  // this chain's code in the code word (LL 6 bits, OF 5, ML 6)
  const uint32_t csh = c == 0 ? 6u : c == 1 ? 11u : 0u, cmask = c == 0 ? 31u : 63u;
  auto code = [&](uint32_t cw) __attribute__((always_inline)) { return (cw >> csh) & cmask; };
  // quad q walks blocks q and q + 4 (8-block frames), one after the other (quad-uniform)
  for (uint32_t blk = (lane >> 2) & 3u; blk < nbk; blk += 4) {
  const uint32_t s0 = w[kWSb + blk], s1 = w[kWSb + blk + 1];
  // the block's last sequence initialises the states (no state bits)
  const uint32_t top = s1 - 1;
  uint32_t st;
  {
    const uint32_t e = tr[code(codes[top])];
    const uint32_t d = tr_d(e);
    const uint32_t nbo = (d + (1u << 15)) >> 16;
    const uint32_t val = (nbo << 16) - d;
    st = tb[(int32_t)(val >> nbo) + tr_f(e)];
  }
  // one chain step: this chain's state bits | count << 12 (only the state table read is on
  // the loop-carried chain)
  auto walk = [&](uint32_t e) __attribute__((always_inline)) {
    const uint32_t nb = (st + tr_d(e)) >> 16;
    const uint32_t out = (st & ((1u << nb) - 1u)) | (nb << 12);
    st = tb[(int32_t)(st >> nb) + tr_f(e)];
    return out;
  };
  if (j < 3) outs[at(top)] = 0;
  // k: sequences top - 1 .. s0, as offsets below top (kk = top - 1 - k')
  const int32_t lo = (int32_t)s0;
  int32_t k = (int32_t)top - 1;
  constexpr int32_t kG = 8;
  // single steps down to a group boundary (k = 8 g + 7)
  for (; k >= lo && (k & 7) != 7; --k) {
    const uint32_t o = walk(tr[code(codes[k])]);
    if (j < 3) outs[at((uint32_t)k)] = (uint16_t)o;
  }
  // groups of 8: the transforms looked up together (independent of the states), then the
  // chain; the lane's 8 outputs stored together
  uint32_t r[kG];
#pragma unroll
  for (int32_t g = 0; g < kG; ++g) r[g] = codes[k - g >= lo ? k - g : lo];
  for (; k >= lo + kG - 1; k -= kG) {
    uint32_t e[kG], o[kG];
#pragma unroll
    for (int32_t g = 0; g < kG; ++g) e[g] = tr[code(r[g])];
#pragma unroll
    for (int32_t g = 0; g < kG; ++g) r[g] = codes[k - kG - g >= lo ? k - kG - g : lo];  // next group
#pragma unroll
    for (int32_t g = 0; g < kG; ++g) o[g] = walk(e[g]);
    if (j < 3) {
      // the group's 8 outputs (sequences k - 7 .. k) as ONE 16-byte store, next to the quad's
      // other two chains': one 48-byte run per quad and group (one stream per chain, 48
      // streams per wave, were written back as partial lines: 3.0 GB of walk writes per GiB
      // against 0.7 GB of state bits)
      const uint4 v = make_uint4(o[7] | (o[6] << 16), o[5] | (o[4] << 16), o[3] | (o[2] << 16),
                                 o[1] | (o[0] << 16));
      *reinterpret_cast<GMEM uint4*>(outs + at((uint32_t)(k - kG + 1))) = v;  // 16-B aligned
    }
  }
  for (; k >= lo; --k) {
    const uint32_t o = walk(tr[code(codes[k])]);
    if (j < 3) outs[at((uint32_t)k)] = (uint16_t)o;
  }
  if (j < 3) w[kWFin + 3 * blk + j] = st;
  }
}

// ---- pass 4: the frame -----------------------------------------------------------------------
// One wave per segment writes the whole frame: the frame header, then per block its literal
// section (Huffman streams of the block's literals with the shared code -- the tree in the
// first Huffman-coded block, Treeless after it -- or raw / RLE, oracle zs_literals_block),
// its sequence section header, the table descriptions (first block) or Repeat_Mode, and its
// sequence bitstream: the fields of 64 sequences per step (highest first) with the state bits
// from pass 3, the final states and the end mark.  Then the block headers, or one raw block
// when the compressed blocks are not smaller than the segment.
#ifndef BITAR_HUF_PER_LANE
#define BITAR_HUF_PER_LANE 8  // literals per lane and step in the Huffman streams (4 or 8)
#endif
#ifndef BITAR_EMIT_WAVES
#define BITAR_EMIT_WAVES 0
#endif
#if BITAR_EMIT_WAVES
#define BITAR_EMIT_ATTR __attribute__((amdgpu_waves_per_eu(BITAR_EMIT_WAVES)))
#else
#define BITAR_EMIT_ATTR
#endif
__global__ __launch_bounds__(64) BITAR_EMIT_ATTR void zstd_emit_kernel(
    const uint8_t* __restrict__ input, uint64_t n_total, uint32_t seg,
    const uint8_t* __restrict__ scratch, uint64_t sstride, uint8_t* __restrict__ slab,
    uint64_t slot_stride, uint8_t* const* __restrict__ dsts, uint32_t* __restrict__ sizes,
    const uint8_t* __restrict__ wscr, uint64_t wstride, const uint32_t* __restrict__ order) {
  using namespace cmp;
  using namespace zse;
  __shared__ __attribute__((aligned(16))) uint8_t obuf[kObuf + kWave];
  __shared__ __attribute__((aligned(16))) uint32_t hcode[256];  // code | length << 16
  __shared__ __attribute__((aligned(16))) uint8_t lst[16 * kWave];  // literal block being encoded
  __shared__ __attribute__((aligned(16))) uint8_t bytes[132 + 256];  // tree; table descriptions
  const uint32_t i_seg = order ? order[blockIdx.x] : blockIdx.x;  // (cost-ordered dispatch)
  const uint64_t seg_off = (uint64_t)i_seg * seg;
  if (seg_off >= n_total) return;
  const GMEM uint32_t* w = global_ptr(reinterpret_cast<const uint32_t*>(wscr + (uint64_t)i_seg * wstride));
  const GMEM uint8_t* wb = reinterpret_cast<const GMEM uint8_t*>(w);
  if (uniform(w[kWHanded]) != 1u) return;
  const uint32_t lane = lane_id();
  for (uint32_t k = lane; k < sizeof(Tabs); k += kWave)
    reinterpret_cast<uint8_t*>(&sT)[k] = reinterpret_cast<const uint8_t*>(&kT)[k];
  const uint32_t n = uniform(w[kWN]), als = uniform(w[kWAls]);
  const uint32_t nb = uniform(w[kWNb]), litw = uniform(w[kWLit]);
  const uint32_t tdesc = uniform(w[kWTdesc]), tbits = uniform(w[kWTb]);
  const uint32_t nlit = uniform(w[kWNlit]);
  const uint32_t lmode = litw & 0xFFu, lrle = (litw >> 8) & 0xFFu, dsz = litw >> 16;
  const uint32_t al_ll = als & 0xFFu, al_of = (als >> 8) & 0xFFu, al_ml = als >> 16;
  if (lmode == 2) {
    for (uint32_t k = lane; k < 256; k += kWave) hcode[k] = w[kWCodeAt + k];
    for (uint32_t k = lane; k < dsz; k += kWave) bytes[k] = wb[4 * kWTreeAt + k];
  }
  for (uint32_t k = lane; k < tdesc; k += kWave) bytes[132 + k] = wb[4 * kWDescAt + k];
  lds_order();
  const GMEM uint8_t* src = global_ptr(input + seg_off);
  const GMEM uint8_t* lits = global_ptr(scratch + (uint64_t)i_seg * sstride);
  const GMEM uint2* seqs = reinterpret_cast<const GMEM uint2*>(lits + lit_cap(seg));
  const GMEM uint16_t* outs = reinterpret_cast<const GMEM uint16_t*>(
      reinterpret_cast<const GMEM uint8_t*>(w) + walk_state_bytes(seg));
  const GMEM uint32_t* wcodes = w + kWWords / 4;
  EntOut o;
  o.ring = obuf;
  o.dst = global_ptr(dsts ? dsts[i_seg] : slab + (uint64_t)i_seg * slot_stride);
  o.cap = slot_stride;
  o.op = 0;
  o.flushed = 0;
  o.overflow = false;
  // the ring starts zeroed (EntOut clears what it flushes: the bit writer ORs into it)
  for (uint32_t k = lane; k < kObuf / 16; k += kWave)
    reinterpret_cast<uint4*>(obuf)[k] = make_uint4(0, 0, 0, 0);
  lds_order();
  // frame header: magic, Single_Segment with the content size (1 byte below 256, else 2)
  const uint32_t fh = n < 256 ? 6u : 7u;
  {
    const uint32_t fcs = n < 256 ? n : n - 256u;
    const uint32_t hb = lane < 4 ? (0xFD2FB528u >> (8 * lane)) & 0xFFu
                        : lane == 4 ? (n < 256 ? 0x20u : 0x60u)
                        : lane == 5 ? fcs & 0xFFu : fcs >> 8;
    o.put(hb, fh);
  }
  // per block (LDS, uniform): its header's position and value, and a Huffman literal
  // section's header and jump table, written at the end (their sizes are known once the
  // streams are): position (0: none), header size, header value (2 words), jump table
  // position (0: none) and stream sizes
  enum : uint32_t { kBPos, kBHdr, kPPos, kPHs, kPH0, kPH1, kPJt, kPZ, kPZ2, kBW };
  __shared__ uint32_t bm[kBlocks][kBW];
  for (uint32_t k = lane; k < kBlocks * kBW; k += kWave) (&bm[0][0])[k] = 0;
  auto bset = [&](uint32_t b, uint32_t f, uint32_t v) __attribute__((always_inline)) {
    lds_order();
    if (lane == 0) bm[b][f] = v;
    lds_order();
  };
  bool tree_sent = false;
  // literals [a, a + m) of the segment's literal area as a Huffman stream (oracle
  // zs_literals_block): symbols from the last, kPerLane x 64 per step, from 1 KiB blocks of aligned
  // 16-B groups staged in LDS, the next one loaded during the current one
  auto huff_stream = [&](uint32_t a, uint32_t b) __attribute__((always_inline)) {
    const uint32_t p0 = o.op;
    uint32_t bits = 0, zeroed = p0;
    const GMEM uint4* l16 = reinterpret_cast<const GMEM uint4*>(lits);
    const int32_t gA = (int32_t)(a >> 4), gB = (int32_t)((b + 15) >> 4);
    int32_t g0 = gB - (int32_t)kWave;
    uint4 blkv = make_uint4(0, 0, 0, 0);
    if (g0 + (int32_t)lane >= gA) blkv = l16[g0 + (int32_t)lane];
    for (;;) {
      lds_order();
      reinterpret_cast<uint4*>(lst)[lane] = blkv;
      const int32_t g1 = g0 - (int32_t)kWave;
      if (g0 > gA && g1 + (int32_t)lane >= gA) blkv = l16[g1 + (int32_t)lane];
      const int32_t lo = max((int32_t)a, 16 * g0), hi = min((int32_t)b, 16 * (g0 + (int32_t)kWave));
      // kPerLane x 64 symbols per step, lane l's are i0 .. i0 + kPerLane - 1, the highest
      // first (the stream runs from the last symbol down; put_bits takes the lanes in
      // descending order, each lane's v0 before its v1): v0 = the codes of the upper half,
      // v1 = those of the lower half, each from its highest symbol (<= kPerLane / 2 x 11 bits).
      // Per-step costs (the bit count's prefix sum, the room check, clearing the ring, the
      // LDS ORs) are shared by kPerLane symbols: 1 -> 2 / 4 / 8 per lane, emit 1.38 -> 1.16 /
      // 0.99 / 0.96 ms (kind 2)
      constexpr int32_t kPerLane = BITAR_HUF_PER_LANE;
      static_assert(kPerLane == 4 || kPerLane == 8, "4 or 8 literals per lane");
      // (steps end at multiples of 8, so a lane's 8 symbol bytes are ONE aligned 8-byte LDS
      // read; symbols outside [lo, hi) are masked)
      static_assert(kPerLane == 8 || kPerLane == 4, "");
      for (int32_t e = (hi + 7) & ~7; e > lo && !o.overflow; e -= kPerLane * (int32_t)kWave) {
        const int32_t i0 = e - kPerLane * (int32_t)kWave + kPerLane * (int32_t)lane;
        const int32_t r0 = i0 - 16 * g0;  // in lst (a multiple of kPerLane)
        lds_order();
        uint32_t sw[2];
        if constexpr (kPerLane == 8) {
          const uint2 v8 = *reinterpret_cast<const uint2*>(lst + (r0 > 0 ? r0 : 0));
          sw[0] = v8.x;
          sw[1] = v8.y;
        } else {
          sw[0] = *reinterpret_cast<const uint32_t*>(lst + (r0 > 0 ? r0 : 0));
          sw[1] = 0;
        }
        // symbols i0 + k + 1 then i0 + k as one field (<= 22 bits)
        auto pair = [&](int32_t k, uint32_t& p, uint32_t& np) __attribute__((always_inline)) {
          const bool a1 = (i0 + k + 1 >= lo) & (i0 + k + 1 < hi);
          const bool a0 = (i0 + k >= lo) & (i0 + k < hi);
          const uint32_t s1 = (sw[(k + 1) >> 2] >> (8 * ((k + 1) & 3))) & 0xFFu;
          const uint32_t s0 = (sw[k >> 2] >> (8 * (k & 3))) & 0xFFu;
          const uint32_t w1 = hcode[s1], w0 = hcode[s0];
          const uint32_t n1 = a1 ? w1 >> 16 : 0u, n0 = a0 ? w0 >> 16 : 0u;
          p = (a1 ? w1 & 0xFFFFu : 0u) | ((a0 ? w0 & 0xFFFFu : 0u) << n1);
          np = n1 + n0;
        };
        uint32_t pa, na, pb, nb;
        pair(kPerLane - 2, pa, na);
        pair(kPerLane - 4, pb, nb);
        if constexpr (kPerLane == 4) {
          o.put_bits(pa, na, pb, nb, p0, bits, zeroed);
        } else {
          uint32_t pc, nc, pd, nd;
          pair(2, pc, nc);
          pair(0, pd, nd);
          o.put_bits(pa | ((uint64_t)pb << na), na + nb, pc | ((uint64_t)pd << nc), nc + nd, p0,
                     bits, zeroed);
        }
      }
      if (g0 <= gA || o.overflow) break;
      g0 = g1;
    }
    o.put_bits(lane == 0 ? 1u : 0u, lane == 0 ? 1u : 0u, 0, 0, p0, bits, zeroed);  // end mark
    o.op = p0 + ((bits + 7) >> 3);
  };
  auto lit_header = [&](uint32_t type, uint32_t m) __attribute__((always_inline)) {
    const uint32_t h = m < 32 ? type | (m << 3)
                       : m < 4096 ? type | (1u << 2) | ((m & 15u) << 4) | ((m >> 4) << 8)
                                  : type | (3u << 2) | ((m & 15u) << 4) | ((m >> 4) << 8);
    const uint32_t hsz = m < 32 ? 1u : m < 4096 ? 2u : 3u;
    o.room(hsz + 1);
    o.put(lane < hsz ? (h >> (8 * (lane < 4 ? lane : 0u))) & 0xFFu : lrle,
          hsz + (type == 1 ? 1u : 0u));
  };
  for (uint32_t b = 0; b < nb && !o.overflow; ++b) {
    const uint32_t blk = o.op;
    bset(b, kBPos, blk);
    o.room(3);
    o.op += 3;  // the block header, written last
    // ---- literal section ----
    const uint32_t a = uniform(w[kWLb + b]), m = uniform(w[kWLb + b + 1]) - a;
    bool coded = false;
    if (lmode == 1 && m > 0) {
      lit_header(1u, m);
      coded = true;
    } else if (lmode == 2 && m > 0) {
      // Huffman when an estimate from the frame's statistics (the block's share of all coded
      // bits) and then the exact sizes both pass zs_literals_block's rule: the streams are
      // encoded once, the header and jump table written at the end with their sizes, and a
      // block the exact rule rejects is rewound and written raw
      const uint32_t ns = m < 256 ? 1u : 4u, q = (m + 3) / 4;
      const uint32_t tsz = tree_sent ? 0u : dsz;
      const int32_t limit = (int32_t)m - (int32_t)((m >> 6) + 2);
      const uint64_t est_bits = (uint64_t)m * tbits / nlit;
      const uint32_t est = tsz + (ns == 4 ? 6u : 0u) + (uint32_t)((est_bits + 8u * ns) / 8u);
      if ((int32_t)est < limit) {
        const uint32_t hs = ns == 1 || m < 1024 ? 3u : m < 16384 ? 4u : 5u;
        const uint32_t sf = ns == 1 ? 0u : m < 1024 ? 1u : m < 16384 ? 2u : 3u;
        const uint32_t sec = o.op;
        o.room(hs);
        o.put(0u, hs);  // (the header, patched at the end)
        o.put_lds(bytes, tsz);
        const uint32_t jt = o.op;
        uint32_t z0 = 0, z1 = 0, z2 = 0;
        if (ns == 4) {
          o.room(6);
          o.put(0u, 6);  // (the jump table, patched at the end)
          uint32_t pk = o.op;
          huff_stream(a, a + q);
          z0 = o.op - pk;
          pk = o.op;
          huff_stream(a + q, a + 2 * q);
          z1 = o.op - pk;
          pk = o.op;
          huff_stream(a + 2 * q, a + 3 * q);
          z2 = o.op - pk;
          huff_stream(a + 3 * q, a + m);
        } else {
          huff_stream(a, a + m);
        }
        const uint32_t total = o.op - sec - hs;
        if (!o.overflow && (int32_t)total < limit) {
          const uint64_t h = (tree_sent ? 3u : 2u) | (sf << 2) | ((uint64_t)m << 4) |
                             ((uint64_t)total << (hs == 3 ? 14 : hs == 4 ? 18 : 22));
          bset(b, kPPos, sec);
          bset(b, kPHs, hs);
          bset(b, kPH0, (uint32_t)h);
          bset(b, kPH1, (uint32_t)(h >> 32));
          bset(b, kPJt, ns == 4 ? jt : 0u);
          bset(b, kPZ, z0 | (z1 << 16));
          bset(b, kPZ2, z2);
          tree_sent = true;
          coded = true;
        } else if (!o.overflow) {  // rewind: raw after all
          // the abandoned streams' bits not yet flushed are still in the ring, whose bytes at
          // and past op must be zero for the bit writer (it ORs): clear them (positions
          // [max(sec, flushed), op), fewer than the ring's size); and the streams' bytes
          // already stored to HBM land before the header and the raw copy overwrite them
          for (uint32_t k = max(sec, o.flushed) + lane; k < o.op; k += kWave) obuf[o.at(k)] = 0;
          lds_order();
          global_fence_wave();
          o.op = sec;
          o.flushed = o.flushed > sec ? sec : o.flushed;
        }
      }
    }
    if (!coded) {  // raw
      lit_header(0u, m);
      if (m) {
        if ((uint64_t)o.op + m > o.cap) {
          o.overflow = true;
        } else {
          o.flush(o.op, true);
          wave_copy_global(o.dst + o.op, lits + a, m);
          o.op += m;
          o.flushed = o.op;
        }
      }
    }
    // ---- sequences section ----
    const uint32_t s0 = uniform(w[kWSb + b]), s1 = uniform(w[kWSb + b + 1]), bn = s1 - s0;
    if (!o.overflow) {
      const uint32_t nh = bn < 128 ? 1u : 2u;
      o.room(nh);
      o.put(nh == 1 ? bn : lane == 0 ? (bn >> 8) + 128u : bn & 0xFFu, nh);
    }
    if (bn && !o.overflow) {
      if (b == 0) {
        o.put_lds(bytes + 132, tdesc);  // modes byte + table descriptions
      } else {
        o.room(1);
        o.put(0xFCu, 1);  // Repeat_Mode for all three tables
      }
      const uint32_t p0 = o.op;
      uint32_t bits = 0, zeroed = p0;
      // the state words of sequence j (OF, ML, LL: bits | count << 12), loaded a step ahead
      // and combined at their use (combined right away, the loads were waited for at once)
      auto load_words = [&](uint32_t j, uint32_t& oo, uint32_t& om, uint32_t& ol)
          __attribute__((always_inline)) {
        const uint32_t sa = walk_state_at(j, 0);
        oo = outs[sa];
        om = outs[sa + 8];
        ol = outs[sa + 16];
      };
      auto word = [&](uint32_t oo, uint32_t om, uint32_t ol) __attribute__((always_inline)) {
        const uint32_t nof = oo >> 12, nml = om >> 12, nll = ol >> 12;
        return (oo & 0xFFFu) | ((om & 0xFFFu) << nof) | ((ol & 0xFFFu) << (nof + nml)) |
               ((nof + nml + nll) << 26);  // OF | ML | LL bits, their count
      };
      const uint32_t lastc = (bn - 1) >> 6;
      uint32_t jn = s0 + lastc * kWave + lane;
      uint2 prec = seqs[jn < s1 ? jn : s1 - 1];
      uint32_t pwc = wcodes[jn < s1 ? jn : s1 - 1];  // codes | offset value << 17 (entropy)
      uint32_t poo, pom, pol;
      load_words(jn < s1 ? jn : s1 - 1, poo, pom, pol);
      for (int32_t c = (int32_t)lastc; c >= 0 && !o.overflow; --c) {
        const uint32_t j = s0 + (uint32_t)c * kWave + lane;
        const bool act = j < s1;
        const uint2 rec = prec;
        const uint32_t wd = word(poo, pom, pol), wc = pwc;
        {  // prefetch the next step (the last step reloads its own: fixed load counts)
          const uint32_t jp = c > 0 ? j - kWave : (j < s1 ? j : s1 - 1);
          prec = seqs[jp];
          pwc = wcodes[jp];
          load_words(jp, poo, pom, pol);
        }
        const uint32_t ll = rec.x & 0x1FFFFu, mlb = rec.y - 3u;
        const uint32_t llc = wc & 63u, ofc = (wc >> 6) & 31u, mlc = (wc >> 11) & 63u, ov = wc >> 17;
        const uint64_t stb = wd & 0x3FFFFFFu;
        const uint32_t stn = wd >> 26;
        const uint32_t llb = sT.ll_bits[llc], mlbits = sT.ml_bits[mlc];
        // part 0: state bits + literal-length extra (<= 26 + 16); part 1: match-length extra,
        // then offset extra (<= 16 + 16)
        const uint64_t f0 = stb | ((uint64_t)(ll & ((1u << llb) - 1u)) << stn);
        const uint64_t f1 = (uint64_t)(mlb & ((1u << mlbits) - 1u)) |
                            ((uint64_t)(ov & ((1u << ofc) - 1u)) << mlbits);
        o.put_bits(act ? f0 : 0u, act ? stn + llb : 0u, act ? f1 : 0u, act ? mlbits + ofc : 0u,
                   p0, bits, zeroed);
      }
      if (!o.overflow) {
        // final states (ML, OF, LL: the decoder reads LL first) and the end mark
        const uint32_t sOF = uniform(w[kWFin + 3 * b]), sML = uniform(w[kWFin + 3 * b + 1]),
                       sLL = uniform(w[kWFin + 3 * b + 2]);
        const uint64_t fin = (uint64_t)(sML & ((1u << al_ml) - 1u)) |
                             ((uint64_t)(sOF & ((1u << al_of) - 1u)) << al_ml) |
                             ((uint64_t)(sLL & ((1u << al_ll) - 1u)) << (al_ml + al_of)) |
                             (1ull << (al_ml + al_of + al_ll));
        const uint32_t fn = al_ml + al_of + al_ll + 1;
        o.put_bits(lane == 0 ? fin : 0u, lane == 0 ? fn : 0u, 0, 0, p0, bits, zeroed);
        o.op = p0 + ((bits + 7) >> 3);
      }
    }
    bset(b, kBHdr, (b + 1 == nb ? 1u : 0u) | (2u << 1) | ((o.op - (blk + 3)) << 3));
  }
  // the blocks, or one raw block when they are not smaller than the segment
  const bool stored = o.overflow || o.op - (fh + 3) >= n;
  if (stored) {
    o.overflow = false;
    if (o.flushed < fh) o.flush(fh, true);  // the frame header may still be staged
    global_fence_wave();                     // earlier stores to this range land first
    wave_copy_global(o.dst + fh + 3, src, n);
    o.op = fh + 3 + n;
    bset(0, kBPos, fh);
    bset(0, kBHdr, 1u | (n << 3));
  } else {
    o.flush(o.op, true);
  }
  global_fence_wave();
  const uint32_t nh = stored ? 1u : nb;
  lds_order();
  if (lane < 3 * nh) {
    const uint32_t bi = lane / 3, byte = lane - 3 * bi;
    o.dst[bm[bi][kBPos] + byte] = (uint8_t)(bm[bi][kBHdr] >> (8 * byte));
  }
  if (!stored) {
    // the Huffman literal sections' headers (lanes 16 b' + k, k < 5) and jump tables (16 b' +
    // 8 + k, k < 6) of blocks b' and b' + 4
    const uint32_t k = lane & 15u;
    for (uint32_t bi = lane >> 4; bi < nb; bi += 4) {
      const uint32_t pp = bm[bi][kPPos], hs = bm[bi][kPHs], jt = bm[bi][kPJt];
      const uint32_t zz = bm[bi][kPZ], z2 = bm[bi][kPZ2];
      const uint64_t hv = (uint64_t)bm[bi][kPH0] | ((uint64_t)bm[bi][kPH1] << 32);
      if (hs && k < hs) o.dst[pp + k] = (uint8_t)(hv >> (8 * k));
      if (jt && k >= 8 && k < 14) {
        const uint32_t e = k - 8, sv = e < 2 ? zz & 0xFFFFu : e < 4 ? zz >> 16 : z2;
        o.dst[jt + e] = (uint8_t)((e & 1u) ? sv >> 8 : sv & 0xFFu);
      }
    }
  }
  if (lane == 0) sizes[i_seg] = o.op;
}

}  // namespace bitar_hip
