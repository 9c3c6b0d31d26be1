// zstd_lanes.hip -- Zstandard frame decode with ONE LANE PER SEGMENT (gfx950).
//
// Why a second decoder: a Zstd sequence section is one backward FSE bitstream whose states
// chain from sequence to sequence, so inside a segment the decode is serial.  The
// wave-per-segment kernel (zstd_decompress.hip) runs that chain on the scalar unit, which
// a CU shares among all its waves -- ~100 scalar instructions per sequence saturate it.
// Here every lane of a wave owns its own segment and runs the chain on the vector ALU:
// 64 sequence chains advance per vector instruction, and the FSE tables (the predefined
// distributions, built at compile time) are one LDS array shared by the lanes.
//
// Scope (the frames zstd_compress_kernel writes, and many libzstd level-1 frames): raw and
// RLE blocks, compressed blocks with raw or RLE literals and predefined (or repeated
// predefined) sequence tables, repeat offsets, single-segment frames with or without the
// content size.  A segment that needs anything else -- Huffman literals, FSE-described or
// RLE sequence tables, a dictionary id, a content checksum -- or that fails ANY of the
// wave kernel's checks is marked kDefer (produced[i]) and left to zstd_decompress_kernel,
// which the runtime launches next in defer-only mode; so acceptance, rejection and error
// reporting are exactly the wave kernel's (= the oracle's, oracle/bitar_zstd.c).
//
// Memory: each lane reads its compressed segment and writes its output with 8-byte
// (unaligned) global accesses; a match reads its history back from the lane's own output
// (same-thread read-after-write through L2).  The 8-byte forms never write past the frame's
// content size (or the capacity when the frame does not state it).  Raw and RLE blocks,
// where lanes would copy up to 64 KiB each, are instead copied by the whole wave, one
// lane's block after another, with coalesced 16-B accesses.
#include "lane_copy.hip.h"
#include "zstd_hand.hip.h"

namespace bitar_hip {

namespace zsl {

using namespace lanes;

constexpr uint32_t kDefer = 0xFFFFFFFEu;

// ---- predefined distributions (RFC 8878 3.1.1.3.2.2) -> decode tables at compile time ----
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
constexpr int16_t kLLNorm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
constexpr int16_t kMLNorm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
constexpr int16_t kOFNorm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

// One decode cell: baseline (17 bits) | extra-bit count << 17 | state bits << 22 |
// next-state base << 25.  The offset table keeps the offset code in the extra-bit field
// (Offset_Value = 2^code + code extra bits) and no baseline.
struct DTab {
  uint32_t c[64];
};

constexpr uint32_t hbc(uint32_t v) {
  uint32_t r = 0;
  while (v >>= 1) ++r;
  return r;
}

// FSE_buildDTable (RFC 8878 4.1.1) for a predefined distribution; kind 0 LL, 1 OF, 2 ML
constexpr DTab build_dtab(const int16_t* norm, uint32_t max_sym, uint32_t al, int kind) {
  DTab d{};
  const uint32_t size = 1u << al, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
  uint32_t high = size - 1;
  uint32_t sym_at[64] = {};
  uint32_t next[64] = {};
  for (uint32_t s = 0; s <= max_sym; ++s) {
    if (norm[s] == -1) {
      sym_at[high--] = s;
      next[s] = 1;
    } else {
      next[s] = (uint32_t)norm[s];
    }
  }
  uint32_t pos = 0;
  for (uint32_t s = 0; s <= max_sym; ++s)
    for (int i = 0; i < norm[s]; ++i) {
      sym_at[pos] = s;
      do {
        pos = (pos + step) & mask;
      } while (pos > high);
    }
  for (uint32_t u = 0; u < size; ++u) {
    const uint32_t s = sym_at[u];
    const uint32_t ns = next[s]++;
    const uint32_t nb = al - hbc(ns);
    const uint32_t base = (ns << nb) - size;
    uint32_t v = 0;
    if (kind == 0) v = kLLBase[s] | ((uint32_t)kLLBits[s] << 17);
    else if (kind == 1) v = s << 17;
    else v = kMLBase[s] | ((uint32_t)kMLBits[s] << 17);
    d.c[u] = v | (nb << 22) | (base << 25);
  }
  return d;
}

constexpr DTab kLLTab = build_dtab(kLLNorm, 35, 6, 0);
constexpr DTab kOFTab = build_dtab(kOFNorm, 28, 5, 1);
constexpr DTab kMLTab = build_dtab(kMLNorm, 52, 6, 2);
__constant__ DTab kTabs[3] = {kLLTab, kOFTab, kMLTab};

// Per-lane backward bit reader over the section [q, end) of the segment: C = the 8 stream
// bytes at [ptr, ptr + 8), bytes below q zeroed; `used` bits consumed from its top.
struct Bits {
  uint64_t C;
  uint32_t used;
  int32_t ptr;
  // branch-free: the load address is clamped into [q - 8, ...) (inside the frame, q >= 12);
  // bytes below q are masked off, all of them when ptr + 8 <= q (an overrun, rejected by
  // the final bit count)
  __device__ __forceinline__ void load(const GMEM uint8_t* src, uint32_t q) {
    const int32_t lo = (int32_t)q - 8;
    const int32_t at = ptr < lo ? lo : ptr;
    const uint64_t v = ld8(src + at);
    const int32_t below = (int32_t)q - ptr;  // bytes of [ptr, ptr + 8) below q
    C = below <= 0 ? v : below >= 8 ? 0ull : v & (~0ull << (8 * (uint32_t)below));
  }
  __device__ __forceinline__ void reload(const GMEM uint8_t* src, uint32_t q) {
    ptr -= (int32_t)(used >> 3);
    used &= 7u;
    load(src, q);
  }
  __device__ __forceinline__ uint32_t read(uint32_t n) {
    const uint32_t sh = (64 - used - n) & 63u;
    const uint32_t v = (uint32_t)(C >> sh) & ((1u << n) - 1u);
    used += n;
    return v;
  }
  __device__ __forceinline__ int32_t remaining(uint32_t q) const {
    return 8 * (ptr - (int32_t)q) + 64 - (int32_t)used;
  }
};

// One compressed block at stream [p, p + len) of lane's segment.  False = defer.
__device__ __forceinline__ bool block(const GMEM uint8_t* src, uint32_t cs, GMEM uint8_t* dst,
                                      uint32_t cap, uint32_t capw, uint32_t& op, uint32_t p, uint32_t len,
                                      uint32_t (&rep)[3], bool& pre, const uint32_t* tab) {
  const uint32_t end = p + len;
  const uint32_t b0 = src[p];
  const uint32_t lt = b0 & 3u, sf = (b0 >> 2) & 3u;
  if (lt >= 2) return false;  // Huffman literals: the wave kernel
  uint32_t regen, hsz;
  if (sf == 0 || sf == 2) { regen = b0 >> 3; hsz = 1; }
  else if (sf == 1) { if (len < 2) return false; regen = ldn(src + p, 2) >> 4; hsz = 2; }
  else { if (len < 3) return false; regen = ldn(src + p, 3) >> 4; hsz = 3; }
  if (regen > (128u << 10) || regen > cap - op) return false;
  uint32_t q = p + hsz;
  uint32_t lit = 0, litb = 0;
  if (lt == 0) {
    if (q + regen > end) return false;
    lit = q;
    q += regen;
  } else {
    if (q + 1 > end) return false;
    litb = src[q];
    q += 1;
  }
  if (q >= end) return false;
  uint32_t nseq = src[q];
  if (nseq < 128) {
    q += 1;
  } else if (nseq < 255) {
    if (q + 2 > end) return false;
    nseq = ((nseq - 128) << 8) + src[q + 1];
    q += 2;
  } else {
    if (q + 3 > end) return false;
    nseq = ldn(src + q + 1, 2) + 0x7F00u;
    q += 3;
  }
  uint32_t lp = 0;
  auto lits = [&](uint32_t n) __attribute__((always_inline)) {
    if (n == 0) return;
    if (lt == 0) {
      copy_lits(dst + op, src + lit + lp, n, op + 16 <= capw && lit + lp + 16 <= cs);
    } else {
      const uint64_t w = 0x0101010101010101ull * litb;
      if (op + n + 8 <= capw) {
        for (uint32_t j = 0; j < n; j += 8) st8(dst + op + j, w);
      } else {
        for (uint32_t j = 0; j < n; ++j) dst[op + j] = (uint8_t)litb;
      }
    }
  };
  if (nseq) {
    if (q >= end) return false;
    const uint32_t modes = src[q];
    q += 1;
    if (modes & 3u) return false;
    // predefined (0) or repeated predefined (3) for all three tables
    for (uint32_t k = 0; k < 3; ++k) {
      const uint32_t m = (modes >> (6 - 2 * k)) & 3u;
      if (m == 1 || m == 2 || (m == 3 && !pre)) return false;
    }
    pre = true;
    if (q >= end) return false;
    Bits b;
    b.ptr = (int32_t)end - 8;
    b.load(src, q);
    const uint32_t last = (uint32_t)(b.C >> 56);
    if (last == 0) return false;
    b.used = 8 - (31u - (uint32_t)__builtin_clz(last));
    uint32_t sll = b.read(6), sof = b.read(5), sml = b.read(6);
    for (uint32_t k = 0; k < nseq; ++k) {
      b.reload(src, q);
      const uint32_t il = tab[sll], io = tab[64 + sof], im = tab[128 + sml];
      const uint32_t ofc = (io >> 17) & 31u;
      const uint32_t ofv = (1u << ofc) + b.read(ofc);
      const uint32_t ml = (im & 0x1FFFFu) + b.read((im >> 17) & 31u);
      if (b.used > 31) b.reload(src, q);
      const uint32_t ll = (il & 0x1FFFFu) + b.read((il >> 17) & 31u);
      if (k + 1 < nseq) {
        sll = (il >> 25) + b.read((il >> 22) & 7u);
        sml = (im >> 25) + b.read((im >> 22) & 7u);
        sof = (io >> 25) + b.read((io >> 22) & 7u);
      }
      uint32_t off;
      // repeat offsets in select form (no exec-mask branches; the three stay in VGPRs)
      const uint32_t c0 = rep[0], c1 = rep[1], c2 = rep[2];
      const uint32_t idx = ofv + (ll == 0 ? 1u : 0u);
      off = ofv > 3 ? ofv - 3 : idx == 1 ? c0 : idx == 2 ? c1 : idx == 3 ? c2 : c0 - 1;
      const bool shift2 = ofv > 3 || idx >= 3, shift1 = ofv > 3 || idx >= 2;
      rep[2] = shift2 ? c1 : c2;
      rep[1] = shift1 ? c0 : c1;
      rep[0] = off;
      if (lp + ll > regen || (uint64_t)op + ml + (regen - lp) > cap) return false;
      if (off == 0 || off > op + ll) return false;  // also the rep0 - 1 == 0 case
      lits(ll);
      op += ll;
      lp += ll;
      copy_match(dst + op, off, ml, op + ml + 32 <= capw);
      op += ml;
    }
    if (b.remaining(q) != 0) return false;
  } else if (q != end) {
    return false;
  }
  if ((uint64_t)op + (regen - lp) > cap) return false;
  lits(regen - lp);
  op += regen - lp;
  return true;
}

}  // namespace zsl

// L segments per wave (lane l < L owns segment blockIdx.x * L + l); the launch has 64 lanes
// per workgroup so the raw/RLE block copies can use the whole wave.
template <uint32_t L>
__global__ __launch_bounds__(64) void zstd_lanes_kernel(
    const uint8_t* const* __restrict__ srcs, const uint8_t* __restrict__ slab,
    uint64_t slot_stride, const uint32_t* __restrict__ csizes, uint32_t nseg, uint32_t seg,
    uint8_t* __restrict__ out, uint32_t* __restrict__ produced) {
  using namespace zsl;
  __shared__ uint32_t tab[3 * 64];
  const uint32_t lane = lane_id();
  tab[lane] = kTabs[0].c[lane];
  tab[64 + lane] = kTabs[1].c[lane];
  tab[128 + lane] = kTabs[2].c[lane];
  lds_order();
  const uint32_t i = blockIdx.x * L + lane;
  bool active = lane < L && i < nseg;
  const GMEM uint8_t* src = nullptr;
  GMEM uint8_t* dst = nullptr;
  uint32_t cs = 0, op = 0, p = 0, fcs = 0, fsz = 0;
  const uint32_t cap = seg;
  if (active) {
    src = global_ptr(srcs ? srcs[i] : slab + (uint64_t)i * slot_stride);
    cs = csizes[i];
    dst = global_ptr(out + (uint64_t)i * seg);
    // frame header
    bool ok = cs >= 6 && ldn(src, 4) == 0xFD2FB528u;
    uint32_t fhd = 0;
    if (ok) {
      fhd = src[4];
      p = 5;
      // reserved bit, content checksum and dictionary ids go to the wave kernel
      ok = (fhd & (8u | 4u | 3u)) == 0;
    }
    if (ok) {
      const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1u;
      if (!single) {
        if (p >= cs) ok = false;
        p++;
      }
      fsz = fcs_flag == 0 ? (single ? 1u : 0u) : fcs_flag == 1 ? 2u : fcs_flag == 2 ? 4u : 8u;
      if (ok && (p + fsz > cs || fsz == 8)) ok = false;
      if (ok) {
        fcs = fsz ? ldn(src + p, fsz) : 0u;
        if (fsz == 2) fcs += 256;
        p += fsz;
        if (fsz && fcs > cap) ok = false;
      }
    }
    if (!ok) {
      produced[i] = kDefer;
      active = false;
    }
  }
  uint32_t rep[3] = {1, 4, 8};
  bool pre = false;
  // block loop: lanes walk their own blocks; all lanes meet at every block header, where
  // raw / RLE blocks are copied by the whole wave
  while (ballot(active)) {
    uint32_t type = 3, bsz = 0;
    bool last = false;
    if (active) {
      if (p + 3 > cs) {
        active = false;
        produced[i] = kDefer;
      } else {
        const uint32_t bh = ldn(src + p, 3);
        p += 3;
        last = bh & 1u;
        type = (bh >> 1) & 3u;
        bsz = bh >> 3;
        bool ok = type != 3;
        if (type == 0) ok = p + bsz <= cs && (uint64_t)op + bsz <= cap;
        else if (type == 1) ok = p + 1 <= cs && (uint64_t)op + bsz <= cap;
        else if (type == 2) ok = bsz <= (128u << 10) && p + bsz <= cs;
        if (!ok) {
          active = false;
          produced[i] = kDefer;
        }
      }
    }
    // raw and RLE blocks: the whole wave copies / fills, one lane's block at a time
    for (uint64_t m = ballot(active && type < 2); m; m &= m - 1) {
      const uint32_t l = (uint32_t)__builtin_ctzll(m);
      const uint64_t d = uniform64(readlane((uint32_t)(uintptr_t)dst, l) |
                                   ((uint64_t)readlane((uint32_t)((uintptr_t)dst >> 32), l) << 32));
      const uint64_t s = uniform64(readlane((uint32_t)(uintptr_t)src, l) |
                                   ((uint64_t)readlane((uint32_t)((uintptr_t)src >> 32), l) << 32));
      const uint32_t lop = readlane(op, l), lp = readlane(p, l), n = readlane(bsz, l);
      GMEM uint8_t* dd = (GMEM uint8_t*)(uintptr_t)d + lop;
      const GMEM uint8_t* ss = (const GMEM uint8_t*)(uintptr_t)s + lp;
      if (readlane(type, l) == 0) {
        wave_copy_global(dd, ss, n);
      } else {
        const uint32_t v = readlane(active ? (uint32_t)src[p] : 0u, l);
        for (uint32_t k = lane; k < n; k += kWave) dd[k] = (uint8_t)v;
      }
      global_fence_wave();  // lane l reads this output back as match history
    }
    if (active) {
      if (type == 0) {
        op += bsz;
        p += bsz;
      } else if (type == 1) {
        op += bsz;
        p += 1;
      } else if (!block(src, cs, dst, cap, fsz ? fcs : cap, op, p, bsz, rep, pre, tab)) {
        active = false;
        produced[i] = kDefer;
      } else {
        p += bsz;
      }
      if (active && last) {
        active = false;
        produced[i] = (p == cs && (!fsz || fcs == op)) ? op : kDefer;
      }
    }
  }
}

// ---- the lane executor of handed-off sequence sections ---------------------------------------
// zstd_decompress_kernel decodes a frame up to the sequence section of its last block (the
// literals -- Huffman-coded ones into the tail of the output slot --, the three decode
// tables, the repeat offsets) and hands the rest over (zstd_decompress.hip kHand*): here
// every lane runs one segment's sequence loop, its decode cells read from the scratch
// (L2-resident, 6 KiB per segment), with the wave kernel's acceptance checks, then the final
// frame checks.  kHand* mirror zstd_decompress.hip.
namespace zsh {
constexpr uint32_t kHandRec = zhand::kRec, kHandCells = zhand::kCells;
constexpr uint64_t kHandStride = zhand::kStride;
constexpr uint32_t kHanded = zhand::kHanded;

// 4 stream bytes at offset a, as loaded: no select on the value, so the load's wait lands
// where the word is first used (below q it reads [q - 4, q) instead; peek masks those bits)
__device__ __forceinline__ uint32_t word_raw(const GMEM uint8_t* s, int32_t a, int32_t lo) {
  uint32_t v;
  __builtin_memcpy(&v, s + (a < lo ? lo : a), 4);
  return v;
}
// 16 bytes {a, b} to d (any alignment)
__device__ __forceinline__ void st16_raw(GMEM uint8_t* d, uint64_t a, uint64_t b) {
  const uint4 v = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
  __builtin_memcpy(d, &v, 16);
}
// 16 stream bytes at s (any alignment)
__device__ __forceinline__ uint4 ld16_raw(const GMEM uint8_t* s) {
  uint4 v;
  __builtin_memcpy(&v, s, 16);
  return v;
}
}  // namespace zsh

// The Huffman literal streams of handed-off blocks (kLitPend): 16 segments per wave, one lane
// per stream (lane 4 l + j = stream j of segment l), the segments' decode tables in LDS; each
// lane decodes its stream backward (one table lookup per symbol, 8 symbols per 8-byte store)
// into the tail of the segment's output slot, where zstd_handoff_kernel reads the literals.
// Acceptance: the stream is consumed exactly (the wave decoder's huf_stream rule).
// It may run alongside zstd_seqdec_kernel (runtime.hip), which needs no literal and moves a
// segment from kHanded to kRecs (records ready) by compare-and-swap: the streams of both
// states are decoded here, and a failure overwrites either.
__device__ __forceinline__ bool lits_pending(uint32_t p) {
  return p == zhand::kHanded || p == zhand::kRecs;
}
// B: the blocks of a segment in the wave (lane 4 B l + 4 b + j = stream j of block b of
// segment l): B = 1 takes the frames that handed their last block only (kNb == 1), B = 4 the
// multi-block hand-offs (kNb >= 2: the streams of all of a frame's blocks run at once, their
// literals going to each block's place in the slot tail, zstd_hand.hip.h kXLit) by units of 4
// blocks (slot l = unit blockIdx.x * S + l: blocks 4 g + b of segment unit >> 1, g = unit & 1).
template <uint32_t S, uint32_t B>
__global__ __launch_bounds__(64) void zstd_hlit_kernel(
    const uint8_t* const* __restrict__ srcs, const uint8_t* __restrict__ slab,
    uint64_t slot_stride, const uint32_t* __restrict__ csizes, uint32_t nseg, uint32_t seg,
    uint8_t* __restrict__ out, uint32_t* __restrict__ produced,
    const uint8_t* __restrict__ hscr, uint32_t* __restrict__ err,
    const uint32_t* __restrict__ order) {
  using namespace zhand;
  static_assert(S * B * 4 <= kWave, "a lane per stream");
  // Per segment: the 2^11-entry table as symbol bytes plus each symbol's code length, 2.25
  // KiB instead of 4 KiB of (symbol | length) entries, so 16 segments take 36 KiB and four
  // workgroups share a CU: every stream of a GiB is resident in one round (two lookups per
  // symbol, the second a tiny table)
  __shared__ uint16_t tab[S][kHufWords];  // two symbol bytes per entry pair
  __shared__ uint8_t len8[S][256];
#ifndef BITAR_HLIT_PRIO
#define BITAR_HLIT_PRIO 3
#endif
  // It runs beside zstd_seqdec_kernel (another stream) and ends after it: its streams are
  // the decode's critical path, so its waves take the issue arbiter first (seqdec has slack)
  if (BITAR_HLIT_PRIO) __builtin_amdgcn_s_setprio(BITAR_HLIT_PRIO);
  const uint32_t lane = lane_id();
  // The wave's segment headers, one lane per segment, loaded together, and each table's
  // words issued before any is used: at about one wave per SIMD every serial load is
  // exposed, and the per-segment form chained three header loads and 16 table loads.
  // (pend: any block's streams pending; hlg: the table log, the same for every block)
  // (order: the segments by literal count, most first, hand_key_kernel: slot x takes
  // segment order[x])
  static_assert(B == 1 || B == kUnitBlocks, "whole units");
  const uint32_t nun = B > 1 ? 2 * nseg : nseg;  // units
  uint32_t p0 = 0, pend = 0, hlg = 0, nbh = 0, il0 = 0, g0 = 0;
  {
    const uint32_t bl = blockIdx.x * S + lane;
    const uint32_t u = bl < nun ? (order ? order[bl] : bl) : bl;
    const uint32_t il = B > 1 ? u >> 1 : u;
    il0 = il;
    g0 = B > 1 ? u & 1u : 0u;
    if (lane < S && bl < nun && il < nseg) {
      const GMEM uint32_t* h = global_ptr(reinterpret_cast<const uint32_t*>(hscr + (uint64_t)il * kStride));
      p0 = produced[il];
      nbh = h[kNb];
      uint32_t pd = 0, lg = 0;
#pragma unroll
      for (uint32_t b = 0; b < B; ++b) {
        const uint32_t bb = B * g0 + b;
        const uint32_t pb = h[blk_at(bb < kMaxBlocks ? bb : 0u) + kLitPend];
        const uint32_t lb = h[blk_at(bb < kMaxBlocks ? bb : 0u) + kHufLog];
        const bool in = bb < nbh && pb == 1u;
        pd |= in ? 1u : 0u;
        lg = in ? lb : lg;
      }
      pend = pd;
      hlg = lg;
    }
  }
  const uint64_t tm = ballot(lits_pending(p0) && pend == 1u && (B == 1 ? nbh == 1u : nbh >= 2u));
  for (uint64_t m = tm; m; m &= m - 1) {
    const uint32_t l = (uint32_t)__builtin_ctzll(m);
    const uint32_t il = readlane(il0, l);
    const GMEM uint32_t* h = global_ptr(reinterpret_cast<const uint32_t*>(hscr + (uint64_t)il * kStride));
    const uint32_t nw = (1u << (readlane(hlg, l) & 0xFFu)) / 2;
    uint32_t wv[kHufWords / kWave];
#pragma unroll
    for (uint32_t k = 0; k < kHufWords / kWave; ++k) {
      const uint32_t u = lane + k * kWave;
      wv[k] = h[kHufAt + (u < nw ? u : 0u)];
    }
#pragma unroll
    for (uint32_t k = 0; k < kHufWords / kWave; ++k) {
      const uint32_t u = lane + k * kWave, w = wv[k];
      if (u < nw) {
        tab[l][u] = (uint16_t)((w & 0xFFu) | ((w >> 8) & 0xFF00u));
        len8[l][w & 0xFFu] = (uint8_t)(w >> 8);  // (every entry of a symbol: the same length)
        len8[l][(w >> 16) & 0xFFu] = (uint8_t)(w >> 24);
      }
    }
  }
  lds_order();
  const uint32_t l = lane / (4 * B), j = lane & 3u;
  // (fetched while every lane is active: a disabled source lane reads as 0)
  const uint32_t i = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((l < S ? l : 0u) << 2), (int)il0);
  const uint32_t g = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((l < S ? l : 0u) << 2), (int)g0);
  const uint32_t bk = B * g + (lane >> 2) % B;  // the block
  if (l >= S || blockIdx.x * S + l >= nun || !((tm >> l) & 1u)) return;
  const GMEM uint32_t* h0 = global_ptr(reinterpret_cast<const uint32_t*>(hscr + (uint64_t)i * kStride));
  if (bk >= h0[kNb]) return;
  const GMEM uint32_t* h = h0 + blk_at(bk);
  if (h[kLitPend] != 1u) return;  // (this block's literals are raw / RLE)
  const uint32_t hl = h[kHufLog], log = hl & 0xFFu, ns = hl >> 8;
  if (j >= ns) return;
  const uint32_t regen = h[kRegen], qq = h[kQQ];
  const uint32_t s1 = h[kS1], s2 = h[kS2], s3 = h[kS3], s4 = h[kS4];
  const uint32_t start = h[kStreams] + (j >= 1 ? s1 : 0u) + (j >= 2 ? s2 : 0u) + (j >= 3 ? s3 : 0u);
  const uint32_t len = j == 0 ? s1 : j == 1 ? s2 : j == 2 ? s3 : s4;
  const uint32_t n = ns == 1 ? regen : j < 3 ? qq : regen - 3 * qq;
  // the block's literals: [cap - kLitAll + kXLit, + regen) of the slot
  const uint32_t lat = (seg - h0[kLitAll]) + h0[kX0 + kXW * bk + kXLit];
  const GMEM uint8_t* src = global_ptr(srcs ? srcs[i] : slab + (uint64_t)i * slot_stride);
  GMEM uint8_t* dst = global_ptr(out + (uint64_t)i * seg + lat + j * qq);
  const uint8_t* t = reinterpret_cast<const uint8_t*>(tab[l]);
  const uint8_t* tl = len8[l];
  bool ok = len > 0;
  uint32_t lastb = 0;
  if (ok) {
    lastb = src[start + len - 1];
    ok = lastb != 0;
  }
  if (ok) {
    // Backward bit reader whose eight words live in FIXED registers W0..W7: phase p decodes
    // from the window W[p]:W[p+1] (W[p] the higher-addressed word) until it has used 32 bits,
    // then reloads W[p] with the word eight below it, which the window reaches seven phases
    // later.  A rotating queue would move each new word on the very next refill and so wait
    // for its load (and, vmcnt being in order, for every store before it) there; the one
    // full wait left is at the loop head, once per eight words.
    // Bits below the stream start q read as zero (masked at the peek, from the position).
    const int32_t q = (int32_t)start, lo = q >= 4 ? q - 4 : 0;
    int32_t top = (int32_t)(start + len);  // stream offset just above the window
#ifndef BITAR_HLIT_NW
#define BITAR_HLIT_NW 8
#endif
#ifndef BITAR_HLIT_X8
#define BITAR_HLIT_X8 1
#endif
    // X8 (multi-block hand-offs): a 16-word window reloaded 8 words (32 bytes) at a time
    constexpr bool X8 = BITAR_HLIT_X8 != 0 && B > 1;
    constexpr uint32_t NW = X8 ? 16u : BITAR_HLIT_NW;
#ifndef BITAR_HLIT_X4
#define BITAR_HLIT_X4 1
#endif
#ifndef BITAR_HLIT_ST16
#define BITAR_HLIT_ST16 1
#endif
    // (multi-block hand-offs only: 16 waves per CU whose scattered lane loads and stores keep
    // the addresser busy; at one wave per SIMD -- the single-block form, long streams -- the
    // longer dependent chain of the 16-byte form costs more than the addresser time it saves:
    // stock libzstd-1 decode 5.38 -> 6.35 ms in hlit with it)
    constexpr bool X4 = BITAR_HLIT_X4 != 0 && NW == 8 && B > 1 && !X8;
    constexpr bool ST16 = BITAR_HLIT_ST16 != 0 && B > 1;
#ifndef BITAR_HLIT_ST32
#define BITAR_HLIT_ST32 1
#endif
    // ST32: 32 symbols per pair of 16-byte stores (with X8: the line of a lane's output run is
    // written in two halves instead of eight 16-byte pieces)
    constexpr bool ST32 = ST16 && X8 && BITAR_HLIT_ST32 != 0;
    uint32_t W[NW];
#pragma unroll
    for (uint32_t w = 0; w < NW; ++w) W[w] = zsh::word_raw(src, top - 4 * (int32_t)(w + 1), lo);
    uint32_t used = 8 - (31u - (uint32_t)__builtin_clz(lastb));  // the end mark and zeros above it
    const uint32_t mask = (1u << log) - 1u;
    uint64_t acc = 0, prev = 0, pv1 = 0, pv2 = 0;
    uint32_t k = 0, ac = 0, half = 0;
    auto phase = [&](uint32_t hi, uint32_t lo32, uint32_t& slot) __attribute__((always_inline)) {
      const uint64_t c = ((uint64_t)hi << 32) | lo32;
      auto emit = [&](uint32_t sym) __attribute__((always_inline)) {
        used += tl[sym];
        acc |= (uint64_t)sym << (8 * ac);
        ++k;
        if (++ac == 8) {
          if constexpr (ST32) {
            // half counts the pending 8-symbol words (prev, pv1, pv2)
            if (half == 3) {
              zsh::st16_raw(dst + k - 32, prev, pv1);
              zsh::st16_raw(dst + k - 16, pv2, acc);
            }
            prev = half == 0 ? acc : prev;
            pv1 = half == 1 ? acc : pv1;
            pv2 = half == 2 ? acc : pv2;
            half = (half + 1) & 3u;
          } else if constexpr (ST16) {
            // 16 symbols per store: half the store addresses
            if (half) zsh::st16_raw(dst + k - 16, prev, acc);
            else prev = acc;
            half ^= 1u;
          } else {
            lanes::st8(dst + k - 8, acc);
          }
          acc = 0;
          ac = 0;
        }
      };
      // A phase reads at most 31 + log <= 42 bits below the window top: with >= 43 stream
      // bits left no peek reaches below the stream start, and the mask leaves the symbol
      // chain (it sat between the shift and the table read of every symbol)
      if (8 * (top - q) - (int32_t)used >= 43) {
        while (used < 32 && k < n) emit(t[(uint32_t)(c >> (64 - used - log)) & mask]);
      } else {
        while (used < 32 && k < n) {
          uint32_t v = (uint32_t)(c >> (64 - used - log)) & mask;
          const int32_t rem = 8 * (top - q) - (int32_t)used;  // stream bits not yet consumed
          if (rem < (int32_t)log) v &= rem <= 0 ? 0u : ~0u << (log - (uint32_t)rem);
          emit(t[v]);
        }
      }
      // (unconditional: a conditional load is a phi the compiler settles with vmcnt(0); when
      // the phase ended on k == n instead, the loop ends and the word is not read)
      if constexpr (!X4 && !X8) slot = zsh::word_raw(src, top - 4 * (int32_t)(NW + 1), lo);
      if (used >= 32) {
        top -= 4;
        used -= 32;
      }
    };
    // X4: the four words a half-round consumed are reloaded by ONE 16-byte load (the
    // addresser handles one address per lane either way, and the lanes' scattered loads bound
    // this kernel: TA busy ~70 % of its cycles with a dword per phase).  The block [top - 32,
    // top - 16) goes to W[h+3] .. W[h] (lowest address first).  Near the stream start the load
    // is clamped to lo and the 128-bit value shifted back into place (the bytes below lo are
    // below the stream and masked at the peek); it only runs after four full phases, so
    // [lo, lo + 16) lies inside the stream.
    auto reload4 = [&](uint32_t& wa, uint32_t& wb, uint32_t& wc, uint32_t& wd) __attribute__((always_inline)) {
      const int32_t A = top - 32;
      const int32_t a = A < lo ? lo : A;
      const uint32_t sh = (uint32_t)(a - A) * 8u;  // 0 except near the start
      const uint4 v = zsh::ld16_raw(src + a);
      const uint64_t l64 = (uint64_t)v.x | ((uint64_t)v.y << 32);
      const uint64_t h64 = (uint64_t)v.z | ((uint64_t)v.w << 32);
      const uint32_t s1 = sh & 63u;
      const uint64_t spill = s1 ? l64 >> (64u - s1) : 0ull;
      const uint64_t rl = sh < 64 ? l64 << s1 : 0ull;
      const uint64_t rh = sh < 64 ? (h64 << s1) | spill : sh < 128 ? l64 << s1 : 0ull;
      wa = (uint32_t)rl;
      wb = (uint32_t)(rl >> 32);
      wc = (uint32_t)rh;
      wd = (uint32_t)(rh >> 32);
    };
    // X8: the eight words a half-round consumed come back as the block [top - 64, top - 32),
    // two 16-byte loads of one 32-byte run (its line is fetched once for both: the lanes'
    // 16-byte reads missed L2 about every time, ~6x the stream bytes, once 8-block frames
    // doubled the concurrent streams); near the stream start word by word (each clamped to
    // lo like the initial fill: a word below lo lies below the stream, masked at the peek)
    auto reload8 = [&](uint32_t h) __attribute__((always_inline)) {
      const int32_t A = top - 64;
      if (A >= lo) {
        const uint4 v0 = zsh::ld16_raw(src + A), v1 = zsh::ld16_raw(src + A + 16);
        W[h + 7] = v0.x;
        W[h + 6] = v0.y;
        W[h + 5] = v0.z;
        W[h + 4] = v0.w;
        W[h + 3] = v1.x;
        W[h + 2] = v1.y;
        W[h + 1] = v1.z;
        W[h] = v1.w;
      } else {
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) W[h + 7 - u] = zsh::word_raw(src, A + 4 * (int32_t)u, lo);
      }
    };
    while (k < n) {
#pragma unroll
      for (uint32_t p = 0; p < NW; ++p) {
        phase(W[p], W[(p + 1) % NW], W[p]);
        if (k >= n) break;
        if constexpr (X4) {
          if (p == 3) reload4(W[3], W[2], W[1], W[0]);
          if (p == 7) reload4(W[7], W[6], W[5], W[4]);
        }
        if constexpr (X8) {
          if (p == 7) reload8(0);
          if (p == 15) reload8(8);
        }
      }
    }
    if (ST32) {  // the pending words, oldest first
      const uint32_t b0 = k - ac - 8 * half;
      if (half >= 1) lanes::st8(dst + b0, prev);
      if (half >= 2) lanes::st8(dst + b0 + 8, pv1);
      if (half >= 3) lanes::st8(dst + b0 + 16, pv2);
    } else if (ST16 && half) {
      lanes::st8(dst + k - ac - 8, prev);
    }
    for (uint32_t r = 0; r < ac; ++r) dst[k - ac + r] = (uint8_t)(acc >> (8 * r));
    ok = 8 * (top - q) - (int32_t)used == 0;
  }
  if (!ok) {
    atomicExch(&produced[i], 0xFFFFFFFFu);  // (over zstd_seqdec_kernel's kRecs, see above)
    atomicOr(err, 1u);
  }
}


template <uint32_t L>
__global__ __launch_bounds__(64) void zstd_handoff_kernel(
    const uint8_t* const* __restrict__ srcs, const uint8_t* __restrict__ slab,
    uint64_t slot_stride, const uint32_t* __restrict__ csizes, uint32_t nseg, uint32_t seg,
    uint8_t* __restrict__ out, uint32_t* __restrict__ produced,
    const uint8_t* __restrict__ hscr, uint32_t* __restrict__ err) {
  using namespace zsl;
  using namespace zsh;
  // baseline | extra-bit count << 24 of every literal-length / match-length code
  __shared__ uint32_t llt[64], mlt[64];
  const uint32_t lane = lane_id();
  llt[lane] = lane < 36 ? kLLBase[lane] | ((uint32_t)kLLBits[lane] << 24) : 0u;
  mlt[lane] = lane < 53 ? kMLBase[lane] | ((uint32_t)kMLBits[lane] << 24) : 0u;
  lds_order();
  const uint32_t i = blockIdx.x * L + lane;
  if (lane >= L || i >= nseg || produced[i] != kHanded) return;
  const GMEM uint32_t* h = global_ptr(reinterpret_cast<const uint32_t*>(hscr + (uint64_t)i * kHandStride));
  if (h[zhand::kNb] != 1u) {  // (multi-block hand-offs belong to zstd_seqdec_kernel, which
    produced[i] = 0xFFFFFFFFu;  // takes or rejects every one: defensive)
    atomicOr(err, 1u);
    return;
  }
  const GMEM uint8_t* src = global_ptr(srcs ? srcs[i] : slab + (uint64_t)i * slot_stride);
  GMEM uint8_t* dst = global_ptr(out + (uint64_t)i * seg);
  const uint32_t cs = csizes[i];
  const uint32_t q = h[0], end = h[1], nseq = h[2], w3 = h[3], litv = h[4], regen = h[5];
  uint32_t op = h[6];
  uint32_t r0 = h[7], r1 = h[8], r2 = h[9];
  const uint32_t fsz = h[10], fcs = h[11];
  const uint32_t al0 = w3 & 0xFFu, al1 = (w3 >> 8) & 0xFFu, al2 = (w3 >> 16) & 0xFFu,
                 lt = w3 >> 24;
  const GMEM uint32_t* tll = h + kHandRec;
  const GMEM uint32_t* tof = tll + kHandCells;
  const GMEM uint32_t* tml = tof + kHandCells;
  const uint32_t cap = seg;
  const uint32_t capw = fsz ? fcs : cap;  // wildcopies stay inside the content size
  // Huffman literals sit at the slot tail [cap - regen, cap): writes stay below the unread
  // part of it
  const GMEM uint8_t* tail = dst + (cap - regen);
  uint32_t lp = 0;
  // (lt 2 and 3 -- a Treeless block reuses the previous block's code -- are both Huffman)
  auto limit = [&]() __attribute__((always_inline)) { return lt >= 2 ? cap - (regen - lp) : capw; };
  auto lits = [&](uint32_t n) __attribute__((always_inline)) {
    if (n == 0) return;
    if (lt == 0) {
      copy_lits(dst + op, src + litv + lp, n, op + n + 16 <= capw && litv + lp + n + 16 <= cs);
    } else if (lt == 1) {
      const uint64_t w = 0x0101010101010101ull * (litv & 0xFFu);
      if (op + n + 8 <= capw) {
        for (uint32_t j = 0; j < n; j += 8) st8(dst + op + j, w);
      } else {
        for (uint32_t j = 0; j < n; ++j) dst[op + j] = (uint8_t)litv;
      }
    } else {
      copy_lits(dst + op, tail + lp, n, op + n + 16 <= cap - (regen - lp) && lp + n + 16 <= regen);
    }
  };
  bool ok = true;
  // backward bit reader with the 8 bytes below its window loaded one reload ahead (the
  // reload is a shift, its load's latency hides behind a sequence)
  struct PBits {
    uint64_t C, N;
    uint32_t used;
    int32_t ptr;
    __device__ __forceinline__ static uint64_t at(const GMEM uint8_t* s, int32_t a, uint32_t q) {
      const int32_t lo = (int32_t)q - 8;
      const uint64_t v = ld8(s + (a < lo ? lo : a));
      const int32_t below = (int32_t)q - a;
      return below <= 0 ? v : below >= 8 ? 0ull : v & (~0ull << (8 * (uint32_t)below));
    }
    __device__ __forceinline__ void reload(const GMEM uint8_t* s, uint32_t q) {
      const uint32_t sb = used >> 3;
      if (sb) {
        C = sb == 8 ? N : (C << (8 * sb)) | (N >> (64 - 8 * sb));
        used &= 7u;
        ptr -= (int32_t)sb;
        N = at(s, ptr - 8, q);
      }
    }
    __device__ __forceinline__ uint32_t read(uint32_t n) {
      const uint32_t sh = (64 - used - n) & 63u;
      const uint32_t v = (uint32_t)(C >> sh) & ((1u << n) - 1u);
      used += n;
      return v;
    }
    __device__ __forceinline__ int32_t remaining(uint32_t q) const {
      return 8 * (ptr - (int32_t)q) + 64 - (int32_t)used;
    }
  } b;
  b.ptr = (int32_t)end - 8;
  b.C = PBits::at(src, b.ptr, q);
  b.N = PBits::at(src, b.ptr - 8, q);
  const uint32_t lastb = (uint32_t)(b.C >> 56);
  if (nseq == 0) {
    ok = q == end;  // no sequences: no bitstream
  } else if (lastb == 0) {
    ok = false;
  }
  if (ok && nseq) {
    b.used = 8 - (31u - (uint32_t)__builtin_clz(lastb));
    uint32_t sll = b.read(al0), sof = b.read(al1), sml = b.read(al2);
    uint32_t cll = tll[sll], cof = tof[sof], cml = tml[sml];
    for (uint32_t k = 0; k < nseq; ++k) {
      b.reload(src, q);
      const uint32_t ofc = cof & 0xFFu;
      const uint32_t ofv = (1u << ofc) + b.read(ofc);
      const uint32_t mle = mlt[cml & 63u];
      const uint32_t ml = (mle & 0xFFFFFFu) + b.read(mle >> 24);
      if (b.used > 20) b.reload(src, q);  // <= 16 extra + 26 state bits follow
      const uint32_t lle = llt[cll & 63u];
      const uint32_t ll = (lle & 0xFFFFFFu) + b.read(lle >> 24);
      if (k + 1 < nseq) {  // the next cells load while this sequence is copied
        sll = (cll >> 16) + b.read((cll >> 8) & 0xFFu);
        sml = (cml >> 16) + b.read((cml >> 8) & 0xFFu);
        sof = (cof >> 16) + b.read((cof >> 8) & 0xFFu);
        cll = tll[sll];
        cof = tof[sof];
        cml = tml[sml];
      }
      // repeat offsets in select form (no exec-mask branches)
      const uint32_t idx = ofv + (ll == 0 ? 1u : 0u);
      const uint32_t off = ofv > 3 ? ofv - 3 : idx == 1 ? r0 : idx == 2 ? r1 : idx == 3 ? r2 : r0 - 1;
      const bool shift2 = ofv > 3 || idx >= 3, shift1 = ofv > 3 || idx >= 2;
      const uint32_t c0 = r0, c1 = r1, c2 = r2;
      r2 = shift2 ? c1 : c2;
      r1 = shift1 ? c0 : c1;
      r0 = off;
      if (lp + ll > regen || (uint64_t)op + ml + (regen - lp) > cap || off == 0 ||
          off > op + ll) {
        ok = false;
        break;
      }
#ifndef BITAR_ZH_NOLIT
      lits(ll);
#endif
      op += ll;
      lp += ll;
#ifndef BITAR_ZH_NOMATCH
      copy_match(dst + op, off, ml, op + ml + 32 <= limit());
#endif
      op += ml;
    }
    if (ok && b.remaining(q) != 0) ok = false;
  }
  if (ok && (uint64_t)op + (regen - lp) > cap) ok = false;
  if (ok) {
    const uint32_t n = regen - lp;
    if (lt >= 2) {  // the tail literals may overlap their destination: forward, 8 B only
                    // where the gap allows
      const uint32_t gap = (cap - (regen - lp)) - op;
      if (gap >= 8) {
        uint32_t j = 0;
        for (; j + 8 <= n; j += 8) st8(dst + op + j, ld8(tail + lp + j));
        for (; j < n; ++j) dst[op + j] = tail[lp + j];
      } else {
        for (uint32_t j = 0; j < n; ++j) dst[op + j] = tail[lp + j];
      }
    } else {
      lits(n);
    }
    op += n;
    ok = end == cs && (!fsz || fcs == op);
  }
  if (ok) {
    produced[i] = op;
  } else {
    produced[i] = 0xFFFFFFFFu;
    atomicOr(err, 1u);
  }
}

template __global__ void zstd_handoff_kernel<16>(const uint8_t* const*, const uint8_t*, uint64_t,
                                                 const uint32_t*, uint32_t, uint32_t, uint8_t*,
                                                 uint32_t*, const uint8_t*, uint32_t*);
template __global__ void zstd_handoff_kernel<4>(const uint8_t* const*, const uint8_t*, uint64_t,
                                                 const uint32_t*, uint32_t, uint32_t, uint8_t*,
                                                 uint32_t*, const uint8_t*, uint32_t*);
template __global__ void zstd_handoff_kernel<8>(const uint8_t* const*, const uint8_t*, uint64_t,
                                                 const uint32_t*, uint32_t, uint32_t, uint8_t*,
                                                 uint32_t*, const uint8_t*, uint32_t*);
#define BITAR_HLIT_INST(S, B)                                                                  \
  template __global__ void zstd_hlit_kernel<S, B>(const uint8_t* const*, const uint8_t*, uint64_t, \
                                                  const uint32_t*, uint32_t, uint32_t, uint8_t*,  \
                                                  uint32_t*, const uint8_t*, uint32_t*,           \
                                                  const uint32_t*);
BITAR_HLIT_INST(4, 1)
BITAR_HLIT_INST(8, 1)
BITAR_HLIT_INST(16, 1)
BITAR_HLIT_INST(4, 4)
#undef BITAR_HLIT_INST

template __global__ void zstd_lanes_kernel<64>(const uint8_t* const*, const uint8_t*, uint64_t,
                                               const uint32_t*, uint32_t, uint32_t, uint8_t*,
                                               uint32_t*);
template __global__ void zstd_lanes_kernel<32>(const uint8_t* const*, const uint8_t*, uint64_t,
                                               const uint32_t*, uint32_t, uint32_t, uint8_t*,
                                               uint32_t*);
template __global__ void zstd_lanes_kernel<8>(const uint8_t* const*, const uint8_t*, uint64_t,
                                              const uint32_t*, uint32_t, uint32_t, uint8_t*,
                                              uint32_t*);
template __global__ void zstd_lanes_kernel<16>(const uint8_t* const*, const uint8_t*, uint64_t,
                                               const uint32_t*, uint32_t, uint32_t, uint8_t*,
                                               uint32_t*);

}  // namespace bitar_hip
