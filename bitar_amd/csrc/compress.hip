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
// The parse itself (input staging, hashing, greedy chain walk) lives in window_parse.hip.h;
// this file holds the two emitters:
//   LZ4: every selected match lane writes its token / length bytes / offset, every
//        literal lane writes its own byte, placed by a wave prefix sum of sequence sizes;
//        rare long runs fall back to a per-sequence path (long literal runs go HBM->HBM);
//   DEFLATE: every position lane contributes its literal code or its match symbol; codes
//        are placed by a prefix sum of bit lengths and OR-ed into an LDS bit ring.
#include "window_parse.hip.h"

namespace bitar_hip {

namespace cmp {

// m's bit for this lane ? a : b (m an SGPR pair used directly as the lane mask)
__device__ __forceinline__ uint32_t lane_sel(uint64_t m, uint32_t a, uint32_t b) {
  uint32_t r;
  __asm__("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(m));
  return r;
}

// ---- LZ4 emitter: sequences batched, output gathered byte by byte ----------------------
// The parse hands each window's matches over as sequence records {match start, distance,
// length}: the chain lanes append them to an LDS list (one store, one mbcnt).  Every <= 64
// records (and before the tail) one flush turns them into LZ4 sequences, one record per
// lane: literal run = [previous match end, match start), sizes by one prefix sum, and then
// the output is GATHERED 64 bytes per step -- output byte o finds its sequence (the latest one
// starting at or before o: sequence starts marked in LDS, a prefix max), fetches that
// sequence's packed header fields (ds_bpermute) and writes exactly one byte: token, length
// byte, literal (from the input ring), offset byte or match-length byte.  Rare sequences --
// literal run >= 270 bytes or outside the input ring, match >= 274 bytes -- and a flush that
// would overrun the slot take the general path, one sequence at a time.
// Round 3's per-window emitter wrote six bytes per POSITION lane (token, length bytes,
// offset, literal; trash bytes for the rest) after two prefix scans per window; with the
// emitter removed the parse ran 30 % faster (1 GiB kinds 1 / 5 / 6), so that is what this
// batching takes aim at.  The output bytes are the same.
#ifndef BITAR_LZ4_GATHER
#define BITAR_LZ4_GATHER 2
#endif
#ifndef BITAR_LZ4_OBUF
#define BITAR_LZ4_OBUF 512
#endif
constexpr uint32_t kLz4Obuf = BITAR_LZ4_OBUF;  // output ring (flushed to HBM in 16-B blocks)
constexpr uint32_t kSeqCap = 64;    // records per flush (a window adds <= 16)
struct Lz4Lds {
#if BITAR_LZ4_GATHER == 2
  uint8_t ring[kLz4Obuf];          // (the gather writes every lane's byte inside the room)
#else
  uint8_t ring[kLz4Obuf + kWave];  // + one trash byte per lane
#endif
  uint2 seqs[kSeqCap + 1];         // + a trash record
  uint32_t marks[kWave + 1];       // sequence starts of the current output step; + trash
};

struct Lz4Out : ByteOutT<kLz4Obuf> {
  Lz4Lds* L;
  uint32_t nseq;      // pending records
  uint32_t last_end;  // end of the last match emitted (the next literal run's start)
  uint32_t step_id;   // output steps so far (tags the marks, so they never need clearing)

  __device__ __forceinline__ void init(Lz4Lds* lds, GMEM uint8_t* d, uint64_t c) {
    L = lds;
    ring = lds->ring;
    dst = d;
    cap = c;
    op = flushed = 0;
    overflow = false;
    nseq = 0;
    last_end = 0;
    step_id = 0;
    lds->marks[lane_id()] = 0;  // (tag 0 never matches a step)
    lds_order();
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
  __device__ __forceinline__ void one(const GMEM uint8_t* in, const InRing& I, uint32_t lit_start,
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

#if BITAR_LZ4_GATHER == 2
  // records of lanes [lo, hi) (all ordinary) as LZ4 sequences, gathered 64 output bytes per
  // step; false (nothing written) if they would overrun the slot.
  // Per step (u = output byte + 1, vs op; lane t holds byte R + t):
  //  * the sequence of each byte: every token in the step marks its byte (LDS, the mark is
  //    the token's u and is cleared once read), one compare turns the marks into the step's
  //    start mask S, and the byte's sequence lane is lo - 1 + (tokens before the step) +
  //    (tokens at bytes R .. R + t): S & 1 on the scalar unit, the rest one v_mbcnt pair;
  //  * the byte itself: one ds_bpermute each of three packed words -- pA = A | T1 << 16
  //    (A = u of the token less the literal-length byte's presence, so r = u - A is 0 / 1 for
  //    the header bytes and >= 2 for literals whether or not that byte exists; T1 = u of the
  //    first offset byte), pH = the two header bytes | (the literal's ring index - u) << 16,
  //    pT = offset | match-length byte << 16 -- then sel = min(u - T1, r + 4, 6) indexes
  //    {pT bytes 0..3, hb0, hb1, literal}: one v_perm builds the upper word, one picks.
  // 18 VALU per 64 output bytes (the mark-tag / prefix-max form: ~50).
  __device__ __forceinline__ bool bulk(const InRing& I, uint32_t lo, uint32_t hi, uint32_t q,
                                       uint32_t lit_start, uint32_t off, uint32_t mlen) {
    const uint32_t lane = lane_id();
    const bool in = (lane >= lo) & (lane < hi);
    const uint32_t lit_len = q - lit_start, ml = mlen - kMinMatch;
    const uint32_t nlx = lit_len >= 15 ? 1u : 0u, nmx = ml >= 15 ? 1u : 0u;
    const uint32_t e = in ? 3u + nlx + nmx + lit_len : 0u;
    const uint32_t incl = wave_incl_sum(e);
    const uint32_t total = readlane(incl, kWave - 1);
    if ((uint64_t)op + total > cap) return false;
    const uint32_t a = incl - e;  // output offset of the sequence's token
    const uint32_t tok = ((lit_len < 15 ? lit_len : 15) << 4) | (ml < 15 ? ml : 15);
    const uint32_t A = a + nlx;
    const uint32_t T1 = a + 2u + nlx + lit_len;
    const uint32_t hb = nlx ? tok | (((lit_len - 15u) & 0xFFu) << 8) : tok << 8;
    const uint32_t D = I.in_lo + lit_start - A - 2u;  // ring index of a literal byte = D + u
    const uint32_t pA = A | (T1 << 16);
    const uint32_t pH = hb | (D << 16);
    const uint32_t pT = (off & 0xFFFFu) | (((ml - 15u) & 0xFFu) << 16);
    // mark slot x4 (lanes outside [lo, hi): the trash slot), and the mark: the token's u
    const uint32_t a4 = in ? a << 2 : 0x7FFFFF00u;
    const uint32_t mark = a + 1u;
    const uint32_t zero = 0;
    const uint32_t rbase = (uint32_t)(uintptr_t)dst + op - 1u;  // ring index = rbase + u
    uint32_t u = lane + 1u;
    uint32_t before = lo - 1u;  // lo - 1 + tokens before the step
    for (uint32_t R = 0; R < total; R += kWave) {
      // (the slot's capacity was checked for the whole batch: only the staging ring's room)
      if (op + kWave - flushed > kLz4Obuf - 64) flush(op, false);
      lds_order();
      const uint32_t slot = min(a4 - (R << 2), (uint32_t)kWave << 2);
      *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(L->marks) + slot) = mark;
      lds_order();
      const uint32_t mk = L->marks[lane];
      L->marks[lane] = zero;
      const uint64_t S = ballot(mk == u);
      const uint32_t base = before + (uint32_t)(S & 1u);
      const uint64_t S1 = S >> 1;
      // (the scalar base added after the shift: one v_lshl_add, no v_mov into the mbcnt)
      const uint32_t idx = __builtin_amdgcn_mbcnt_hi((uint32_t)(S1 >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)S1, 0u));
      before += (uint32_t)__builtin_popcountll(S);
      const int src = (int)((idx << 2) + (base << 2));
      const uint32_t qA = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)pA);
      const uint32_t qH = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)pH);
      const uint32_t qT = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)pT);
      const uint32_t r = u - (qA & 0xFFFFu);
      const uint32_t t = u - (qA >> 16);
      const uint32_t sel = min(min(t, r + 4u), 6u);
      const uint32_t litb = I.ring[(((u << 16) + qH) >> 16) & I.mask];
      // [hb0, hb1, literal, 0] then {pT bytes, that}[sel]
      const uint32_t hi4 = __builtin_amdgcn_perm(litb, qH, 0x0C040100u);
      const uint32_t b = __builtin_amdgcn_perm(hi4, qT, sel);
      const uint32_t nb = total - R < kWave ? total - R : kWave;
      // all 64 bytes are written: those past nb lie at or past the new op, inside the room
      // just made, and are rewritten before they are flushed
      ring[(rbase + u) & kMask] = (uint8_t)b;
      lds_order();
      op += nb;
      u += kWave;
    }
    return true;
  }
#else
  // records of lanes [lo, hi) (all ordinary) as LZ4 sequences, gathered 64 output bytes per
  // step; false (nothing written) if they would overrun the slot
  __device__ __forceinline__ bool bulk(const InRing& I, uint32_t lo, uint32_t hi, uint32_t q,
                                       uint32_t lit_start, uint32_t off, uint32_t mlen) {
    const uint32_t lane = lane_id();
    const bool in = (lane >= lo) & (lane < hi);
    const uint32_t lit_len = q - lit_start, ml = mlen - kMinMatch;
    const uint32_t nlx = lit_len >= 15 ? 1u : 0u, nmx = ml >= 15 ? 1u : 0u;
    const uint32_t e = in ? 3u + nlx + nmx + lit_len : 0u;
    const uint32_t incl = wave_incl_sum(e);
    const uint32_t total = readlane(incl, kWave - 1);
    if ((uint64_t)op + total > cap) return false;
    const uint32_t a = incl - e;  // output offset of the sequence's token
    const uint32_t tok = ((lit_len < 15 ? lit_len : 15) << 4) | (ml < 15 ? ml : 15);
    const uint32_t p0 = a | (lit_len << 16) | (nlx << 25) | (nmx << 26);
    const uint32_t p1 = lit_start | (tok << 16);
    const uint32_t p2 = (off & 0xFFFFu) | (((ml - 15u) & 0xFFu) << 16) | ((lit_len - 15u) << 24);
    for (uint32_t R = 0; R < total; R += kWave) {
      room(kWave);
      step_id += 1;
      // the sequences starting in this step mark their first byte; every byte then takes the
      // latest sequence starting at or before it (those before the step: counted by a ballot)
      const bool st = in & (a - R < kWave);
      lds_order();
      L->marks[st ? a - R : kWave] = (step_id << 8) | (lane + 1);
      lds_order();
      const uint32_t mk = L->marks[lane];
      const uint32_t before = (uint32_t)__builtin_popcountll(ballot(in & (a < R)));
      const uint32_t carry = before ? lo + before : 0u;
      const uint32_t v = (mk >> 8) == step_id ? (mk & 0xFFu) : 0u;
      const uint32_t s1 = max(wave_incl_max(v), carry);  // >= 1: lane lo starts at offset 0
      const int src = (int)((s1 - 1) << 2);
      const uint32_t q0 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)p0);
      const uint32_t q1 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)p1);
      const uint32_t q2 = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)p2);
      const uint32_t r = R + lane - (q0 & 0xFFFFu);  // byte of its sequence
      const uint32_t ll = (q0 >> 16) & 511u;
      const uint32_t L0 = 1u + ((q0 >> 25) & 1u), h = L0 + ll;
      const uint32_t litb = I.byte((q1 & 0xFFFFu) + r - L0);
      uint32_t b = r == h + 2 ? (q2 >> 16) & 0xFFu : (q2 >> 8) & 0xFFu;  // ml byte / off high
      b = r == h ? q2 & 0xFFu : b;
      b = r < h ? litb : b;
      b = r < L0 ? q2 >> 24 : b;  // (r == 1 with a literal-length byte)
      b = r == 0 ? (q1 >> 16) & 0xFFu : b;
      const uint32_t nb = total - R < kWave ? total - R : kWave;
      lds_order();
      ring[lane < nb ? at(op + lane) : kLz4Obuf + lane] = (uint8_t)b;
      lds_order();
      op += nb;
    }
    return true;
  }
#endif

  // every pending record as LZ4 sequences
  __device__ __forceinline__ void flush_seqs(const GMEM uint8_t* in, const InRing& I) {
    const uint32_t cnt = nseq;
    nseq = 0;
    if (!cnt || overflow) return;
    const uint32_t lane = lane_id();
    lds_order();
    const uint2 rec = L->seqs[lane < cnt ? lane : kSeqCap];
    const uint32_t q = rec.x & 0xFFFFu, off = (rec.x >> 16) + 1u, mlen = rec.y;
    const uint32_t end = q + mlen;
    const uint32_t prev = wave_shr1(end);
    const uint32_t lit_start = lane == 0 ? last_end : prev;
    const uint32_t lit_len = q - lit_start;
    last_end = readlane(end, cnt - 1);
    // rare sequences (and a flush that would overrun the slot) take the general path
    const uint64_t live = cnt < kWave ? (1ull << cnt) - 1 : ~0ull;
    uint64_t special = (ballot(lit_len >= 270u) | ballot(mlen >= 270u + kMinMatch) |
                        ballot(lit_start < I.lo)) & live;
    uint32_t lo = 0;
    for (;;) {
      const uint32_t k = special ? (uint32_t)__builtin_ctzll(special) : cnt;
      if (k > lo && !bulk(I, lo, k, q, lit_start, off, mlen)) {
        for (uint32_t j = lo; j < k && !overflow; ++j)  // (the slot's end: exact checks)
          one(in, I, readlane(lit_start, j), readlane(lit_len, j), readlane(off, j),
              readlane(mlen, j));
      }
      if (k >= cnt || overflow) break;
      one(in, I, readlane(lit_start, k), readlane(lit_len, k), readlane(off, k),
          readlane(mlen, k));
      special &= special - 1;
      lo = k + 1;
    }
  }

  // the tail literals (and whatever is pending before them)
  __device__ __forceinline__ void sequence(const GMEM uint8_t* in, const InRing& I,
                                           uint32_t lit_start, uint32_t lit_len, uint32_t off,
                                           uint32_t mlen) {
    flush_seqs(in, I);
    one(in, I, lit_start, lit_len, off, mlen);
  }
  // the tail sequence starts at the last match's end
  __device__ __forceinline__ uint32_t pending_from(uint32_t anchor, uint32_t) const { return anchor; }

  // between windows: flush the records once the next window could overfill the list
  __device__ __forceinline__ void between(const GMEM uint8_t* in, const InRing& I) {
    if (nseq > kSeqCap - 16) flush_seqs(in, I);
  }
  // One window: its matches appended as records (<= 16: matches are >= 4 bytes)
  __device__ __forceinline__ void window(const GMEM uint8_t*, const InRing&, const Window& W,
                                         uint32_t, uint32_t) {
    if (!W.chain) return;
    const uint64_t chain = W.chain;
    // (the record index: v_mbcnt adds its second operand, so no separate add)
    const uint32_t idx = __builtin_amdgcn_mbcnt_hi((uint32_t)(chain >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)chain, nseq));
    const uint32_t lane = lane_id();
    lds_order();
    L->seqs[lane_sel(chain, idx, kSeqCap)] =
        make_uint2((W.x + lane) | (W.dm1 << 16), W.mlen);
    lds_order();
    nseq += (uint32_t)__builtin_popcountll(chain);
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

#ifndef BITAR_DFL_BULK
#define BITAR_DFL_BULK 1
#endif
struct DflLds {
  uint2 recs[kSeqCap + 1];    // + a trash record
  uint32_t marks[kWave + 1];  // zero between steps; + trash
};
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
    // only lanes with bits for a word take part in its atomic (same-address lanes serialize;
    // kind 1 6.14 -> 5.60 ms, kind 6 8.18 -> 5.95 ms)
    if (nb) atomicOr(&stage[w & kBitMask], val << sh);
    if (sh + nb > 32) atomicOr(&stage[(w + 1) & kBitMask], spill);
    lds_order();
    bits += total;
    const uint32_t full = (uint32_t)(bits >> 5);
    if (full - wflushed >= kBitWords - 80) flush_words(full);  // a window adds <= 63 words
  }
  __device__ __forceinline__ void put_one(uint32_t val, uint32_t nb) {
    put_lanes(lane_id() == 0 ? val : 0u, lane_id() == 0 ? nb : 0u);
  }
  // literal codes of [s, s+n) (from the input ring when it holds them, else from HBM)
  __device__ __forceinline__ void literals(const GMEM uint8_t* in, const InRing& I, uint32_t s,
                                           uint32_t n) {
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
#if BITAR_DFL_BULK
  // Batched (as the LZ4 emitter): a window appends its matches {start | distance << 16,
  // length} to an LDS list; every <= 48 records (and before the tail) one flush codes their
  // symbols -- each record's literal run [previous match end, start), then its match --
  // 64 symbols per step: every run marks its first symbol (the run's u = symbol offset + 1),
  // one compare gives the step's start mask, a v_mbcnt pair the run, three ds_bpermute its
  // literal ring offset, match-symbol position + code length and match code (coded once per
  // record); a literal lane codes its byte from the input ring.  Only real symbols are coded
  // (the per-window form coded all 64 positions, the ones inside matches too).  Runs starting
  // below the input ring take the per-run path.  Same bitstream.
  DflLds* L;
  uint32_t npend, last_end;

  __device__ __forceinline__ void bulk(const InRing& I, uint32_t lo, uint32_t hi,
                                       uint32_t lit_start, uint32_t ll, uint32_t mv, uint32_t mb) {
    const uint32_t lane = lane_id();
    const bool in = (lane >= lo) & (lane < hi);
    const uint32_t e = in ? ll + 1u : 0u;
    const uint32_t incl = wave_incl_sum(e);
    const uint32_t total = readlane(incl, kWave - 1);
    const uint32_t a = incl - e;  // the run's first symbol
    const uint32_t D = I.in_lo + lit_start - a - 1u;  // ring index of a literal = D + u
    const uint32_t pX = ((a + ll + 1u) << 16) | mb;   // u of the match symbol | its length
    const uint32_t a4 = in ? a << 2 : 0x7FFFFF00u;
    const uint32_t mark = a + 1u;
    const uint32_t zero = 0;
    uint32_t u = lane + 1u;
    uint32_t before = lo - 1u;
    for (uint32_t R = 0; R < total && !overflow; R += kWave) {
      lds_order();
      const uint32_t slot = min(a4 - (R << 2), (uint32_t)kWave << 2);
      *reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(L->marks) + slot) = mark;
      lds_order();
      const uint32_t mk = L->marks[lane];
      L->marks[lane] = zero;
      const uint64_t S = ballot(mk == u);
      const uint32_t base = before + (uint32_t)(S & 1u);
      const uint64_t S1 = S >> 1;
      const uint32_t k = __builtin_amdgcn_mbcnt_hi((uint32_t)(S1 >> 32),
                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)S1, 0u));
      before += (uint32_t)__builtin_popcountll(S);
      const int src = (int)((k << 2) + (base << 2));
      const uint32_t qD = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)D);
      const uint32_t qX = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)pX);
      const uint32_t qM = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)mv);
      const uint32_t b = I.ring[(qD + u) & I.mask];
      uint32_t lb;
      const uint32_t lv = fixed_code(b, lb);
      const bool ism = u == (qX >> 16);
      const bool live = u <= total;
      put_lanes(ism ? qM : lv, live ? (ism ? (qX & 63u) : lb) : 0u);
      u += kWave;
    }
  }
  // every pending record's literal run and match
  __device__ __forceinline__ void flush_seqs(const GMEM uint8_t* in, const InRing& I) {
    const uint32_t cnt = npend;
    npend = 0;
    if (!cnt || overflow) return;
    const uint32_t lane = lane_id();
    lds_order();
    const uint2 rec = L->recs[lane < cnt ? lane : kSeqCap];
    const uint32_t q = rec.x & 0xFFFFu, off = (rec.x >> 16) + 1u, mlen = rec.y;
    const uint32_t end = q + mlen;
    const uint32_t prev = wave_shr1(end);
    const uint32_t lit_start = lane == 0 ? last_end : prev;
    const uint32_t ll = q - lit_start;
    last_end = readlane(end, cnt - 1);
    uint32_t mb;
    const uint32_t mv = match_code(lane < cnt ? mlen : 3u, lane < cnt ? off : 1u, mb);
    const uint64_t live = cnt < kWave ? (1ull << cnt) - 1 : ~0ull;
    uint64_t special = ballot(lit_start < I.lo) & ballot(ll != 0u) & live;
    uint32_t lo = 0;
    for (;;) {
      const uint32_t k = special ? (uint32_t)__builtin_ctzll(special) : cnt;
      if (k > lo) bulk(I, lo, k, lit_start, ll, mv, mb);
      if (k >= cnt || overflow) break;
      literals(in, I, readlane(lit_start, k), readlane(ll, k));
      put_one(readlane(mv, k), readlane(mb, k));
      special &= special - 1;
      lo = k + 1;
    }
  }
  // the tail literals start at the last match's end (after whatever is pending)
  __device__ __forceinline__ uint32_t pending_from(uint32_t anchor, uint32_t) const { return anchor; }
  __device__ __forceinline__ void between(const GMEM uint8_t* in, const InRing& I) {
    if (npend > kSeqCap - 16) flush_seqs(in, I);
  }
  // the tail literals (matches end >= 5 bytes before the segment end, so this always runs)
  __device__ __forceinline__ void sequence(const GMEM uint8_t* in, const InRing& I, uint32_t s,
                                           uint32_t n, uint32_t, uint32_t) {
    flush_seqs(in, I);
    literals(in, I, s, n);
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
    L->recs[lane_sel(chain, idx, kSeqCap)] =
        make_uint2((W.x + lane) | (W.dm1 << 16), W.mlen);
    lds_order();
    npend += (uint32_t)__builtin_popcountll(chain);
  }
#else
  // literals are emitted window by window: the tail starts where output stopped
  __device__ __forceinline__ uint32_t pending_from(uint32_t, uint32_t emitted) const { return emitted; }
  __device__ __forceinline__ void between(const GMEM uint8_t*, const InRing&) {}
  __device__ __forceinline__ void sequence(const GMEM uint8_t* in, const InRing& I, uint32_t s,
                                           uint32_t n, uint32_t, uint32_t) {
    literals(in, I, s, n);
  }

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
    const uint32_t mv = match_code(cl ? W.mlen : 3u, cl ? W.off() : 1u, mb);
    const uint32_t lv = fixed_code(W.byte, lb);
    const bool lit = !cl && !covered && q < n;
    put_lanes(cl ? mv : lit ? lv : 0u, cl ? mb : lit ? lb : 0u);
  }
#endif
};

}  // namespace cmp

// RING / HLOG: the parse's input ring and hash table -- 4 KiB / 1024 entries (distance cap
// 2560: BITAR_HIP_CODEC_LZ4, 21 waves per CU), or 16 KiB / 4096 entries (cap 14848:
// BITAR_HIP_CODEC_LZ4_WIDE, the ratio operating point; 27.3 KiB of LDS, 5 waves per CU)
#ifndef BITAR_LZ4C_WAVES
#define BITAR_LZ4C_WAVES 0  // tuning knob: waves per SIMD the register allocation must allow
#endif
#if BITAR_LZ4C_WAVES
#define BITAR_LZ4C_ATTR __attribute__((amdgpu_waves_per_eu(BITAR_LZ4C_WAVES)))
#else
#define BITAR_LZ4C_ATTR
#endif
template <uint32_t RING, uint32_t HLOG>
__global__ __launch_bounds__(64) BITAR_LZ4C_ATTR void lz4_compress_kernel(
    const uint8_t* __restrict__ input, uint64_t n_total, uint32_t seg,
    uint8_t* __restrict__ slab, uint64_t slot_stride, uint8_t* const* __restrict__ dsts,
    uint32_t* __restrict__ sizes, uint32_t* __restrict__ err, const uint32_t* __restrict__ order) {
  using namespace cmp;
  // (+ one trash entry: probe lanes past the segment insert there, see parse)
  __shared__ __attribute__((aligned(16))) uint16_t table[(1u << HLOG) + 8];
  __shared__ __attribute__((aligned(16))) uint8_t inring[RING + kInPad];
  __shared__ __attribute__((aligned(16))) Lz4Lds olds;
  // cost-ordered dispatch (seg_order_kernel): workgroup b compresses segment order[b]
  const uint32_t i_seg = order ? order[blockIdx.x] : blockIdx.x;
  const uint64_t seg_off = (uint64_t)i_seg * seg;
  if (seg_off >= n_total) return;
  const uint32_t n = (uint32_t)((n_total - seg_off) < seg ? (n_total - seg_off) : seg);
  Lz4Out o;
  o.init(&olds, global_ptr(dsts ? dsts[i_seg] : slab + (uint64_t)i_seg * slot_stride), slot_stride);
#ifndef BITAR_CMP_LZ4_SKIP
#define BITAR_CMP_LZ4_SKIP 1  // tuning knob: 0 = the plain window scan (not the oracle's LZ4 parse)
#endif
  parse<Lz4Out, false, BITAR_CMP_LZ4_SKIP != 0, RING, HLOG>(global_ptr(input + seg_off), n,
                                         global_ptr(input + n_total), table, inring,
                                         RING - 1536u, 0xFFFFFFFFu, o);
  o.flush(o.op, true);
  if (lane_id() == 0) {
    sizes[i_seg] = o.overflow ? 0xFFFFFFFFu : o.op;
    if (o.overflow) atomicOr(err, 2u);
  }
}

template __global__ void lz4_compress_kernel<cmp::kIn, cmp::kHashLog>(
    const uint8_t*, uint64_t, uint32_t, uint8_t*, uint64_t, uint8_t* const*, uint32_t*, uint32_t*,
    const uint32_t*);
template __global__ void lz4_compress_kernel<16384, 12>(
    const uint8_t*, uint64_t, uint32_t, uint8_t*, uint64_t, uint8_t* const*, uint32_t*, uint32_t*,
    const uint32_t*);

__global__ __launch_bounds__(64) void deflate_compress_kernel(
    const uint8_t* __restrict__ input, uint64_t n_total, uint32_t seg,
    uint8_t* __restrict__ slab, uint64_t slot_stride, uint8_t* const* __restrict__ dsts,
    uint32_t* __restrict__ sizes, uint32_t* __restrict__ err, const uint32_t* __restrict__ order) {
  using namespace cmp;
  __shared__ __attribute__((aligned(16))) uint16_t table[1u << kHashLog];
  __shared__ __attribute__((aligned(16))) uint8_t inring[kIn + kInPad];
  __shared__ __attribute__((aligned(16))) uint32_t stage[kBitWords];
#if BITAR_DFL_BULK
  __shared__ __attribute__((aligned(16))) DflLds dl;
#endif
  const uint32_t i_seg = order ? order[blockIdx.x] : blockIdx.x;  // (cost-ordered dispatch)
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
#if BITAR_DFL_BULK
  o.L = &dl;
  o.npend = 0;
  o.last_end = 0;
  dl.marks[lane_id()] = 0;
  lds_order();
#endif
  o.put_one(1u | (1u << 1), 3);  // BFINAL = 1, BTYPE = 01 (fixed Huffman)
  parse(global_ptr(input + seg_off), n, global_ptr(input + n_total), table, inring, kMaxDist,
        258u, o);
  uint32_t eb;
  const uint32_t eob = fixed_code(256, eb);
  o.put_one(eob, eb);
  o.flush_words((uint32_t)((o.bits + 31) >> 5));
  // stored blocks instead unless the fixed-Huffman block is smaller by at least n / 16
  // (incompressible input: the fixed code spends 9 bits on bytes >= 144; a nearly
  // incompressible segment coded anyway decodes a literal at a time, the slowest segment of
  // its decode launch) -- blocks of <= 65535 bytes, the last one final (oracle
  // bo_deflate_fixed_block, BO_STORE_MARGIN)
  uint32_t size = (uint32_t)((o.bits + 7) >> 3);
  const uint32_t nblk = (n + 65534u) / 65535u;
  const uint32_t stored = nblk * 5u + n;
  if (!o.overflow && stored < size + (n >> 4)) {  // (oracle BO_STORE_MARGIN)
    GMEM uint8_t* d = reinterpret_cast<GMEM uint8_t*>(o.dst);
    const GMEM uint8_t* in = global_ptr(input + seg_off);
    global_fence_wave();  // the fixed-Huffman stores to this range land first
    uint32_t p = 0, q = 0;
    for (uint32_t b = 0; b < nblk; ++b) {
      const uint32_t len = n - p < 65535u ? n - p : 65535u;
      const uint32_t lane = lane_id();
      const uint32_t hv = lane == 0 ? (b + 1 == nblk ? 1u : 0u)
                          : lane == 1 ? len & 0xFFu : lane == 2 ? len >> 8
                          : lane == 3 ? ~len & 0xFFu : (~len >> 8) & 0xFFu;
      if (lane < 5) d[q + lane] = (uint8_t)hv;
      wave_copy_global(d + q + 5, in + p, len);
      p += len;
      q += 5 + len;
    }
    size = stored;
  }
  if (lane_id() == 0) {
    sizes[i_seg] = o.overflow ? 0xFFFFFFFFu : size;
    if (o.overflow) atomicOr(err, 2u);
  }
}

}  // namespace bitar_hip
