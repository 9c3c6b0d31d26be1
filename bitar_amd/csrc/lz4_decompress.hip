// lz4_decompress.hip -- LZ4 block decode, one wavefront per segment (gfx950).
//
// Replaces the inflate op the reference hands to the BlueField engine per segment
// (reference src/memory.cc:432-505 assembles one op per compressed buffer; output slice
// i*seg of the caller's buffer).  Acceptance rules are exactly those of the oracle's
// bo_lz4_decompress_block (oracle/bitar_oracle.c), so malformed input fails identically:
// the block format's end conditions (final literal run >= 5 bytes, last match >= 12 bytes
// before the end) and liblz4's two limits on length-extension bytes included.  Batches
// never meet those (they stop >= 132 stream bytes before the end), so the general path
// checks them, the last match's length coming from the general path or -- when the final
// token directly follows a batch -- from a re-walk of that batch's headers.
//
// Per wave LDS (one wave per workgroup):
//   win[kWin]   the compressed stream, staged from HBM 16 B per lane (dwordx4), refilled
//               when the parse leaves it; token / length / offset / short-literal bytes are
//               read from here.
//   ring[kRing] the last kRing output bytes, indexed by ABSOLUTE output address & mask so a
//               16-B-aligned ring block is a 16-B-aligned HBM block.  Matches read their
//               history from the ring (LDS latency, no HBM round trip); completed 16-B
//               blocks are flushed to HBM with dwordx4 stores, 1 KiB per wave instruction.
//   Matches reaching further back than the ring read HBM, behind a lazily placed fence.
//   Literal runs >= kLongLit bypass the ring and stream HBM -> HBM (wave_copy_global).
#include "stream_ring.hip.h"

#include <type_traits>

// diagnostic build: count batches, their bytes, general-path sequences and why walks end
// (BITAR_HIP_PATH_LZ4_* 11..15; costs a few SALU per batch, so off by default)
#ifndef BITAR_LZ4D_PROFILE
#define BITAR_LZ4D_PROFILE 0
#endif
// tuning knob: 0 builds a decoder WITHOUT the end-of-block checks (timing A/B only; it is
// looser than the oracle)
#ifndef BITAR_LZ4D_ENDRULES
#define BITAR_LZ4D_ENDRULES 1
#endif

namespace bitar_hip {



namespace lz4d {

using namespace sr;

// stream bytes the batch path may touch past ip: 64 candidate tokens, each with up to two
// length bytes and <= 60 literals, plus its offset
constexpr uint32_t kBatchIn = 132;
// output bytes one batch may produce: two per lane, as two halves of 64 (lane t holds
// output bytes t and 64 + t); one sequence of the batch produces at most kSeqOut of them
constexpr uint32_t kBatchOut = 2 * kWave;
constexpr uint32_t kSeqOut = kWave;
// Largest next-token lane of an ELIGIBLE token (colen <= kSeqOut, minmatch 4): lane 63 +
// token + 2 offset bytes + a literal-length byte + max(60 literals with no match-length byte,
// 45 literals + a match-length byte, since an extended match is >= 19 bytes).  The walk
// record keeps it in 7 bits; widening eligibility must keep this <= 127.
constexpr uint32_t kMaxEligibleNext =
    (kWave - 1) + 3 + 1 + ((kSeqOut - 4) > (kSeqOut - 19) + 1 ? (kSeqOut - 4)
                                                                : (kSeqOut - 19) + 1);
static_assert(kMaxEligibleNext <= 127, "next-token lane overflows the walk record's 7 bits");

// 256 stream bytes held in ONE register, dword-packed: lane l holds bytes vb+4l .. vb+4l+3
// (vb 4-byte aligned in absolute address terms).  The parse reads tokens, extensions and
// offsets with v_readlane instead of LDS round trips.
struct SVec {
  uint32_t v;
  uint32_t vb;  // stream position of byte 0 (may be up to 3 below the first wanted byte)

  __device__ __forceinline__ void load(State& s, uint8_t* win, uint32_t pos) {
    const uint64_t abs = (uint64_t)(uintptr_t)(s.src + pos);
    const uint32_t mis = (uint32_t)(abs & 3u);
    uint32_t need = s.csize - pos + mis;
    if (need > 256) need = 256;
    // the window is 16-B aligned, so these dword reads are aligned
    const uint32_t w = win_at_abs(s, win, abs - mis, need);
    lds_order();
    v = *reinterpret_cast<const uint32_t*>(win + w + 4 * lane_id());
    vb = pos - mis;  // modular: may sit up to 3 below position 0
  }
  __device__ __forceinline__ bool covers(uint32_t pos, uint32_t n) const {
    return pos - vb <= 256u - n;  // modular difference: huge when pos < vb
  }
  // byte at stream position pos (covered)
  __device__ __forceinline__ uint32_t byte(uint32_t pos) const {
    const uint32_t k = pos - vb;
    return (readlane(v, k >> 2) >> ((k & 3u) * 8)) & 0xFFu;
  }
  // little-endian 16-bit value at pos (covered, pos+1 too)
  __device__ __forceinline__ uint32_t u16(uint32_t pos) const {
    const uint32_t k = pos - vb;
    const uint32_t d = k >> 2;
    const uint64_t w = (uint64_t)readlane(v, d) | ((uint64_t)readlane(v, (d + 1) & 63) << 32);
    return (uint32_t)(w >> ((k & 3u) * 8)) & 0xFFFFu;
  }
  __device__ __forceinline__ uint32_t get(State& s, uint8_t* win, uint32_t pos) {
    if (!covers(pos, 1)) load(s, win, pos);
    return byte(pos);
  }
};

// LZ4 length extension from the register vector; long runs (> 32 bytes of 255s) fall back
// to the 64-byte ballot scan.
__device__ __forceinline__ bool ext_len(State& s, uint8_t* win, SVec& sv, uint32_t& len) {
  for (uint32_t n = 0; n < 32; ++n) {
    if (s.ip >= s.csize) return false;
    const uint32_t b = sv.get(s, win, s.ip);
    s.ip += 1;
    len += b;
    if (b != 255u) return true;
  }
  return read_ext(s, win, len);
}


// The batch's token walk: from lane 0, follow the chain of candidate tokens while each
// sequence is eligible and fits in lim (<= 128) output bytes, and mark the lane of each
// sequence's first output byte with the sequence's token lane (v_writelane), in v0 for
// sequences starting in the first half (output bytes 0..63), in v1 for the second (64..127;
// the lane select is m0 mod 64).  Written out because the scalar chain is the batch's bound
// (one SALU per SIMD every 4 cycles, shared by the CU).  pw = next lane clamped to 63 (bits
// 0..5) | output length (bits 6..13, 255: not eligible) | kWordTag (bit 20: a written word
// is never 0) | unclamped next lane (bits 24..30: the stream advance when the walk ends after
// this sequence).  The word of the sequence before is what is written: its bits 0..5 are
// this sequence's token lane (the first sequence's "word before" is kWordTag alone: lane 0,
// advance 0), so the walk reads one word per sequence and the records stay in their token
// lanes.  Lane 63 is a sentinel that never qualifies, so "the next token lies past the
// parsed lanes" needs no compare of its own.  The room is kept as a remainder (one s_sub_u32
// both subtracts and tests: its borrow is "does not fit"), the word read is itself the next
// lane select (v_readlane takes the low 6 bits of its lane-select SGPR; >= 4 instructions
// separate each VALU write of e / e2 from its use as a lane select), each loop is unrolled
// twice: 3 SALU + 2 VALU per sequence.  Phase A's room ends at byte 64, so its loop never
// tests the half; the sequence that crosses byte 64 (or starts at it) is placed once by the
// hand-over code, then phase B runs with the whole room.  `adv` = the stream bytes consumed.
constexpr uint32_t kWordTag = 1u << 20;
__device__ __forceinline__ uint32_t walk_tokens2h(uint32_t pw, uint32_t lim, uint32_t& adv,
                                                  uint32_t& v0, uint32_t& v1) {
  uint32_t out, e, e2, ol, rem, m0_saved;
  __asm__ volatile(
      "s_mov_b32 %[m0s], m0\n"
      "s_mov_b32 %[e], %[tag]\n"
      "s_mov_b32 %[e2], 0\n"
      "s_min_u32 %[rem], %[lim], 64\n"
      "s_mov_b32 m0, 0\n"
      // phase A: sequences ending at or before byte 64 (or lim)
      "L_a_%=:\n"
      "v_readlane_b32 %[e2], %[pw], %[e]\n"
      "s_bfe_u32 %[ol], %[e2], 0x80006\n"
      "s_sub_u32 %[rem], %[rem], %[ol]\n"
      "s_cbranch_scc1 L_xa_%=\n"
      "v_writelane_b32 %[v0], %[e], m0\n"
      "s_add_u32 m0, m0, %[ol]\n"
      "v_readlane_b32 %[e], %[pw], %[e2]\n"
      "s_bfe_u32 %[ol], %[e], 0x80006\n"
      "s_sub_u32 %[rem], %[rem], %[ol]\n"
      "s_cbranch_scc1 L_xb_%=\n"
      "v_writelane_b32 %[v0], %[e2], m0\n"
      "s_add_u32 m0, m0, %[ol]\n"
      "s_branch L_a_%=\n"
      // hand-over, failing word in e2 (word before: e): fits the whole room?
      "L_xa_%=:\n"
      "s_sub_u32 %[rem], %[lim], m0\n"
      "s_sub_u32 %[rem], %[rem], %[ol]\n"
      "s_cbranch_scc1 L_da_%=\n"
      "s_cmp_lt_u32 m0, 64\n"
      "s_cbranch_scc0 L_xa1_%=\n"
      "v_writelane_b32 %[v0], %[e], m0\n"
      "s_add_u32 m0, m0, %[ol]\n"
      "s_branch L_b_%=\n"
      "L_xa1_%=:\n"
      "v_writelane_b32 %[v1], %[e], m0\n"
      "s_add_u32 m0, m0, %[ol]\n"
      "s_branch L_b_%=\n"
      // hand-over, failing word in e (word before: e2)
      "L_xb_%=:\n"
      "s_sub_u32 %[rem], %[lim], m0\n"
      "s_sub_u32 %[rem], %[rem], %[ol]\n"
      "s_cbranch_scc1 L_db_%=\n"
      "s_cmp_lt_u32 m0, 64\n"
      "s_cbranch_scc0 L_xb1_%=\n"
      "v_writelane_b32 %[v0], %[e2], m0\n"
      "s_add_u32 m0, m0, %[ol]\n"
      "s_branch L_b2_%=\n"
      "L_xb1_%=:\n"
      "v_writelane_b32 %[v1], %[e2], m0\n"
      "s_add_u32 m0, m0, %[ol]\n"
      "s_branch L_b2_%=\n"
      // phase B: every later sequence starts past byte 64
      "L_b_%=:\n"
      "v_readlane_b32 %[e], %[pw], %[e2]\n"
      "s_bfe_u32 %[ol], %[e], 0x80006\n"
      "s_sub_u32 %[rem], %[rem], %[ol]\n"
      "s_cbranch_scc1 L_db_%=\n"
      "v_writelane_b32 %[v1], %[e2], m0\n"
      "s_add_u32 m0, m0, %[ol]\n"
      "L_b2_%=:\n"
      "v_readlane_b32 %[e2], %[pw], %[e]\n"
      "s_bfe_u32 %[ol], %[e2], 0x80006\n"
      "s_sub_u32 %[rem], %[rem], %[ol]\n"
      "s_cbranch_scc1 L_da_%=\n"
      "v_writelane_b32 %[v1], %[e], m0\n"
      "s_add_u32 m0, m0, %[ol]\n"
      "s_branch L_b_%=\n"
      "L_da_%=:\n"
      "s_lshr_b32 %[e], %[e], 24\n"
      "s_branch L_out_%=\n"
      "L_db_%=:\n"
      "s_lshr_b32 %[e], %[e2], 24\n"
      "L_out_%=:\n"
      "s_mov_b32 %[out], m0\n"
      "s_mov_b32 m0, %[m0s]\n"
      : [e] "=&s"(e), [e2] "=&s"(e2), [out] "=&s"(out), [ol] "=&s"(ol), [rem] "=&s"(rem),
        [m0s] "=&s"(m0_saved), [v0] "+v"(v0), [v1] "+v"(v1)
      : [pw] "v"(pw), [lim] "s"(lim), [tag] "i"(kWordTag)
      : "scc");
  adv = e;
  return out;
}

}  // namespace lz4d

// Two instantiations, launched back to back by the runtime:
//   FARK = false  every segment; batches admit offsets within the ring only (our own streams
//                 never go beyond it).  A segment whose next sequence could be batched only
//                 with far history (stock streams: offsets up to 65535) is deferred
//                 (produced = kDefer) as soon as that is seen.
//   FARK = true   the deferred segments only (the others exit at once): FAR batches read far
//                 history back from HBM, and stay FAR while they meet it.
// Keeping the far machinery out of the first kernel keeps its batch path as short as before
// (measured: 4-8 % on our own streams when both share one kernel).
constexpr uint32_t kDefer = 0xFFFFFFFEu;

template <bool FARK>
__global__ __launch_bounds__(64) void lz4_decompress_kernel(
    const uint8_t* const* __restrict__ srcs, const uint8_t* __restrict__ slab,
    uint64_t slot_stride, const uint32_t* __restrict__ csizes, uint32_t nseg, uint32_t seg,
    uint8_t* __restrict__ out, uint32_t* __restrict__ produced, uint32_t* __restrict__ err,
    unsigned long long* __restrict__ stats, const uint32_t* __restrict__ order) {
  using namespace lz4d;
  // the ring at LDS address 0: a history source is then (address & mask), one add fewer
  __shared__ __attribute__((aligned(16))) uint8_t lds[kRing + kWin];
  uint8_t* ring = lds;
  uint8_t* win = lds + kRing;
  if (blockIdx.x >= nseg) return;
  // cost-ordered dispatch (seg_order_kernel): workgroup b decodes segment order[b]
  const uint32_t i = order ? order[blockIdx.x] : blockIdx.x;
  if (FARK && produced[i] != kDefer) return;

  State s;
  s.src = global_ptr(srcs ? srcs[i] : slab + (uint64_t)i * slot_stride);
  s.csize = csizes[i];
  s.dst = global_ptr(out + (uint64_t)i * seg);
  s.cap = seg;
  s.ip = 0;
  s.op = 0;
  s.flushed = 0;
  s.fenced = 0;
  s.wb = ~0ull;  // nothing staged
  s.wlen = 0;

  bool ok = s.csize != 0;
  SVec sv;
  sv.vb = 0xFFFFFF00u;  // nothing loaded
  sv.v = 0;
  const uint32_t lane = lane_id();
  const uint32_t base = (uint32_t)(uintptr_t)s.dst;  // ring index = absolute address & mask
  const uint32_t src_lo = (uint32_t)(uintptr_t)s.src;
  bool want_far = false, stay_far = false;
  // end-of-block conditions: the last match's length (0 = it was in the batch at bip)
  uint32_t last_ml = 0, bip = 0, fin_lit = 0, fin_tok = 0;
  [[maybe_unused]] uint32_t p_batches = 0, p_bytes = 0, p_general = 0, p_stop_parse = 0,
                            p_stop_inel = 0;
  while (ok) {
    // ---- batch fast path: up to kBatchOut output bytes of short sequences per step ------
    // 1. every lane l decodes "a token at stream position ip+l" from the LDS window
    //    (token, literal count, match length, offset): a speculative parse of 64 candidates;
    // 2. a scalar walk follows the real token chain from ip (one v_readlane per sequence)
    //    while the sequences are short (no length extension), not last, and fit the batch;
    //    it drops each sequence's record into the lane of its first output byte
    //    (v_writelane), and a DPP prefix max hands every output byte its sequence's record
    //    (the output start sits in the top bits, so the latest start wins);
    // 3. each output byte (lane t holds bytes t, t+64, ...) finds its source: a literal byte
    //    in the window, a history byte in the ring, or -- for a match reaching into this
    //    batch -- another byte of the batch, resolved by pointer doubling;
    // 4. one ds_read per 64 bytes gathers the batch, one ds_write stores it into the ring.
    // Bytes past the batch are written too: their ring slots are >= kRing - kBatchOut
    // behind the output, older than any near source and already flushed, and are rewritten
    // before use.
    // one batch; FAR = false admits offsets within the ring only (the common case, no far
    // bookkeeping), FAR = true any offset (far history read from HBM); returns the output
    // byte count, 0 if the first token does not qualify
    auto batch = [&](auto far_tag) __attribute__((always_inline)) -> uint32_t {
      constexpr bool FAR = decltype(far_tag)::value;
      if (s.op + kBatchOut - s.flushed > kFlushAt) flush(s, ring, s.op, false);
      uint32_t wrel = src_lo + s.ip - (uint32_t)s.wb;  // window index of ip (mod 2^32)
      if (wrel > kWin - kBatchIn) {
        win_at(s, win, s.ip, kBatchIn);
        wrel = src_lo + s.ip - (uint32_t)s.wb;
      }
      // (1) speculative parse, one candidate token per lane: token, optional literal
      //     length byte, literals, offset, optional match length byte
      lds_order();
      const uint32_t wc = wrel + lane;
      // the literal gather's base, LDS address of this lane's stream byte (kept in a VGPR
      // of its own: folded into the parse's reads, it costs every literal address an add)
      uint32_t wck = kRing + wc;
      __asm__("" : "+v"(wck));
      const uint32_t tok = win[wc];
      const uint32_t b1 = win[wc + 1];
      const uint32_t cm4 = tok & 15u;
      const bool lx = (tok >> 4) == 15u, mx = cm4 == 15u;
      const uint32_t cL = lx ? 15u + b1 : tok >> 4;
      const uint32_t ob = wc + 1 + (lx ? 1u : 0u) + cL;  // offset position
      const uint32_t cb0 = win[ob], cb1 = win[ob + 1], b2 = win[ob + 2];
      const uint32_t coff = cb0 | (cb1 << 8);
      const uint32_t cml = 4 + (mx ? 15u + b2 : cm4);
      const uint32_t colen = cL + cml;
      // eligible: <= 64 output bytes (so <= 60 literals; a length byte of 255, which would
      // continue the length, makes colen >= 274, so this also means "one length byte each"),
      // a real offset (within the ring, or any distance in a FAR batch: far sources are read
      // back from HBM below), not before the segment start (conservatively, as if this token
      // opened the batch)
      // bitwise on the compares: short-circuit forms compile to an exec-mask branch
      const bool cfar = (colen <= kSeqOut) & (coff - 1u < s.op + cL);
      const bool csimple = cfar && (FAR || coff <= kNearOff);
      // walk word: next token lane (7 bits, <= 127 for an eligible token, see
      // kMaxEligibleNext; the walk stops at a lane >= 64, which was not parsed, after
      // consuming the sequence) | output length (255: not eligible, the walk's one compare
      // then stops; an ineligible token's wider nxt only ORs into those already-set bits).
      // Sequence record (stays in the token lane): offset (16 bits) | literal count (byte 2;
      // <= 60 when eligible) | lane of the first literal (byte 3: lane + 1 + lx <= 64).
      const uint32_t nxt = lane + 3 + (lx ? 1u : 0u) + (mx ? 1u : 0u) + cL;
      const uint32_t pr = coff | (cL << 16) | ((lane + 1u + (lx ? 1u : 0u)) << 24);
      // (2) scalar walk over the real tokens (capacity: checked once for the whole batch)
      const uint32_t room = s.cap - s.op;
      const uint32_t lim = room < kBatchOut ? room : kBatchOut;
      // (lanes the walk does not write keep bit 31: negative keys for the signed prefix max)
      uint32_t k, vrec0 = 0x80000000u, vrec1 = 0x80000000u;
      const bool celig = csimple && lane < kWave - 1;  // lane 63: the walk's sentinel
      const uint32_t pw = (nxt < kWave - 1 ? nxt : kWave - 1) | ((celig ? colen : 255u) << 6) |
                          kWordTag | (nxt << 24);
      const uint32_t out = walk_tokens2h(pw, lim, k, vrec0, vrec1);
      if (out == 0) {
        // the first token qualifies only for a FAR batch: worth trying one
        if (!FAR) want_far = (ballot(cfar) & 1ull) != 0;
        return 0u;
      }
      if constexpr (BITAR_LZ4D_PROFILE != 0) {
        p_batches += 1;
        p_bytes += out;
        if (k >= kWave - 1) p_stop_parse += 1;
        else if ((readlane(pw, k) >> 6 & 255u) == 255u) p_stop_inel += 1;
      }
      // FAR batches (entered only where a near batch could not start: stock streams with
      // offsets beyond the ring's reach; ours stay <= 2560) read far history from HBM
      constexpr bool big = FAR;
      if (big) stay_far = false;
      // (3)+(4) for the output bytes 64h .. 64h+63 (lane t: byte 64h + t); `key` is the
      // byte's sequence: its token lane (bits 0..5) and output start (bits 24..30)
      auto prep = [&](auto h_tag, uint32_t key) __attribute__((always_inline)) -> uint32_t {
        constexpr uint32_t H = decltype(h_tag)::value;
        const uint32_t q = lane + H * kWave;  // output byte of this lane (vs op)
        // sources: window literal / ring history / HBM history (far) / alias of an earlier
        // byte of this half (branch-free: every lane computes every form).  bit31: alias
        // (low 6 bits: the source lane); bit30: far (low 16 bits: the output position); else
        // an LDS byte address.  Bytes of the first half are in the ring already when the
        // second half reads them.
        const uint32_t ostart = key >> 24;
        // the record from its token lane (ds_bpermute reads address bits 2..7 only)
        const uint32_t rec =
            (uint32_t)__builtin_amdgcn_ds_bpermute((int)(key << 2), (int)pr);
        const uint32_t ms = ostart + ((rec >> 16) & 0xFFu);  // the match's first byte (vs op)
        const bool is_lit = q < ms;
        // a match byte's source: q - off (vs op; SDWA takes the offset's 16 bits in place)
        int32_t srel;
        __asm__("v_sub_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD "
                "src0_sel:DWORD src1_sel:WORD_0"
                : "=v"(srel) : "v"(q), "v"(rec));
        // overlapping copy (source inside the match itself: q - off >= ms): fold the source
        // into the first period, ms + (m mod off) - off with m = q - ms (exact in fp32 for
        // m, off < 64); skipped when no byte needs it
        if (ballot(srel >= (int32_t)ms && q < out)) {
          const uint32_t joff = rec & 0xFFFFu;
          const uint32_t m = (q - ms) & 63u;
          const float qf = floorf(((float)m + 0.5f) *
                                  __builtin_amdgcn_rcpf((float)(joff > 1u ? joff : 1u)));
          const int32_t sf = (int32_t)(ms + m - (uint32_t)qf * joff) - (int32_t)joff;
          srel = srel >= (int32_t)ms ? sf : srel;  // (a select: no exec-mask branch)
        }
        const uint32_t hist = (base + s.op + (uint32_t)srel) & kRingMask;  // ring at 0
        const uint32_t lit_addr = wck + H * kWave + (rec >> 24) - ostart;
        // every form computed before the selects (the empty asm pins them), so the compiler
        // does not turn the selects into an exec-mask if / else
        uint32_t lit_a = lit_addr, hist_a = hist, alias_a = (uint32_t)srel | 0x80000000u;
        __asm__("" : "+v"(lit_a), "+v"(hist_a), "+v"(alias_a));
        uint32_t st = srel >= (int32_t)(H * kWave) ? alias_a : hist_a;
        st = is_lit ? lit_a : st;
        if (big && srel < -(int32_t)kNearOff && !is_lit)
          st = (s.op + (uint32_t)srel) | 0x40000000u;  // far: the output position
        return st;
      };
      // pointer doubling, the gather and the store of a half whose sources prep gave
      auto finish = [&](auto h_tag, uint32_t st) __attribute__((always_inline)) {
        constexpr uint32_t H = decltype(h_tag)::value;
        const uint32_t q = lane + H * kWave;  // output byte of this lane (vs op)
        // pointer doubling until no byte of the half aliases another: every alias chain
        // strictly descends (srel <= q - 1, past-the-end bytes included), so <= 6 rounds
        // (written out: the compiler's form of this loop spends three branches on the
        // usual zero rounds; ds_bpermute reads its lane from address bits 2..7 only)
        {
          uint32_t a, o;
          __asm__ volatile(
              "L_dbl_%=:\n"
              "v_cmp_gt_i32_e32 vcc, 0, %[st]\n"
              "s_cbranch_vccz L_dbe_%=\n"
              "v_lshlrev_b32_e32 %[a], 2, %[st]\n"
              "ds_bpermute_b32 %[o], %[a], %[st]\n"
              "s_waitcnt lgkmcnt(0)\n"
              "v_cndmask_b32_e32 %[st], %[st], %[o], vcc\n"
              "s_branch L_dbl_%=\n"
              "L_dbe_%=:\n"
              : [st] "+v"(st), [a] "=&v"(a), [o] "=&v"(o)
              :
              : "vcc", "memory");
        }
        // one gather (LDS, or HBM for far history), one store
        lds_order();
        // (near batches: every resolved source is an LDS address < kRing + kWin)
        uint32_t g = lds[big ? st & 0x3FFFu : st];
        if (big) {
          const bool gfar = (st >> 30) == 1u && q < out;
          const uint64_t farm = ballot(gfar);
          // history only in HBM: make this wave's flushed stores visible to its loads
          if (farm && (ballot((st & 0xFFFFu) >= s.fenced) & farm)) {
            global_fence_wave();
            s.fenced = s.flushed;
          }
          if (gfar) g = s.dst[st & 0xFFFFu];
          stay_far |= farm != 0;  // keep to FAR batches while they meet far history
        }
        ring[(base + s.op + q) & kRingMask] = (uint8_t)g;
        lds_order();
      };
      auto half = [&](auto h_tag, uint32_t key) __attribute__((always_inline)) {
        finish(h_tag, prep(h_tag, key));
      };
      // every output byte takes the record of the latest sequence starting at or before it
      // (a written word has bit 31 clear, so its key is >= 0; the first sequence's, at lane
      // 0, is 0, so every half-0 key ends >= 0)
#ifndef BITAR_LZ4D_KEYS2
#define BITAR_LZ4D_KEYS2 1
#endif
      const uint32_t key0 =
          (uint32_t)wave_incl_max_i((int32_t)((vrec0 & 0x8000003Fu) | (lane << 24)));
#if BITAR_LZ4D_KEYS2
      // (both halves' scans side by side: each DPP step's two wait states filled by the
      // other scan's; the second is wasted on a batch of <= 64 bytes)
      const int32_t key1 =
          wave_incl_max_i((int32_t)((vrec1 & 0x8000003Fu) | ((lane + kWave) << 24)));
#endif
#ifndef BITAR_LZ4D_SPLIT
#define BITAR_LZ4D_SPLIT 1
#endif
#if BITAR_LZ4D_KEYS2 && BITAR_LZ4D_SPLIT
      // both halves' sources worked out before either gathers (independent work side by
      // side; the second half's is wasted on a batch of <= 64 bytes), then half 0's gather and
      // store, then half 1's, which may read half 0's bytes from the ring
      {
        const uint32_t st0 = prep(std::integral_constant<uint32_t, 0>{}, key0);
        const int32_t carry = (int32_t)readlane(key0, kWave - 1);
        const uint32_t st1 = prep(std::integral_constant<uint32_t, 1>{},
                                  (uint32_t)(key1 > carry ? key1 : carry));
        finish(std::integral_constant<uint32_t, 0>{}, st0);
        if (out > kWave) finish(std::integral_constant<uint32_t, 1>{}, st1);
      }
      if (false) {
#else
      half(std::integral_constant<uint32_t, 0>{}, key0);
#endif
      if (out > kWave) {
        // second half: its own starts (all past byte 64), else the first half's last record
#if !BITAR_LZ4D_KEYS2
        const int32_t key1 =
            wave_incl_max_i((int32_t)((vrec1 & 0x8000003Fu) | ((lane + kWave) << 24)));
#endif
        const int32_t carry = (int32_t)readlane(key0, kWave - 1);
        half(std::integral_constant<uint32_t, 1>{}, (uint32_t)(key1 > carry ? key1 : carry));
      }
#if BITAR_LZ4D_KEYS2 && BITAR_LZ4D_SPLIT
      }
#endif
      if constexpr (BITAR_LZ4D_ENDRULES == 1 || BITAR_LZ4D_ENDRULES == 2) {
        bip = s.ip;
        last_ml = 0;
      }
      s.ip += __builtin_amdgcn_readfirstlane(k);  // (k is an SGPR: keeps the add scalar)
      s.op += out;
      return out;
    };
    if constexpr (!FARK) {
      // one loop condition computed at the end of each batch (the for / continue / break
      // form compiles to ~12 SALU of uniform-bool bookkeeping per batch)
      want_far = false;
      if (s.ip + kBatchIn <= s.csize) {
        uint32_t t;
        do {
          const uint32_t o = batch(std::false_type{});
          // "a batch was made and the next one fits the stream": one compare (the select
          // in asm, so the compiler keeps it a single scalar branch)
          const uint32_t rest = s.csize - s.ip;
          __asm__("s_cmp_lg_u32 %1, 0\n s_cselect_b32 %0, %2, 0" : "=s"(t) : "s"(o), "s"(rest)
                  : "scc");
        } while (t >= kBatchIn);
      }
    } else
    for (;;) {
      if (s.ip + kBatchIn > s.csize) break;
      if constexpr (FARK) {
        if (stay_far) {
          if (batch(std::true_type{})) continue;
          stay_far = false;
        }
        want_far = false;
        if (batch(std::false_type{})) continue;
        if (!want_far || !batch(std::true_type{})) break;
      } else {
        want_far = false;
        if (batch(std::false_type{})) continue;
        break;
      }
    }
    if (!FARK && want_far) break;  // defer the segment to the FAR kernel
    // ---- general path: one sequence, any shape -----------------------------------------
    if constexpr (BITAR_LZ4D_PROFILE != 0) p_general += 1;
    if (s.ip >= s.csize) { ok = false; break; }
    const uint32_t tok_at = s.ip;
    const uint32_t token = sv.get(s, win, s.ip);
    s.ip += 1;
    uint32_t lit = token >> 4;
    // (a literal-length extension must start > 15 bytes before the end: liblz4)
    if (lit == 15 && (s.ip + 15 >= s.csize || !ext_len(s, win, sv, lit))) { ok = false; break; }
    if ((uint64_t)s.ip + lit > s.csize || (uint64_t)s.op + lit > s.cap) { ok = false; break; }
    if (lit >= kLongLit) literals_long(s, win, ring, lit);
    else if (lit) literals_short(s, win, ring, lit);
    if (s.ip == s.csize) {  // last sequence: literals only (end conditions: below)
      fin_lit = lit;
      fin_tok = tok_at;
      break;
    }
    if (s.ip + 2 > s.csize) { ok = false; break; }
    const uint32_t o0 = sv.get(s, win, s.ip);
    const uint32_t o1 = sv.get(s, win, s.ip + 1);
    s.ip += 2;
    const uint32_t off = o0 | (o1 << 8);
    if (off == 0 || off > s.op) { ok = false; break; }
    uint32_t m = token & 15u;
    // (a match-length extension must end > 4 bytes before the end: liblz4)
    if (m == 15 && (!ext_len(s, win, sv, m) || s.ip + 4 >= s.csize)) { ok = false; break; }
    m += 4;
    if ((uint64_t)s.op + m > s.cap) { ok = false; break; }
    match_copy(s, ring, off, m);
    last_ml = m;
  }
  if constexpr (BITAR_LZ4D_PROFILE != 0) {
    if (stats && lane_id() == 0) {
      atomicAdd(stats + BITAR_HIP_PATH_LZ4_BATCHES, (unsigned long long)p_batches);
      atomicAdd(stats + BITAR_HIP_PATH_LZ4_BATCH_BYTES, (unsigned long long)p_bytes);
      atomicAdd(stats + BITAR_HIP_PATH_LZ4_GENERAL_SEQS, (unsigned long long)p_general);
      atomicAdd(stats + BITAR_HIP_PATH_LZ4_STOP_PARSE, (unsigned long long)p_stop_parse);
      atomicAdd(stats + BITAR_HIP_PATH_LZ4_STOP_INELIGIBLE, (unsigned long long)p_stop_inel);
    }
  }
  // the block format's end conditions, if the block had a match: >= 5 final literals, the
  // last match >= 12 bytes before the end (its length: from the general path, or -- the
  // final token right after a batch -- re-walked from that batch's first token; ml >= 4
  // settles fin_lit >= 8).  Out of the decode loop: inside it, this code cost the loop 6 %.
  if ((BITAR_LZ4D_ENDRULES == 1 || BITAR_LZ4D_ENDRULES == 3) && ok && s.op > fin_lit &&
      !(!FARK && want_far)) {
    uint32_t ml = last_ml;
    if (ml == 0 && fin_lit >= 5 && fin_lit < 8) {
      for (uint32_t p = bip; p < fin_tok;) {
        const uint32_t t = sv.get(s, win, p);
        uint32_t ll = t >> 4, mm = t & 15u;
        p += 1;
        if (ll == 15) ll += sv.get(s, win, p++);  // (batch sequences: <= 1 length byte)
        p += ll + 2;
        if (mm == 15) mm += sv.get(s, win, p++);
        ml = mm + 4;
      }
    }
    if (fin_lit < 5 || fin_lit + ml < 12) ok = false;
  }
  if (!FARK && want_far) {
    if (lane_id() == 0) {
      produced[i] = kDefer;
      if (stats) atomicAdd(stats + BITAR_HIP_PATH_LZ4_FAR, 1ull);
    }
  } else if (ok) {
    flush(s, ring, s.op, true);
    if (lane_id() == 0) produced[i] = s.op;
  } else if (lane_id() == 0) {
    produced[i] = 0xFFFFFFFFu;
    atomicOr(err, 1u);
  }
}

template __global__ void lz4_decompress_kernel<false>(const uint8_t* const*, const uint8_t*,
                                                     uint64_t, const uint32_t*, uint32_t,
                                                     uint32_t, uint8_t*, uint32_t*, uint32_t*,
                                                     unsigned long long*, const uint32_t*);
template __global__ void lz4_decompress_kernel<true>(const uint8_t* const*, const uint8_t*,
                                                    uint64_t, const uint32_t*, uint32_t, uint32_t,
                                                    uint8_t*, uint32_t*, uint32_t*,
                                                    unsigned long long*, const uint32_t*);

}  // namespace bitar_hip
