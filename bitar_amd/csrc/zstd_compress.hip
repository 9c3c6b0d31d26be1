// zstd_compress.hip -- Zstandard (RFC 8878) frame per segment, one wavefront per segment
// (gfx950): zstd_compress_kernel, BASELINE configs[5].
//
// The frame is exactly the one the oracle's bo_zstd_compress_block (oracle/bitar_zstd.c)
// writes: single-segment frame header with the content size, then blocks of <= 256
// sequences found by the shared window-scan parse (window_parse.hip.h, restated by
// bo_window_parse), each block = raw literals section + sequences coded with the predefined
// FSE distributions (RFC 8878 3.1.1.3.2.2), offsets as Offset_Value = distance + 3 (no
// repeat offsets); a block that does not shrink is stored raw.
#include "window_parse.hip.h"

namespace bitar_hip {

namespace zse {

constexpr uint32_t kMaxSeq = 256;  // sequences per block (oracle ZS_MAX_SEQ)

// ---- predefined distributions and code tables (RFC 8878 3.1.1.3.2.1-2) ---------------------
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
constexpr uint8_t kOFBits[29] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14,
                                 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28};
constexpr int16_t kLLNorm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
constexpr int16_t kMLNorm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
constexpr int16_t kOFNorm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

// FSE compression table of one predefined distribution (FSE_buildCTable; the oracle's
// zs_build_ctable): state[] = next-state table, per symbol {deltaNbBits, deltaFindState |
// extra-bit count << 16}.
struct CTab {
  uint16_t state[64];
  uint2 sym[64];
};

constexpr CTab build_ctab(const int16_t* norm, uint32_t max_sym, uint32_t al,
                          const uint8_t* extra) {
  CTab c{};
  const uint32_t size = 1u << al, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
  uint32_t high = size - 1;
  uint8_t sym_at[64] = {};
  uint32_t cumul[65] = {};
  for (uint32_t s = 1; s <= max_sym + 1; ++s) {
    if (norm[s - 1] == -1) {
      cumul[s] = cumul[s - 1] + 1;
      sym_at[high--] = (uint8_t)(s - 1);
    } else {
      cumul[s] = cumul[s - 1] + (uint32_t)norm[s - 1];
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
  for (uint32_t u = 0; u < size; ++u) c.state[cumul[sym_at[u]]++] = (uint16_t)(size + u);
  int32_t total = 0;
  for (uint32_t s = 0; s <= max_sym; ++s) {
    int32_t dnb = 0, dfs = 0;
    if (norm[s] == 0) {
      dnb = (int32_t)(((al + 1) << 16) - size);
    } else if (norm[s] == -1 || norm[s] == 1) {
      dnb = (int32_t)((al << 16) - size);
      dfs = total - 1;
      total += 1;
    } else {
      uint32_t hb = 0;  // highbit(norm - 1)
      for (uint32_t v = (uint32_t)norm[s] - 1; v > 1; v >>= 1) ++hb;
      const uint32_t mbo = al - hb;
      const uint32_t msp = (uint32_t)norm[s] << mbo;
      dnb = (int32_t)((mbo << 16) - msp);
      dfs = total - norm[s];
      total += norm[s];
    }
    c.sym[s] = uint2{(uint32_t)dnb, ((uint32_t)dfs & 0xFFFFu) | ((uint32_t)extra[s] << 16)};
  }
  return c;
}

// code of a literal length < 64 / of a match length - 3 < 128 (ZSTD_LLcode / ZSTD_MLcode;
// longer lengths: highbit + 19 / + 36)
struct Codes {
  uint8_t ll[64];
  uint8_t ml[128];
};
constexpr Codes build_codes() {
  Codes t{};
  for (uint32_t v = 0; v < 64; ++v) {
    uint32_t c = 35;
    while (kLLBase[c] > v) --c;
    t.ll[v] = (uint8_t)c;
  }
  for (uint32_t v = 0; v < 128; ++v) {
    uint32_t c = 52;
    while (kMLBase[c] > v + 3) --c;
    t.ml[v] = (uint8_t)c;
  }
  return t;
}

__constant__ CTab kCtLL = build_ctab(kLLNorm, 35, 6, kLLBits);
__constant__ CTab kCtML = build_ctab(kMLNorm, 52, 6, kMLBits);
__constant__ CTab kCtOF = build_ctab(kOFNorm, 28, 5, kOFBits);
__constant__ Codes kCodes = build_codes();

__device__ __forceinline__ uint32_t hb32(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }



using cmp::InRing;
using cmp::Window;
using cmp::kObuf;
using cmp::kObufMask;

// Emitter, per parsed window: literal lanes write their byte straight into the literal
// section (placed by mbcnt), staged in the LDS output ring; match lanes append {literal
// length, offset, match length} to a 2 KiB LDS table; a block closes right after its 256th
// match (the window is split at that lane).
struct ZstdOut : cmp::ByteOut {
  uint2* seqs;              // LDS, kMaxSeq records {ll | offset_value << 16, match length}
  uint32_t* ew;             // LDS, 4 x 64: per-chain symbol transforms / state bits
  const uint8_t* tabs;      // LDS, the OF / ML / LL next-state tables at 0 / 64 / 128
  const GMEM uint8_t* src;  // the segment's input (raw blocks are copied from it)
  uint32_t blk;             // output offset of the open block's header
  uint32_t in0;             // input position the open block starts at
  uint32_t nlit, nseq;

  __device__ __forceinline__ void begin_block(uint32_t in_pos) {
    blk = op;
    in0 = in_pos;
    nlit = 0;
    nseq = 0;
    // block header (3) + raw-literals header (3), patched in HBM when the block closes
    if (room(6)) op += 6;
  }

  // literal bytes [s, s + len) of the input, appended to the literal section
  __device__ __forceinline__ void literals(const GMEM uint8_t* in, const InRing& I, uint32_t s,
                                           uint32_t len) {
    if (overflow || !len) return;
    const uint32_t lane = lane_id();
    if (len <= 256 && s >= I.lo) {
      for (uint32_t k = 0; k < len; k += kWave) {
        const uint32_t step = len - k < kWave ? len - k : kWave;
        if (!room(step)) return;
        lds_order();
        const uint32_t b = I.byte(s + k + (lane < step ? lane : 0u));
        put(b, step);
      }
    } else {  // long run (or not in the input ring): drain the ring, then HBM -> HBM
      if ((uint64_t)op + len > cap) {
        overflow = true;
        return;
      }
      flush(op, true);
      wave_copy_global(dst + op, in + s, len);
      op += len;
      flushed = op;
    }
    nlit += len;
  }

  // the literal tail of the segment (and the whole segment when it is too short to parse)
  __device__ __forceinline__ void sequence(const GMEM uint8_t* in, const InRing& I, uint32_t s,
                                           uint32_t len, uint32_t, uint32_t) {
    literals(in, I, s, len);
  }
  // literals are written window by window: the tail starts where output stopped
  __device__ __forceinline__ uint32_t pending_from(uint32_t, uint32_t emitted) const {
    return emitted;
  }

  // the literal lanes `litm` and match lanes `chm` of one window
  __device__ __forceinline__ void part(const Window& W, uint32_t ll, uint64_t litm, uint64_t chm) {
    const uint32_t lane = lane_id();
    const uint32_t nl = (uint32_t)__builtin_popcountll(litm);
    if (nl) {
      if (!room(nl)) return;
      const uint32_t li = __builtin_amdgcn_mbcnt_hi((uint32_t)(litm >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)litm, 0u));
      lds_order();
      ring[(litm >> lane) & 1 ? at(op + li) : kObuf + lane] = (uint8_t)W.byte;
      lds_order();
      op += nl;
      nlit += nl;
    }
    const uint32_t ns = (uint32_t)__builtin_popcountll(chm);
    if (ns) {
      const uint32_t si = __builtin_amdgcn_mbcnt_hi((uint32_t)(chm >> 32),
                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)chm, 0u));
      lds_order();
      if ((chm >> lane) & 1) seqs[nseq + si] = uint2{ll | ((W.off + 3u) << 16), W.mlen};
      lds_order();
      nseq += ns;
    }
  }

  __device__ __forceinline__ void window(const GMEM uint8_t*, const InRing&, const Window& W,
                                         uint32_t anchor, uint32_t n) {
    if (overflow) return;
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
    const uint32_t cnt = (uint32_t)__builtin_popcountll(W.chain);
    if (nseq + cnt < kMaxSeq) {
      part(W, ll, litm, W.chain);
      return;
    }
    // the block's last match is the (kMaxSeq - nseq)-th chain lane: split the window there
    uint64_t m = W.chain;
    for (uint32_t r = kMaxSeq - nseq - 1; r; --r) m &= m - 1;
    const uint32_t ls = (uint32_t)__builtin_ctzll(m);
    const uint64_t lo = ls == 63 ? ~0ull : (2ull << ls) - 1;
    part(W, ll, litm & lo, W.chain & lo);
    const uint32_t end = W.x + ls + readlane(W.mlen, ls);
    close_block(false, end);
    begin_block(end);
    part(W, ll, litm & ~lo, W.chain & ~lo);
  }

  // OR the lanes' bit fields (v, nb), in DESCENDING lane order, into the bitstream that
  // starts at output byte p0; bits = bits written so far; zeroed = first ring byte not yet
  // cleared for the bitstream
  __device__ __forceinline__ void put_bits(uint64_t v, uint32_t nb, uint32_t p0, uint32_t& bits,
                                           uint32_t& zeroed) {
    const uint32_t lane = lane_id();
    const uint32_t incl = wave_incl_sum(nb);
    const uint32_t total = readlane(incl, 63);
    op = p0 + (bits >> 3);
    if (!room((total >> 3) + 16)) return;
    const uint32_t end = p0 + ((bits + total + 7) >> 3);
    lds_order();
    for (uint32_t b = zeroed + lane; b < end; b += kWave) ring[at(b)] = 0;
    if (end > zeroed) zeroed = end;
    const uint32_t pos = bits + total - incl;  // lanes above come first
    const uint32_t a = ((((uint32_t)(uintptr_t)dst + p0) & kObufMask) << 3) + pos;
    const uint32_t wmask = kObufMask >> 2;
    const uint32_t w = (a >> 5) & wmask, sh = a & 31u;
    const uint32_t x0 = (uint32_t)(v << sh);
    const uint32_t x1 = (uint32_t)((v << sh) >> 32);
    const uint32_t x2 = sh ? (uint32_t)(v >> (64 - sh)) : 0u;
    uint32_t* r32 = reinterpret_cast<uint32_t*>(ring);
    lds_order();
    atomicOr(&r32[w], x0);
    atomicOr(&r32[(w + 1) & wmask], x1);
    atomicOr(&r32[(w + 2) & wmask], x2);
    lds_order();
    bits += total;
    op = p0 + (bits >> 3);
  }

  // The sequences bitstream of the open block (nseq >= 1), oracle zs_close_block.  Per 64
  // sequences (highest first): every lane computes its sequence's codes and symbol
  // transforms and stores them chain-major in LDS (ew[4 k + c]: c = 0 OF, 1 ML, 2 LL,
  // deltaNbBits | deltaFindState << 24); then lanes 0..2 walk the three FSE state chains on
  // the vector ALU, one chain per lane, sequence 63 down to 0, each step one LDS read of the
  // transform and one of the chain's state table (tabs), writing the state bits back over
  // the transform; finally every lane assembles its sequence's field (state bits + extra
  // bits, <= 61 bits), placed by a prefix sum.  The walk costs a few scalar instructions per
  // sequence: the scalar unit stays with the parse, which every wave of the CU shares.
  __device__ __forceinline__ void encode_sequences() {
    const uint32_t lane = lane_id();
    const uint32_t p0 = op;
    uint32_t bits = 0, zeroed = p0;
    uint32_t st = 0;  // lane c < 3: the state of chain c
    const uint32_t top = nseq - 1;
    // chain of this lane: its table base in tabs (lanes >= 3 walk a dummy chain whose
    // reads stay inside the tables and whose writes go to ew[4 k + 3])
    const uint32_t cl = lane < 3 ? lane : 3u;
    const uint32_t tb = cl == 0 ? 0u : cl == 1 ? 64u : cl == 2 ? 128u : 192u;
    for (int32_t c = (int32_t)(top >> 6); c >= 0; --c) {
      const uint32_t j = (uint32_t)c * kWave + lane;
      const bool act = j < nseq;
      lds_order();
      const uint2 rec = seqs[act ? j : top];
      const uint32_t ll = rec.x & 0xFFFFu, of = rec.x >> 16, mlb = rec.y - 3u;
      const uint32_t llc = ll < 64 ? kCodes.ll[ll] : hb32(ll) + 19u;
      const uint32_t mlc = mlb < 128 ? kCodes.ml[mlb] : hb32(mlb) + 36u;
      const uint32_t ofc = hb32(of);
      const uint2 eLL = kCtLL.sym[llc], eML = kCtML.sym[mlc], eOF = kCtOF.sym[ofc];
      auto pack = [](uint2 e) { return e.x | (e.y << 24); };  // d < 2^19, f in [-64, 64)
      ew[4 * lane + 0] = pack(eOF);
      ew[4 * lane + 1] = pack(eML);
      ew[4 * lane + 2] = pack(eLL);
      ew[4 * lane + 3] = 0u;
      lds_order();
      int32_t k = 63;
      if (c == (int32_t)(top >> 6)) {  // the last sequence initialises the three states
        k = (int32_t)(top & 63u);
        const uint32_t e = ew[4 * (uint32_t)k + cl];
        const uint32_t d = e & 0xFFFFFFu;
        const int32_t f = (int32_t)e >> 24;
        const uint32_t nbo = (d + (1u << 15)) >> 16;
        const uint32_t val = (nbo << 16) - d;
        st = tabs[(tb + (uint32_t)((int32_t)(val >> nbo) + f)) & 255u];
        lds_order();
        ew[4 * (uint32_t)k + cl] = 0u;  // no state bits
        --k;
      }
      for (; k >= 0; --k) {
        lds_order();
        const uint32_t e = ew[4 * (uint32_t)k + cl];
        const uint32_t nb = (st + (e & 0xFFFFFFu)) >> 16;
        const uint32_t out = st & ((1u << nb) - 1u);
        st = tabs[(tb + (uint32_t)((int32_t)(st >> nb) + ((int32_t)e >> 24))) & 255u];
        ew[4 * (uint32_t)k + cl] = out | (nb << 24);
      }
      lds_order();
      const uint32_t w0 = ew[4 * lane + 0], w1 = ew[4 * lane + 1], w2 = ew[4 * lane + 2];
      const uint32_t nof = w0 >> 24, nml = w1 >> 24, nll = w2 >> 24;
      const uint32_t stb = ((w0 & 0xFFFFFFu) | ((w1 & 0xFFFFFFu) << nof) |
                            ((w2 & 0xFFFFFFu) << (nof + nml))) & 0xFFFFFFu;
      // each lane's field: state bits, then literal-length, match-length and offset extras
      const uint32_t stn = nof + nml + nll;
      const uint32_t llb = eLL.y >> 16, mlbits = eML.y >> 16;
      const uint64_t llx = ll & ((1u << llb) - 1u);
      const uint64_t mlx = mlb & ((1u << mlbits) - 1u);
      const uint64_t ofx = of & ((1u << ofc) - 1u);
      uint64_t v = (uint64_t)stb | (llx << stn) | (mlx << (stn + llb)) |
                   (ofx << (stn + llb + mlbits));
      uint32_t nb = stn + llb + mlbits + ofc;
      if (!act) {
        v = 0;
        nb = 0;
      }
      put_bits(v, nb, p0, bits, zeroed);
      if (overflow) return;
    }
    // final states (ML, OF, LL: the decoder reads LL first) and the end mark
    const uint32_t sOF = readlane(st, 0), sML = readlane(st, 1), sLL = readlane(st, 2);
    const uint32_t fin = (sML & 63u) | ((sOF & 31u) << 6) | ((sLL & 63u) << 11) | (1u << 17);
    put_bits(lane == 0 ? fin : 0u, lane == 0 ? 18u : 0u, p0, bits, zeroed);
    op = p0 + ((bits + 7) >> 3);
  }

  // close the open block; in_end = input position it ends at (oracle zs_close_block)
  __device__ __forceinline__ void close_block(bool last, uint32_t in_end) {
    if (overflow) return;
    const uint32_t lane = lane_id();
    // Number_of_Sequences (1 or 2 bytes) + Symbol_Compression_Modes (0: all predefined)
    const uint32_t nh = nseq == 0 ? 1u : nseq < 128 ? 2u : 3u;
    if (!room(nh)) return;
    const uint32_t b0 = nseq < 128 ? nseq : (nseq >> 8) + 128u;
    const uint32_t b1 = nseq < 128 ? 0u : nseq & 0xFFu;
    lds_order();
    if (lane < nh) ring[at(op + lane)] = (uint8_t)(lane == 0 ? b0 : lane == 1 ? b1 : 0u);
    lds_order();
    op += nh;
    if (nseq) encode_sequences();
    if (overflow) return;
    const uint32_t csz = op - (blk + 3), raw = in_end - in0;
    uint32_t hdr;
    const bool stored = csz >= raw;
    if (stored) {  // did not shrink: the block's input, raw
      if (flushed < blk) flush(blk, true);  // bytes before the block are still staged
      global_fence_wave();                  // earlier stores to this range land first
      wave_copy_global(dst + blk + 3, src + in0, raw);
      op = blk + 3 + raw;
      flushed = op;
      hdr = (last ? 1u : 0u) | (raw << 3);
    } else {
      flush(op, true);
      hdr = (last ? 1u : 0u) | (2u << 1) | (csz << 3);
    }
    global_fence_wave();
    // block header; compressed blocks also get their raw-literals header (20-bit size)
    uint32_t hb = 0;
    if (lane < 3) hb = hdr >> (8 * lane);
    else if (lane == 3) hb = (3u << 2) | ((nlit & 15u) << 4);
    else if (lane == 4) hb = nlit >> 4;
    else if (lane == 5) hb = nlit >> 12;
    if (lane < (stored ? 3u : 6u)) dst[blk + lane] = (uint8_t)hb;
  }
};

}  // namespace zse

__global__ __launch_bounds__(64) void zstd_compress_kernel(
    const uint8_t* __restrict__ input, uint64_t n_total, uint32_t seg,
    uint8_t* __restrict__ slab, uint64_t slot_stride, uint8_t* const* __restrict__ dsts,
    uint32_t* __restrict__ sizes, uint32_t* __restrict__ err) {
  using namespace cmp;
  __shared__ __attribute__((aligned(16))) uint16_t table[1u << kHashLog];
  __shared__ __attribute__((aligned(16))) uint8_t inring[kIn + kInPad];
  __shared__ __attribute__((aligned(16))) uint8_t obuf[kObuf + kWave];  // + trash bytes
  __shared__ __attribute__((aligned(16))) uint2 seqs[zse::kMaxSeq];
  __shared__ __attribute__((aligned(16))) uint32_t ew[4 * kWave];
  __shared__ __attribute__((aligned(16))) uint8_t tabs[256];
  const uint32_t i_seg = blockIdx.x;
  const uint64_t seg_off = (uint64_t)i_seg * seg;
  if (seg_off >= n_total) return;
  const uint32_t n = (uint32_t)((n_total - seg_off) < seg ? (n_total - seg_off) : seg);
  const uint32_t lane = lane_id();
  zse::ZstdOut o;
  o.ring = obuf;
  o.dst = global_ptr(dsts ? dsts[i_seg] : slab + (uint64_t)i_seg * slot_stride);
  o.cap = slot_stride;
  o.op = 0;
  o.flushed = 0;
  o.overflow = false;
  o.seqs = seqs;
  o.ew = ew;
  o.tabs = tabs;
  tabs[lane] = (uint8_t)zse::kCtOF.state[lane & 31u];
  tabs[64 + lane] = (uint8_t)zse::kCtML.state[lane];
  tabs[128 + lane] = (uint8_t)zse::kCtLL.state[lane];
  tabs[192 + lane] = 0;
  o.src = global_ptr(input + seg_off);
  // frame header: magic, Single_Segment with the content size (1 byte below 256, else 2)
  const uint32_t fh = n < 256 ? 6u : 7u;
  const uint32_t fcs = n < 256 ? n : n - 256u;
  const uint32_t hb = lane < 4 ? (0xFD2FB528u >> (8 * lane)) & 0xFFu
                      : lane == 4 ? (n < 256 ? 0x20u : 0x60u)
                      : lane == 5 ? fcs & 0xFFu : fcs >> 8;
  if (lane < fh) obuf[o.at(lane)] = (uint8_t)hb;
  lds_order();
  o.op = fh;
  o.begin_block(0);
  parse(o.src, n, global_ptr(input + n_total), table, inring, kMaxDist, 0xFFFFFFFFu, o);
  o.close_block(true, n);
  o.flush(o.op, true);
  if (lane == 0) {
    sizes[i_seg] = o.overflow ? 0xFFFFFFFFu : o.op;
    if (o.overflow) atomicOr(err, 2u);
  }
}

}  // namespace bitar_hip
