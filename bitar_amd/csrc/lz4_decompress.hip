// lz4_decompress.hip -- LZ4 block decode, one wavefront per segment (gfx950).
//
// Replaces the inflate op the reference hands to the BlueField engine per segment
// (reference src/memory.cc:432-505 assembles one op per compressed buffer; output slice
// i*seg of the caller's buffer).  Acceptance rules are exactly those of the oracle's
// bo_lz4_decompress_block (oracle/bitar_oracle.c), so malformed input fails identically.
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

namespace bitar_hip {



namespace lz4d {

using namespace sr;

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

}  // namespace lz4d

__global__ __launch_bounds__(64) void lz4_decompress_kernel(
    const uint8_t* const* __restrict__ srcs, const uint8_t* __restrict__ slab,
    uint64_t slot_stride, const uint32_t* __restrict__ csizes, uint32_t nseg, uint32_t seg,
    uint8_t* __restrict__ out, uint32_t* __restrict__ produced, uint32_t* __restrict__ err) {
  using namespace lz4d;
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWin + kRing];
  uint8_t* win = lds;
  uint8_t* ring = lds + kWin;
  const uint32_t i = blockIdx.x;
  if (i >= nseg) return;

  State s;
  s.src = srcs ? srcs[i] : slab + (uint64_t)i * slot_stride;
  s.csize = csizes[i];
  s.dst = out + (uint64_t)i * seg;
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
  while (ok) {
    // ---- fast path: short sequence fully inside the register vector and the window -----
    // token, no length extensions, not the last sequence, near match, room in the ring.
    // Every output byte of the sequence is gathered with ONE ds_read (literal bytes from the
    // window, match bytes from the ring -- a match byte whose source lies in this sequence's
    // own literals is read from the window too) and stored with ONE ds_write.
    if (s.ip + 20 <= s.csize && s.op + 64 - s.flushed <= kFlushAt) {
      if (!sv.covers(s.ip, 20)) sv.load(s, win, s.ip);
      const int64_t wrel = (int64_t)((uintptr_t)(s.src + s.ip) - s.wb);  // ip inside win
      const uint32_t token = sv.byte(s.ip);
      const uint32_t L = token >> 4, m4 = token & 15u;
      if (L < 15 && m4 < 15 && wrel >= 0 && wrel + 20 <= (int64_t)kWin) {
        const uint32_t off = sv.u16(s.ip + 1 + L);
        const uint32_t M = m4 + 4;
        const uint32_t opl = s.op + L;
        if (off != 0 && off <= opl && off <= kNearOff && opl + M <= s.cap) {
          const uint32_t t = lane;
          const uint32_t lit0 = (uint32_t)wrel + 1;  // window index of the first literal
          uint32_t addr;
          if (t < L) {
            addr = lit0 + t;
          } else {
            const uint32_t r = t - L;
            uint32_t rel = r;
            if (off <= r) {  // overlap: r mod off (exact for r, off < 64)
              const float q = floorf(((float)r + 0.5f) * __builtin_amdgcn_rcpf((float)off));
              rel = r - (uint32_t)q * off;
            }
            const uint32_t src = opl - off + rel;  // < opl
            addr = src >= s.op ? lit0 + (src - s.op) : kWin + ((base + src) & kRingMask);
          }
          lds_order();
          const uint32_t b = t < L + M ? (uint32_t)lds[addr] : 0u;
          if (t < L + M) ring[(base + s.op + t) & kRingMask] = (uint8_t)b;
          lds_order();
          s.ip += 3 + L;
          s.op = opl + M;
          continue;
        }
      }
    }
    // ---- general path: one sequence, any shape -----------------------------------------
    if (s.ip >= s.csize) { ok = false; break; }
    const uint32_t token = sv.get(s, win, s.ip);
    s.ip += 1;
    uint32_t lit = token >> 4;
    if (lit == 15 && !ext_len(s, win, sv, lit)) { ok = false; break; }
    if ((uint64_t)s.ip + lit > s.csize || (uint64_t)s.op + lit > s.cap) { ok = false; break; }
    if (lit >= kLongLit) literals_long(s, win, ring, lit);
    else if (lit) literals_short(s, win, ring, lit);
    if (s.ip == s.csize) break;  // last sequence: literals only
    if (s.ip + 2 > s.csize) { ok = false; break; }
    const uint32_t o0 = sv.get(s, win, s.ip);
    const uint32_t o1 = sv.get(s, win, s.ip + 1);
    s.ip += 2;
    const uint32_t off = o0 | (o1 << 8);
    if (off == 0 || off > s.op) { ok = false; break; }
    uint32_t m = token & 15u;
    if (m == 15 && !ext_len(s, win, sv, m)) { ok = false; break; }
    m += 4;
    if ((uint64_t)s.op + m > s.cap) { ok = false; break; }
    match_copy(s, ring, off, m);
  }
  if (ok) {
    flush(s, ring, s.op, true);
    if (lane_id() == 0) produced[i] = s.op;
  } else if (lane_id() == 0) {
    produced[i] = 0xFFFFFFFFu;
    atomicOr(err, 1u);
  }
}

}  // namespace bitar_hip
