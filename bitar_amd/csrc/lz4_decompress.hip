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



__global__ __launch_bounds__(64) void lz4_decompress_kernel(
    const uint8_t* const* __restrict__ srcs, const uint8_t* __restrict__ slab,
    uint64_t slot_stride, const uint32_t* __restrict__ csizes, uint32_t nseg, uint32_t seg,
    uint8_t* __restrict__ out, uint32_t* __restrict__ produced, uint32_t* __restrict__ err) {
  using namespace sr;
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
  while (ok) {
    if (s.ip >= s.csize) { ok = false; break; }
    const uint32_t token = byte_u(s, win, s.ip);
    s.ip += 1;
    uint32_t lit = token >> 4;
    if (lit == 15 && !read_ext(s, win, lit)) { ok = false; break; }
    if ((uint64_t)s.ip + lit > s.csize || (uint64_t)s.op + lit > s.cap) { ok = false; break; }
    if (lit >= kLongLit) literals_long(s, win, ring, lit);
    else if (lit) literals_short(s, win, ring, lit);
    if (s.ip == s.csize) break;  // last sequence: literals only
    if (s.ip + 2 > s.csize) { ok = false; break; }
    const uint32_t o0 = byte_u(s, win, s.ip);
    const uint32_t o1 = byte_u(s, win, s.ip + 1);
    s.ip += 2;
    const uint32_t off = o0 | (o1 << 8);
    if (off == 0 || off > s.op) { ok = false; break; }
    uint32_t m = token & 15u;
    if (m == 15 && !read_ext(s, win, m)) { ok = false; break; }
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
