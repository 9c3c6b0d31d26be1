// lz4_chain.hip -- LZ4 frames with LINKED blocks (LZ4 frame format, Block_Independence = 0:
// a block's matches may reach back into the output of the blocks before it, up to 64 KiB),
// the default of liblz4's frame API and of Arrow's LZ4_FRAME codec.  The blocks of one frame
// depend on each other, so one wavefront decodes them in order: the token walk is scalar,
// literal runs and matches move 64 bytes per step through the LDS output ring of
// stream_ring.hip.h (history older than the ring is read back from HBM), and the ring keeps
// running across block boundaries, so a match into the previous block is an ordinary match.
// Acceptance: the block format of bo_lz4_decompress_block (oracle/bitar_oracle.c) applied to
// the concatenated output -- a match offset must be 1..(bytes produced so far), every block
// ends right after a literal run.
#include "stream_ring.hip.h"

namespace bitar_hip {

// blocks: nblocks pairs {offset of the block data in src, size | 1u << 31 when stored}
__global__ __launch_bounds__(64) void lz4_chain_kernel(const uint8_t* __restrict__ src,
                                                       uint32_t csize,
                                                       const uint32_t* __restrict__ blocks,
                                                       uint32_t nblocks, uint8_t* __restrict__ out,
                                                       uint32_t cap, uint32_t* __restrict__ produced,
                                                       uint32_t* __restrict__ err) {
  using namespace sr;
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWin + kRing];
  uint8_t* win = lds;
  uint8_t* ring = lds + kWin;
  State s;
  s.src = global_ptr(src);
  s.csize = csize;
  s.dst = global_ptr(out);
  s.cap = cap;
  s.ip = 0;
  s.op = 0;
  s.flushed = 0;
  s.fenced = 0;
  s.wb = ~0ull;
  s.wlen = 0;
  auto lits = [&](uint32_t n) __attribute__((always_inline)) {
    if (n >= kLongLit) literals_long(s, win, ring, n);
    else if (n) literals_short(s, win, ring, n);
  };
  bool ok = true;
  for (uint32_t b = 0; b < nblocks && ok; ++b) {
    const uint32_t bo = uniform(blocks[2 * b]), bw = uniform(blocks[2 * b + 1]);
    const uint32_t bsz = bw & 0x7FFFFFFFu;
    const uint32_t end = bo + bsz;
    if (end < bo || end > csize) {
      ok = false;
      break;
    }
    s.ip = bo;
    if (bw >> 31) {  // stored block: its bytes are output as they are
      if ((uint64_t)s.op + bsz > cap) {
        ok = false;
        break;
      }
      lits(bsz);
      continue;
    }
    for (;;) {
      if (s.ip >= end) {
        ok = false;
        break;
      }
      const uint32_t token = byte_u(s, win, s.ip++);
      uint32_t ll = token >> 4;
      if (ll == 15 && !read_ext(s, win, ll)) {
        ok = false;
        break;
      }
      if (s.ip > end || ll > end - s.ip || (uint64_t)s.op + ll > cap) {
        ok = false;
        break;
      }
      lits(ll);
      if (s.ip == end) break;  // the block's last sequence: literals only
      if (s.ip + 2 > end) {
        ok = false;
        break;
      }
      const uint32_t off = byte_u(s, win, s.ip) | (byte_u(s, win, s.ip + 1) << 8);
      s.ip += 2;
      uint32_t ml = token & 15u;
      if (ml == 15 && !read_ext(s, win, ml)) {
        ok = false;
        break;
      }
      ml += 4;
      if (s.ip > end || off == 0 || off > s.op || (uint64_t)s.op + ml > cap) {
        ok = false;
        break;
      }
      match_copy(s, ring, off, ml);
    }
  }
  if (ok) flush(s, ring, s.op, true);
  if (lane_id() == 0) {
    produced[0] = ok ? s.op : 0xFFFFFFFFu;
    if (!ok) atomicOr(err, 1u);
  }
}

}  // namespace bitar_hip
