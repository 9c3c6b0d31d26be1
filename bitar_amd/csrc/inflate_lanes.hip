// inflate_lanes.hip -- raw DEFLATE (RFC 1951) decode with ONE LANE PER SEGMENT (gfx950).
//
// The symbol chain of a Huffman-coded DEFLATE block is serial: every code's position in
// the bitstream depends on the lengths of all codes before it.  The wave-per-segment
// inflate_kernel (inflate.hip) attacks that with speculative decoding of 256 candidate bit
// offsets per step (~45 VALU + ~34 SALU per symbol).  Here each lane owns one segment and
// walks its own symbol chain on the vector ALU -- L chains per vector instruction -- with
// the fixed literal/length and distance codes (RFC 1951 3.2.6) as compile-time tables in
// LDS shared by the lanes.
//
// Scope: stored and fixed-Huffman blocks (every stream deflate_compress_kernel writes, and
// zlib's level-0 / Z_FIXED streams).  A segment with a dynamic-Huffman block or one that
// fails ANY of the wave kernel's checks is marked kDefer (produced[i]) and left to
// inflate_kernel, which the runtime launches next in defer-only mode; acceptance and error
// reporting are therefore exactly the wave kernel's (= the oracle's bo_inflate_raw).
//
// Memory: the bit buffer is refilled with 8-byte (unaligned) loads of the lane's stream;
// literals are single-byte stores, matches use the copy helpers of lane_copy.hip.h.
// Stored blocks are copied by the whole wave, one lane's block at a time (coalesced).
// Bytes of a segment's output slot past its produced size are unspecified (match
// wildcopies may write up to 32 bytes past the current output position, inside the slot).
#include "lane_copy.hip.h"

namespace bitar_hip {

namespace infl_lanes {

using namespace lanes;

constexpr uint32_t kDefer = 0xFFFFFFFEu;

constexpr uint16_t kLenBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                   31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
constexpr uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                   2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
constexpr uint16_t kDistBase[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                    33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                    1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
constexpr uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2,  3,  3,  4,  4,  5,  5,  6,
                                    6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

constexpr uint32_t rev(uint32_t v, uint32_t n) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < n; ++i) r |= ((v >> i) & 1u) << (n - 1 - i);
  return r;
}

// Fixed-code tables, indexed by the next 9 (literal/length) or 5 (distance) stream bits,
// LSB first.  Literal/length entry: kind (0 literal, 1 length, 2 end of block, 3 invalid
// symbol 286/287) << 30 | code length << 24 | extra-bit count << 16 | literal byte or length
// base.  Distance entry: valid << 31 | extra-bit count << 16 | base (codes 30, 31 invalid).
struct Fixed {
  uint32_t lit[512];
  uint32_t dist[32];
};
constexpr Fixed build_fixed() {
  Fixed f{};
  for (uint32_t s = 0; s < 288; ++s) {
    const uint32_t n = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
    const uint32_t code = s < 144 ? 0x30 + s : s < 256 ? 0x190 + (s - 144) : s < 280 ? s - 256
                                                                                     : 0xC0 + (s - 280);
    uint32_t e = 0;
    if (s < 256) e = (0u << 30) | s;
    else if (s == 256) e = 2u << 30;
    else if (s < 286) e = (1u << 30) | ((uint32_t)kLenExtra[s - 257] << 16) | kLenBase[s - 257];
    else e = 3u << 30;
    e |= n << 24;
    const uint32_t r = rev(code, n);
    for (uint32_t hi = 0; hi < (1u << (9 - n)); ++hi) f.lit[r | (hi << n)] = e;
  }
  for (uint32_t d = 0; d < 32; ++d) {
    const uint32_t r = rev(d, 5);
    f.dist[r] = d < 30 ? (1u << 31) | ((uint32_t)kDistExtra[d] << 16) | kDistBase[d] : 0u;
  }
  return f;
}
__constant__ Fixed kFixed = build_fixed();

// LSB-first bit buffer over the lane's stream [0, cs): bytes past cs read as zeros; the
// consumed bit count (8 ip - left) is checked against 8 cs once, at the end.
struct Bits {
  uint64_t buf;
  uint32_t left;  // valid bits in buf
  uint32_t ip;    // next stream byte to load
  __device__ __forceinline__ void refill(const GMEM uint8_t* src, uint32_t cs) {
    // top up to >= 56 bits: load the 8 bytes at ip (zeros past the stream's end)
    uint64_t v;
    if (ip + 8 <= cs) {
      v = ld8(src + ip);
    } else if (ip >= cs) {
      v = 0;
    } else if (cs >= 8) {  // the last cs - ip bytes, from an in-bounds 8-byte load
      v = ld8(src + cs - 8) >> (8 * (ip + 8 - cs));
    } else {
      v = 0;
      for (uint32_t k = ip; k < cs; ++k) v |= (uint64_t)src[k] << (8 * (k - ip));
    }
    buf |= v << left;
    const uint32_t nb = (63 - left) >> 3;
    ip += nb;
    left += 8 * nb;
  }
  __device__ __forceinline__ uint32_t peek(uint32_t n) const {
    return (uint32_t)buf & ((1u << n) - 1u);
  }
  __device__ __forceinline__ void skip(uint32_t n) {
    buf >>= n;
    left -= n;
  }
  __device__ __forceinline__ uint64_t used() const { return 8ull * ip - left; }
};

}  // namespace infl_lanes

template <uint32_t L>
__global__ __launch_bounds__(64) void inflate_lanes_kernel(
    const uint8_t* const* __restrict__ srcs, const uint8_t* __restrict__ slab,
    uint64_t slot_stride, const uint32_t* __restrict__ csizes, uint32_t nseg, uint32_t seg,
    uint8_t* __restrict__ out, uint32_t* __restrict__ produced) {
  using namespace infl_lanes;
  __shared__ uint32_t tlit[512];
  __shared__ uint32_t tdist[32];
  const uint32_t lane = lane_id();
#pragma unroll
  for (uint32_t k = 0; k < 512; k += kWave) tlit[k + lane] = kFixed.lit[k + lane];
  if (lane < 32) tdist[lane] = kFixed.dist[lane];
  lds_order();
  const uint32_t i = blockIdx.x * L + lane;
  bool active = lane < L && i < nseg;
  const GMEM uint8_t* src = nullptr;
  GMEM uint8_t* dst = nullptr;
  uint32_t cs = 0, op = 0;
  const uint32_t cap = seg;
  Bits b = {0ull, 0u, 0u};
  if (active) {
    src = global_ptr(srcs ? srcs[i] : slab + (uint64_t)i * slot_stride);
    cs = csizes[i];
    dst = global_ptr(out + (uint64_t)i * seg);
  }
  // block loop: all lanes meet at every block header, where stored blocks are copied by the
  // whole wave
  while (ballot(active)) {
    uint32_t type = 3, last = 0, sp = 0, slen = 0;
    if (active) {
      b.refill(src, cs);
      const uint32_t hdr = b.peek(3);
      b.skip(3);
      last = hdr & 1u;
      type = hdr >> 1;
      if (type == 0) {
        // stored: align to a byte, LEN / NLEN, LEN raw bytes (oracle bo_inflate_raw)
        const uint32_t pos = (uint32_t)((b.used() + 7) >> 3);
        bool ok = pos + 4 <= cs;
        if (ok) {
          const uint32_t ln = ldn(src + pos, 4);
          slen = ln & 0xFFFFu;
          ok = slen == (~(ln >> 16) & 0xFFFFu) && pos + 4 + slen <= cs && op + slen <= cap;
          sp = pos + 4;
        }
        if (!ok) {
          active = false;
          produced[i] = kDefer;
          type = 3;
        }
      } else if (type != 1) {  // dynamic Huffman (the wave kernel) or reserved
        active = false;
        produced[i] = kDefer;
      }
    }
    for (uint64_t m = ballot(active && type == 0); m; m &= m - 1) {
      const uint32_t l = (uint32_t)__builtin_ctzll(m);
      const uint64_t d = uniform64(readlane((uint32_t)(uintptr_t)dst, l) |
                                   ((uint64_t)readlane((uint32_t)((uintptr_t)dst >> 32), l) << 32));
      const uint64_t s = uniform64(readlane((uint32_t)(uintptr_t)src, l) |
                                   ((uint64_t)readlane((uint32_t)((uintptr_t)src >> 32), l) << 32));
      wave_copy_global((GMEM uint8_t*)(uintptr_t)d + readlane(op, l),
                       (const GMEM uint8_t*)(uintptr_t)s + readlane(sp, l), readlane(slen, l));
      global_fence_wave();  // lane l reads this output back as match history
    }
    if (active && type == 0) {
      op += slen;
      b = {0ull, 0u, sp + slen};  // the bit reader restarts after the stored bytes
    }
    if (active && type == 1) {
      // fixed-Huffman symbols until end of block
      bool eob = false;
      while (!eob) {
        b.refill(src, cs);  // >= 56 bits: one code (<= 9) + length extra (<= 5) + distance
                            // code (5) + its extra (<= 13)
        const uint32_t e = tlit[b.peek(9)];
        b.skip((e >> 24) & 15u);
        const uint32_t kind = e >> 30;
        if (kind == 0) {
          if (op >= cap) break;
          dst[op++] = (uint8_t)e;
          // up to five more literals on the same refill (>= 56 bits after it, each literal
          // takes <= 9); anything else is decoded at the loop head
#pragma unroll
          for (uint32_t r = 0; r < 5; ++r) {
            const uint32_t e2 = tlit[b.peek(9)];
            if ((e2 >> 30) != 0 || op >= cap) break;
            b.skip((e2 >> 24) & 15u);
            dst[op++] = (uint8_t)e2;
          }
          continue;
        }
        if (kind != 1) {  // end of block, or an invalid symbol (286 / 287)
          eob = kind == 2;
          break;
        }
        const uint32_t len = (e & 0xFFFFu) + b.peek((e >> 16) & 7u);
        b.skip((e >> 16) & 7u);
        const uint32_t de = tdist[b.peek(5)];
        b.skip(5);
        if (!(de >> 31)) break;  // distance code 30 / 31
        const uint32_t dx = (de >> 16) & 15u;
        const uint32_t dist = (de & 0xFFFFu) + b.peek(dx);
        b.skip(dx);
        if (dist > op || op + len > cap) break;
        copy_match(dst + op, dist, len, op + len + 32 <= cap);
        op += len;
        // the match took <= 32 of the >= 56 bits: up to two literals more before the refill
#pragma unroll
        for (uint32_t r = 0; r < 2; ++r) {
          const uint32_t e2 = tlit[b.peek(9)];
          if ((e2 >> 30) != 0 || op >= cap) break;
          b.skip((e2 >> 24) & 15u);
          dst[op++] = (uint8_t)e2;
        }
      }
      if (!eob) {
        active = false;
        produced[i] = kDefer;
      }
    }
    if (active && last) {
      active = false;
      produced[i] = b.used() <= 8ull * cs ? op : kDefer;
    }
  }
}

template __global__ void inflate_lanes_kernel<4>(const uint8_t* const*, const uint8_t*, uint64_t,
                                                 const uint32_t*, uint32_t, uint32_t, uint8_t*,
                                                 uint32_t*);
template __global__ void inflate_lanes_kernel<8>(const uint8_t* const*, const uint8_t*, uint64_t,
                                                 const uint32_t*, uint32_t, uint32_t, uint8_t*,
                                                 uint32_t*);
template __global__ void inflate_lanes_kernel<16>(const uint8_t* const*, const uint8_t*, uint64_t,
                                                  const uint32_t*, uint32_t, uint32_t, uint8_t*,
                                                  uint32_t*);
template __global__ void inflate_lanes_kernel<32>(const uint8_t* const*, const uint8_t*, uint64_t,
                                                  const uint32_t*, uint32_t, uint32_t, uint8_t*,
                                                  uint32_t*);

}  // namespace bitar_hip
