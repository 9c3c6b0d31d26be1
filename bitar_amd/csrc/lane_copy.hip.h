// lane_copy.hip.h -- per-lane (one lane = one segment) global-memory access and LZ77 copy
// helpers of the lane-per-segment decoders (zstd_lanes.hip, inflate_lanes.hip).  Every
// access is unaligned-capable (gfx950 global memory); the 8-byte "wildcopy" forms write
// up to 32 bytes past the copied range, so callers pass room = that much is inside the
// segment's output.  A match reads its history back from the lane's own output
// (same-thread read-after-write: program order, no fence).
#pragma once

#include "wave.hip.h"

namespace bitar_hip {

namespace lanes {

// ---- per-lane global access -------------------------------------------------------------
__device__ __forceinline__ uint64_t ld8(const GMEM uint8_t* p) {
  uint64_t v;
  __builtin_memcpy(&v, p, 8);
  return v;
}
__device__ __forceinline__ void st8(GMEM uint8_t* p, uint64_t v) { __builtin_memcpy(p, &v, 8); }
__device__ __forceinline__ void st16(GMEM uint8_t* p, uint4 v) { __builtin_memcpy(p, &v, 16); }
// little-endian value of the n <= 4 bytes at p (byte loads: never reads past p + n)
__device__ __forceinline__ uint32_t ldn(const GMEM uint8_t* p, uint32_t n) {
  uint32_t v = 0;
  for (uint32_t k = 0; k < n; ++k) v |= (uint32_t)p[k] << (8 * k);
  return v;
}

// n literal bytes s -> d (no overlap).  Wildcopy when both sides have 16 bytes of room.
__device__ __forceinline__ void copy_lits(GMEM uint8_t* d, const GMEM uint8_t* s, uint32_t n,
                                         bool room) {
  if (n <= 16 && room) {  // both loads in flight, then the stores
    const uint64_t a = ld8(s), b = ld8(s + 8);
    st8(d, a);
    if (n > 8) st8(d + 8, b);
    return;
  }
  uint32_t j = 0;
  for (; j + 32 <= n; j += 32) {
    const uint64_t a = ld8(s + j), b = ld8(s + j + 8), c = ld8(s + j + 16), e = ld8(s + j + 24);
    st8(d + j, a);
    st8(d + j + 8, b);
    st8(d + j + 16, c);
    st8(d + j + 24, e);
  }
  for (; j + 8 <= n; j += 8) st8(d + j, ld8(s + j));
  for (; j < n; ++j) d[j] = s[j];
}

// n bytes of a match at distance off (1 <= off <= d - segment start): d[j] = d[j - off]
__device__ __forceinline__ void copy_match(GMEM uint8_t* d, uint32_t off, uint32_t n,
                                           bool room) {
  const GMEM uint8_t* s = d - off;
  if (room) {  // d + n + 32 <= end of the segment
    if (off >= 16 && n <= 16) {  // the common short match: two loads, then two stores
      const uint64_t a = ld8(s), b = ld8(s + 8);
      st8(d, a);
      st8(d + 8, b);
    } else if (off >= 32) {  // 32-byte steps: four loads in flight, then four stores
      for (uint32_t j = 0; j < n; j += 32) {
        const uint64_t a = ld8(s + j), b = ld8(s + j + 8), c = ld8(s + j + 16),
                       e = ld8(s + j + 24);
        st8(d + j, a);
        st8(d + j + 8, b);
        st8(d + j + 16, c);
        st8(d + j + 24, e);
      }
    } else if (off >= 16) {  // 16-byte steps
      for (uint32_t j = 0; j < n; j += 16) {
        const uint64_t a = ld8(s + j), b = ld8(s + j + 8);
        st8(d + j, a);
        st8(d + j + 8, b);
      }
    } else if (off >= 8) {
      for (uint32_t j = 0; j < n; j += 8) st8(d + j, ld8(s + j));
    } else {
      // the first `off` bytes repeat: build an 8-byte word of the pattern, store it every
      // `step` bytes (the largest multiple of off <= 8)
      uint64_t rep = ld8(s) & (~0ull >> (64 - 8 * off));
      for (uint32_t len = off; len < 8; len *= 2) rep |= rep << (8 * len);
      const uint32_t step = 8 - (8 % off);
      for (uint32_t j = 0; j < n; j += step) st8(d + j, rep);
    }
    return;
  }
  for (uint32_t j = 0; j < n; ++j) d[j] = s[j];
}

}  // namespace lanes

}  // namespace bitar_hip
