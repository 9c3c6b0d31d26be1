// stream_ring.hip.h -- per-wave stream window + output history ring shared by the decoders
// (LZ4 block decode and raw-DEFLATE inflate).  One wavefront per segment, LDS private to it.
//
//   win[kWin]   the compressed stream, staged from HBM 16 B per lane (dwordx4), refilled
//               when the parse leaves it.
//   ring[kRing] the last kRing output bytes, indexed by ABSOLUTE output address & mask so a
//               16-B-aligned ring block is a 16-B-aligned HBM block.  Matches read their
//               history from the ring (LDS latency, no HBM round trip); completed 16-B
//               blocks are flushed to HBM with dwordx4 stores, 1 KiB per wave instruction.
//   Matches reaching further back than the ring read HBM behind a lazily placed fence;
//   long literal runs bypass the ring and stream HBM -> HBM (wave_copy_global).
#pragma once
#include "wave.hip.h"
#include "../../include/bitar_hip.h"  // BITAR_HIP_PATH_* counter indices

namespace bitar_hip {

namespace sr {

#ifndef BITAR_DEC_RING
#define BITAR_DEC_RING 4096
#endif
#ifndef BITAR_DEC_WIN
#define BITAR_DEC_WIN 1024
#endif
constexpr uint32_t kRing = BITAR_DEC_RING;
constexpr uint32_t kRingMask = kRing - 1;
constexpr uint32_t kWin = BITAR_DEC_WIN;  // dwordx4 per lane per refill step
constexpr uint32_t kLongLit = 1024;    // literal runs at least this long go HBM -> HBM
constexpr uint32_t kFlushAt = kRing / 2;
constexpr uint32_t kNearOff = kRing - 2 * kWave - 16;  // ring holds the source

struct State {
  const GMEM uint8_t* src;  // compressed segment
  uint32_t csize;
  GMEM uint8_t* dst;        // output segment base
  uint32_t cap;
  uint32_t ip;         // stream position
  uint32_t op;         // output position
  uint32_t flushed;    // out[0, flushed) written to HBM
  uint32_t fenced;     // out[0, fenced) visible to this wave's loads
  uint64_t wb;         // absolute address of win[0] (16-aligned)
  uint32_t wlen;       // bytes of the stream covered by win: [wb, wb + wlen) ∩ segment
  uint32_t nbatch;     // batches run (inflate_kernel's path counter)
};

// Stage the stream bytes starting at absolute address `abs` (rounded down to 16 B) into
// win.  Blocks that hold no byte of the segment are skipped (never read: every read is
// bounds-checked against csize first).
__device__ __forceinline__ void refill_abs(State& s, uint8_t* win, uint64_t abs) {
  const uint64_t a = abs & ~(uint64_t)15;
  const uint64_t lo = (uint64_t)(uintptr_t)s.src, hi = lo + s.csize;
  const uint32_t lane = lane_id();
#pragma unroll
  for (uint32_t j = 0; j < kWin / (16 * kWave); ++j) {
    const uint64_t blk = a + 16ull * (lane + j * kWave);
    if (blk < hi && blk + 16 > lo) {
      const uint4 v = *reinterpret_cast<const GMEM uint4*>(s.src + (int64_t)(blk - lo));
      *reinterpret_cast<uint4*>(win + 16 * (lane + j * kWave)) = v;
    }
  }
  lds_order();
  s.wb = a;
}

__device__ __forceinline__ void refill(State& s, uint8_t* win, uint32_t pos) {
  refill_abs(s, win, (uint64_t)(uintptr_t)(s.src + pos));
}

// window index of absolute address abs, refilling so that [abs, abs+need) is staged
// (need <= kWin - 15)
__device__ __forceinline__ uint32_t win_at_abs(State& s, uint8_t* win, uint64_t abs, uint32_t need) {
  if (abs < s.wb || abs + need > s.wb + kWin) refill_abs(s, win, abs);
  return (uint32_t)(abs - s.wb);
}

// window-relative index of stream position pos, refilling so that [pos, pos+need) is staged
__device__ __forceinline__ uint32_t win_at(State& s, uint8_t* win, uint32_t pos, uint32_t need) {
  return win_at_abs(s, win, (uint64_t)(uintptr_t)(s.src + pos), need);
}

__device__ __forceinline__ uint32_t byte_u(State& s, uint8_t* win, uint32_t pos) {
  const uint32_t w = win_at(s, win, pos, 1);
  lds_order();
  return uniform((uint32_t)win[w]);
}

// LZ4 length extension: bytes of 255 continue the run.  64 bytes examined per step with a
// ballot.  Returns false if the run leaves the segment.
__device__ __forceinline__ bool read_ext(State& s, uint8_t* win, uint32_t& len) {
  const uint32_t lane = lane_id();
  for (;;) {
    if (s.ip >= s.csize) return false;
    uint32_t avail = s.csize - s.ip;
    if (avail > kWave) avail = kWave;
    const uint32_t w = win_at(s, win, s.ip, avail);
    lds_order();
    const uint32_t b = lane < avail ? (uint32_t)win[w + lane] : 0u;
    const uint64_t stop = ballot(lane < avail && b != 255u);
    if (stop == 0) {
      len += 255u * avail;
      s.ip += avail;
      continue;
    }
    const uint32_t k = (uint32_t)__builtin_ctzll(stop);
    len += 255u * k + readlane(b, k);
    s.ip += k + 1;
    return true;
  }
}

// Write out[flushed, upto) from the ring to HBM.  Whole 16-B blocks only unless `final`.
__device__ __forceinline__ void flush(State& s, const uint8_t* ring, uint32_t upto, bool final) {
  const uint32_t lane = lane_id();
  const uintptr_t base = (uintptr_t)s.dst;
  uint32_t f = s.flushed;
  lds_order();
  uint32_t head = (uint32_t)((16u - ((base + f) & 15u)) & 15u);
  if (head > upto - f) head = upto - f;
  if (head) {
    if (lane < head) s.dst[f + lane] = ring[(base + f + lane) & kRingMask];
    f += head;
  }
  const uint32_t nb = (upto - f) >> 4;
  for (uint32_t b = lane; b < nb; b += kWave) {
    const uint32_t k = f + 16u * b;
    const uint4 v = *reinterpret_cast<const uint4*>(ring + ((base + k) & kRingMask));
    *reinterpret_cast<GMEM uint4*>(s.dst + k) = v;
  }
  f += nb << 4;
  if (final && f < upto) {
    if (lane < upto - f) s.dst[f + lane] = ring[(base + f + lane) & kRingMask];
    f = upto;
  }
  s.flushed = f;
}

__device__ __forceinline__ void make_room(State& s, const uint8_t* ring, uint32_t n) {
  if (s.op + n - s.flushed > kFlushAt) flush(s, ring, s.op, false);
}

// out[op, op+n) <- stream[ip, ip+n) through the window into the ring
__device__ __forceinline__ void literals_short(State& s, uint8_t* win, uint8_t* ring,
                                               uint32_t n) {
  const uint32_t lane = lane_id();
  const uintptr_t base = (uintptr_t)s.dst;
  while (n) {
    const uint32_t step = n < kWave ? n : kWave;
    make_room(s, ring, step);
    const uint32_t w = win_at(s, win, s.ip, step);
    lds_order();
    if (lane < step) ring[(base + s.op + lane) & kRingMask] = win[w + lane];
    lds_order();
    s.ip += step;
    s.op += step;
    n -= step;
  }
}

__device__ __forceinline__ void literals_long(State& s, uint8_t* win, uint8_t* ring,
                                              uint32_t n) {
  const uint32_t lane = lane_id();
  const uintptr_t base = (uintptr_t)s.dst;
  flush(s, ring, s.op, true);
  wave_copy_global(s.dst + s.op, s.src + s.ip, n);
  const bool more = s.ip + n < s.csize;
  if (more) {
    // Seed the ring with the run's last kRing bytes so the ring stays hole-free: every
    // match with off <= kNearOff then finds its history in LDS.
    uint32_t keep = n < kRing ? n : kRing;
    uint32_t k = n - keep;
    while (k < n) {
      uint32_t step = n - k;
      if (step > kWin - 16) step = kWin - 16;
      const uint32_t w = win_at(s, win, s.ip + k, step);
      lds_order();
      for (uint32_t t = lane; t < step; t += kWave)
        ring[(base + s.op + k + t) & kRingMask] = win[w + t];
      lds_order();
      k += step;
    }
  }
  s.ip += n;
  s.op += n;
  s.flushed = s.op;  // written straight to HBM (not yet fenced)
}

// out[op, op+m) <- out[op-off, ...) with LZ4 overlap semantics: byte t copies
// out[op - off + (t mod off)], which is always already final.
__device__ __forceinline__ void match_copy(State& s, uint8_t* ring, uint32_t off, uint32_t m) {
  const uint32_t lane = lane_id();
  const uintptr_t base = (uintptr_t)s.dst;
  const bool near = off <= kNearOff;
  while (m) {
    const uint32_t step = m < kWave ? m : kWave;
    make_room(s, ring, step);
    uint32_t rel = lane;
    if (off < step) {  // lane mod off, exact for lane, off < 64
      const float q = floorf(((float)lane + 0.5f) * __builtin_amdgcn_rcpf((float)off));
      rel = lane - (uint32_t)q * off;
    }
    const uint32_t from = s.op - off + rel;
    uint32_t v = 0;
    if (near) {
      lds_order();
      if (lane < step) v = ring[(base + from) & kRingMask];
    } else {
      if (s.op - off + step > s.fenced) {  // history only in HBM: make our stores visible
        global_fence_wave();
        s.fenced = s.flushed;
      }
      if (lane < step) v = s.dst[from];
    }
    lds_order();
    if (lane < step) ring[(base + s.op + lane) & kRingMask] = (uint8_t)v;
    lds_order();
    s.op += step;
    m -= step;
  }
}

}  // namespace sr

}  // namespace bitar_hip
