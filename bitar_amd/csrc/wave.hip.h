// wave.hip.h -- wavefront-level primitives shared by the codec kernels (gfx950, wave64).
//
// Every kernel in this engine gives ONE 64-lane wavefront to ONE segment.  Control flow is
// wave-uniform (scalars come from readfirstlane), byte work is spread over the 64 lanes,
// and LDS is private to the wave (one wave per workgroup), so intra-wave LDS traffic needs
// no barrier: a wave's DS instructions execute in issue order.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bitar_hip {

constexpr int kWave = 64;

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

template <typename T>
__device__ __forceinline__ T uniform(T v) {
  return (T)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ uint32_t readlane(uint32_t v, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
// Compiler barrier: keeps LDS accesses in program order (the hardware already executes a
// wave's DS instructions in order).
__device__ __forceinline__ void lds_order() { __asm__ volatile("" ::: "memory"); }

// Global stores of this wave visible to its own later global loads (workgroup scope ==
// this wave, one wave per workgroup).
__device__ __forceinline__ void global_fence_wave() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ uint32_t shfl_down1(uint32_t v) {
  // ds_bpermute: lane l reads lane l+1 (lane 63 reads itself; callers patch it)
  const int src = (int)((lane_id() + 1) & 63) << 2;
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)v);
}

// byte-shift funnel: bytes [r, r+4) of the little-endian pair (lo, hi)
__device__ __forceinline__ uint32_t funnel(uint32_t lo, uint32_t hi, uint32_t r) {
  return __builtin_amdgcn_alignbyte(hi, lo, r);
}

// Copy `len` bytes from global `s` to global `d` (no overlap), all 64 lanes cooperating,
// 16 B per lane per step with aligned dwordx4 loads + stores.  Source blocks that contain
// no byte of [s, s+len) are never loaded.  len, s, d wave-uniform.
__device__ __forceinline__ void wave_copy_global(uint8_t* d, const uint8_t* s, uint64_t len) {
  const uint32_t lane = lane_id();
  uint32_t head = (uint32_t)((16u - ((uintptr_t)d & 15u)) & 15u);
  if (head > len) head = (uint32_t)len;
  if (lane < head) d[lane] = s[lane];
  d += head;
  s += head;
  len -= head;
  const uint64_t nb = len >> 4;
  const uint32_t sh = (uint32_t)((uintptr_t)s & 15u);
  const uint4* sa = reinterpret_cast<const uint4*>((uintptr_t)s & ~(uintptr_t)15);
  uint4* da = reinterpret_cast<uint4*>(d);
  if (sh == 0) {
    for (uint64_t b = lane; b < nb; b += kWave) da[b] = sa[b];
  } else {
    const uint32_t q = sh >> 2, r = sh & 3u;
    for (uint64_t base = 0; base < nb; base += kWave) {
      const uint64_t b = base + lane;
      const bool act = b < nb;
      uint4 x = act ? sa[b] : make_uint4(0, 0, 0, 0);
      uint4 y;
      y.x = shfl_down1(x.x);
      y.y = shfl_down1(x.y);
      y.z = shfl_down1(x.z);
      y.w = shfl_down1(x.w);
      if (act && (lane == kWave - 1 || b + 1 == nb)) y = sa[b + 1];  // holds s+16b+15
      const uint32_t w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
      uint4 o;
      // q is wave-uniform: the switch is a scalar branch
      switch (q) {
        case 0: o = make_uint4(funnel(w[0], w[1], r), funnel(w[1], w[2], r), funnel(w[2], w[3], r), funnel(w[3], w[4], r)); break;
        case 1: o = make_uint4(funnel(w[1], w[2], r), funnel(w[2], w[3], r), funnel(w[3], w[4], r), funnel(w[4], w[5], r)); break;
        case 2: o = make_uint4(funnel(w[2], w[3], r), funnel(w[3], w[4], r), funnel(w[4], w[5], r), funnel(w[5], w[6], r)); break;
        default: o = make_uint4(funnel(w[3], w[4], r), funnel(w[4], w[5], r), funnel(w[5], w[6], r), funnel(w[6], w[7], r)); break;
      }
      if (act) da[b] = o;
    }
  }
  const uint64_t done = nb << 4;
  const uint32_t tail = (uint32_t)(len - done);
  if (lane < tail) d[done + lane] = s[done + lane];
}

}  // namespace bitar_hip
