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
// (ballot of a single compare is one v_cmp into an SGPR pair; ballot of a compound
// condition costs a v_cndmask + v_cmp more -- AND single-compare ballots instead)
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ uint32_t readlane(uint32_t v, uint32_t l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}
// v with lane l replaced by the (wave-uniform) x
__device__ __forceinline__ uint32_t writelane(uint32_t v, uint32_t x, uint32_t l) {
  uint32_t r;
  // two SGPR operands break the constant-bus limit: the lane select goes through m0
  __asm__("v_writelane_b32 %0, %1, m0" : "=v"(r) : "s"(x), "{m0}"(l), "0"(v));
  return r;
}
// Pointers into global memory (HBM) are typed GMEM (address space 1).  A generic pointer
// (loaded from a slot table, or rebuilt from an integer) makes the compiler emit FLAT
// accesses: those count against both vmcnt and lgkmcnt, and every later LDS access must
// wait for outstanding FLAT stores (they may alias LDS).  GMEM pointers give global_load /
// global_store.  A cast back to a generic pointer loses the address space, so kernel
// state keeps GMEM-typed pointers.
// (The host compilation pass parses device code too; there the qualifier is dropped.)
#ifdef __HIP_DEVICE_COMPILE__
#define GMEM __attribute__((address_space(1)))
#else
#define GMEM
#endif
template <typename T>
__device__ __forceinline__ GMEM T* global_ptr(T* p) {
  return (GMEM T*)p;
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

// byte-shift funnel: bytes [r, r+4) of the little-endian pair (lo, hi); only r's low 2 bits
// count (v_alignbyte_b32), so callers may pass an unmasked byte address
__device__ __forceinline__ uint32_t funnel(uint32_t lo, uint32_t hi, uint32_t r) {
  return __builtin_amdgcn_alignbyte(hi, lo, r);
}

// Copy `len` bytes from global `s` to global `d` (no overlap), all 64 lanes cooperating,
// 16 B per lane per step with aligned dwordx4 loads + stores.  Source blocks that contain
// no byte of [s, s+len) are never loaded.  len, s, d wave-uniform.
__device__ __forceinline__ void wave_copy_global(GMEM uint8_t* d, const GMEM uint8_t* s, uint64_t len) {
  const uint32_t lane = lane_id();
  uint32_t head = (uint32_t)((16u - ((uintptr_t)d & 15u)) & 15u);
  if (head > len) head = (uint32_t)len;
  if (lane < head) d[lane] = s[lane];
  d += head;
  s += head;
  len -= head;
  const uint64_t nb = len >> 4;
  const uint32_t sh = (uint32_t)((uintptr_t)s & 15u);
  const GMEM uint4* sa = reinterpret_cast<const GMEM uint4*>(s - sh);
  GMEM uint4* da = reinterpret_cast<GMEM uint4*>(d);
  if (sh == 0) {
    uint64_t b = lane;
    for (; b + 3 * kWave < nb; b += 4 * kWave) {  // 4 KiB per wave in flight
      const uint4 x0 = sa[b], x1 = sa[b + kWave], x2 = sa[b + 2 * kWave], x3 = sa[b + 3 * kWave];
      da[b] = x0;
      da[b + kWave] = x1;
      da[b + 2 * kWave] = x2;
      da[b + 3 * kWave] = x3;
    }
    for (; b < nb; b += kWave) da[b] = sa[b];
  } else {
    const uint32_t q = sh >> 2, r = sh & 3u;
    // funnel one 16-B output block from its source block x and the next one y
    auto emit = [&](uint64_t b, uint4 x, uint4 y) {
      const uint32_t w[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
      uint4 o;
      switch (q) {  // q is wave-uniform: a scalar branch
        case 0: o = make_uint4(funnel(w[0], w[1], r), funnel(w[1], w[2], r), funnel(w[2], w[3], r), funnel(w[3], w[4], r)); break;
        case 1: o = make_uint4(funnel(w[1], w[2], r), funnel(w[2], w[3], r), funnel(w[3], w[4], r), funnel(w[4], w[5], r)); break;
        case 2: o = make_uint4(funnel(w[2], w[3], r), funnel(w[3], w[4], r), funnel(w[4], w[5], r), funnel(w[5], w[6], r)); break;
        default: o = make_uint4(funnel(w[3], w[4], r), funnel(w[4], w[5], r), funnel(w[5], w[6], r), funnel(w[6], w[7], r)); break;
      }
      da[b] = o;
    };
    uint64_t base = 0;
    // main body: 4 wave-contiguous 1 KiB rows per step (4 KiB in flight per wave); a lane's
    // next source block comes from lane+1, lane 63 takes lane 0 of the next row
    auto next = [&](uint4 x, uint4 row_after) {
      uint4 y;
      y.x = shfl_down1(x.x);
      y.y = shfl_down1(x.y);
      y.z = shfl_down1(x.z);
      y.w = shfl_down1(x.w);
      if (lane == kWave - 1) {
        y.x = readlane(row_after.x, 0);
        y.y = readlane(row_after.y, 0);
        y.z = readlane(row_after.z, 0);
        y.w = readlane(row_after.w, 0);
      }
      return y;
    };
    for (; base + 4 * kWave <= nb; base += 4 * kWave) {
      const uint64_t b = base + lane;
      const uint4 x0 = sa[b], x1 = sa[b + kWave], x2 = sa[b + 2 * kWave], x3 = sa[b + 3 * kWave];
      uint4 x4 = make_uint4(0, 0, 0, 0);
      if (lane == 0) x4 = sa[base + 4 * kWave];  // in bounds
      emit(b, x0, next(x0, x1));
      emit(b + kWave, x1, next(x1, x2));
      emit(b + 2 * kWave, x2, next(x2, x3));
      emit(b + 3 * kWave, x3, next(x3, x4));
    }
    for (; base < nb; base += kWave) {
      const uint64_t b = base + lane;
      const bool act = b < nb;
      uint4 x = make_uint4(0, 0, 0, 0);
      if (act) x = sa[b];
      uint4 y;
      y.x = shfl_down1(x.x);
      y.y = shfl_down1(x.y);
      y.z = shfl_down1(x.z);
      y.w = shfl_down1(x.w);
      if (act && (lane == kWave - 1 || b + 1 == nb)) y = sa[b + 1];  // holds s+16b+15
      if (act) emit(b, x, y);
    }
  }
  const uint64_t done = nb << 4;
  const uint32_t tail = (uint32_t)(len - done);
  if (lane < tail) d[done + lane] = s[done + lane];
}

// inclusive prefix sum over the wave's 64 lanes (DPP row shifts + row broadcasts)
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
  int x = (int)v;
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return (uint32_t)x;
}

// inclusive prefix max (unsigned) over the wave's 64 lanes
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
  uint32_t x = v;
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
  return x;
}
// signed form (lanes out of the DPP pattern read INT_MIN, the identity of the max)
__device__ __forceinline__ int32_t wave_incl_max_i(int32_t v) {
  constexpr int32_t lo = (int32_t)0x80000000u;
  int32_t x = v;
  x = max(x, __builtin_amdgcn_update_dpp(lo, x, 0x111, 0xf, 0xf, false));
  x = max(x, __builtin_amdgcn_update_dpp(lo, x, 0x112, 0xf, 0xf, false));
  x = max(x, __builtin_amdgcn_update_dpp(lo, x, 0x114, 0xf, 0xf, false));
  x = max(x, __builtin_amdgcn_update_dpp(lo, x, 0x118, 0xf, 0xf, false));
  x = max(x, __builtin_amdgcn_update_dpp(lo, x, 0x142, 0xa, 0xf, false));
  x = max(x, __builtin_amdgcn_update_dpp(lo, x, 0x143, 0xc, 0xf, false));
  return x;
}
// lane l gets lane l-1's value, lane 0 gets 0 (DPP wave_shr:1)
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}


}  // namespace bitar_hip
