// util_kernels.hip -- frame packing (prefix sum + gather) and the synthetic-input generator.
#include "order.hip.h"
#include "wave.hip.h"

namespace bitar_hip {

// A size larger than `limit` (the slot stride; BITAR_HIP_SEGMENT_ERROR of a failed op in
// particular) counts as 0 bytes and raises bit 2 of the stream's error word: pack must
// never copy past a slot.
__device__ __forceinline__ uint32_t clamp_size(uint32_t v, uint64_t limit,
                                               uint32_t* __restrict__ err) {
  if ((uint64_t)v > limit) {
    atomicOr(err, 4u);
    return 0u;
  }
  return v;
}

// Exclusive prefix sum of nseg sizes -> offsets[0..nseg], one 1024-thread workgroup.
// nseg is at most a few hundred thousand (8 GiB / 64 KiB = 131072): a single block walks
// the array in 1024-element tiles with a carried base.
__global__ __launch_bounds__(1024) void scan_sizes_kernel(const uint32_t* __restrict__ sizes,
                                                          uint32_t nseg, uint64_t limit,
                                                          uint64_t* __restrict__ offsets,
                                                          uint32_t* __restrict__ err) {
  __shared__ uint64_t part[1024 / kWave];
  __shared__ uint64_t carry;
  const uint32_t t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) carry = 0;
  __syncthreads();
  for (uint32_t base = 0; base < nseg; base += 1024) {
    const uint32_t idx = base + t;
    uint64_t v = idx < nseg ? (uint64_t)clamp_size(sizes[idx], limit, err) : 0ull;
    uint64_t incl = v;  // inclusive wave scan (Hillis-Steele over 64 lanes)
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint64_t y = __shfl_up(incl, d, 64);
      if (lane >= d) incl += y;
    }
    if (lane == 63) part[w] = incl;
    __syncthreads();
    if (t < 64) {
      uint64_t pv = t < 1024 / kWave ? part[t] : 0ull;
      uint64_t pin = pv;
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(pin, d, 64);
        if (t >= d) pin += y;
      }
      if (t < 1024 / kWave) part[t] = pin - pv;  // exclusive wave bases
    }
    __syncthreads();
    const uint64_t c = carry;
    if (idx < nseg) offsets[idx] = c + part[w] + incl - v;
    __syncthreads();
    if (t == 1023) carry = c + part[w] + incl;
    __syncthreads();
  }
  if (t == 0) offsets[nseg] = carry;
}

// Gather slot i (sizes[i] bytes at slab + i*stride) to frame + offsets[i]; one wave per slot.
__global__ __launch_bounds__(64) void pack_kernel(const uint8_t* __restrict__ slab,
                                                  uint64_t stride,
                                                  const uint32_t* __restrict__ sizes,
                                                  const uint64_t* __restrict__ offsets,
                                                  uint32_t nseg, uint8_t* __restrict__ frame) {
  const uint32_t i = blockIdx.x;
  if (i >= nseg) return;
  // the same clamp as the scan (which already flagged it): a failed slot packs 0 bytes
  const uint32_t len = (uint64_t)sizes[i] > stride ? 0u : sizes[i];
  wave_copy_global(global_ptr(frame + offsets[i]), global_ptr(slab + (uint64_t)i * stride), len);
}

// Batched copy: entry i moves sizes[i] bytes from srcs[i] to dsts[i]; one wave per entry.
// Splits a chained op's output over its slots and joins chained inputs (max_sgl_segs > 1).
__global__ __launch_bounds__(64) void copy_batch_kernel(const uint8_t* const* __restrict__ srcs,
                                                        uint8_t* const* __restrict__ dsts,
                                                        const uint32_t* __restrict__ sizes,
                                                        uint32_t n) {
  const uint32_t i = blockIdx.x;
  if (i >= n) return;
  const uint32_t len = sizes[i];
  if (len) wave_copy_global(global_ptr(dsts[i]), global_ptr(srcs[i]), len);
}

// LZ4 frame data blocks (lz4 frame format, independent blocks): framed size of block i =
// 4-byte size field + the compressed block, or the raw slice when it did not shrink (a
// compressed block may not exceed the frame's maximum block size).
__global__ __launch_bounds__(256) void lz4f_sizes_kernel(const uint32_t* __restrict__ sizes,
                                                         uint32_t nseg, uint64_t n, uint32_t seg,
                                                         uint32_t* __restrict__ framed) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i >= nseg) return;
  const uint64_t off = (uint64_t)i * seg;
  const uint32_t len = (uint32_t)(n - off < seg ? n - off : seg);
  framed[i] = 4 + (sizes[i] < len ? sizes[i] : len);  // a failed op (SEGMENT_ERROR) ships raw
}

// block i at frame + offsets[i]: LE32 size (| 1 << 31 when stored raw) + its bytes
__global__ __launch_bounds__(64) void lz4f_pack_kernel(const uint8_t* __restrict__ in, uint64_t n,
                                                       uint32_t seg, const uint8_t* __restrict__ slab,
                                                       uint64_t stride,
                                                       const uint32_t* __restrict__ sizes,
                                                       const uint64_t* __restrict__ offsets,
                                                       uint32_t nseg, uint8_t* __restrict__ frame) {
  const uint32_t i = blockIdx.x;
  if (i >= nseg) return;
  const uint64_t off = (uint64_t)i * seg;
  const uint32_t len = (uint32_t)(n - off < seg ? n - off : seg);
  const bool raw = sizes[i] >= len;
  const uint32_t body = raw ? len : sizes[i];
  const uint32_t field = raw ? (len | 0x80000000u) : body;
  GMEM uint8_t* d = global_ptr(frame + offsets[i]);
  if (lane_id() < 4) d[lane_id()] = (uint8_t)(field >> (8 * lane_id()));
  wave_copy_global(d + 4, raw ? global_ptr(in + off) : global_ptr(slab + (uint64_t)i * stride), body);
}

// ---- synthetic input: a device restatement-free generator; tests check it against the
// oracle's bo_fill byte for byte.  One thread per 64-byte line.
__device__ __forceinline__ uint64_t sm64(uint64_t seed, uint64_t k) {
  uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ void put_dec(uint8_t* p, uint32_t v, int width) {
  for (int i = width - 1; i >= 0; --i) { p[i] = (uint8_t)('0' + v % 10); v /= 10; }
}

__device__ __forceinline__ void put_str(uint8_t* p, const char* s, int n) {
  for (int i = 0; i < n; ++i) p[i] = (uint8_t)s[i];
}

__device__ void log_line(uint64_t seed, uint64_t j, uint8_t* l) {
  const char* kLevel = "INFO WARN DEBUGERROR";
  const char* kComp = "device   driver   memory   pool     queuepairconfig   burst    dequeue  ";
  const char* kStat = "OK    OK    EAGAINOK    ";
  const uint64_t h = sm64(seed ^ 0x5bd1e995ull, j);
  for (int i = 0; i < 64; ++i) l[i] = ' ';
  const uint64_t ms = j * 7;
  put_dec(l + 0, (uint32_t)((ms / 3600000) % 24), 2); l[2] = ':';
  put_dec(l + 3, (uint32_t)((ms / 60000) % 60), 2); l[5] = ':';
  put_dec(l + 6, (uint32_t)((ms / 1000) % 60), 2); l[8] = '.';
  put_dec(l + 9, (uint32_t)(ms % 1000), 3);
  const uint32_t lv = (uint32_t)(h & 15);
  put_str(l + 13, kLevel + 5 * (lv < 12 ? 0 : lv < 14 ? 1 : lv < 15 ? 2 : 3), 5);
  put_str(l + 19, kComp + 9 * ((h >> 4) & 7), 9);
  put_str(l + 29, "qp=", 3);
  put_dec(l + 32, (uint32_t)((h >> 8) % 32), 2);
  put_str(l + 35, "seg=", 4);
  put_dec(l + 39, (uint32_t)((h >> 16) % 100000), 5);
  put_str(l + 45, "status=", 7);
  put_str(l + 52, kStat + 6 * ((h >> 40) & 3), 6);
  l[63] = '\n';
}

// Bytes [off, off + n) of the stream (off a multiple of 64): out[b] = stream[off + b].  A
// rank generates only the batches of a job it was dealt (bitar_amd/job.py).
__global__ __launch_bounds__(256) void fill_kernel(int kind, uint64_t seed, uint64_t off,
                                                   uint8_t* __restrict__ out, uint64_t n) {
  const uint64_t nlines = (n + 63) / 64;
  const uint64_t line0 = off / 64;
  for (uint64_t jl = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; jl < nlines;
       jl += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t j = line0 + jl;  // line of the whole stream (the generator's index)
    __attribute__((aligned(16))) uint8_t line[64];
    uint64_t w[8];
    const uint64_t k0 = j * 8;
    bool text = false;
    uint64_t tseed = seed;
    switch (kind) {
      case 0:
        for (int i = 0; i < 8; ++i) w[i] = sm64(seed, k0 + i);
        break;
      case 1: {
        const uint64_t region = ((j * 64) >> 20) % 3;
        if (region == 0) {
          for (int i = 0; i < 8; ++i) w[i] = sm64(seed ^ 0x1111ull, k0 + i) % 1000;
        } else if (region == 1) {
          text = true;
        } else {
          for (int i = 0; i < 8; ++i) w[i] = sm64(seed ^ 0x2222ull, k0 + i);
        }
        break;
      }
      case 2: {
        const uint64_t col = ((j * 64) >> 20) & 3;
        if (col == 3) { text = true; tseed = seed ^ 0x4444ull; break; }
        for (int i = 0; i < 8; ++i) {
          const uint64_t r = sm64(seed ^ (0x3333ull + col), k0 + i);
          if (col == 0) {
            w[i] = r % 1000;
          } else if (col == 1) {
            const int64_t s = (int64_t)(r & 0xFFFF) + (int64_t)((r >> 16) & 0xFFFF) +
                              (int64_t)((r >> 32) & 0xFFFF) + (int64_t)(r >> 48) - 131070;
            const double d = (double)s / 37837.0;
            w[i] = (uint64_t)__double_as_longlong(d);
          } else {
            w[i] = (r & 63) | (((r >> 32) & 63) << 32);
          }
        }
        break;
      }
      case 3:
        for (int i = 0; i < 8; ++i) w[i] = 0x6161616161616161ull;
        break;
      case 5:
        for (int i = 0; i < 8; ++i) w[i] = sm64(seed ^ 0x1111ull, k0 + i) % 1000;
        break;
      case 6:
        text = true;
        break;
      default:
        for (int b = 0; b < 64; ++b) line[b] = (uint8_t)(((j * 64 + b) % 251) * 7);
        break;
    }
    if (text) {
      log_line(tseed, j, line);
    } else if ((kind >= 0 && kind <= 3) || kind == 5) {
      for (int i = 0; i < 8; ++i)
        for (int b = 0; b < 8; ++b) line[i * 8 + b] = (uint8_t)(w[i] >> (8 * b));
    }
    const uint64_t base = jl * 64;  // output position
    if (base + 64 <= n) {
      uint4* d = reinterpret_cast<uint4*>(out + base);
      const uint4* s = reinterpret_cast<const uint4*>(line);
      if (((uintptr_t)d & 15) == 0) {
        for (int q = 0; q < 4; ++q) d[q] = s[q];
      } else {
        for (int b = 0; b < 64; ++b) out[base + b] = line[b];
      }
    } else {
      for (uint64_t b = 0; base + b < n; ++b) out[base + b] = line[b];
    }
  }
}

// ---- cost-ordered dispatch ----------------------------------------------------------------
// One wave per segment holds a CU slot for the segment's whole (serial) parse or decode, so a
// launch ends with a drain of ~one segment's duration in which the CUs empty out.  When the
// segments differ in cost (a mix of text, columns and incompressible data), the drain is
// shortest if the expensive segments run first and the cheap ones fill the end (longest
// processing time first).  The runtime dispatches segment order[b] as workgroup b, order =
// the segments sorted by an estimated cost key (lowest key = most expensive first).

// Compress: the number of distinct byte values in a 128-byte sample of the segment (4 x 32 B
// at its quarter points) -- incompressible data shows ~100, the parse skips through it.
__global__ __launch_bounds__(64) void seg_cost_kernel(const uint8_t* __restrict__ in,
                                                       uint64_t n, uint32_t seg, uint32_t nseg,
                                                       uint32_t* __restrict__ keys) {
  // four threads per segment, one 32-byte sample each; the four 256-bit byte sets are OR-ed
  // across the quad (a thread per segment issued 128 selects per byte set: 25 -> 12 us per
  // GiB with 16-byte loads, this splits the rest four ways)
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t i = t >> 2, q = t & 3u;
  const bool live = i < nseg;
  const uint64_t s0 = (uint64_t)(live ? i : 0u) * seg;
  const uint32_t len = live ? (uint32_t)(n - s0 < seg ? n - s0 : seg) : 0u;
  uint32_t bm[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto add = [&](uint32_t b) __attribute__((always_inline)) {
    const uint32_t bit = 1u << (b & 31u), w = b >> 5;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) bm[j] |= w == j ? bit : 0u;
  };
  const uint32_t at = (uint32_t)(((uint64_t)len * q) / 4);
  if (len >= 128) {
    uint4 v[2];
    __builtin_memcpy(&v[0], in + s0 + at, 16);
    __builtin_memcpy(&v[1], in + s0 + at + 16, 16);
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) {
      const uint32_t w4[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
      for (uint32_t b = 0; b < 16; ++b) add((w4[b >> 2] >> (8 * (b & 3u))) & 0xFFu);
    }
  } else if (live) {
    const uint32_t cnt = len - at < 32 ? len - at : 32;
    for (uint32_t k = 0; k < cnt; ++k) add(in[s0 + at + k]);
  }
  uint32_t d = 0;
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j) {
    uint32_t x = bm[j];
    x |= (uint32_t)__shfl_xor((int)x, 1, 64);
    x |= (uint32_t)__shfl_xor((int)x, 2, 64);
    d += (uint32_t)__builtin_popcount(x);
  }
  if (live && q == 0) keys[i] = d;
}

// Zstd chain walk (zstd_walk_kernel, 4 segments x 4 blocks per wave): the sequence count,
// most first, so a wave walks chains of similar length and the longest go in the first round.
__global__ __launch_bounds__(64) void walk_key_kernel(const uint2* __restrict__ meta, uint32_t nseg,
                                                      uint32_t* __restrict__ keys) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nseg) return;
  const uint32_t q = meta[i].y >> 6;
  keys[i] = kOrderBins - 1u - (q < kOrderBins - 1u ? q : kOrderBins - 1u);
}

// order = 0..nseg-1 sorted by key (< kOrderBins) ascending: a counting sort over tiles of
// `tile` consecutive segments, in two launches of one-wave workgroups (order_hist_kernel: the
// tiles' histograms; order_scatter_kernel: every tile's bin offsets from all histograms, then
// its segments).  One-wave workgroups take a CU slot as soon as any wave of another grid
// ends, so the sort of one queue pair's call no longer waits for a CU to drain while another
// queue pair's compress grid holds the chip (a 1024-thread workgroup did: 4.7 ms per call in
// the configs[3] record batch, 0.03 ms alone).  The order within a key is not fixed (it does
// not matter for the output).  keys == null: the decompress key from the compressed sizes
// (csizes): the largest coded segments first (a decoder's cost grows with the symbols or
// sequences it reads), the stored / incompressible ones (csize >= seg: raw blocks, stored
// blocks, one literal run) last, as they decode as copies.  (Measured against smallest-first:
// LZ4 kind 1 decode 1.74 -> 1.67 ms, fixed-Huffman DEFLATE 10.6 -> 7.9 ms, Zstd kind 1 6.53
// -> 6.42 ms.)  Each lane takes a contiguous run of its tile's segments and adds runs of
// equal keys with one LDS atomic (neighbouring segments often share a key: one address for
// all of them would serialize).
__device__ __forceinline__ uint32_t order_key(const uint32_t* keys, const uint32_t* csizes,
                                              uint32_t seg, uint32_t i) {
  if (keys) return keys[i] < kOrderBins ? keys[i] : kOrderBins - 1u;
  const uint32_t c = csizes[i];
  return c >= seg ? kOrderBins - 1u
                  : kOrderBins - 2u - (uint32_t)((uint64_t)c * (kOrderBins - 2u) / seg);
}

// lane l of tile b visits the segments [b tile + l per, + per), per = tile / 64; runs of equal
// keys go to f(key, run start, run length)
template <class F>
__device__ __forceinline__ void order_runs(const uint32_t* keys, const uint32_t* csizes,
                                           uint32_t seg, uint32_t nseg, uint32_t tile, F f) {
  const uint32_t per = tile / kWave;
  const uint32_t i0 = blockIdx.x * tile + lane_id() * per;
  const uint32_t i1 = i0 + per < nseg ? i0 + per : nseg;
  constexpr uint32_t kB = 16;  // keys read 16 at a time, all loads issued before the first use
  uint32_t cur = 0, cnt = 0, start = i0;
  for (uint32_t b = i0; b < i1; b += kB) {
    uint32_t kk[kB];
#pragma unroll
    for (uint32_t j = 0; j < kB; ++j) kk[j] = b + j < i1 ? order_key(keys, csizes, seg, b + j) : 0u;
#pragma unroll
    for (uint32_t j = 0; j < kB; ++j) {
      if (b + j >= i1) break;
      if (cnt && kk[j] != cur) {
        f(cur, start, cnt);
        cnt = 0;
      }
      if (!cnt) start = b + j;
      cur = kk[j];
      ++cnt;
    }
  }
  if (cnt) f(cur, start, cnt);
}

__global__ __launch_bounds__(64) void order_hist_kernel(const uint32_t* __restrict__ keys,
                                                        const uint32_t* __restrict__ csizes,
                                                        uint32_t seg, uint32_t nseg, uint32_t tile,
                                                        uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[kOrderBins];
  const uint32_t lane = lane_id();
  for (uint32_t k = lane; k < kOrderBins; k += kWave) h[k] = 0;
  __syncthreads();
  order_runs(keys, csizes, seg, nseg, tile,
             [&](uint32_t key, uint32_t, uint32_t cnt) { atomicAdd(&h[key], cnt); });
  __syncthreads();
  for (uint32_t k = lane; k < kOrderBins; k += kWave) hist[blockIdx.x * kOrderBins + k] = h[k];
}

__global__ __launch_bounds__(64) void order_scatter_kernel(const uint32_t* __restrict__ keys,
                                                           const uint32_t* __restrict__ csizes,
                                                           uint32_t seg, uint32_t nseg,
                                                           uint32_t tile, uint32_t ntiles,
                                                           const uint32_t* __restrict__ hist,
                                                           uint32_t* __restrict__ order) {
  static_assert(kOrderBins == 4 * kWave, "four bins per lane");
  __shared__ uint32_t base[kOrderBins];
  const uint32_t lane = lane_id(), me = blockIdx.x;
  // lane l owns bins 4l .. 4l + 3: their totals and the counts of the tiles before this one
  uint32_t tot[4] = {0, 0, 0, 0}, pre[4] = {0, 0, 0, 0};
  const uint4* h4 = reinterpret_cast<const uint4*>(hist);
  for (uint32_t t = 0; t < ntiles; ++t) {
    const uint4 v = h4[t * (kOrderBins / 4) + lane];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      tot[j] += w[j];
      pre[j] += t < me ? w[j] : 0u;
    }
  }
  // exclusive scan of the totals over the bins (4 per lane, then across the lanes)
  const uint32_t s4 = tot[0] + tot[1] + tot[2] + tot[3];
  uint32_t incl = s4;
#pragma unroll
  for (uint32_t d = 1; d < kWave; d <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, d, kWave);
    if (lane >= d) incl += y;
  }
  uint32_t run = incl - s4;
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j) {
    base[4 * lane + j] = run + pre[j];
    run += tot[j];
  }
  __syncthreads();
  order_runs(keys, csizes, seg, nseg, tile, [&](uint32_t key, uint32_t start, uint32_t cnt) {
    const uint32_t pos = atomicAdd(&base[key], cnt);
    for (uint32_t j = 0; j < cnt; ++j) order[pos + j] = start + j;
  });
}

}  // namespace bitar_hip
