// order.hip.h -- cost-ordered dispatch: the key range and the tiling of the counting sort
// (util_kernels.hip order_hist_kernel / order_scatter_kernel; runtime.hip SegOrder).
#pragma once
#include <stdint.h>

namespace bitar_hip {

constexpr uint32_t kOrderBins = 256;  // sort keys are < kOrderBins (lowest first)
constexpr uint32_t kOrderMaxTiles = 64;

// segments per tile: a multiple of 1024 (16 per lane), at most kOrderMaxTiles tiles
__host__ __device__ inline uint32_t order_tile(uint32_t nseg) {
  const uint32_t t = (nseg + kOrderMaxTiles - 1) / kOrderMaxTiles;
  return ((t < 1024u ? 1024u : t) + 1023u) & ~1023u;
}

}  // namespace bitar_hip
