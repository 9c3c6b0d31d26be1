// huffman.hip.h -- length-limited Huffman code lengths for one wavefront (gfx950), shared by
// the dynamic-Huffman DEFLATE encoder (deflate_dyn.hip, limit 15 / 7) and the Zstandard
// literal encoder (zstd_compress.hip, limit 11).  Restated by the oracle's bo_huff_lengths
// (oracle/bitar_deflate_dyn.c): a two-queue Huffman tree over the used symbols sorted by
// (frequency, symbol), depths capped as zlib's gen_bitlen does.
#pragma once

#include "wave.hip.h"

namespace bitar_hip {

namespace huf {

constexpr uint32_t kMaxSym = 286;  // DEFLATE literal/length alphabet (the largest user)

struct TreeLds {
  uint32_t fw[kMaxSym];      // frequencies (padded)
  uint32_t w[2 * kMaxSym];   // node weights
  uint16_t parent[2 * kMaxSym];
  uint16_t order[2 * kMaxSym];
  uint16_t leaf[kMaxSym];
  uint8_t nlen[2 * kMaxSym];
  uint16_t blc[16];        // bl_count / next_code
};

// Length-limited Huffman code lengths of nsym symbols (bo_huff_lengths).
static __device__ void huff_lengths(const uint32_t* freq, uint32_t nsym, uint32_t maxlen, uint8_t* lens,
                             TreeLds& T) {
  const uint32_t lane = lane_id();
  uint32_t m = 0;
  lds_order();
  for (uint32_t s0 = 0; s0 < nsym; s0 += kWave) {
    const uint32_t s = s0 + lane;
    const uint32_t f = s < nsym ? freq[s] : 0u;
    if (s < nsym) {
      T.fw[s] = f;
      lens[s] = 0;
    }
    m += (uint32_t)__builtin_popcountll(ballot(f != 0));
  }
  lds_order();
  if (m < 2 && lane == 0) {
    for (uint32_t s = 0; s < nsym && m < 2; ++s)
      if (!T.fw[s]) { T.fw[s] = 1; ++m; }
  }
  lds_order();
  m = m < 2 ? 2u : m;
  // leaves in (frequency, symbol) order: rank of every used symbol.  Keys (f << 9 | s) are
  // unique; an unused symbol's key is ~0 (never below a used one).  Each lane holds the keys
  // of symbols lane + 64 k in registers and counts the smaller keys of all symbols via
  // readlane: no LDS round trip per comparison.
  constexpr uint32_t kMaxChunks = (kMaxSym + kWave - 1) / kWave;  // 5
  const uint32_t nch = (nsym + kWave - 1) / kWave;
  uint32_t key[kMaxChunks], rank[kMaxChunks];
#pragma unroll
  for (uint32_t c = 0; c < kMaxChunks; ++c) {
    const uint32_t s = c * kWave + lane;
    const uint32_t f = c < nch && s < nsym ? T.fw[s] : 0u;
    key[c] = f ? (f << 9) | s : ~0u;
    rank[c] = 0;
  }
  for (uint32_t c2 = 0; c2 < nch; ++c2) {
    uint32_t kc = key[0];
#pragma unroll
    for (uint32_t c = 1; c < kMaxChunks; ++c) kc = c2 == c ? key[c] : kc;  // (c2 uniform)
    for (uint32_t t = 0; t < kWave; ++t) {
      const uint32_t kt = readlane(kc, t);
#pragma unroll
      for (uint32_t c = 0; c < kMaxChunks; ++c) rank[c] += kt < key[c] ? 1u : 0u;
    }
  }
  lds_order();
#pragma unroll
  for (uint32_t c = 0; c < kMaxChunks; ++c)
    if (key[c] != ~0u) T.leaf[rank[c]] = (uint16_t)(key[c] & 511u);
  lds_order();
  if (lane == 0) {
    for (uint32_t k = 0; k < m; ++k) T.w[k] = T.fw[T.leaf[k]];
    uint32_t i = 0, j = m, next = m, no = 0;
    for (uint32_t step = 0; step + 1 < m; ++step) {
      uint32_t ab[2];
      for (int t = 0; t < 2; ++t) {
        const bool take_leaf = i < m && (j >= next || T.w[i] <= T.w[j]);
        ab[t] = take_leaf ? i++ : j++;
        T.order[no++] = (uint16_t)ab[t];
      }
      T.w[next] = T.w[ab[0]] + T.w[ab[1]];
      T.parent[ab[0]] = (uint16_t)next;
      T.parent[ab[1]] = (uint16_t)next;
      ++next;
    }
    const uint32_t root = 2 * m - 2;
    T.order[no++] = (uint16_t)root;
    for (uint32_t b = 0; b < 16; ++b) T.blc[b] = 0;
    int overflow = 0;
    T.nlen[root] = 0;
    for (int k = (int)no - 2; k >= 0; --k) {
      const uint32_t nd = T.order[k];
      uint32_t bits = T.nlen[T.parent[nd]] + 1u;
      if (bits > maxlen) { bits = maxlen; ++overflow; }
      T.nlen[nd] = (uint8_t)bits;
      if (nd < m) T.blc[bits]++;
    }
    if (overflow) {
      do {
        uint32_t bits = maxlen - 1;
        while (T.blc[bits] == 0) --bits;
        T.blc[bits]--;
        T.blc[bits + 1] += 2;
        T.blc[maxlen]--;
        overflow -= 2;
      } while (overflow > 0);
      uint32_t h = 0;
      for (uint32_t bits = maxlen; bits != 0; --bits) {
        uint32_t n = T.blc[bits];
        while (n != 0) {
          const uint32_t nd = T.order[h++];
          if (nd >= m) continue;
          T.nlen[nd] = (uint8_t)bits;
          --n;
        }
      }
    }
    for (uint32_t k = 0; k < m; ++k) lens[T.leaf[k]] = T.nlen[k];
  }
  lds_order();
}

}  // namespace huf

}  // namespace bitar_hip
