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
  uint32_t fw[kMaxSym];     // frequencies (padded)
  uint32_t w[2 * kMaxSym];  // leaf weights in rank order [0, m), internal weights [m, 2m - 1)
  uint16_t leaf[kMaxSym];   // rank -> symbol
  uint16_t up[kMaxSym];     // internal node -> its parent (pointer jumping)
  uint16_t dep[kMaxSym];    // internal node depth (pointer jumping)
  uint16_t blc[16];         // bl_count
};

// elements of the non-decreasing a[a0, a0 + n) below x (le: not above x); branch-free binary
// search, n < 512
__device__ __forceinline__ uint32_t count_below(const uint32_t* a, uint32_t a0, uint32_t n,
                                                uint32_t x, bool le) {
  uint32_t p = 0;
  for (uint32_t st = 256; st != 0; st >>= 1) {
    const uint32_t q = p + st;
    const uint32_t y = q <= n ? a[a0 + q - 1] : ~0u;
    p = (le ? y <= x : y < x) && q <= n ? q : p;
  }
  return p;
}

// Length-limited Huffman code lengths of nsym symbols (bo_huff_lengths), identical to the
// oracle's two-queue construction but with only its merge left serial:
//   1. leaves ranked by (frequency, symbol) in parallel;
//   2. one lane merges the two queues for the internal weights I[0, m-1) alone (no parent or
//      order arrays);
//   3. the merge consumed the nodes in the stable merge of the sorted leaves L and the
//      (non-decreasing) internal weights I, leaves first on ties -- a leaf taken while its
//      internal rival does not exist yet is that rival's child, so never heavier -- and the
//      nodes consumed at positions 2t and 2t+1 are internal node t's children.  So every
//      node's position is a merge rank (binary search), its parent internal node position/2,
//      and the depths follow by pointer jumping, all lanes at once;
//   4. zlib's gen_bitlen capping: a node deeper than maxlen counts one overflow (internal
//      nodes too); on overflow bl_count is repaired as zlib does (one lane, <= 16 entries)
//      and the lengths handed out to the leaves in consumption (= rank) order, in parallel.
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
    if (key[c] != ~0u) {
      T.leaf[rank[c]] = (uint16_t)(key[c] & 511u);
      T.w[rank[c]] = key[c] >> 9;
    }
  lds_order();
  // leaf weights T.w[0, m), internal weights T.w[m, m + ni)
  const uint32_t ni = m - 1;  // internal nodes; the last, ni - 1, is the root
  if (lane == 0) {
    uint32_t i = 0, j = 0;
    for (uint32_t t = 0; t < ni; ++t) {
      uint32_t v = 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t a = T.w[i], b = T.w[m + j];
        const bool lf = i < m && (j >= t || a <= b);
        v += lf ? a : b;
        i += lf ? 1u : 0u;
        j += lf ? 0u : 1u;
      }
      T.w[m + t] = v;
    }
  }
  lds_order();
  // positions in the consumption order: leaf k after the internal nodes lighter than it,
  // internal node t after the leaves not heavier than it (branch-free binary searches)
  uint32_t dl[kMaxChunks], ti[kMaxChunks];
#pragma unroll
  for (uint32_t c = 0; c < kMaxChunks; ++c) {
    const uint32_t t = c * kWave + lane;
    ti[c] = t;
    if (t < ni) {
      const uint32_t up = t + 1 == ni ? t : (t + count_below(T.w, 0, m, T.w[m + t], true)) >> 1;
      T.up[t] = (uint16_t)up;
      T.dep[t] = t + 1 == ni ? 0u : 1u;
    }
  }
  // depths of the internal nodes: pointer jumping (the root points at itself, depth 0);
  // a depth is < ni, so ceil(log2(ni)) rounds
  for (uint32_t span = 1; span < ni; span <<= 1) {
    uint32_t nd[kMaxChunks], nu[kMaxChunks];
    lds_order();
#pragma unroll
    for (uint32_t c = 0; c < kMaxChunks; ++c) {
      if (ti[c] < ni) {
        const uint32_t u = T.up[ti[c]];
        nd[c] = T.dep[ti[c]] + T.dep[u];
        nu[c] = T.up[u];
      }
    }
    lds_order();
#pragma unroll
    for (uint32_t c = 0; c < kMaxChunks; ++c) {
      if (ti[c] < ni) {
        T.dep[ti[c]] = (uint16_t)nd[c];
        T.up[ti[c]] = (uint16_t)nu[c];
      }
    }
  }
  lds_order();
  // leaf depths, capped; overflow = nodes deeper than maxlen, root excluded
  uint32_t over = 0;
#pragma unroll
  for (uint32_t c = 0; c < kMaxChunks; ++c) {
    const uint32_t k = c * kWave + lane;
    dl[c] = 0;
    if (k < m) dl[c] = T.dep[(k + count_below(T.w, m, ni, T.w[k], false)) >> 1] + 1u;
    const bool deep_int = k + 1 < ni && T.dep[k] > maxlen;
    over += (uint32_t)__builtin_popcountll(ballot(k < m && dl[c] > maxlen)) +
            (uint32_t)__builtin_popcountll(ballot(deep_int));
    dl[c] = dl[c] > maxlen ? maxlen : dl[c];
  }
  if (over) {  // (uniform)
    // bl_count from the capped lengths (ballots: one count per length)
    for (uint32_t b = 1; b <= maxlen; ++b) {
      uint32_t cnt = 0;
#pragma unroll
      for (uint32_t c = 0; c < kMaxChunks; ++c)
        cnt += (uint32_t)__builtin_popcountll(ballot(c * kWave + lane < m && dl[c] == b));
      if (lane == 0) T.blc[b] = (uint16_t)cnt;
    }
    lds_order();
    if (lane == 0) {
      int32_t ov = (int32_t)over;
      do {
        uint32_t bits = maxlen - 1;
        while (T.blc[bits] == 0) --bits;
        T.blc[bits]--;
        T.blc[bits + 1] += 2;
        T.blc[maxlen]--;
        ov -= 2;
      } while (ov > 0);
    }
    lds_order();
    // the lengths again, maxlen first, to the leaves in rank order
    uint32_t cum = 0;
    for (uint32_t b = maxlen; b != 0; --b) {
      const uint32_t nb = T.blc[b];
#pragma unroll
      for (uint32_t c = 0; c < kMaxChunks; ++c) {
        const uint32_t k = c * kWave + lane;
        if (k >= cum && k < cum + nb) dl[c] = b;
      }
      cum += nb;
    }
  }
#pragma unroll
  for (uint32_t c = 0; c < kMaxChunks; ++c) {
    const uint32_t k = c * kWave + lane;
    if (k < m) lens[T.leaf[k]] = (uint8_t)dl[c];
  }
  lds_order();
}

}  // namespace huf

}  // namespace bitar_hip
