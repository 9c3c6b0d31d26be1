// zstd_layout.hip.h -- scratch layout of the Zstd encoder's four launches (zstd_compress.hip),
// shared with the runtime that allocates it (runtime.hip).
#pragma once
#include <cstdint>

namespace bitar_hip {
namespace zse {

// parse scratch per segment: the literal area, then 8-byte sequence records
// {literal length | match distance << 17, match length}
__host__ __device__ constexpr uint64_t lit_cap(uint32_t seg) { return ((uint64_t)seg + 15u) & ~15ull; }
__host__ __device__ constexpr uint64_t scratch_stride(uint32_t seg) {
  return (lit_cap(seg) + 8ull * (seg / 4u + 2u) + 255u) & ~255ull;
}

// Blocks per frame (oracle zs_nblocks): a frame with >= kMultiMin sequences is 4 compressed
// blocks of equal sequence counts -- 8 (kBlocks) with >= kWideLit literal bytes -- sharing one
// literal code and one set of sequence tables; block b holds sequences [b nseq / B,
// (b + 1) nseq / B).
constexpr uint32_t kBlocks = 8, kMultiMin = 64, kWideLit = 32768;
__host__ __device__ constexpr uint32_t frame_blocks(uint32_t nseq, uint32_t nlit) {
  return nseq < kMultiMin ? 1u : nlit >= kWideLit ? 8u : 4u;
}

// walk scratch (zstd_entropy_kernel -> zstd_walk_kernel -> zstd_emit_kernel), per segment: a
// record of kW* words; the Huffman codes (256 u32: code | length << 16); the FSE state tables
// (u16, kTabDummy + 1) and transforms (3 x 64 u32); then per sequence its three codes (u32:
// LL | OF << 6 | ML << 11 | the offset value << 17, written by the entropy kernel) and each
// chain's state bits | their count << 12 (u16) in groups of 8 sequences: group g holds the
// OF, ML and LL words of sequences 8g .. 8g + 7, 8 of each chain (walk_state_at)
enum : uint32_t {
  kWHanded = 0,  // 1: the emit kernel writes this segment's frame
  kWTrash = 1,   // the target of idle lanes' stores (fixed store counts in loops)
  kWN = 3,       // segment bytes
  kWNseq,        // sequences
  kWAls,         // accuracy logs LL | OF << 8 | ML << 16
  kWNb = 9,      // blocks
  kWLit,         // literal code: mode (0 raw, 1 RLE, 2 Huffman) | RLE byte << 8 | tree bytes << 16
  kWNlit,        // literal bytes
  kWTdesc,       // bytes of the modes byte + table descriptions (kWDescAt)
  kWTb,          // coded bits of all literals (sum of length x count): the blocks' estimate
  kWSb = 16,     // kBlocks + 1 words: first sequence of each block (then nseq)
  kWLb = 25,     // kBlocks + 1 words: first literal of each block (then nlit)
  kWStep = 34,   // kBlocks words (unused)
  kWFin = 42,    // kBlocks x 3 words: each block's final states (OF, ML, LL)
  kWTreeAt = 68,  // the Huffman tree description (<= 130 bytes)
  kWDescAt = 104,  // modes byte + sequence table descriptions (<= 256 bytes)
  kWCodeAt = 168   // 256 words: literal codes
};
static_assert(kWLb == kWSb + kBlocks + 1 && kWStep == kWLb + kBlocks + 1 &&
                  kWFin == kWStep + kBlocks && kWTreeAt >= kWFin + 3 * kBlocks &&
                  kWDescAt >= kWTreeAt + 33 && kWCodeAt >= kWDescAt + 64,
              "record areas");
constexpr uint32_t kWTabs = 4 * 424, kWTr = kWTabs + 2 * 1284, kWWords = kWTr + 3 * 64 * 4;
static_assert(kWCodeAt + 256 <= kWTabs / 4, "record words before the tables");
static_assert(kWTabs % 16 == 0 && kWWords % 8 == 0, "aligned areas");
__host__ __device__ constexpr uint32_t walk_cap(uint32_t seg) { return seg / 4u + 2u; }  // >= nseq
// u16 index of chain c's state word of sequence k in the state area (chains 0 OF, 1 ML, 2 LL)
__host__ __device__ constexpr uint32_t walk_state_at(uint32_t k, uint32_t c) {
  return (k >> 3) * 24u + c * 8u + (k & 7u);
}
__host__ __device__ constexpr uint64_t walk_state_bytes(uint32_t seg) {  // bytes, from the record (16-B aligned)
  return ((uint64_t)kWWords + 4ull * walk_cap(seg) + 15u) & ~15ull;
}
__host__ __device__ constexpr uint64_t walk_stride(uint32_t seg) {
  return (walk_state_bytes(seg) + 48ull * ((walk_cap(seg) + 7u) / 8u) + 255u) & ~255ull;
}

}  // namespace zse
}  // namespace bitar_hip
