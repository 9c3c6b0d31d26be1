// zstd_hand.hip.h -- the scratch record through which the wave Zstd decoder
// (zstd_decompress.hip) hands a frame's last block over to the lane kernels
// (zstd_lanes.hip): zstd_hlit_kernel decodes its Huffman literal streams, zstd_handoff_kernel
// executes its sequences.  Per segment kStride bytes: kRec record words, the LL / OF / ML
// decode cells (kCells words each, cell = sym | nbits << 8 | base << 16), then the Huffman
// table (2^11 u16 entries, sym | nbits << 8).
#pragma once

#include <cstdint>

namespace bitar_hip {

namespace zhand {

constexpr uint32_t kRec = 32, kCells = 512, kHufWords = 1024;
constexpr uint32_t kCellsAt = kRec, kHufAt = kRec + 3 * kCells;
constexpr uint64_t kStride = 4ull * (kRec + 3 * kCells + kHufWords);
constexpr uint32_t kHanded = 0xFFFFFFFDu;  // produced[i] while the lane kernels own segment i
constexpr uint32_t kRecs = 0xFFFFFFFCu;    // produced[i]: zstd_seqdec_kernel's records ready

// record words
enum : uint32_t {
  kQ = 0,      // sequence bitstream [kQ, kEnd) (frame offsets)
  kEnd,
  kNseq,
  kAls,        // al_LL | al_OF << 8 | al_ML << 16 | literal type << 24
  kLitV,       // raw literals: their frame offset; RLE: the byte
  kRegen,      // literal count
  kOp,         // output bytes before the block
  kRep0, kRep1, kRep2,
  kFsz, kFcs,  // frame content size field size and value (final check)
  kLitPend,    // 1: the Huffman streams below still have to be decoded to the slot tail
  kHufLog,     // table log | stream count << 8
  kStreams,    // frame offset of the first stream
  kS1, kS2, kS3, kS4,  // stream lengths
  kQQ,         // literals per stream (the last one: regen - 3 kQQ)
};

}  // namespace zhand

}  // namespace bitar_hip
