// zstd_hand.hip.h -- the scratch record through which the wave Zstd decoder
// (zstd_decompress.hip) hands a frame's trailing blocks over to the lane kernels
// (zstd_lanes.hip, zstd_seq.hip): zstd_hlit_kernel decodes their Huffman literal streams,
// zstd_seqdec_kernel walks their FSE chains, zstd_exec_kernel (or the lane executor
// zstd_handoff_kernel) executes the sequences.  Per segment kStride bytes: kRec record words,
// the LL / OF / ML decode cells (kCells words each, cell = sym | nbits << 8 | base << 16),
// then the Huffman table (2^11 u16 entries, sym | nbits << 8).
//
// A frame hands over either its last block (any frame without a checksum), or -- the frames
// of this engine's encoder (zstd_compress.hip: up to kMaxBlocks compressed blocks sharing one
// literal code and one set of tables) -- all of its blocks: the first may define tables and
// the tree, the others use Repeat_Mode and Treeless / raw / RLE literals.  Block b's
// sub-record (kQ .. kQQ) is at blk_at(b); block 0's also holds the frame-level words (kOp,
// kRep*, kFsz, kFcs).
#pragma once

#include <cstdint>

namespace bitar_hip {

namespace zhand {

constexpr uint32_t kMaxBlocks = 8;
constexpr uint32_t kRec = 256, kCells = 512, kHufWords = 1024;
constexpr uint32_t kCellsAt = kRec, kHufAt = kRec + 3 * kCells;
constexpr uint64_t kStride = 4ull * (kRec + 3 * kCells + kHufWords);
constexpr uint32_t kHanded = 0xFFFFFFFDu;  // produced[i] while the lane kernels own segment i
constexpr uint32_t kRecs = 0xFFFFFFFCu;    // produced[i]: zstd_seqdec_kernel's records ready

// sub-record words of a handed block
enum : uint32_t {
  kQ = 0,      // sequence bitstream [kQ, kEnd) (frame offsets)
  kEnd,
  kNseq,
  kAls,        // al_LL | al_OF << 8 | al_ML << 16 | literal type << 24
  kLitV,       // raw literals: their frame offset; RLE: the byte
  kRegen,      // literal count
  kOp,         // (block 0) output bytes before the first handed block
  kRep0, kRep1, kRep2,  // (block 0) the repeat offsets before it
  kFsz, kFcs,  // (block 0) frame content size field size and value (final check)
  kLitPend,    // 1: the Huffman streams below still have to be decoded to the slot tail
  kHufLog,     // table log | stream count << 8
  kStreams,    // frame offset of the first stream
  kS1, kS2, kS3, kS4,  // stream lengths
  kQQ,         // literals per stream (the last one: regen - 3 kQQ)
};
constexpr uint32_t kBlkW = 20;
__host__ __device__ constexpr uint32_t blk_at(uint32_t b) { return b == 0 ? 0u : 32u + kBlkW * (b - 1); }

// frame-level words: handed blocks, their sequences and literals in all; then per block b at
// kX0 + kXW b: its first record (zstd_seqdec_kernel's records, in block order), its literals'
// offset in the slot tail [cap - kLitAll, cap), and its final repeat offsets (written by
// zstd_seqdec_kernel: for b >= 1 in terms of the history before the block, see zstd_seq.hip)
enum : uint32_t { kNb = 176, kNseqAll, kLitAll, kX0 = 180 };
enum : uint32_t { kXRec = 0, kXLit, kXFin0, kXFin1, kXFin2 };
constexpr uint32_t kXW = 8;
static_assert(blk_at(kMaxBlocks - 1) + kBlkW <= kNb && kX0 + kXW * kMaxBlocks <= kRec, "layout");
// The multi-block lane kernels take a frame's blocks in groups of 4 ("units": unit 2 i + g =
// blocks 4 g .. 4 g + 3 of segment i); a frame of <= 4 blocks has one unit.
constexpr uint32_t kUnitBlocks = 4;

}  // namespace zhand

}  // namespace bitar_hip
