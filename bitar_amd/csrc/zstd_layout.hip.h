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

// walk scratch (pass 2 -> zstd_walk_kernel -> zstd_emit_kernel), per segment: a 16-word record
// (kW*), the FSE state tables (u16, kTabDummy + 1) and transforms (3 x 64 u32); then per
// sequence its three codes (u32: LL | OF << 6 | ML << 11, written by pass 2) and each
// chain's state bits | their count << 12 (u16, chains OF, ML, LL one array each); then per
// step of 64 sequences the repeat-offset history before it (3 u32, written by pass 2), from
// which zstd_emit_kernel re-derives the offset values of the step
enum : uint32_t { kWHanded = 0, kWP0, kWBlk, kWN, kWNseq, kWAls, kWSt0, kWSt1, kWSt2 };
constexpr uint32_t kWTabs = 64, kWTr = kWTabs + 2 * 1284, kWWords = kWTr + 3 * 64 * 4;
__host__ __device__ constexpr uint32_t walk_cap(uint32_t seg) { return seg / 4u + 2u; }  // >= nseq
__host__ __device__ constexpr uint32_t walk_steps(uint32_t seg) { return (walk_cap(seg) + 63u) / 64u; }
__host__ __device__ constexpr uint64_t walk_hist_at(uint32_t seg) {  // bytes, from the record (16-B aligned)
  return ((uint64_t)kWWords + 10ull * walk_cap(seg) + 15u) & ~15ull;
}
__host__ __device__ constexpr uint64_t walk_stride(uint32_t seg) {
  return (walk_hist_at(seg) + 12ull * walk_steps(seg) + 255u) & ~255ull;
}

}  // namespace zse
}  // namespace bitar_hip
