// bitar/memory_pool.h -- arrow::MemoryPool backends (reference src/include/memory_pool.h).
//
// Rtemalloc / Rtememzone (DPDK hugepage memory the BlueField DMAs from) become HipHost
// (pinned host memory, hipHostMalloc) and HipDevice (HBM on the current device, hipMalloc).
// The reference names are kept as aliases so callers compile unchanged.
#pragma once

#include <cstddef>
#include <cstdint>
#include <mutex>
#include <unordered_map>

namespace arrow {
class MemoryPool;
}  // namespace arrow

namespace bitar {

enum class MemoryPoolBackend : std::uint8_t {
  System,
  Jemalloc,
  Mimalloc,
  HipHost,
  HipDevice,
  Rtemalloc = HipHost,   // reference name (memory_pool.h:65-71)
  Rtememzone = HipDevice
};

struct HipAllocation {
  std::uint8_t* addr;
  std::int64_t size;
  int device;   // -1 for pinned host
  bool device_memory;
};

/// Address -> allocation map of every allocation made through the HIP pools (the
/// RtememzoneAllocatorTracker analogue, memory_pool.h:38-63).  Unlike the reference, every
/// access takes the mutex (Emplace/Of ran unlocked there).
class HipAllocationTracker {
 public:
  /// Exact start-address lookup; false if `addr` is not the start of a tracked allocation.
  bool Of(const std::uint8_t* addr, HipAllocation* out) const;
  [[nodiscard]] std::size_t count() const;
  static HipAllocationTracker* Instance();

  void Emplace(const HipAllocation& a);
  void Release(const std::uint8_t* addr);

 private:
  mutable std::mutex mutex_;
  std::unordered_map<const std::uint8_t*, HipAllocation> allocations_;
};

/// \brief Get the memory pool for the selected backend.  HipDevice allocates on the device
/// selected by SetHipPoolDevice (default 0).
arrow::MemoryPool* GetMemoryPool(MemoryPoolBackend backend);

/// Device ordinal the HipDevice pool allocates on (per thread).
void SetHipPoolDevice(int device);
int HipPoolDevice();

}  // namespace bitar
