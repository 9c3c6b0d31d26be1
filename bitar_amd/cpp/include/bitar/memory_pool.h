// bitar/memory_pool.h -- arrow::MemoryPool backends (reference src/include/memory_pool.h).
//
// Rtemalloc / Rtememzone (DPDK hugepage memory: host memory the CPU writes and the BlueField
// DMAs from, memory_pool.cc:70-188) become HipHost: pinned host memory (hipHostMalloc), which
// the CPU reads and writes and the GPU's copy engines reach at full link rate.  The reference
// names alias HipHost, so the demo's flow -- fill a memzone buffer on the CPU, Compress,
// Decompress into another, compare on the CPU (demo_app.cc:121-122, 589-592) -- runs
// unchanged.  HipDevice is HBM of the current device (hipMalloc): the fast path, but Arrow's
// PoolBuffer tags every pool allocation with the CPU memory manager, so HipDevice buffers
// report is_cpu() == true although the host must not touch them; bitar::AllocateDeviceBuffer
// (hip_device.h) gives HBM buffers with the kROCM memory manager instead.
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
  Rtemalloc = HipHost,   // reference names (memory_pool.h:65-71): host memory the engine reads
  Rtememzone = HipHost
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

/// Whether this build of the pools writes the debug poison bytes (reference
/// memory_pool.cc:190-263 under `#ifndef NDEBUG`): false for the shipped release libbitar.so,
/// true for the debug variant (lib/debug/libbitar.so).
bool PoolPoisons();

}  // namespace bitar
