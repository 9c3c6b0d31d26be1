// memory_pool.cc -- arrow::MemoryPool backends over HBM and pinned host memory
// (reference src/memory_pool.cc:70-350: RtemallocAllocator / RtememzoneAllocator /
// BaseMemoryPoolImpl / RtememzoneAllocatorTracker / GetMemoryPool).
#include "bitar/memory_pool.h"

#include <arrow/memory_pool.h>
#include <arrow/status.h>
#include <arrow/util/logging.h>

#include <cstdlib>
#include <limits>
#include <mutex>
#include <unordered_map>

#include "hip_ctx.h"

namespace bitar {

namespace internal {

arrow::Result<bitar_hip_ctx*> HelperContext(int device) {
  static std::mutex mu;
  static std::unordered_map<int, bitar_hip_ctx*> ctxs;
  const std::lock_guard<std::mutex> lock(mu);
  auto it = ctxs.find(device);
  if (it != ctxs.end()) return it->second;
  bitar_hip_config cfg{1, 0};
  bitar_hip_ctx* ctx = nullptr;
  BITAR_ABI(bitar_hip_open(device, &cfg, &ctx), "bitar_hip_open");
  ctxs.emplace(device, ctx);
  return ctx;
}

}  // namespace internal

namespace {

thread_local int g_pool_device = 0;

// A static piece of memory for 0-size allocations, so as to return an aligned non-null
// pointer (as the reference does, memory_pool.cc:60-66).
alignas(64) std::int64_t zero_size_area[1] = {0};
std::uint8_t* const kZeroSizeArea = reinterpret_cast<std::uint8_t*>(&zero_size_area);

#ifndef NDEBUG
// Debug builds mark the first and last byte of a fresh allocation, of the grown part of a
// reallocation and (host pool) of a freed buffer, as the reference's pools do
// (memory_pool.cc:190-263), so that reads of uninitialised or freed pool memory show a
// recognisable value.  HBM bytes are written through the ABI's copy on the helper context,
// which no other user of a fresh allocation can race with.  Release builds (-DNDEBUG, the
// shipped libbitar.so) do none of it.
constexpr std::uint8_t kAllocPoison = 0xBC;
constexpr std::uint8_t kReallocPoison = 0xBD;
constexpr std::uint8_t kDeallocPoison = 0xBE;

void PoisonByte(bitar_hip_ctx* ctx, bool device, std::uint8_t* at, std::uint8_t value) {
  if (!device) {
    *at = value;
    return;
  }
  static const std::uint8_t kValues[3] = {kAllocPoison, kReallocPoison, kDeallocPoison};
  const std::uint8_t* src = &kValues[value - kAllocPoison];
  if (bitar_hip_memcpy(ctx, at, src, 1, nullptr) == 0) (void)bitar_hip_sync(ctx, nullptr);
}

void PoisonEnds(bitar_hip_ctx* ctx, bool device, std::uint8_t* lo, std::uint8_t* last,
                std::uint8_t value) {
  PoisonByte(ctx, device, lo, value);
  if (last != lo) PoisonByte(ctx, device, last, value);
}
#endif

template <bool kDevice>
class HipPool : public arrow::MemoryPool {
 public:
  arrow::Status Allocate(int64_t size, int64_t /*alignment: HIP gives >= 256 B*/,
                         uint8_t** out) override {
    if (size < 0) return arrow::Status::Invalid("negative malloc size");
    if (static_cast<std::uint64_t>(size) >= std::numeric_limits<std::size_t>::max())
      return arrow::Status::OutOfMemory("malloc size overflows size_t");
    if (size == 0) {
      *out = kZeroSizeArea;
      return arrow::Status::OK();
    }
    const int device = kDevice ? g_pool_device : 0;
    ARROW_ASSIGN_OR_RAISE(auto* ctx, internal::HelperContext(device));
    void* p = nullptr;
    const int rc = kDevice ? bitar_hip_alloc(ctx, static_cast<uint64_t>(size), &p)
                           : bitar_hip_host_alloc(ctx, static_cast<uint64_t>(size), &p);
    if (rc != 0) return arrow::Status::OutOfMemory("allocation of size ", size, " failed");
    *out = static_cast<uint8_t*>(p);
#ifndef NDEBUG
    PoisonEnds(ctx, kDevice, *out, *out + size - 1, kAllocPoison);
#endif
    HipAllocationTracker::Instance()->Emplace({*out, size, kDevice ? device : -1, kDevice});
    stats_.DidAllocateBytes(size);
    return arrow::Status::OK();
  }

  arrow::Status Reallocate(int64_t old_size, int64_t new_size, int64_t alignment,
                           uint8_t** ptr) override {
    if (new_size < 0) return arrow::Status::Invalid("negative realloc size");
    if (static_cast<std::uint64_t>(new_size) >= std::numeric_limits<std::size_t>::max())
      return arrow::Status::OutOfMemory("realloc overflows size_t");
    uint8_t* prev = *ptr;
    uint8_t* fresh = nullptr;
    ARROW_RETURN_NOT_OK(Allocate(new_size, alignment, &fresh));
    const int64_t keep = std::min(old_size, new_size);
    if (keep > 0 && prev != kZeroSizeArea) {
      HipAllocation a{};
      const int device = HipAllocationTracker::Instance()->Of(prev, &a) ? a.device : 0;
      ARROW_ASSIGN_OR_RAISE(auto* ctx, internal::HelperContext(device < 0 ? 0 : device));
      BITAR_ABI(bitar_hip_memcpy(ctx, fresh, prev, static_cast<uint64_t>(keep), nullptr),
                "realloc copy");
      BITAR_ABI(bitar_hip_sync(ctx, nullptr), "realloc sync");
    }
#ifndef NDEBUG
    if (new_size > old_size) {
      ARROW_ASSIGN_OR_RAISE(auto* ctx, internal::HelperContext(kDevice ? g_pool_device : 0));
      PoisonEnds(ctx, kDevice, fresh + old_size, fresh + new_size - 1, kReallocPoison);
    }
#endif
    Free(prev, old_size, alignment);
    *ptr = fresh;
    return arrow::Status::OK();
  }

  void Free(uint8_t* buffer, int64_t size, int64_t /*alignment*/) override {
    if (buffer == kZeroSizeArea || buffer == nullptr) return;
    HipAllocation a{};
    const bool known = HipAllocationTracker::Instance()->Of(buffer, &a);
    const int device = known && a.device >= 0 ? a.device : 0;
    auto ctx = internal::HelperContext(device);
    if (ctx.ok()) {
#ifndef NDEBUG
      // (host memory only: HBM is returned to the driver right away, and a copy on the helper
      // context's stream would not be ordered after work still queued on a queue pair's
      // stream that reads the buffer)
      if (!kDevice && size > 0) PoisonEnds(*ctx, kDevice, buffer, buffer + size - 1, kDeallocPoison);
#endif
      if (kDevice) (void)bitar_hip_free(*ctx, buffer);
      else (void)bitar_hip_host_free(*ctx, buffer);
    }
    HipAllocationTracker::Instance()->Release(buffer);
    stats_.DidFreeBytes(size);
  }

  int64_t bytes_allocated() const override { return stats_.bytes_allocated(); }
  int64_t max_memory() const override { return stats_.max_memory(); }
  int64_t total_bytes_allocated() const override { return stats_.total_bytes_allocated(); }
  int64_t num_allocations() const override { return stats_.num_allocations(); }
  std::string backend_name() const override { return kDevice ? "hip_device" : "hip_host"; }

 private:
  arrow::internal::MemoryPoolStats stats_;
};

}  // namespace

bool HipAllocationTracker::Of(const std::uint8_t* addr, HipAllocation* out) const {
  const std::lock_guard<std::mutex> lock(mutex_);
  auto it = allocations_.find(addr);
  if (it == allocations_.end()) return false;
  if (out) *out = it->second;
  return true;
}

std::size_t HipAllocationTracker::count() const {
  const std::lock_guard<std::mutex> lock(mutex_);
  return allocations_.size();
}

HipAllocationTracker* HipAllocationTracker::Instance() {
  static HipAllocationTracker instance;
  return &instance;
}

void HipAllocationTracker::Emplace(const HipAllocation& a) {
  const std::lock_guard<std::mutex> lock(mutex_);
  allocations_[a.addr] = a;
}

void HipAllocationTracker::Release(const std::uint8_t* addr) {
  const std::lock_guard<std::mutex> lock(mutex_);
  allocations_.erase(addr);
}

bool PoolPoisons() {
#ifndef NDEBUG
  return true;
#else
  return false;
#endif
}

void SetHipPoolDevice(int device) { g_pool_device = device; }
int HipPoolDevice() { return g_pool_device; }

arrow::MemoryPool* GetMemoryPool(MemoryPoolBackend backend) {
  arrow::MemoryPool* out = nullptr;
  switch (backend) {
    case MemoryPoolBackend::System:
      return arrow::system_memory_pool();
    case MemoryPoolBackend::Jemalloc:
      if (arrow::jemalloc_memory_pool(&out).ok()) return out;
      return arrow::default_memory_pool();
    case MemoryPoolBackend::Mimalloc:
      if (arrow::mimalloc_memory_pool(&out).ok()) return out;
      return arrow::default_memory_pool();
    case MemoryPoolBackend::HipHost: {
      static HipPool<false> host_pool;
      return &host_pool;
    }
    case MemoryPoolBackend::HipDevice: {
      static HipPool<true> device_pool;
      return &device_pool;
    }
  }
  ARROW_LOG(FATAL) << "Internal error: unimplemented memory pool";
  return nullptr;
}

}  // namespace bitar
