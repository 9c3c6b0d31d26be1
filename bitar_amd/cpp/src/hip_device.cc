// hip_device.cc -- arrow::Device / MemoryManager for MI355X HBM (see bitar/hip_device.h).
#include "bitar/hip_device.h"

#include <arrow/memory_pool.h>

#include <mutex>
#include <unordered_map>

#include "bitar/memory_pool.h"
#include "hip_ctx.h"

namespace bitar {

namespace {

// An owning HBM buffer tied to a HipMemoryManager.
class HipBuffer : public arrow::ResizableBuffer {
 public:
  HipBuffer(std::shared_ptr<HipMemoryManager> mm, bitar_hip_ctx* ctx)
      : arrow::ResizableBuffer(nullptr, 0, mm), ctx_(ctx) {}
  ~HipBuffer() override {
    if (data_) (void)bitar_hip_free(ctx_, const_cast<uint8_t*>(data_));
  }

  arrow::Status Reserve(const int64_t new_capacity) override {
    if (new_capacity <= capacity_) return arrow::Status::OK();
    void* p = nullptr;
    BITAR_ABI(bitar_hip_alloc(ctx_, static_cast<uint64_t>(new_capacity), &p), "hip alloc");
    if (size_ > 0) {
      BITAR_ABI(bitar_hip_memcpy(ctx_, p, data_, static_cast<uint64_t>(size_), nullptr), "copy");
      BITAR_ABI(bitar_hip_sync(ctx_, nullptr), "sync");
    }
    if (data_) (void)bitar_hip_free(ctx_, const_cast<uint8_t*>(data_));
    data_ = static_cast<uint8_t*>(p);
    capacity_ = new_capacity;
    return arrow::Status::OK();
  }

  arrow::Status Resize(const int64_t new_size, bool /*shrink_to_fit*/) override {
    if (new_size < 0) return arrow::Status::Invalid("negative buffer resize");
    ARROW_RETURN_NOT_OK(Reserve(new_size));
    size_ = new_size;
    return arrow::Status::OK();
  }

 private:
  bitar_hip_ctx* ctx_;
};

arrow::Result<std::unique_ptr<HipBuffer>> MakeHipBuffer(int64_t size, int device_id) {
  ARROW_ASSIGN_OR_RAISE(auto* ctx, internal::HelperContext(device_id));
  auto buf = std::make_unique<HipBuffer>(hip_memory_manager(device_id), ctx);
  ARROW_RETURN_NOT_OK(buf->Resize(size, false));
  return buf;
}

}  // namespace

std::shared_ptr<HipDevice> HipDevice::Make(int device_id) {
  static std::mutex mu;
  static std::unordered_map<int, std::shared_ptr<HipDevice>> devices;
  const std::lock_guard<std::mutex> lock(mu);
  auto& d = devices[device_id];
  if (!d) d = std::make_shared<HipDevice>(device_id);
  return d;
}

std::string HipDevice::ToString() const {
  return "HipDevice(gfx950, id=" + std::to_string(device_id_) + ")";
}

bool HipDevice::Equals(const arrow::Device& other) const {
  return other.device_type() == device_type() && other.device_id() == device_id_;
}

std::shared_ptr<arrow::MemoryManager> HipDevice::default_memory_manager() {
  return hip_memory_manager(device_id_);
}

std::shared_ptr<HipMemoryManager> hip_memory_manager(int device_id) {
  static std::mutex mu;
  static std::unordered_map<int, std::shared_ptr<HipMemoryManager>> mms;
  const std::lock_guard<std::mutex> lock(mu);
  auto& m = mms[device_id];
  if (!m) m = std::make_shared<HipMemoryManager>(HipDevice::Make(device_id));
  return m;
}

arrow::Result<std::shared_ptr<arrow::io::RandomAccessFile>> HipMemoryManager::GetBufferReader(
    std::shared_ptr<arrow::Buffer>) {
  return arrow::Status::NotImplemented("HBM buffers are not host-readable; copy to CPU first");
}

arrow::Result<std::shared_ptr<arrow::io::OutputStream>> HipMemoryManager::GetBufferWriter(
    std::shared_ptr<arrow::Buffer>) {
  return arrow::Status::NotImplemented("HBM buffers are not host-writable");
}

arrow::Result<std::unique_ptr<arrow::Buffer>> HipMemoryManager::AllocateBuffer(int64_t size) {
  ARROW_ASSIGN_OR_RAISE(auto b, MakeHipBuffer(size, device_id()));
  return std::unique_ptr<arrow::Buffer>(std::move(b));
}

arrow::Result<std::shared_ptr<arrow::Buffer>> HipMemoryManager::CopyBufferFrom(
    const std::shared_ptr<arrow::Buffer>& buf, const std::shared_ptr<arrow::MemoryManager>& from) {
  ARROW_ASSIGN_OR_RAISE(auto b, CopyNonOwnedFrom(*buf, from));
  return std::shared_ptr<arrow::Buffer>(std::move(b));
}

arrow::Result<std::shared_ptr<arrow::Buffer>> HipMemoryManager::CopyBufferTo(
    const std::shared_ptr<arrow::Buffer>& buf, const std::shared_ptr<arrow::MemoryManager>& to) {
  ARROW_ASSIGN_OR_RAISE(auto b, CopyNonOwnedTo(*buf, to));
  if (!b) return std::shared_ptr<arrow::Buffer>();
  return std::shared_ptr<arrow::Buffer>(std::move(b));
}

arrow::Result<std::unique_ptr<arrow::Buffer>> HipMemoryManager::CopyNonOwnedFrom(
    const arrow::Buffer& buf, const std::shared_ptr<arrow::MemoryManager>& from) {
  if (!from->is_cpu() && from->device()->device_type() != arrow::DeviceAllocationType::kROCM)
    return std::unique_ptr<arrow::Buffer>();
  ARROW_ASSIGN_OR_RAISE(auto dst, MakeHipBuffer(buf.size(), device_id()));
  ARROW_ASSIGN_OR_RAISE(auto* ctx, internal::HelperContext(device_id()));
  BITAR_ABI(bitar_hip_memcpy(ctx, reinterpret_cast<void*>(dst->mutable_address()),
                             reinterpret_cast<const void*>(buf.address()),
                             static_cast<uint64_t>(buf.size()), nullptr),
            "copy to HBM");
  BITAR_ABI(bitar_hip_sync(ctx, nullptr), "sync");
  return std::unique_ptr<arrow::Buffer>(std::move(dst));
}

arrow::Result<std::unique_ptr<arrow::Buffer>> HipMemoryManager::CopyNonOwnedTo(
    const arrow::Buffer& buf, const std::shared_ptr<arrow::MemoryManager>& to) {
  if (!to->is_cpu()) return std::unique_ptr<arrow::Buffer>();
  ARROW_ASSIGN_OR_RAISE(auto dst, to->AllocateBuffer(buf.size()));
  ARROW_ASSIGN_OR_RAISE(auto* ctx, internal::HelperContext(device_id()));
  BITAR_ABI(bitar_hip_memcpy(ctx, dst->mutable_data(), reinterpret_cast<const void*>(buf.address()),
                             static_cast<uint64_t>(buf.size()), nullptr),
            "copy to host");
  BITAR_ABI(bitar_hip_sync(ctx, nullptr), "sync");
  return dst;
}

arrow::Result<std::unique_ptr<arrow::Buffer>> AllocateDeviceBuffer(int64_t size, int device_id) {
  ARROW_ASSIGN_OR_RAISE(auto b, MakeHipBuffer(size, device_id));
  return std::unique_ptr<arrow::Buffer>(std::move(b));
}

arrow::Result<std::unique_ptr<arrow::ResizableBuffer>> AllocateResizableDeviceBuffer(
    int64_t capacity, int device_id) {
  ARROW_ASSIGN_OR_RAISE(auto b, MakeHipBuffer(0, device_id));
  ARROW_RETURN_NOT_OK(b->Reserve(capacity));
  return std::unique_ptr<arrow::ResizableBuffer>(std::move(b));
}

}  // namespace bitar
