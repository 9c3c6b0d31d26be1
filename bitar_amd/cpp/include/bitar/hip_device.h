// bitar/hip_device.h -- arrow::Device / arrow::MemoryManager for MI355X HBM.
//
// Buffers tied to HipMemoryManager report is_cpu() == false and
// device_type() == DeviceAllocationType::kROCM, so Arrow code never dereferences HBM on the
// host; arrow::Buffer::Copy(buf, arrow::default_cpu_memory_manager()) brings one back.
#pragma once

#include <arrow/buffer.h>
#include <arrow/device.h>
#include <arrow/result.h>

#include <memory>
#include <string>

namespace bitar {

class HipDevice : public arrow::Device {
 public:
  static std::shared_ptr<HipDevice> Make(int device_id);

  const char* type_name() const override { return "hip_gfx950"; }
  std::string ToString() const override;
  bool Equals(const arrow::Device& other) const override;
  int64_t device_id() const override { return device_id_; }
  arrow::DeviceAllocationType device_type() const override {
    return arrow::DeviceAllocationType::kROCM;
  }
  std::shared_ptr<arrow::MemoryManager> default_memory_manager() override;

  explicit HipDevice(int device_id) : arrow::Device(/*is_cpu=*/false), device_id_(device_id) {}

 private:
  int device_id_;
  std::weak_ptr<arrow::MemoryManager> mm_;
};

class HipMemoryManager : public arrow::MemoryManager {
 public:
  explicit HipMemoryManager(const std::shared_ptr<arrow::Device>& device)
      : arrow::MemoryManager(device) {}

  int device_id() const { return static_cast<int>(device()->device_id()); }

  arrow::Result<std::shared_ptr<arrow::io::RandomAccessFile>> GetBufferReader(
      std::shared_ptr<arrow::Buffer> buf) override;
  arrow::Result<std::shared_ptr<arrow::io::OutputStream>> GetBufferWriter(
      std::shared_ptr<arrow::Buffer> buf) override;
  /// HBM allocation, freed with the buffer.
  arrow::Result<std::unique_ptr<arrow::Buffer>> AllocateBuffer(int64_t size) override;

 protected:
  arrow::Result<std::shared_ptr<arrow::Buffer>> CopyBufferFrom(
      const std::shared_ptr<arrow::Buffer>& buf,
      const std::shared_ptr<arrow::MemoryManager>& from) override;
  arrow::Result<std::shared_ptr<arrow::Buffer>> CopyBufferTo(
      const std::shared_ptr<arrow::Buffer>& buf,
      const std::shared_ptr<arrow::MemoryManager>& to) override;
  arrow::Result<std::unique_ptr<arrow::Buffer>> CopyNonOwnedFrom(
      const arrow::Buffer& buf, const std::shared_ptr<arrow::MemoryManager>& from) override;
  arrow::Result<std::unique_ptr<arrow::Buffer>> CopyNonOwnedTo(
      const arrow::Buffer& buf, const std::shared_ptr<arrow::MemoryManager>& to) override;
};

/// The memory manager of device `device_id` (one per device, process-wide).
std::shared_ptr<HipMemoryManager> hip_memory_manager(int device_id);

/// HBM buffer on `device_id` (is_cpu() == false).
arrow::Result<std::unique_ptr<arrow::Buffer>> AllocateDeviceBuffer(int64_t size, int device_id);

/// Resizable HBM buffer on `device_id`: the decompression target of CompressDevice::Decompress
/// when the output should stay in HBM.
arrow::Result<std::unique_ptr<arrow::ResizableBuffer>> AllocateResizableDeviceBuffer(
    int64_t capacity, int device_id);

}  // namespace bitar
