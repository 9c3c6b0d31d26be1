// driver.cc -- device discovery and worker -> queue-pair mapping (reference src/driver.cc).
#include "bitar/driver.h"

#include <algorithm>
#include <cstdlib>
#include <sstream>

#include "bitar_hip.h"
#include "hip_ctx.h"

namespace bitar {

namespace {

arrow::Status HasDeviceIds(const std::vector<std::uint8_t>& avail_dev_ids,
                           const std::vector<std::uint8_t>& device_ids) {  // driver.cc:55-73
  std::vector<std::uint8_t> missing;
  for (const auto& id : device_ids) {
    if (std::find(avail_dev_ids.begin(), avail_dev_ids.end(), id) == avail_dev_ids.end())
      missing.push_back(id);
  }
  if (!missing.empty()) {
    std::ostringstream os;
    for (std::size_t i = 0; i < missing.size(); ++i) os << (i ? ", " : "") << +missing[i];
    return arrow::Status::Invalid("Not available device ids: ", os.str());
  }
  return arrow::Status::OK();
}

// Map workers to devices as evenly as possible, each device getting at least one
// (driver.cc:100-116); worker ids play the role of lcore ids (1-based, 0 = main thread).
arrow::Result<std::vector<std::unique_ptr<HipGfx950CompressDevice>>> CreateDevices(
    const std::vector<std::uint8_t>& device_ids, const std::vector<std::uint32_t>& workers) {
  const auto min_per_dev = workers.size() / device_ids.size();
  auto remaining = workers.size() % device_ids.size();
  auto it = workers.begin();
  std::vector<std::unique_ptr<HipGfx950CompressDevice>> devices;
  devices.reserve(device_ids.size());
  for (const auto& id : device_ids) {
    const auto n = min_per_dev + (remaining > 0 ? 1 : 0);
    ARROW_ASSIGN_OR_RAISE(auto* device, DeviceManager::Instance()->Create<Class_HIP_GFX950>(
                                            id, std::vector<std::uint32_t>(it, it + n)));
    devices.emplace_back(device);
    it += static_cast<std::ptrdiff_t>(n);
    if (remaining > 0) --remaining;
  }
  return devices;
}

}  // namespace

template <typename Class, typename Enable>
CompressDriver<Class>* CompressDriver<Class, Enable>::Instance() {
  static CompressDriver<Class> instance;
  return &instance;
}

template <>
arrow::Result<std::vector<std::uint8_t>> CompressDriver<Class_HIP_GFX950>::ListAvailableDeviceIds() {
  int count = 0;
  BITAR_ABI(bitar_hip_device_count(&count), "device count");
  if (count == 0) {
    return arrow::Status::Invalid("No compress device is available with driver name: ",
                                  driver_name());
  }
  std::vector<std::uint8_t> ids(static_cast<std::size_t>(count));
  for (int i = 0; i < count; ++i) ids[static_cast<std::size_t>(i)] = static_cast<std::uint8_t>(i);
  return ids;
}

template <>
arrow::Result<std::vector<std::unique_ptr<HipGfx950CompressDevice>>>
CompressDriver<Class_HIP_GFX950>::GetDevices(const std::vector<std::uint8_t>& device_ids) {
  ARROW_ASSIGN_OR_RAISE(auto avail, ListAvailableDeviceIds());
  ARROW_RETURN_NOT_OK(HasDeviceIds(avail, device_ids));
  if (device_ids.empty()) return arrow::Status::Invalid("No device ids requested");
  std::uint32_t num_workers = num_workers_;
  if (num_workers == 0) {
    const char* env = std::getenv("BITAR_NUM_WORKERS");
    num_workers = env ? static_cast<std::uint32_t>(std::strtoul(env, nullptr, 10)) : 0;
  }
  if (num_workers == 0) num_workers = 4 * static_cast<std::uint32_t>(device_ids.size());
  if (device_ids.size() > num_workers) {
    return arrow::Status::Invalid("The number of devices to set up (", device_ids.size(),
                                  ") is greater than the number of available worker "
                                  "lcores (", num_workers, ").");
  }
  std::vector<std::uint32_t> workers(num_workers);
  for (std::uint32_t i = 0; i < num_workers; ++i) workers[i] = i + 1;
  return CreateDevices(device_ids, workers);
}

template class CompressDriver<Class_HIP_GFX950>;

}  // namespace bitar
