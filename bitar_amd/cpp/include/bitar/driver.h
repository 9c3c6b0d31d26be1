// bitar/driver.h -- device discovery (reference src/include/driver.h:36-68).
#pragma once

#include <arrow/result.h>

#include <cstdint>
#include <memory>
#include <vector>

#include "bitar/config.h"
#include "bitar/device.h"

namespace bitar {

template <typename Class,
          typename = internal::IsEnumConstant<internal::DriverClass, Class>>
class CompressDriver {
 public:
  CompressDriver(const CompressDriver&) = delete;
  CompressDriver& operator=(const CompressDriver&) = delete;

  /// \brief Return the global CompressDriver instance of the type.
  static CompressDriver<Class>* Instance();

  /// \brief Devices for \p device_ids.  The worker count (the reference's
  /// rte_lcore_count() - 1, driver.cc:199) is set_num_workers() or BITAR_NUM_WORKERS
  /// (default: 4 per requested device); workers are spread over the devices as evenly as
  /// possible, each device getting one queue pair per worker (driver.cc:100-157).
  arrow::Result<std::vector<std::unique_ptr<CompressDevice<Class>>>> GetDevices(
      const std::vector<std::uint8_t>& device_ids);

  /// \brief All gfx950 devices on this machine.
  arrow::Result<std::vector<std::uint8_t>> ListAvailableDeviceIds();

  void set_num_workers(std::uint32_t n) { num_workers_ = n; }

 protected:
  [[nodiscard]] static const char* driver_name() noexcept { return "HIP_GFX950"; }

 private:
  CompressDriver() = default;
  ~CompressDriver() = default;
  std::uint32_t num_workers_ = 0;
};

}  // namespace bitar
