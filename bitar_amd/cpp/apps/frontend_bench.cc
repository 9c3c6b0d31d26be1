// frontend_bench.cc -- throughput THROUGH the drop-in C++ API (namespace bitar): what a
// reference user measures with demo_app's EvaluateSync (reference apps/demo_app.cc:332-357,
// PrintPerfNumbers 82-89), as one JSON line for bench.py.
//
//   frontend_bench [--bytes N] [--seg N] [--kind K] [--codec lz4|deflate|zstd]
//                  [--steps K] [--warmup W] [--no-host]
//
// Leg "frontend": an HBM-resident arrow::Buffer of N bytes (the synthetic input of kind K,
// generated on the device), K timed round trips of CompressDevice::Compress (qp 0) +
// Decompress (qp 0, into an HBM ResizableBuffer) + Recycle, each phase timed on the host
// clock; the output is compared with the input once after the loop.
// Leg "h2d_d2h": the same round trip with HOST-resident data (pinned HipHost pool buffers):
// Compress stages the input to HBM, Decompress stages the output back -- the PCIe-inclusive
// rate -- plus the raw 1-way copy rates of the link for the same byte count.
#include <arrow/api.h>
#include <arrow/buffer.h>
#include <arrow/memory_pool.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "bitar/bitar.h"
#include "bitar_hip.h"

namespace {

using Clock = std::chrono::steady_clock;
using Device = bitar::CompressDevice<bitar::Class_HIP_GFX950>;

double Secs(Clock::time_point a, Clock::time_point b) {
  return std::chrono::duration<double>(b - a).count();
}

[[noreturn]] void Die(const std::string& what, const arrow::Status& st) {
  std::fprintf(stderr, "frontend_bench: %s: %s\n", what.c_str(), st.ToString().c_str());
  std::exit(1);
}
#define OK_OR_DIE(expr, what)        \
  do {                               \
    auto _s = (expr);                \
    if (!_s.ok()) Die((what), _s);   \
  } while (0)

struct Times {
  double comp = 0, dec = 0, rec = 0, total = 0;
  double best_total = 1e30;
};

// K timed round trips of Compress + Decompress + Recycle (W untimed first)
Times RoundTrips(Device& d, const std::shared_ptr<arrow::Buffer>& in,
                 const std::unique_ptr<arrow::ResizableBuffer>& out, int steps, int warmup,
                 double* ratio) {
  Times t;
  for (int s = 0; s < warmup + steps; ++s) {
    const auto t0 = Clock::now();
    auto comp = d.Compress(0, in);
    const auto t1 = Clock::now();
    OK_OR_DIE(comp.status(), "Compress");
    OK_OR_DIE(d.Decompress(0, *comp, out), "Decompress");
    const auto t2 = Clock::now();
    if (s == 0) {
      int64_t c = 0;
      for (const auto& b : *comp) c += b->size();
      *ratio = static_cast<double>(in->size()) / static_cast<double>(c);
    }
    const size_t back = d.Recycle(*comp);
    const auto t3 = Clock::now();
    if (back != comp->size()) {
      std::fprintf(stderr, "frontend_bench: Recycle returned %zu of %zu\n", back, comp->size());
      std::exit(1);
    }
    if (s >= warmup) {
      t.comp += Secs(t0, t1);
      t.dec += Secs(t1, t2);
      t.rec += Secs(t2, t3);
      t.total += Secs(t0, t3);
      t.best_total = std::min(t.best_total, Secs(t0, t3));
    }
  }
  t.comp /= steps;
  t.dec /= steps;
  t.rec /= steps;
  t.total /= steps;
  return t;
}

std::string Json(const char* name, const Times& t, int64_t n, double ratio) {
  const double gib = static_cast<double>(n) / (1u << 30);
  char buf[1024];
  std::snprintf(buf, sizeof buf,
                "\"%s\": {\"roundtrip_gibs\": %.3f, \"best_roundtrip_gibs\": %.3f, "
                "\"compress_call_ms\": %.4f, \"decompress_call_ms\": %.4f, "
                "\"recycle_call_ms\": %.4f, \"ms_per_roundtrip\": %.4f, \"ratio\": %.4f}",
                name, gib / t.total, gib / t.best_total, t.comp * 1e3, t.dec * 1e3, t.rec * 1e3,
                t.total * 1e3, ratio);
  return buf;
}

}  // namespace

int main(int argc, char** argv) {
  int64_t n = int64_t{1} << 30;
  uint32_t seg = 65536;
  int kind = 1, steps = 10, warmup = 3;
  bool host = true;
  std::string codec = "lz4";
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&]() { return i + 1 < argc ? std::string(argv[++i]) : std::string(); };
    if (a == "--bytes") n = std::stoll(next());
    else if (a == "--seg") seg = static_cast<uint32_t>(std::stoul(next()));
    else if (a == "--kind") kind = std::stoi(next());
    else if (a == "--steps") steps = std::stoi(next());
    else if (a == "--warmup") warmup = std::stoi(next());
    else if (a == "--codec") codec = next();
    else if (a == "--no-host") host = false;
    else {
      std::fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  const uint64_t nseg = (static_cast<uint64_t>(n) + seg - 1) / seg;

  auto* driver = bitar::CompressDriver<bitar::Class_HIP_GFX950>::Instance();
  auto ids = driver->ListAvailableDeviceIds();
  OK_OR_DIE(ids.status(), "ListAvailableDeviceIds");
  if (ids->empty()) Die("devices", arrow::Status::Invalid("no gfx950 device"));
  driver->set_num_workers(1);  // one queue pair
  auto devs = driver->GetDevices({(*ids)[0]});
  OK_OR_DIE(devs.status(), "GetDevices");
  Device& d = *(*devs)[0];
  auto cfg = std::make_unique<bitar::HipConfiguration>(bitar::HipConfiguration::Defaults());
  cfg->set_codec(codec == "zstd" ? bitar::Codec::ZSTD
                 : codec == "deflate" ? bitar::Codec::DEFLATE : bitar::Codec::LZ4);
  cfg->set_decompressed_seg_size32(seg);
  // the slot pool holds a whole call's outputs from the start (no critical-path growth)
  cfg->set_max_preallocate_memzones(
      static_cast<uint16_t>(std::min<uint64_t>(nseg, bitar::internal::kMaxPreallocateSlots)));
  OK_OR_DIE(d.Initialize(std::move(cfg)), "Initialize");

  // HBM input generated on the device through the C ABI (same generator as bench.py)
  bitar_hip_config hc{1, 0};
  bitar_hip_ctx* ctx = nullptr;
  if (bitar_hip_open((*ids)[0], &hc, &ctx) != 0) Die("bitar_hip_open", arrow::Status::IOError(bitar_hip_last_error()));
  auto din = bitar::AllocateDeviceBuffer(n, (*ids)[0]);
  OK_OR_DIE(din.status(), "AllocateDeviceBuffer");
  std::shared_ptr<arrow::Buffer> in = std::move(*din);
  if (bitar_hip_fill(ctx, nullptr, kind, 0, reinterpret_cast<void*>(in->address()), n) != 0 ||
      bitar_hip_sync(ctx, nullptr) != 0)
    Die("fill", arrow::Status::IOError(bitar_hip_last_error()));
  auto dout = bitar::AllocateResizableDeviceBuffer(static_cast<int64_t>(nseg * seg), (*ids)[0]);
  OK_OR_DIE(dout.status(), "AllocateResizableDeviceBuffer");
  std::unique_ptr<arrow::ResizableBuffer> out = std::move(*dout);

  double ratio = 0;
  const Times dev_t = RoundTrips(d, in, out, steps, warmup, &ratio);
  // byte equality of the last round trip (host copies of both, once)
  std::vector<uint8_t> a(n), b(n);
  if (bitar_hip_memcpy(ctx, a.data(), reinterpret_cast<const void*>(in->address()), n, nullptr) ||
      bitar_hip_memcpy(ctx, b.data(), reinterpret_cast<const void*>(out->address()), n, nullptr) ||
      bitar_hip_sync(ctx, nullptr))
    Die("readback", arrow::Status::IOError(bitar_hip_last_error()));
  const bool ok = out->size() == n && std::memcmp(a.data(), b.data(), n) == 0;

  std::string line = "{\"workload\": \"CompressDevice<Class_HIP_GFX950>::Compress + Decompress "
                     "+ Recycle on queue pair 0, " + codec + ", " + std::to_string(seg) +
                     "-B segments, kind " + std::to_string(kind) + ", " + std::to_string(n) +
                     " B\", \"bytes\": " + std::to_string(n) + ", \"segments\": " +
                     std::to_string(nseg) + ", \"steps\": " + std::to_string(steps) +
                     ", \"roundtrip_ok\": " + (ok ? "true" : "false") + ", " +
                     Json("hbm", dev_t, n, ratio);

  if (host) {
    // pinned host input / output (the HipHost pool: the reference's Rtemalloc analogue)
    auto* hpool = bitar::GetMemoryPool(bitar::MemoryPoolBackend::HipHost);
    auto hin = arrow::AllocateBuffer(n, hpool);
    OK_OR_DIE(hin.status(), "host input");
    std::memcpy((*hin)->mutable_data(), a.data(), n);
    std::shared_ptr<arrow::Buffer> host_in = std::move(*hin);
    auto hout = arrow::AllocateResizableBuffer(static_cast<int64_t>(nseg * seg), hpool);
    OK_OR_DIE(hout.status(), "host output");
    std::unique_ptr<arrow::ResizableBuffer> host_out = std::move(*hout);
    double r2 = 0;
    const Times host_t = RoundTrips(d, host_in, host_out, std::max(2, steps / 3), 1, &r2);
    const bool ok2 = host_out->size() == n && std::memcmp(host_out->data(), a.data(), n) == 0;
    // the link alone: one-way copies of the same n bytes, pinned host <-> HBM
    double h2d = 1e30, d2h = 1e30;
    for (int r = 0; r < 3; ++r) {
      auto t0 = Clock::now();
      if (bitar_hip_memcpy(ctx, reinterpret_cast<void*>(in->address()), host_in->data(), n, nullptr) ||
          bitar_hip_sync(ctx, nullptr))
        Die("h2d", arrow::Status::IOError(bitar_hip_last_error()));
      auto t1 = Clock::now();
      if (bitar_hip_memcpy(ctx, host_out->mutable_data(), reinterpret_cast<const void*>(in->address()), n, nullptr) ||
          bitar_hip_sync(ctx, nullptr))
        Die("d2h", arrow::Status::IOError(bitar_hip_last_error()));
      auto t2 = Clock::now();
      h2d = std::min(h2d, Secs(t0, t1));
      d2h = std::min(d2h, Secs(t1, t2));
    }
    const double gib = static_cast<double>(n) / (1u << 30);
    char buf[256];
    std::snprintf(buf, sizeof buf,
                  ", \"host_roundtrip_ok\": %s, \"h2d_gibs\": %.3f, \"d2h_gibs\": %.3f, "
                  "\"h2d_ms\": %.3f, \"d2h_ms\": %.3f",
                  ok2 ? "true" : "false", gib / h2d, gib / d2h, h2d * 1e3, d2h * 1e3);
    line += ", " + Json("host", host_t, n, r2) + buf;
  }
  line += "}";
  std::printf("%s\n", line.c_str());
  bitar_hip_close(ctx);
  return ok ? 0 : 1;
}
