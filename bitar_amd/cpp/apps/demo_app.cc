// demo_app.cc -- the bitar demo/benchmark harness on MI355X (reference apps/demo_app.cc).
//
//   demo_app --file|-f PATH [--bytes|-b N] [--mode|-m 0|1] [--codec deflate|lz4|zstd]
//            [--seg N] [--devices N] [--workers N] [--ipc-codec none|zstd|lz4]
//   demo_app --synthetic N ...      (no file: N bytes of a generated mixed buffer)
//
// ReadData (demo_app.cc:295-330):
//   mode 0 (raw)      the first --bytes of the file (ReadRawData, demo_app.cc:113-140);
//   mode 1 (content)  a .parquet (parquet::arrow reader) or .feather (ipc::feather reader)
//                     table, serialized to an Arrow IPC stream (SerializeTable,
//                     demo_app.cc:142-195) -- optionally with the body compression the
//                     reference leaves commented out (demo_app.cc:148-150), here the GPU
//                     codec adapter (--ipc-codec) -- checked by deserializing it back
//                     (DeserializeTable, demo_app.cc:236-250) and cut to --bytes.
// then the reference's two flows:
//   EvaluateSync  (demo_app.cc:487-546): Compress -> Decompress -> memcmp on device 0,
//                 kNumTests times each;
//   EvaluateAsync (demo_app.cc:548-693): the input split into one part per (device, queue
//                 pair), dealt round-robin (Advance, demo_app.cc:249-256); CompressAsync on
//                 every worker, WaitLcore, DecompressAsync, WaitLcore, per-part memcmp;
// printing "Duration / Throughput (Gbps)" like PrintPerfNumbers (demo_app.cc:82-89).
#include <arrow/api.h>
#include <arrow/buffer.h>
#include <arrow/io/file.h>
#include <arrow/io/memory.h>
#include <arrow/ipc/api.h>
#include <arrow/ipc/feather.h>
#include <arrow/memory_pool.h>
#include <parquet/arrow/reader.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "bitar/bitar.h"

namespace {

constexpr int kNumTests = 3;  // demo_app.h:45
using Clock = std::chrono::steady_clock;
using Device = bitar::CompressDevice<bitar::Class_HIP_GFX950>;

void PrintPerfNumbers(int64_t total_bytes, Clock::time_point start,
                      Clock::time_point end = Clock::now()) {
  const double s = std::chrono::duration<double>(end - start).count();
  std::printf("-> Duration: %.2f microseconds\t\tThroughput: %.2f Gbps\n", s * 1e6,
              static_cast<double>(total_bytes) * 8 / 1e9 / s);
}

void PrintHeader(const std::string& s) {
  std::printf("\n================================================================\n%s\n"
              "================================================================\n",
              s.c_str());
}

bool EndsWith(const std::string& s, const std::string& suf) {
  return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}

int64_t BytesToRead(int64_t want, int64_t max) { return want <= 0 ? max : std::min(want, max); }

std::shared_ptr<arrow::Buffer> Synthetic(int64_t n) {  // 1/3 small ints, 1/3 text, 1/3 random
  auto buf = *arrow::AllocateBuffer(n);
  uint8_t* v = buf->mutable_data();
  uint64_t x = 0x9E3779B97F4A7C15ull;
  const char* text = "2026-10-15 12:00:00.000 INFO device qp=3 seg=59460 status=OK\n";
  const size_t tl = std::strlen(text);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t region = (i >> 20) % 3;
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    v[i] = region == 0 ? ((i & 7) == 0 ? static_cast<uint8_t>(x % 100) : 0)
           : region == 1 ? static_cast<uint8_t>(text[i % tl]) : static_cast<uint8_t>(x);
  }
  return std::shared_ptr<arrow::Buffer>(std::move(buf));
}

arrow::Result<std::shared_ptr<arrow::Buffer>> SerializeTable(
    const std::shared_ptr<arrow::Table>& table, const std::string& ipc_codec) {
  auto opts = arrow::ipc::IpcWriteOptions::Defaults();
  if (ipc_codec == "zstd" || ipc_codec == "lz4") {
    ARROW_ASSIGN_OR_RAISE(auto codec, bitar::MakeArrowCodec(ipc_codec == "zstd"
                                                                 ? arrow::Compression::ZSTD
                                                                 : arrow::Compression::LZ4_FRAME));
    opts.codec = std::shared_ptr<arrow::util::Codec>(std::move(codec));
  }
  std::shared_ptr<arrow::Buffer> out;
  for (int t = 0; t < kNumTests; ++t) {
    ARROW_ASSIGN_OR_RAISE(auto sink, arrow::io::BufferOutputStream::Create());
    ARROW_ASSIGN_OR_RAISE(auto writer, arrow::ipc::MakeStreamWriter(sink, table->schema(), opts));
    const auto start = Clock::now();
    ARROW_RETURN_NOT_OK(writer->WriteTable(*table));
    ARROW_RETURN_NOT_OK(writer->Close());
    ARROW_ASSIGN_OR_RAISE(out, sink->Finish());
    PrintPerfNumbers(out->size(), start);
  }
  std::printf("Compression type for serialization: %s\n",
              opts.codec ? opts.codec->name().c_str() : "uncompressed");
  return out;
}

arrow::Status DeserializeTable(const std::shared_ptr<arrow::Buffer>& buffer,
                               const std::shared_ptr<arrow::Table>& expect) {
  PrintHeader("Deserialize Table (buffer_size: " + std::to_string(buffer->size()) + ")");
  for (int t = 0; t < kNumTests; ++t) {
    ARROW_ASSIGN_OR_RAISE(auto reader, arrow::ipc::RecordBatchStreamReader::Open(
                                           std::make_shared<arrow::io::BufferReader>(buffer)));
    const auto start = Clock::now();
    ARROW_ASSIGN_OR_RAISE(auto table, reader->ToTable());
    PrintPerfNumbers(buffer->size(), start);
    if (!table->Equals(*expect)) return arrow::Status::Invalid("IPC round trip changed the table");
  }
  return arrow::Status::OK();
}

arrow::Result<std::shared_ptr<arrow::Buffer>> ReadData(const std::string& path, int mode,
                                                       int64_t want, const std::string& ipc_codec) {
  PrintHeader("Serialize Data (num_bytes_want: " + std::to_string(want) + ", mode: " +
              (mode ? "kContent" : "kRaw") + ", file: '" + path + "')");
  ARROW_ASSIGN_OR_RAISE(auto file, arrow::io::MemoryMappedFile::Open(path, arrow::io::FileMode::READ));
  ARROW_ASSIGN_OR_RAISE(const int64_t size, file->GetSize());
  if (mode == 0) {
    const int64_t n = BytesToRead(want, size);
    ARROW_ASSIGN_OR_RAISE(auto buf, arrow::AllocateBuffer(n));
    for (int t = 0; t < kNumTests; ++t) {
      const auto start = Clock::now();
      ARROW_ASSIGN_OR_RAISE(const int64_t got, file->ReadAt(0, n, buf->mutable_data()));
      if (got != n) return arrow::Status::IOError("Unable to read ", n, " bytes from file");
      PrintPerfNumbers(n, start);
    }
    std::printf("Read raw file %lld bytes out of a total %lld bytes\n",
                static_cast<long long>(n), static_cast<long long>(size));
    return std::shared_ptr<arrow::Buffer>(std::move(buf));
  }
  std::shared_ptr<arrow::Table> table;
  if (EndsWith(path, ".parquet")) {
    std::unique_ptr<parquet::arrow::FileReader> reader;
    ARROW_ASSIGN_OR_RAISE(reader, parquet::arrow::OpenFile(file, arrow::default_memory_pool()));
    ARROW_ASSIGN_OR_RAISE(table, reader->ReadTable());
  } else if (EndsWith(path, ".feather")) {
    ARROW_ASSIGN_OR_RAISE(auto reader, arrow::ipc::feather::Reader::Open(file));
    ARROW_RETURN_NOT_OK(reader->Read(&table));
  } else {
    return arrow::Status::Invalid("Unsupported file type: kContent mode only supports "
                                  "'.parquet' or '.feather' file as input");
  }
  ARROW_ASSIGN_OR_RAISE(auto buffer, SerializeTable(table, ipc_codec));
  ARROW_RETURN_NOT_OK(DeserializeTable(buffer, table));
  const int64_t n = BytesToRead(want, buffer->size());
  std::printf("Read serialized table %lld bytes out of a total %lld bytes\n",
              static_cast<long long>(n), static_cast<long long>(buffer->size()));
  return arrow::SliceBuffer(buffer, 0, n);
}

// Compress -> Decompress -> memcmp on device 0, queue pair 0 (demo_app.cc:487-546)
arrow::Status EvaluateSync(const std::unique_ptr<Device>& dev, int device_id,
                           const std::shared_ptr<arrow::Buffer>& host, uint32_t seg) {
  PrintHeader("Evaluate Sync (" + std::to_string(host->size()) + " bytes)");
  ARROW_ASSIGN_OR_RAISE(auto in, arrow::Buffer::Copy(host, bitar::hip_memory_manager(device_id)));
  const int64_t nseg = (host->size() + seg - 1) / seg;
  bitar::BufferVector comp;
  for (int t = 0; t < kNumTests; ++t) {
    if (!comp.empty()) dev->Recycle(comp);
    const auto start = Clock::now();
    ARROW_ASSIGN_OR_RAISE(comp, dev->Compress(0, in));
    PrintPerfNumbers(host->size(), start);
  }
  int64_t csize = 0;
  for (auto& b : comp) csize += b->size();
  std::printf("Compression ratio: %.3f (%lld segments)\n",
              static_cast<double>(host->size()) / static_cast<double>(csize),
              static_cast<long long>(nseg));
  ARROW_ASSIGN_OR_RAISE(auto out, bitar::AllocateResizableDeviceBuffer(nseg * seg, device_id));
  std::unique_ptr<arrow::ResizableBuffer> dout = std::move(out);
  for (int t = 0; t < kNumTests; ++t) {
    const auto start = Clock::now();
    ARROW_RETURN_NOT_OK(dev->Decompress(0, comp, dout));
    PrintPerfNumbers(host->size(), start);
  }
  ARROW_ASSIGN_OR_RAISE(auto back, arrow::Buffer::Copy(std::shared_ptr<arrow::Buffer>(std::move(dout)),
                                                       arrow::default_cpu_memory_manager()));
  if (dev->Recycle(comp) != comp.size()) return arrow::Status::Invalid("Recycle count mismatch");
  if (back->size() != host->size() || std::memcmp(back->data(), host->data(), host->size()) != 0)
    return arrow::Status::Invalid("The decompressed data is not the same as the input buffer");
  std::printf("The decompressed data is equivalent to the input buffer\n");
  return arrow::Status::OK();
}

// one part per (device, queue pair), round-robin; CompressAsync / DecompressAsync on every
// worker, per-part memcmp (demo_app.cc:548-693)
arrow::Status EvaluateAsync(const std::vector<std::unique_ptr<Device>>& devs,
                            const std::vector<uint8_t>& ids,
                            const std::shared_ptr<arrow::Buffer>& host, uint32_t seg) {
  std::vector<std::pair<size_t, uint16_t>> slots;  // (device index, qp), Advance order
  for (size_t d = 0; d < devs.size(); ++d)
    for (uint16_t q = 0; q < devs[d]->num_qps(); ++q) slots.emplace_back(d, q);
  const int64_t k = static_cast<int64_t>(slots.size());
  PrintHeader("Evaluate Async (" + std::to_string(host->size()) + " bytes over " +
              std::to_string(k) + " queue pairs)");
  // parts of whole segments, so every part but the last is a multiple of seg
  const int64_t nseg = (host->size() + seg - 1) / seg;
  const int64_t per = (nseg + k - 1) / k * seg;
  std::vector<std::shared_ptr<arrow::Buffer>> parts(k);
  std::vector<int64_t> offs(k);
  for (int64_t i = 0; i < k; ++i) {
    offs[i] = std::min<int64_t>(i * per, host->size());
    const int64_t len = std::min<int64_t>(per, host->size() - offs[i]);
    ARROW_ASSIGN_OR_RAISE(parts[i], arrow::Buffer::Copy(arrow::SliceBuffer(host, offs[i], len),
                                                       bitar::hip_memory_manager(ids[slots[i].first])));
  }
  std::vector<bitar::BufferVector> comp(k);
  std::vector<Clock::time_point> ends(k);
  auto ccb = [&](uint8_t device_id, uint16_t qp, arrow::Result<bitar::BufferVector>&& r) -> int {
    if (!r.ok()) {
      std::fprintf(stderr, "async compress failed on device %u qp %u: %s\n", device_id, qp,
                   r.status().ToString().c_str());
      return EXIT_FAILURE;
    }
    for (int64_t i = 0; i < k; ++i)
      if (ids[slots[i].first] == device_id && slots[i].second == qp) {
        comp[i] = std::move(r).ValueUnsafe();
        ends[i] = Clock::now();
      }
    return bitar::kAsyncReturnOK;
  };
  using CParam = bitar::CompressParam<bitar::Class_HIP_GFX950, decltype(ccb)>;
  std::vector<std::unique_ptr<CParam>> cps;
  auto start = Clock::now();
  for (int64_t i = 0; i < k; ++i) {
    cps.push_back(std::make_unique<CParam>(devs[slots[i].first], slots[i].second, parts[i], ccb));
    if (bitar::CompressAsync(cps.back()) != 0) return arrow::Status::IOError("CompressAsync busy");
  }
  bool ok = true;
  for (int64_t i = 0; i < k; ++i)
    ok &= bitar::WaitLcore(devs[slots[i].first]->LcoreOf(slots[i].second)) == bitar::kAsyncReturnOK;
  if (!ok) return arrow::Status::IOError("Failed to complete async compression");
  PrintPerfNumbers(host->size(), start, *std::max_element(ends.begin(), ends.end()));
  std::vector<std::unique_ptr<arrow::ResizableBuffer>> outs(k);
  for (int64_t i = 0; i < k; ++i) {
    ARROW_ASSIGN_OR_RAISE(auto o, bitar::AllocateResizableDeviceBuffer(
                                      std::max<int64_t>(1, static_cast<int64_t>(comp[i].size()) * seg),
                                      ids[slots[i].first]));
    outs[i] = std::move(o);
  }
  auto dcb = [&](uint8_t device_id, uint16_t qp, const arrow::Status& st) -> int {
    if (!st.ok()) {
      std::fprintf(stderr, "async decompress failed on device %u qp %u: %s\n", device_id, qp,
                   st.ToString().c_str());
      return EXIT_FAILURE;
    }
    for (int64_t i = 0; i < k; ++i)
      if (ids[slots[i].first] == device_id && slots[i].second == qp) ends[i] = Clock::now();
    return bitar::kAsyncReturnOK;
  };
  using DParam = bitar::DecompressParam<bitar::Class_HIP_GFX950, decltype(dcb)>;
  std::vector<std::unique_ptr<DParam>> dps;
  start = Clock::now();
  for (int64_t i = 0; i < k; ++i) {
    dps.push_back(std::make_unique<DParam>(devs[slots[i].first], slots[i].second, comp[i], outs[i], dcb));
    if (bitar::DecompressAsync(dps.back()) != 0) return arrow::Status::IOError("DecompressAsync busy");
  }
  for (int64_t i = 0; i < k; ++i)
    ok &= bitar::WaitLcore(devs[slots[i].first]->LcoreOf(slots[i].second)) == bitar::kAsyncReturnOK;
  if (!ok) return arrow::Status::IOError("Failed to complete async decompression");
  PrintPerfNumbers(host->size(), start, *std::max_element(ends.begin(), ends.end()));
  for (int64_t i = 0; i < k; ++i) {
    ARROW_ASSIGN_OR_RAISE(auto back, arrow::Buffer::Copy(std::shared_ptr<arrow::Buffer>(std::move(outs[i])),
                                                         arrow::default_cpu_memory_manager()));
    if (back->size() != parts[i]->size() ||
        std::memcmp(back->data(), host->data() + offs[i], static_cast<size_t>(back->size())) != 0)
      return arrow::Status::Invalid("Decompressed segment ", i, " is not the same as the input buffer");
    if (devs[slots[i].first]->Recycle(comp[i]) != comp[i].size())
      return arrow::Status::Invalid("Recycle count mismatch");
  }
  std::printf("The aggregated decompressed data from %lld parts is equivalent to the input buffer\n",
              static_cast<long long>(k));
  return arrow::Status::OK();
}

}  // namespace

int main(int argc, char** argv) {
  std::string file, codec_name = "deflate", ipc_codec = "none";
  int64_t bytes = 0, synthetic = 0;
  int mode = 0;
  uint32_t seg = 59460, ndev = 1, workers = 4;
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string a = argv[i], v = argv[i + 1];
    if (a == "--file" || a == "-f") file = v;
    else if (a == "--bytes" || a == "-b") bytes = std::stoll(v);
    else if (a == "--mode" || a == "-m") mode = std::stoi(v);
    else if (a == "--synthetic") synthetic = std::stoll(v);
    else if (a == "--codec") codec_name = v;
    else if (a == "--seg") seg = static_cast<uint32_t>(std::stoul(v));
    else if (a == "--devices") ndev = static_cast<uint32_t>(std::stoul(v));
    else if (a == "--workers") workers = static_cast<uint32_t>(std::stoul(v));
    else if (a == "--ipc-codec") ipc_codec = v;
    else { std::cerr << "unknown option " << a << "\n"; return 2; }
  }
  std::shared_ptr<arrow::Buffer> host;
  if (!file.empty()) {
    auto r = ReadData(file, mode, bytes, ipc_codec);
    if (!r.ok()) { std::cerr << r.status().ToString() << "\n"; return 1; }
    host = *r;
  } else if (synthetic > 0) {
    host = Synthetic(synthetic);
  } else {
    std::cerr << "Missing argument for '--file' (or --synthetic N)\n";
    return 1;
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
        std::min<int64_t>(65535, host->size() / seg + 64)));
    auto st = d->Initialize(std::move(cfg));
    if (!st.ok()) { std::cerr << st.ToString() << "\n"; return 1; }
  }
  auto st = EvaluateSync((*devs)[0], use[0], host, seg);
  if (st.ok()) st = EvaluateAsync(*devs, use, host, seg);
  if (!st.ok()) { std::cerr << st.ToString() << "\n"; return 1; }
  return 0;
}
