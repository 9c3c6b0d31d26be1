// frontend_test.cc -- tests of the bitar C++ front-end (namespace bitar) on MI355X.
//
// Modes: `cpu` (no GPU needed: configuration rules, discovery errors), `gpu <in> <outdir>`
// (Compress/Decompress/Recycle/async through real devices; compressed segments are written
// to <outdir> so the Python side can check them with zlib / liblz4), `arrow <in> <outdir>`
// (the util::Codec adapters) and `pool <0|1> <in>` (the pools' debug poisoning, expected on
// or off, and buffers the front-end did not allocate: hipHostRegister'd host memory and HBM
// owned by another context).  Built twice: against the release libbitar.so (-DNDEBUG) and
// the debug variant (lib/debug/libbitar.so).  Mirrors the reference's
// only behavioural checks (apps/demo_app.cc:288-290, 500-501, 534-543, 671-686).
#include <arrow/api.h>
#include <arrow/buffer.h>
#include <arrow/io/memory.h>
#include <arrow/ipc/api.h>
#include <arrow/memory_pool.h>
#include <arrow/util/compression.h>

#include <hip/hip_runtime_api.h>  // (hipHostRegister: a caller-pinned buffer, PoolTests)

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "bitar/bitar.h"
#include "bitar_hip.h"

namespace {

int g_failures = 0;
#define CHECK(cond)                                                           \
  do {                                                                        \
    if (!(cond)) {                                                            \
      std::cerr << __FILE__ << ":" << __LINE__ << " CHECK failed: " #cond "\n"; \
      ++g_failures;                                                           \
    }                                                                         \
  } while (0)
#define CHECK_OK(expr)                                                                 \
  do {                                                                                 \
    auto _s = (expr);                                                                  \
    if (!_s.ok()) {                                                                    \
      std::cerr << __FILE__ << ":" << __LINE__ << " not OK: " << _s.ToString() << "\n"; \
      ++g_failures;                                                                    \
    }                                                                                  \
  } while (0)

std::unique_ptr<bitar::HipConfiguration> MakeConfig(bitar::Codec codec, std::uint32_t seg) {
  auto c = std::make_unique<bitar::HipConfiguration>(bitar::HipConfiguration::Defaults());
  c->set_codec(codec);
  c->set_decompressed_seg_size32(seg);
  c->set_burst_size(32);
  c->set_max_preallocate_memzones(64);
  return c;
}

// INTEGRATION.md's minimal program, verbatim between the markers (tests/test_frontend.py
// checks that the two texts are identical)
// --- INTEGRATION.md minimal program ---
// `data`, `n`: the caller's bytes on the host
arrow::Status RoundTrip(const std::uint8_t* data, std::int64_t n) {
  auto* driver = bitar::CompressDriver<bitar::Class_HIP_GFX950>::Instance();
  ARROW_ASSIGN_OR_RAISE(auto ids, driver->ListAvailableDeviceIds());
  ARROW_ASSIGN_OR_RAISE(auto devices, driver->GetDevices({ids[0]}));
  auto& dev = devices[0];
  auto cfg = std::make_unique<bitar::HipConfiguration>(bitar::HipConfiguration::Defaults());
  cfg->set_codec(bitar::Codec::LZ4);
  cfg->set_decompressed_seg_size32(65536);
  ARROW_RETURN_NOT_OK(dev->Initialize(std::move(cfg)));

  // (a) host-filled buffers: the pinned HipHost pool (= the reference's Rtememzone), written
  //     and read by the CPU; Compress / Decompress stream them over PCIe in chunks
  auto* pinned = bitar::GetMemoryPool(bitar::MemoryPoolBackend::HipHost);
  ARROW_ASSIGN_OR_RAISE(std::shared_ptr<arrow::Buffer> input, arrow::AllocateBuffer(n, pinned));
  std::memcpy(input->mutable_data(), data, static_cast<std::size_t>(n));  // host write
  ARROW_ASSIGN_OR_RAISE(auto frames, dev->Compress(/*qp=*/0, input));
  const auto cap = static_cast<std::int64_t>(frames.size()) * 65536;
  ARROW_ASSIGN_OR_RAISE(std::unique_ptr<arrow::ResizableBuffer> out,
                        arrow::AllocateResizableBuffer(cap, pinned));
  ARROW_RETURN_NOT_OK(dev->Decompress(0, frames, out));
  if (out->size() != n || std::memcmp(out->data(), data, static_cast<std::size_t>(n)) != 0)
    return arrow::Status::IOError("round trip differs");
  dev->Recycle(frames);

  // (b) HBM-resident buffers (the fast path: no PCIe): copy in through the ROCm memory
  //     manager, decompress into an HBM buffer; both report is_cpu() == false
  ARROW_ASSIGN_OR_RAISE(auto d_in, arrow::Buffer::Copy(input, bitar::hip_memory_manager(0)));
  ARROW_ASSIGN_OR_RAISE(auto frames2, dev->Compress(0, d_in));
  ARROW_ASSIGN_OR_RAISE(std::unique_ptr<arrow::ResizableBuffer> d_out,
                        bitar::AllocateResizableDeviceBuffer(cap, 0));
  ARROW_RETURN_NOT_OK(dev->Decompress(0, frames2, d_out));
  ARROW_ASSIGN_OR_RAISE(auto back, arrow::Buffer::Copy(std::shared_ptr<arrow::Buffer>(std::move(d_out)),
                                                       arrow::default_cpu_memory_manager()));
  if (back->size() != n || std::memcmp(back->data(), data, static_cast<std::size_t>(n)) != 0)
    return arrow::Status::IOError("HBM round trip differs");
  dev->Recycle(frames2);
  return arrow::Status::OK();
}
// --- end ---

void CpuTests() {
  // slot sizing rule of the reference (config.cc:59-73)
  bitar::HipConfiguration c;
  c.set_decompressed_seg_size(2048);
  CHECK(c.compressed_seg_size() == 4096);
  c.set_decompressed_seg_size(59460);
  CHECK(c.compressed_seg_size() == 65406);
  c.set_decompressed_seg_size(32768);
  CHECK(c.compressed_seg_size() == 36044);
  c.set_decompressed_seg_size(16384);
  CHECK(c.compressed_seg_size() == 32768);
  CHECK(bitar::internal::kMaxSegSize == 59460);
  CHECK(c.ToString().find("checksum_type: NONE") != std::string::npos);
  CHECK(c.type_name() == bitar::kHipConfigurationTypeName);
  // memory pools exist; the reference's DPDK pools are host memory the engine reads
  // (memory_pool.cc:70-188), so both names alias the pinned host pool
  CHECK(bitar::GetMemoryPool(bitar::MemoryPoolBackend::Rtememzone) ==
        bitar::GetMemoryPool(bitar::MemoryPoolBackend::HipHost));
  CHECK(bitar::GetMemoryPool(bitar::MemoryPoolBackend::Rtemalloc) ==
        bitar::GetMemoryPool(bitar::MemoryPoolBackend::HipHost));
  CHECK(bitar::GetMemoryPool(bitar::MemoryPoolBackend::HipDevice) !=
        bitar::GetMemoryPool(bitar::MemoryPoolBackend::HipHost));
  CHECK(c.level() == 1 && c.ToString().find("level: 1") != std::string::npos);
  CHECK(bitar::GetMemoryPool(bitar::MemoryPoolBackend::System) != nullptr);
  uint8_t* p = nullptr;
  CHECK_OK(bitar::GetMemoryPool(bitar::MemoryPoolBackend::HipDevice)->Allocate(0, 64, &p));
  CHECK(p != nullptr);  // zero-size sentinel, no device needed
}

std::vector<uint8_t> ReadFile(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

void WriteSegments(const std::string& path, const bitar::BufferVector& bufs) {
  // [u32 size][bytes]... via Arrow's device -> CPU copy
  std::ofstream f(path, std::ios::binary);
  for (const auto& b : bufs) {
    auto view = std::make_shared<arrow::Buffer>(reinterpret_cast<const uint8_t*>(b->address()),
                                                b->size(), b->memory_manager());
    auto copied = arrow::Buffer::Copy(view, arrow::default_cpu_memory_manager());
    if (!copied.ok()) {
      std::cerr << "copy failed: " << copied.status().ToString() << "\n";
      ++g_failures;
      return;
    }
    const uint32_t sz = static_cast<uint32_t>(b->size());
    f.write(reinterpret_cast<const char*>(&sz), 4);
    f.write(reinterpret_cast<const char*>((*copied)->data()), sz);
  }
}

void GpuTests(const std::string& input_path, const std::string& outdir) {
  auto* driver = bitar::CompressDriver<bitar::Class_HIP_GFX950>::Instance();
  auto ids = driver->ListAvailableDeviceIds();
  CHECK_OK(ids.status());
  if (!ids.ok()) return;
  driver->set_num_workers(2);
  auto devs = driver->GetDevices({(*ids)[0]});
  CHECK_OK(devs.status());
  if (!devs.ok()) return;
  CHECK(devs->size() == 1 && (*devs)[0]->num_qps() == 2);
  CHECK((*devs)[0]->LcoreOf(0) == 1 && (*devs)[0]->LcoreOf(1) == 2);
  auto bad = driver->GetDevices({200});
  CHECK(bad.status().IsInvalid());

  const auto data = ReadFile(input_path);
  CHECK(data.size() > 100000);
  auto host_in = std::make_shared<arrow::Buffer>(data.data(), static_cast<int64_t>(data.size()));

  // DEFLATE with the reference's default DYNAMIC Huffman (config.h:151) and with FIXED
  struct Case {
    bitar::Codec codec;
    bitar::HuffmanEncoding huff;
    const char* file;
  };
  for (const Case& cs : {Case{bitar::Codec::DEFLATE, bitar::HuffmanEncoding::DYNAMIC, "/deflate.segs"},
                         Case{bitar::Codec::DEFLATE, bitar::HuffmanEncoding::FIXED, "/deflate_fixed.segs"},
                         Case{bitar::Codec::LZ4, bitar::HuffmanEncoding::DEFAULT, "/lz4.segs"},
                         Case{bitar::Codec::ZSTD, bitar::HuffmanEncoding::DEFAULT, "/zstd.segs"}}) {
    const auto codec = cs.codec;
    const std::uint32_t seg = codec == bitar::Codec::DEFLATE ? 59460 : 65536;
    auto& dev = (*devs)[0];
    // not initialized yet -> Invalid (EntryGuard, device.cc:446-451)
    if (codec == bitar::Codec::DEFLATE) CHECK(dev->Compress(0, host_in).status().IsInvalid());
    // wrong configuration type is rejected
    // (a fresh device per codec: the reference initializes a device once)
    auto fresh = driver->GetDevices({(*ids)[0]});
    CHECK_OK(fresh.status());
    auto& d = (*fresh)[0];
    auto cfg = MakeConfig(codec, seg);
    if (codec == bitar::Codec::DEFLATE) {
      CHECK(cfg->huffman_enc() == bitar::HuffmanEncoding::DYNAMIC);  // the reference default
      cfg->set_huffman_enc(cs.huff);
    }
    CHECK_OK(d->Initialize(std::move(cfg)));
    CHECK(d->Compress(5, host_in).status().IsInvalid());  // qp out of range

    // sync round trip from a HOST buffer (staged to HBM by the device)
    auto comp = d->Compress(0, host_in);
    CHECK_OK(comp.status());
    if (!comp.ok()) continue;
    const auto nseg = (data.size() + seg - 1) / seg;
    CHECK(comp->size() == nseg);
    for (const auto& b : *comp) CHECK(!b->is_cpu());
    WriteSegments(outdir + cs.file, *comp);

    auto out = arrow::AllocateResizableBuffer(static_cast<int64_t>(nseg * seg));
    CHECK_OK(out.status());
    std::unique_ptr<arrow::ResizableBuffer> host_out = std::move(*out);
    CHECK_OK(d->Decompress(1, *comp, host_out));
    CHECK(host_out->size() == static_cast<int64_t>(data.size()));
    CHECK(std::memcmp(host_out->data(), data.data(), data.size()) == 0);

    // capacity rule (device.cc:248-254)
    // (Arrow pads capacities to 64 B, so stay a full pad below the requirement)
    auto small = arrow::AllocateResizableBuffer(static_cast<int64_t>(nseg * seg - 128));
    std::unique_ptr<arrow::ResizableBuffer> small_out = std::move(*small);
    CHECK(d->Decompress(0, *comp, small_out).IsCapacityError());

    // HBM-resident input and output (no staging), via the Arrow device API
    auto dev_in = arrow::Buffer::Copy(host_in, bitar::hip_memory_manager(0));
    CHECK_OK(dev_in.status());
    auto comp2 = d->Compress(0, *dev_in);
    CHECK_OK(comp2.status());
    auto dev_out = bitar::AllocateResizableDeviceBuffer(static_cast<int64_t>(nseg * seg), 0);
    CHECK_OK(dev_out.status());
    std::unique_ptr<arrow::ResizableBuffer> dout = std::move(*dev_out);
    CHECK_OK(d->Decompress(0, *comp2, dout));
    CHECK(!dout->is_cpu() && dout->size() == static_cast<int64_t>(data.size()));
    auto back = arrow::Buffer::Copy(std::shared_ptr<arrow::Buffer>(std::move(dout)),
                                    arrow::default_cpu_memory_manager());
    CHECK_OK(back.status());
    if (back.ok()) CHECK(std::memcmp((*back)->data(), data.data(), data.size()) == 0);

    // corrupted stream -> IOError (per-op status, device.cc:512-520)
    {
      auto bogus = std::make_shared<arrow::Buffer>(reinterpret_cast<const uint8_t*>("\x07\x07\x07\x07"), 4);
      bitar::BufferVector bv;
      bv.emplace_back(std::make_unique<arrow::Buffer>(bogus->data(), 4));
      auto o = arrow::AllocateResizableBuffer(seg);
      std::unique_ptr<arrow::ResizableBuffer> ob = std::move(*o);
      if (codec != bitar::Codec::LZ4) CHECK(d->Decompress(0, bv, ob).IsIOError());
    }

    // async on both queue pairs (CompressAsync / WaitLcore, util.h:216-236)
    int calls = 0;
    bitar::BufferVector async_out[2];
    auto cb = [&](std::uint8_t, std::uint16_t qp, arrow::Result<bitar::BufferVector>&& r) {
      ++calls;
      if (!r.ok()) return 1;
      async_out[qp] = std::move(r).ValueUnsafe();
      return bitar::kAsyncReturnOK;
    };
    using Param = bitar::CompressParam<bitar::Class_HIP_GFX950, decltype(cb)>;
    auto p0 = std::make_unique<Param>(d, 0, host_in, cb);
    auto p1 = std::make_unique<Param>(d, 1, *dev_in, cb);
    CHECK(bitar::CompressAsync(p0) == 0);
    CHECK(bitar::CompressAsync(p1) == 0);
    CHECK(bitar::WaitLcore(d->LcoreOf(0)) == bitar::kAsyncReturnOK);
    CHECK(bitar::WaitLcore(d->LcoreOf(1)) == bitar::kAsyncReturnOK);
    CHECK(calls == 2);
    auto dcb = [&](std::uint8_t, std::uint16_t, const arrow::Status& s) {
      return s.ok() ? bitar::kAsyncReturnOK : 1;
    };
    auto o2 = arrow::AllocateResizableBuffer(static_cast<int64_t>(nseg * seg));
    std::unique_ptr<arrow::ResizableBuffer> aout = std::move(*o2);
    using DParam = bitar::DecompressParam<bitar::Class_HIP_GFX950, decltype(dcb)>;
    auto dp = std::make_unique<DParam>(d, 1, async_out[0], aout, dcb);
    CHECK(bitar::DecompressAsync(dp) == 0);
    CHECK(bitar::WaitLcore(d->LcoreOf(1)) == bitar::kAsyncReturnOK);
    CHECK(aout->size() == static_cast<int64_t>(data.size()) &&
          std::memcmp(aout->data(), data.data(), data.size()) == 0);

    // concurrent failure on one queue pair: qp 1 decodes a malformed segment while qp 0
    // decodes a valid frame; only qp 1 may report IOError (per-queue-pair status,
    // reference device.cc:84-110, 512-520).  Repeated so the two calls overlap.
    {
      static const uint8_t kBad[3] = {0, 0, 0};  // LZ4: offset 0; DEFLATE/Zstd: truncated
      bitar::BufferVector bad;
      bad.emplace_back(std::make_unique<arrow::Buffer>(kBad, 3));
      for (int rep = 0; rep < 8; ++rep) {
        arrow::Status st[2];
        auto scb = [&](std::uint8_t, std::uint16_t qp, const arrow::Status& s) {
          st[qp] = s;
          return bitar::kAsyncReturnOK;
        };
        auto g0 = arrow::AllocateResizableBuffer(static_cast<int64_t>(nseg * seg));
        auto g1 = arrow::AllocateResizableBuffer(static_cast<int64_t>(seg));
        std::unique_ptr<arrow::ResizableBuffer> good_out = std::move(*g0);
        std::unique_ptr<arrow::ResizableBuffer> bad_out = std::move(*g1);
        using SParam = bitar::DecompressParam<bitar::Class_HIP_GFX950, decltype(scb)>;
        auto q1 = std::make_unique<SParam>(d, 1, bad, bad_out, scb);
        auto q0 = std::make_unique<SParam>(d, 0, async_out[0], good_out, scb);
        CHECK(bitar::DecompressAsync(q1) == 0);
        CHECK(bitar::DecompressAsync(q0) == 0);
        CHECK(bitar::WaitLcore(d->LcoreOf(1)) == bitar::kAsyncReturnOK);
        CHECK(bitar::WaitLcore(d->LcoreOf(0)) == bitar::kAsyncReturnOK);
        CHECK(st[0].ok());
        CHECK(st[1].IsIOError());
        CHECK(good_out->size() == static_cast<int64_t>(data.size()) &&
              std::memcmp(good_out->data(), data.data(), data.size()) == 0);
      }
    }

    // Recycle returns every slot exactly once (demo_app.cc:288-290)
    CHECK(d->Recycle(*comp) == comp->size());
    CHECK(d->Recycle(*comp) == 0);
    CHECK(d->Recycle(*comp2) == comp2->size());
    CHECK(d->Recycle(async_out[0]) == async_out[0].size());
    CHECK(d->Recycle(async_out[1]) == async_out[1].size());
  }
  // checksum_type (config.h:169-182): per-segment CRC32 | Adler32 << 32 of the uncompressed
  // side of each call -- the compress input and the decompress output (written for the
  // Python side to check against zlib)
  {
    auto fresh = driver->GetDevices({(*ids)[0]});
    CHECK_OK(fresh.status());
    auto& d = (*fresh)[0];
    const std::uint32_t seg = 65536;
    auto cfg = MakeConfig(bitar::Codec::LZ4, seg);
    cfg->set_checksum_type(bitar::ChecksumType::CRC32_ADLER32);
    CHECK_OK(d->Initialize(std::move(cfg)));
    auto comp = d->Compress(0, host_in);
    CHECK_OK(comp.status());
    const auto nseg = (data.size() + seg - 1) / seg;
    const std::vector<std::uint64_t> cs = d->checksums(0);
    CHECK(cs.size() == nseg);
    if (comp.ok()) {
      auto o = arrow::AllocateResizableBuffer(static_cast<int64_t>(nseg * seg));
      std::unique_ptr<arrow::ResizableBuffer> out = std::move(*o);
      CHECK_OK(d->Decompress(1, *comp, out));
      CHECK(d->checksums(1) == cs);  // round trip: same uncompressed bytes
      std::ofstream f(outdir + "/checksums.bin", std::ios::binary);
      f.write(reinterpret_cast<const char*>(cs.data()), static_cast<std::streamsize>(8 * cs.size()));
      CHECK(d->Recycle(*comp) == comp->size());
    }
  }
  // chained ops (max_sgl_segs = 4, reference memory.cc:350-505): one stream per 4 segments,
  // spread over 4 slots (trailing ones empty); Decompress regroups 4 buffers per op; one
  // checksum per op; an op larger than 64 KiB is refused
  for (const auto codec : {bitar::Codec::LZ4, bitar::Codec::DEFLATE, bitar::Codec::ZSTD}) {
    const std::uint32_t seg = 16384, k = 4;
    {
      auto fresh = driver->GetDevices({(*ids)[0]});
      CHECK_OK(fresh.status());
      auto cfg = MakeConfig(codec, seg * 2);
      cfg->set_max_sgl_segs(k);
      CHECK((*fresh)[0]->Initialize(std::move(cfg)).IsInvalid());
    }
    auto fresh = driver->GetDevices({(*ids)[0]});
    CHECK_OK(fresh.status());
    auto& d = (*fresh)[0];
    auto cfg = MakeConfig(codec, seg);
    cfg->set_max_sgl_segs(k);
    cfg->set_checksum_type(bitar::ChecksumType::CRC32);
    CHECK_OK(d->Initialize(std::move(cfg)));
    auto comp = d->Compress(0, host_in);
    CHECK_OK(comp.status());
    if (!comp.ok()) continue;
    const auto nseg = (data.size() + seg - 1) / seg;
    const auto nops = (nseg + k - 1) / k;
    CHECK(comp->size() == nseg);
    CHECK(d->checksums(0).size() == nops);
    const std::vector<std::uint64_t> cs = d->checksums(0);
    WriteSegments(outdir + (codec == bitar::Codec::LZ4       ? "/sgl_lz4.segs"
                            : codec == bitar::Codec::DEFLATE ? "/sgl_deflate.segs"
                                                             : "/sgl_zstd.segs"),
                  *comp);
    auto o = arrow::AllocateResizableBuffer(static_cast<int64_t>(nseg * seg));
    std::unique_ptr<arrow::ResizableBuffer> out = std::move(*o);
    CHECK_OK(d->Decompress(1, *comp, out));
    CHECK(out->size() == static_cast<int64_t>(data.size()) &&
          std::memcmp(out->data(), data.data(), data.size()) == 0);
    CHECK(d->checksums(1) == cs);
    // HBM in and out
    auto dev_in = arrow::Buffer::Copy(host_in, bitar::hip_memory_manager(0));
    CHECK_OK(dev_in.status());
    auto comp2 = d->Compress(1, *dev_in);
    CHECK_OK(comp2.status());
    auto dev_out = bitar::AllocateResizableDeviceBuffer(static_cast<int64_t>(nseg * seg), 0);
    std::unique_ptr<arrow::ResizableBuffer> dout = std::move(*dev_out);
    CHECK_OK(d->Decompress(0, *comp2, dout));
    auto back = arrow::Buffer::Copy(std::shared_ptr<arrow::Buffer>(std::move(dout)),
                                    arrow::default_cpu_memory_manager());
    CHECK_OK(back.status());
    if (back.ok())
      CHECK((*back)->size() == static_cast<int64_t>(data.size()) &&
            std::memcmp((*back)->data(), data.data(), data.size()) == 0);
    CHECK(d->Recycle(*comp) == comp->size());
    CHECK(d->Recycle(*comp2) == comp2->size());
  }
  // the reference's demo flow over its memzone pool (demo_app.cc:121-122, 589-592): the
  // input is written on the CPU into an Rtememzone buffer, compressed, decompressed into
  // another Rtememzone buffer and compared on the CPU
  {
    auto fresh = driver->GetDevices({(*ids)[0]});
    CHECK_OK(fresh.status());
    auto& d = (*fresh)[0];
    CHECK_OK(d->Initialize(MakeConfig(bitar::Codec::LZ4, 65536)));
    auto* pool = bitar::GetMemoryPool(bitar::MemoryPoolBackend::Rtememzone);
    auto in = arrow::AllocateBuffer(static_cast<int64_t>(data.size()), pool);
    CHECK_OK(in.status());
    std::shared_ptr<arrow::Buffer> zin = std::move(*in);
    std::memcpy(zin->mutable_data(), data.data(), data.size());  // host write (rte_memcpy)
    auto comp = d->Compress(0, zin);
    CHECK_OK(comp.status());
    const auto nseg = (data.size() + 65535) / 65536;
    auto out = arrow::AllocateResizableBuffer(static_cast<int64_t>(nseg * 65536), pool);
    CHECK_OK(out.status());
    std::unique_ptr<arrow::ResizableBuffer> zout = std::move(*out);
    if (comp.ok()) {
      CHECK_OK(d->Decompress(0, *comp, zout));
      CHECK(zout->size() == static_cast<int64_t>(data.size()) &&
            std::memcmp(zout->data(), data.data(), data.size()) == 0);  // host read
      CHECK(d->Recycle(*comp) == comp->size());
    }
    // Reallocate keeps the bytes (the reference copies memzones with rte_memcpy, 151-174)
    CHECK_OK(zout->Resize(static_cast<int64_t>(nseg * 65536 + 4096)));
    CHECK(std::memcmp(zout->data(), data.data(), data.size()) == 0);
  }
  // LZ4 at level 2 = the wide parse (the ratio point): smaller output, same round trip;
  // <outdir>/lz4_wide.segs is checked against the oracle's wide parse by the Python side
  {
    auto fresh = driver->GetDevices({(*ids)[0]});
    CHECK_OK(fresh.status());
    auto& d = (*fresh)[0];
    auto cfg = MakeConfig(bitar::Codec::LZ4, 65536);
    cfg->set_level(2);
    const auto* wide_cfg = cfg.get();  // (owned by the device after Initialize)
    CHECK_OK(d->Initialize(std::move(cfg)));
    auto comp = d->Compress(0, host_in);
    CHECK_OK(comp.status());
    if (comp.ok()) {
      WriteSegments(outdir + "/lz4_wide.segs", *comp);
      auto out = arrow::AllocateResizableBuffer(static_cast<int64_t>(comp->size() * 65536));
      std::unique_ptr<arrow::ResizableBuffer> o = std::move(*out);
      CHECK_OK(d->Decompress(0, *comp, o));
      CHECK(o->size() == static_cast<int64_t>(data.size()) &&
            std::memcmp(o->data(), data.data(), data.size()) == 0);
    }
    CHECK(wide_cfg->window_size() == 14);  // the wide parse reaches 14848 B
    auto bad = driver->GetDevices({(*ids)[0]});
    CHECK_OK(bad.status());
    auto cfg0 = MakeConfig(bitar::Codec::LZ4, 65536);
    cfg0->set_level(0);
    CHECK((*bad)[0]->Initialize(std::move(cfg0)).IsInvalid());
  }
  // window_size reports the encoder's reach (2560 B -> 12); a larger requested window is
  // accepted (the streams are valid for it), a smaller one or one past the format's maximum is
  // refused; DEFLATE and ZSTD refuse levels other than 1 instead of ignoring them
  {
    struct W {
      bitar::Codec codec;
      int window, level;
      bool ok;
    };
    for (const W& w : {W{bitar::Codec::LZ4, 0, 1, true}, W{bitar::Codec::DEFLATE, 15, 1, true},
                       W{bitar::Codec::ZSTD, 16, 1, true}, W{bitar::Codec::LZ4, 11, 1, false},
                       W{bitar::Codec::DEFLATE, 16, 1, false}, W{bitar::Codec::DEFLATE, 0, 2, false},
                       W{bitar::Codec::ZSTD, 0, 3, false}, W{bitar::Codec::LZ4, 0, 9, true}}) {
      auto fresh = driver->GetDevices({(*ids)[0]});
      CHECK_OK(fresh.status());
      auto& d = (*fresh)[0];
      auto cfg = MakeConfig(w.codec, w.codec == bitar::Codec::DEFLATE ? 59460 : 65536);
      cfg->set_window_size(static_cast<std::uint8_t>(w.window));
      cfg->set_level(static_cast<std::uint8_t>(w.level));
      const auto* c = cfg.get();
      const auto st = d->Initialize(std::move(cfg));
      CHECK(st.ok() == w.ok);
      // (a requested window is kept, 0 is answered with the reach; encoder_window() is the
      // reach either way)
      const int reach = w.level >= 2 ? 14 : 12;
      if (st.ok()) CHECK(c->window_size() == (w.window ? w.window : reach));
      if (st.ok()) CHECK(d->encoder_window() == reach);
    }
  }
  // INTEGRATION.md's minimal program, run as written
  CHECK_OK(RoundTrip(data.data(), static_cast<std::int64_t>(data.size())));
  // empty input -> empty vector (device.cc:161-164); empty vector -> OK
  auto& d0 = (*devs)[0];
  CHECK_OK(d0->Initialize(MakeConfig(bitar::Codec::LZ4, 65536)));
  auto empty = d0->Compress(0, std::make_shared<arrow::Buffer>(nullptr, 0));
  CHECK(empty.ok() && empty->empty());
  std::unique_ptr<arrow::ResizableBuffer> none;
  CHECK_OK(d0->Decompress(0, bitar::BufferVector{}, none));
}

// The Arrow util::Codec adapters (bitar/arrow_codec.h): round trips,
// the stock Arrow codecs decode what they write, and an Arrow IPC stream written with GPU
// body compression reads back with the stock reader.  Writes <outdir>/arrow_{zstd,lz4f}.bin
// and <outdir>/ipc_{zstd,lz4f}.arrows for the Python side (pyarrow) to check.
std::shared_ptr<arrow::RecordBatch> IpcBatch() {
  // deterministic: int64 i * 7 % 1000, utf8 "row" + (i % 977), for i < 200000
  arrow::Int64Builder ib;
  arrow::StringBuilder sb;
  for (int64_t i = 0; i < 200000; ++i) {
    (void)ib.Append(i * 7 % 1000);
    (void)sb.Append("row" + std::to_string(i % 977));
  }
  std::shared_ptr<arrow::Array> a, b;
  (void)ib.Finish(&a);
  (void)sb.Finish(&b);
  auto schema = arrow::schema({arrow::field("v", arrow::int64()), arrow::field("s", arrow::utf8())});
  return arrow::RecordBatch::Make(schema, a->length(), {a, b});
}

void ArrowCodecTests(const std::string& input_path, const std::string& outdir) {
  std::ifstream f(input_path, std::ios::binary);
  std::vector<uint8_t> data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  CHECK(!bitar::MakeArrowCodec(arrow::Compression::SNAPPY).ok());
  for (auto type : {arrow::Compression::ZSTD, arrow::Compression::LZ4_FRAME}) {
    const std::string tag = type == arrow::Compression::ZSTD ? "zstd" : "lz4f";
    auto codec = bitar::MakeArrowCodec(type, 0);
    CHECK_OK(codec.status());
    if (!codec.ok()) continue;
    auto& c = *codec;
    CHECK(c->compression_type() == type);
    for (size_t n : {data.size(), size_t(0), size_t(1), size_t(65536), size_t(65537)}) {
      if (n > data.size()) continue;
      const int64_t max = c->MaxCompressedLen(static_cast<int64_t>(n), data.data());
      std::vector<uint8_t> comp(static_cast<size_t>(max));
      auto clen = c->Compress(static_cast<int64_t>(n), data.data(), max, comp.data());
      CHECK_OK(clen.status());
      if (!clen.ok()) continue;
      std::vector<uint8_t> back(n + 1);
      auto dlen = c->Decompress(*clen, comp.data(), static_cast<int64_t>(n), back.data());
      CHECK_OK(dlen.status());
      CHECK(dlen.ok() && *dlen == static_cast<int64_t>(n) &&
            std::memcmp(back.data(), data.data(), n) == 0);
      // the stock Arrow codec decodes the GPU stream
      auto stock = arrow::util::Codec::Create(type);
      CHECK_OK(stock.status());
      if (stock.ok()) {
        std::vector<uint8_t> sb(n + 1);
        auto r = (*stock)->Decompress(*clen, comp.data(), static_cast<int64_t>(n), sb.data());
        CHECK_OK(r.status());
        CHECK(r.ok() && *r == static_cast<int64_t>(n) && std::memcmp(sb.data(), data.data(), n) == 0);
      }
      if (n == data.size()) {
        std::ofstream o(outdir + "/arrow_" + tag + ".bin", std::ios::binary);
        o.write(reinterpret_cast<const char*>(comp.data()), *clen);
      }
    }
    // streams the stock codec wrote (one frame: Zstd frames of any size, LZ4 frames with
    // linked blocks): decoded on the GPU
    for (const size_t n : {size_t{60000}, data.size()}) {
      auto stock = arrow::util::Codec::Create(type);
      if (!stock.ok()) break;
      const int64_t max = (*stock)->MaxCompressedLen(static_cast<int64_t>(n), data.data());
      std::vector<uint8_t> comp(static_cast<size_t>(max));
      auto clen = (*stock)->Compress(static_cast<int64_t>(n), data.data(), max, comp.data());
      CHECK_OK(clen.status());
      if (!clen.ok()) break;
      std::vector<uint8_t> back(n);
      auto r = c->Decompress(*clen, comp.data(), static_cast<int64_t>(n), back.data());
      CHECK_OK(r.status());
      CHECK(r.ok() && *r == static_cast<int64_t>(n) && std::memcmp(back.data(), data.data(), n) == 0);
    }
    // stock streams written by the Python side (pyarrow's codecs = the IPC writer's per-buffer
    // frames; liblz4 / libzstd with block + content checksums, content sizes):
    // <outdir>/stock.txt lines "zstd|lz4f <stream file> <plain file>"
    {
      std::ifstream man(outdir + "/stock.txt");
      std::string kind, sf, pf;
      int count = 0;
      while (man >> kind >> sf >> pf) {
        if ((kind == "zstd") != (type == arrow::Compression::ZSTD)) continue;
        const auto comp = ReadFile(outdir + "/" + sf);
        const auto plain = ReadFile(outdir + "/" + pf);
        std::vector<uint8_t> back(plain.size() + 64);
        auto r = c->Decompress(static_cast<int64_t>(comp.size()), comp.data(),
                               static_cast<int64_t>(back.size()), back.data());
        CHECK_OK(r.status());
        CHECK(r.ok() && *r == static_cast<int64_t>(plain.size()) &&
              std::memcmp(back.data(), plain.data(), plain.size()) == 0);
        if (!r.ok() || *r != static_cast<int64_t>(plain.size())) std::cerr << "stock stream " << sf << "\n";
        // a corrupted copy returns (an error, or bytes: these formats carry no checksum
        // unless the frame asks for one), it never faults
        auto bad = comp;
        bad[bad.size() / 2] ^= 0x5A;
        (void)c->Decompress(static_cast<int64_t>(bad.size()), bad.data(),
                            static_cast<int64_t>(back.size()), back.data());
        ++count;
      }
      std::cout << "stock streams decoded: " << count << "\n";
    }
    // Arrow IPC with GPU body compression, read back by the stock reader
    auto batch = IpcBatch();
    auto opts = arrow::ipc::IpcWriteOptions::Defaults();
    opts.codec = std::shared_ptr<arrow::util::Codec>(std::move(c));
    auto sink = arrow::io::BufferOutputStream::Create();
    CHECK_OK(sink.status());
    auto writer = arrow::ipc::MakeStreamWriter(*sink, batch->schema(), opts);
    CHECK_OK(writer.status());
    if (!writer.ok()) continue;
    CHECK_OK((*writer)->WriteRecordBatch(*batch));
    CHECK_OK((*writer)->Close());
    auto buf = (*sink)->Finish();
    CHECK_OK(buf.status());
    auto reader = arrow::ipc::RecordBatchStreamReader::Open(
        std::make_shared<arrow::io::BufferReader>(*buf));
    CHECK_OK(reader.status());
    if (reader.ok()) {
      std::shared_ptr<arrow::RecordBatch> got;
      CHECK_OK((*reader)->ReadNext(&got));
      CHECK(got && got->Equals(*batch));
    }
    std::ofstream o(outdir + "/ipc_" + tag + ".arrows", std::ios::binary);
    o.write(reinterpret_cast<const char*>((*buf)->data()), (*buf)->size());
  }
}


// arrow pools over memory the front-end did not allocate: (a) malloc'd host memory pinned by
// hipHostRegister (its device address may differ from the host one, so the device must stage
// it by copy, runtime.hip bitar_hip_pointer_info); (b) HBM of another bitar context
class RegisteredPool : public arrow::MemoryPool {
 public:
  arrow::Status Allocate(int64_t size, int64_t, uint8_t** out) override {
    void* p = nullptr;
    if (posix_memalign(&p, 4096, static_cast<std::size_t>(size ? size : 1)) != 0)
      return arrow::Status::OutOfMemory("posix_memalign");
    if (hipHostRegister(p, static_cast<std::size_t>(size ? size : 1), hipHostRegisterDefault) != hipSuccess) {
      std::free(p);
      return arrow::Status::IOError("hipHostRegister");
    }
    *out = static_cast<uint8_t*>(p);
    bytes_ += size;
    return arrow::Status::OK();
  }
  arrow::Status Reallocate(int64_t old_size, int64_t new_size, int64_t a, uint8_t** ptr) override {
    uint8_t* fresh = nullptr;
    ARROW_RETURN_NOT_OK(Allocate(new_size, a, &fresh));
    std::memcpy(fresh, *ptr, static_cast<std::size_t>(std::min(old_size, new_size)));
    Free(*ptr, old_size, a);
    *ptr = fresh;
    return arrow::Status::OK();
  }
  void Free(uint8_t* p, int64_t size, int64_t) override {
    (void)hipHostUnregister(p);
    std::free(p);
    bytes_ -= size;
  }
  int64_t bytes_allocated() const override { return bytes_; }
  std::string backend_name() const override { return "host_registered"; }
  int64_t max_memory() const override { return -1; }
  int64_t total_bytes_allocated() const override { return 0; }
  int64_t num_allocations() const override { return 0; }

 private:
  int64_t bytes_ = 0;
};

class OtherContextPool : public arrow::MemoryPool {
 public:
  explicit OtherContextPool(bitar_hip_ctx* ctx) : ctx_(ctx) {}
  arrow::Status Allocate(int64_t size, int64_t, uint8_t** out) override {
    void* p = nullptr;
    if (bitar_hip_alloc(ctx_, static_cast<uint64_t>(size ? size : 1), &p) != 0)
      return arrow::Status::OutOfMemory("bitar_hip_alloc");
    *out = static_cast<uint8_t*>(p);
    bytes_ += size;
    return arrow::Status::OK();
  }
  arrow::Status Reallocate(int64_t, int64_t, int64_t, uint8_t**) override {
    return arrow::Status::NotImplemented("fixed-size test pool");
  }
  void Free(uint8_t* p, int64_t size, int64_t) override {
    (void)bitar_hip_free(ctx_, p);
    bytes_ -= size;
  }
  int64_t bytes_allocated() const override { return bytes_; }
  std::string backend_name() const override { return "other_context"; }
  int64_t max_memory() const override { return -1; }
  int64_t total_bytes_allocated() const override { return 0; }
  int64_t num_allocations() const override { return 0; }

 private:
  bitar_hip_ctx* ctx_;
  int64_t bytes_ = 0;
};

// one HBM byte back to the host
uint8_t DeviceByte(bitar_hip_ctx* ctx, const uint8_t* at) {
  uint8_t v = 0;
  CHECK(bitar_hip_memcpy(ctx, &v, at, 1, nullptr) == 0);
  CHECK(bitar_hip_sync(ctx, nullptr) == 0);
  return v;
}

void PoolTests(bool expect_poison, const std::string& input_path) {
  CHECK(bitar::PoolPoisons() == expect_poison);
  bitar_hip_config cfg{1, 0};
  bitar_hip_ctx* other = nullptr;
  CHECK(bitar_hip_open(0, &cfg, &other) == 0);
  if (!other) return;
  if (expect_poison) {
    // debug-build pool poisoning (reference memory_pool.cc:190-263): 0xBC at both ends of a
    // fresh allocation, 0xBD at both ends of a reallocation's grown part, kept bytes intact;
    // 0xBE at both ends of a freed host buffer (HBM is returned to the driver unpoisoned)
    auto* pool = bitar::GetMemoryPool(bitar::MemoryPoolBackend::HipHost);
    uint8_t* p = nullptr;
    CHECK_OK(pool->Allocate(100, 64, &p));
    CHECK(p[0] == 0xBC && p[99] == 0xBC);
    std::memset(p, 7, 100);
    CHECK_OK(pool->Reallocate(100, 300, 64, &p));
    CHECK(p[0] == 7 && p[99] == 7 && p[100] == 0xBD && p[299] == 0xBD);
    pool->Free(p, 300, 64);
    // the HBM pool, read back through the ABI's copy
    auto* dpool = bitar::GetMemoryPool(bitar::MemoryPoolBackend::HipDevice);
    uint8_t* d = nullptr;
    CHECK_OK(dpool->Allocate(4096, 64, &d));
    CHECK(DeviceByte(other, d) == 0xBC && DeviceByte(other, d + 4095) == 0xBC);
    static const uint8_t k7[2] = {7, 7};
    CHECK(bitar_hip_memcpy(other, d, k7, 1, nullptr) == 0 &&
          bitar_hip_memcpy(other, d + 4095, k7, 1, nullptr) == 0 &&
          bitar_hip_sync(other, nullptr) == 0);
    CHECK_OK(dpool->Reallocate(4096, 10000, 64, &d));
    CHECK(DeviceByte(other, d) == 7 && DeviceByte(other, d + 4095) == 7);
    CHECK(DeviceByte(other, d + 4096) == 0xBD && DeviceByte(other, d + 9999) == 0xBD);
    dpool->Free(d, 10000, 64);
    CHECK(pool->bytes_allocated() == 0 && dpool->bytes_allocated() == 0);
  }
  // buffers the front-end did not allocate, through Compress and Decompress
  const auto data = ReadFile(input_path);
  CHECK(data.size() > 100000);
  auto* driver = bitar::CompressDriver<bitar::Class_HIP_GFX950>::Instance();
  auto ids = driver->ListAvailableDeviceIds();
  CHECK_OK(ids.status());
  if (!ids.ok()) return;
  RegisteredPool registered;
  OtherContextPool foreign(other);
  for (const auto codec : {bitar::Codec::LZ4, bitar::Codec::DEFLATE, bitar::Codec::ZSTD}) {
    const std::uint32_t seg = codec == bitar::Codec::DEFLATE ? 59460 : 65536;
    const auto nseg = (data.size() + seg - 1) / seg;
    auto devs = driver->GetDevices({(*ids)[0]});
    CHECK_OK(devs.status());
    if (!devs.ok()) return;
    auto& d = (*devs)[0];
    CHECK_OK(d->Initialize(MakeConfig(codec, seg)));
    for (arrow::MemoryPool* pool : {static_cast<arrow::MemoryPool*>(&registered),
                                    static_cast<arrow::MemoryPool*>(&foreign)}) {
      const bool host = pool == &registered;
      auto in = arrow::AllocateBuffer(static_cast<int64_t>(data.size()), pool);
      CHECK_OK(in.status());
      if (!in.ok()) continue;
      std::shared_ptr<arrow::Buffer> input = std::move(*in);
      if (host) {
        std::memcpy(input->mutable_data(), data.data(), data.size());
      } else {
        CHECK(bitar_hip_memcpy(other, input->mutable_data(), data.data(), data.size(), nullptr) == 0);
        CHECK(bitar_hip_sync(other, nullptr) == 0);
      }
      auto comp = d->Compress(0, input);
      CHECK_OK(comp.status());
      if (!comp.ok()) continue;
      CHECK(comp->size() == nseg);
      auto o = arrow::AllocateResizableBuffer(static_cast<int64_t>(nseg * seg), pool);
      CHECK_OK(o.status());
      if (!o.ok()) continue;
      std::unique_ptr<arrow::ResizableBuffer> out = std::move(*o);
      // (the foreign pool cannot grow a buffer: the output is allocated at full capacity)
      CHECK_OK(d->Decompress(0, *comp, out));
      CHECK(out->size() == static_cast<int64_t>(data.size()));
      std::vector<uint8_t> back(data.size());
      if (host) {
        std::memcpy(back.data(), out->data(), data.size());
      } else {
        CHECK(bitar_hip_memcpy(other, back.data(), out->data(), data.size(), nullptr) == 0);
        CHECK(bitar_hip_sync(other, nullptr) == 0);
      }
      CHECK(std::memcmp(back.data(), data.data(), data.size()) == 0);
      CHECK(d->Recycle(*comp) == comp->size());
    }
  }
  CHECK(registered.bytes_allocated() == 0 && foreign.bytes_allocated() == 0);
  CHECK(bitar_hip_close(other) == 0);
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "cpu";
  CpuTests();
  if (mode == "cpu") {
    // no GPU in the build container: discovery must fail cleanly, not crash
    auto ids = bitar::CompressDriver<bitar::Class_HIP_GFX950>::Instance()->ListAvailableDeviceIds();
    if (!ids.ok()) CHECK(ids.status().IsInvalid());
  } else if (argc >= 4 && mode == "pool") {
    PoolTests(std::string(argv[2]) == "1", argv[3]);
  } else if (argc >= 4 && mode == "arrow") {
    ArrowCodecTests(argv[2], argv[3]);
  } else if (argc >= 4) {
    GpuTests(argv[2], argv[3]);
  } else {
    std::cerr << "usage: frontend_test cpu | gpu <input> <outdir> | arrow <input> <outdir> | pool <0|1> <input>\n";
    return 2;
  }
  std::cout << (g_failures ? "FAILED " : "PASSED ") << g_failures << " failures\n";
  return g_failures ? 1 : 0;
}
