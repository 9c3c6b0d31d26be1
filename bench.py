#!/usr/bin/env python3
"""bench.py -- the driver-facing benchmark of the MI355X segment codec engine.

Headline (BASELINE.json metric "GiB/s compress+decompress on 1-GiB Arrow buffer";
configs[2]): a job of N GiB of the Silesia-style mix (kind 1) cut into 64 KiB
segments, dealt to the N ranks in round-robin batches of 256 segments (bitar_amd.dist,
apps/demo_app.cc:249-256), so every GPU holds 1 GiB in HBM (weak scaling).  One step = LZ4
compress of the rank's segments into per-segment slots + the RCCL all-gather of the
per-segment compressed sizes and the global frame index + LZ4 decompress of every slot.
value = uncompressed bytes round-tripped by all ranks / wall time (max over ranks).

Beside it, on the same JSON line:
  recordbatch   BASELINE configs[3]: an 8 GiB Arrow record-batch job (64 KiB chunks), the
                same round-robin batches, K queue-pair streams per GPU running concurrently
                (CompressAsync / DecompressAsync, util.h:216-236), RCCL size all-gather;
                total work fixed (strong scaling), at every N.
  secondary     BASELINE configs[1]: 1 GiB random bytes, LZ4 decompress only (N = 1).
  zstd          BASELINE configs[4]: Zstd frames on Arrow record-batch bodies (weak).
  deflate       the reference's own codec (raw DEFLATE, 59460-B segments; weak).
  stock_decode  GPU decode of streams the STOCK libraries wrote on the host (liblz4 default,
                zlib level 1 raw DEFLATE = the reference's codec, libzstd level 1), N = 1.
  stock_ratio   the stock libraries' ratio on the headline input, beside ours.
  cpu_baseline  stock liblz4 / zlib-1 on this host's cores, 1 core and all cores, plus
                BASELINE configs[0] (1 MiB Arrow IPC of a Parquet-like table, 1 core).

Launch: python bench.py [--gpus N --steps K --warmup W].  With --gpus N > 1 and no launcher
around it, the process starts N rank processes itself (bitar_amd.launch; the parent never
touches the GPU); under torch.distributed.run the ranks come from the environment.  Rank 0
prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--bytes", type=int, default=1 << 30, help="headline bytes per rank")
    p.add_argument("--seg", type=int, default=65536)
    p.add_argument("--kind", type=int, default=1, help="0 random, 1 mixed, 2 arrow")
    p.add_argument("--codec", default="lz4",
                   choices=["lz4", "deflate", "zstd", "deflate_dyn", "lz4_wide"])
    p.add_argument("--streams", type=int, default=4,
                   help="queue-pair streams per GPU in the configs[3] record-batch leg")
    p.add_argument("--record-bytes", type=int, default=8 << 30,
                   help="total job bytes of the configs[3] record-batch leg")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=256 << 20)
    p.add_argument("--no-secondary", action="store_true",
                   help="skip the random-data decompress-only line (BASELINE configs[1])")
    p.add_argument("--no-zstd", action="store_true")
    p.add_argument("--no-deflate", action="store_true")
    p.add_argument("--no-recordbatch", action="store_true")
    p.add_argument("--no-lz4-arrow", action="store_true",
                   help="skip the kind-2 (Arrow record batch) LZ4 round-trip line")
    p.add_argument("--no-lz4-wide", action="store_true",
                   help="skip the wide-parse LZ4 leg (the ratio operating point)")
    p.add_argument("--no-stock", action="store_true",
                   help="skip the stock-stream GPU decode legs")
    p.add_argument("--no-qp2", action="store_true",
                   help="skip the headline job over two queue-pair streams (informational)")
    p.add_argument("--only", default=None,
                   help="comma list of legs to run besides the headline (profiling runs)")
    p.add_argument("--traffic-json", default=os.path.join(HERE, "profiles", "traffic.json"))
    return p.parse_args()


# every kernel one compress / decompress call launches (a "+" list: the HIP events bracket
# them together and the PMC traffic is their sum; a templated kernel counts all its
# instantiations -- lz4_decompress_kernel<false> then <true> for the deferred segments)
KERNELS = {"lz4": ("lz4_compress_kernel", "lz4_decompress_kernel"),
           # the wide parse (16 KiB history): same kernels, other template instance; offsets
           # past the decoder's LDS ring take lz4_decompress_kernel<true> (far history)
           "lz4_wide": ("lz4_compress_kernel", "lz4_decompress_kernel"),
           # decompress = inflate_fixed_kernel (inflate.hip built with the 9/8-bit tables of
           # the fixed code, picked on the FIXED hint; the lane-per-segment
           # inflate_lanes_kernel runs in front only when a context turns it on)
           "deflate": ("deflate_compress_kernel", "inflate_fixed_kernel"),
           # compress = zstd_parse_kernel + zstd_entropy_kernel + zstd_walk_kernel (FSE state
           # chains, a lane per chain) + zstd_emit_kernel (sequence bitstream); decompress =
           # zstd_lanes_kernel (predefined-table frames) + zstd_decompress_kernel (headers,
           # tables) + zstd_hlit_kernel (Huffman literals) + zstd_seqdec_kernel (FSE chains ->
           # records, lane per segment) + zstd_exec_kernel (records -> output, wave per
           # segment) + zstd_handoff_kernel (what seqdec did not take)
           "zstd": ("zstd_parse_kernel+zstd_entropy_kernel+zstd_walk_kernel+zstd_emit_kernel",
                    "zstd_lanes_kernel+zstd_decompress_kernel+zstd_hlit_kernel+"
                    "zstd_seqdec_kernel+zstd_exec_kernel+zstd_handoff_kernel"),
           # compress = deflate_dyn_parse_kernel + deflate_dyn_emit_kernel (one event pair
           # brackets both); decompress = inflate_kernel (10/9-bit tables, the DYNAMIC hint)
           "deflate_dyn": ("deflate_dyn_parse_kernel+deflate_dyn_emit_kernel",
                           "inflate_kernel")}
CODEC_NAMES = {"lz4": "lz4-block", "deflate": "deflate-raw-fixed", "zstd": "zstd-frame",
               "deflate_dyn": "deflate-raw-dynamic", "lz4_wide": "lz4-block (wide parse)"}


def codec_id(name):
    import bitar_amd
    return {"lz4": bitar_amd.CODEC_LZ4, "deflate": bitar_amd.CODEC_DEFLATE,
            "zstd": bitar_amd.CODEC_ZSTD, "deflate_dyn": bitar_amd.CODEC_DEFLATE_DYNAMIC,
            "lz4_wide": bitar_amd.CODEC_LZ4_WIDE}[name]


def reduce_max_sum(vals_max, vals_sum, world):
    """MAX over ranks of vals_max, SUM over ranks of vals_sum (float64 lists); a collective
    whenever a process group is up (also a one-rank RCCL group)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return list(vals_max), list(vals_sum)
    # RCCL reduces device tensors; gloo (the one-GPU rehearsal) host tensors
    dev = f"cuda:{torch.cuda.current_device()}" if dist.get_backend() == "nccl" else "cpu"
    a = torch.tensor(list(vals_max), dtype=torch.float64, device=dev)
    b = torch.tensor(list(vals_sum), dtype=torch.float64, device=dev)
    dist.all_reduce(a, op=dist.ReduceOp.MAX)
    dist.all_reduce(b, op=dist.ReduceOp.SUM)
    return a.tolist(), b.tolist()


def run_job(eng, codec_name, kind, job_bytes, seg, nstreams, steps, warmup, world, rank,
            seed=0):
    """K timed steps of a sharded job (bitar_amd.job.ShardedJob): compress on every part's
    stream, RCCL size all-gather + global frame index, decompress.  Returns the timings
    (max over ranks), the byte-equality verdict (all ranks) and the job's sizes."""
    import torch
    import torch.distributed as dist
    from bitar_amd.job import ShardedJob
    job = ShardedJob(eng, codec_id(codec_name), job_bytes, seg, world, rank, nstreams)
    job.generate(kind, seed)
    dev = eng.device
    ev = []  # per step: {part stream: (c0, c1)}, {part stream: (d0, d1)}

    def step(timed):
        if timed:
            ce = {p.stream: (torch.cuda.Event(enable_timing=True),
                             torch.cuda.Event(enable_timing=True)) for p in job.layout.parts}
            de = {p.stream: (torch.cuda.Event(enable_timing=True),
                             torch.cuda.Event(enable_timing=True)) for p in job.layout.parts}
            ev.append((ce, de))
        else:
            ce = de = None
        job.compress(ce)
        job.gather_index()
        job.decompress(de)

    for _ in range(warmup):
        step(False)
    job.sync()
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        step(True)
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    job.sync()  # raises if any segment op failed
    ok = job.verify()
    csize = job.local_compressed_bytes()
    ok = ok and int(job.index[-1].item()) >= csize  # the global index spans the job
    # per-launch durations (each event pair brackets exactly one kernel launch)
    comp_ms = [c0.elapsed_time(c1) for ce, _ in ev for c0, c1 in ce.values()]
    dec_ms = [d0.elapsed_time(d1) for _, de in ev for d0, d1 in de.values()]

    def span(evs):  # first start to last end of one step's concurrent launches (ms)
        ref = next(iter(evs.values()))[0]
        return (max(ref.elapsed_time(e1) for _, e1 in evs.values()) -
                min(ref.elapsed_time(e0) for e0, _ in evs.values()))
    comp_span = [span(ce) for ce, _ in ev]
    dec_span = [span(de) for _, de in ev]
    local = {"nbytes": job.layout.local_bytes, "nseg": job.layout.local_nseg,
             "parts": len(job.layout.parts)}
    total_c = int(job.index[-1].item())
    job.free()
    t_comp, t_dec = sum(comp_ms) / len(comp_ms) / 1e3, sum(dec_ms) / len(dec_ms) / 1e3
    # max over ranks, and the per-rank spread (min through the max of the negation), so the
    # first multi-GPU run can be diagnosed from its line: a slow rank shows as max/min > 1
    (elapsed, bad, tc_max, td_max, n_el, n_tc, n_td), (csum,) = reduce_max_sum(
        [elapsed, 0.0 if ok else 1.0, t_comp, t_dec, -elapsed, -t_comp, -t_dec], [float(csize)], world)
    spread = {"elapsed_s": [round(-n_el, 6), round(elapsed, 6)],
              "compress_launch_ms": [round(-n_tc * 1e3, 4), round(tc_max * 1e3, 4)],
              "decompress_launch_ms": [round(-n_td * 1e3, 4), round(td_max * 1e3, 4)],
              "elapsed_max_over_min": round(elapsed / -n_el, 4) if n_el else None}
    return {"elapsed": elapsed, "ok": bad == 0.0, "csize_local": csize, "csize_total": total_c,
            "rank_spread": spread,
            "t_comp": t_comp, "t_dec": t_dec,
            "t_comp_span": sum(comp_span) / len(comp_span) / 1e3,
            "t_dec_span": sum(dec_span) / len(dec_span) / 1e3,
            "local": local, "job_bytes": job_bytes}


def kernel_lines(codec_name, r, traffic_json, leg="headline"):
    """roofline of the dominant kernel + per-kernel averages.  Durations are HIP events
    bracketing each launch on its own stream; algorithmic bytes per launch =
    U + C (+ 4 B per segment for compress) of the part that launch covered."""
    parts = r["local"]["parts"]
    U = float(r["local"]["nbytes"]) / parts
    C = float(r["csize_local"]) / parts
    nseg = float(r["local"]["nseg"]) / parts
    comp_bytes = U + C + 4.0 * nseg
    dec_bytes = U + C
    kc, kd = KERNELS[codec_name]
    t_comp, t_dec = r["t_comp"], r["t_dec"]
    dominant = (kc, comp_bytes, t_comp) if t_comp >= t_dec else (kd, dec_bytes, t_dec)
    if parts > 1:
        # the parts' launches run at once on their queue-pair streams: one launch's duration
        # is not its share of the GPU.  The roofline is the step's launches together: all
        # parts' bytes over first start to last end.
        tc, td = r["t_comp_span"], r["t_dec_span"]
        dominant = ((f"{kc} x{parts} concurrent", comp_bytes * parts, tc) if tc >= td else
                    (f"{kd} x{parts} concurrent", dec_bytes * parts, td))
    achieved = dominant[1] / dominant[2] / 1e9
    traffic = None
    try:
        with open(traffic_json) as f:
            # per-launch HBM bytes of this leg's kernel(s), from its own PMC passes
            tj = json.load(f)
            per = [tj.get(f"{leg}/{k}") for k in dominant[0].split(" ")[0].split("+")]
            # (concurrent parts: the roofline covers all of the step's launches of the kernel)
            traffic = sum(per) * parts if all(p is not None for p in per) else None
    except (OSError, ValueError):
        pass
    roof = {"bound": "hbm", "kernel": dominant[0], "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            # traffic is not measured in this run: a bench run under --pmc would perturb the
            # timing, so it is the per-launch PMC figure of this leg's kernels from the
            # committed profile (scripts/gpu_bench.sh PROFILE=1 -> scripts/collect_profile.py)
            "traffic_source": (f"committed PMC profile {os.path.relpath(traffic_json, HERE)} "
                               f"(FETCH_SIZE x2 + WRITE_SIZE per launch, separate --pmc passes)"
                               if traffic is not None else None),
            "algorithmic_bytes_per_launch": dominant[1],
            "avg_launch_ms": round(dominant[2] * 1e3, 4)}
    kernels = {kc: {"avg_ms": round(t_comp * 1e3, 4), "alg_GBs": round(comp_bytes / t_comp / 1e9, 2)},
               kd: {"avg_ms": round(t_dec * 1e3, 4), "alg_GBs": round(dec_bytes / t_dec / 1e9, 2)}}
    return roof, kernels


def leg_summary(name, r, world, steps, traffic_json, workload, leg=None):
    roof, kern = kernel_lines(name, r, traffic_json, leg or name)
    U = float(r["job_bytes"])
    return {"workload": workload,
            "value": round(U * steps / r["elapsed"] / GIB, 3), "unit": "GiB/s",
            "ms_per_step": round(r["elapsed"] / steps * 1e3, 4),
            "compression_ratio": round(U / r["csize_total"], 4) if r["csize_total"] else None,
            "compress_gibs_per_launch": round(r["local"]["nbytes"] / r["local"]["parts"] / r["t_comp"] / GIB, 3),
            "decompress_gibs_per_launch": round(r["local"]["nbytes"] / r["local"]["parts"] / r["t_dec"] / GIB, 3),
            "roundtrip_ok": r["ok"], "roofline": roof, "kernels": kern,
            **({"rank_spread": r["rank_spread"]} if world > 1 else {})}


def random_decompress(eng, n, seg, args):
    """BASELINE configs[1]: 1 GiB random bytes, LZ4 decompress only."""
    import torch
    import bitar_amd
    codec = bitar_amd.CODEC_LZ4
    nseg = (n + seg - 1) // seg
    stride = bitar_amd.slot_size(codec, seg)
    data = eng.empty(n)
    slab = eng.empty(nseg * stride)
    sizes = eng.empty(nseg, dtype=torch.int32)
    out = eng.empty(nseg * seg)
    prod = eng.empty(nseg, dtype=torch.int32)
    stream = torch.cuda.current_stream()
    eng.fill(0, 1, data)
    eng.compress_into(codec, data, seg, slab, stride, sizes, n=n)
    eng.sync()
    c_rand = float(sizes.to(torch.int64).sum().item())
    evs = []
    for i in range(args.warmup + args.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        eng.decompress_slab_into(codec, slab, stride, sizes, nseg, seg, out, prod,
                                 capacity=nseg * seg)
        e1.record(stream)
        if i >= args.warmup:
            evs.append((e0, e1))
    torch.cuda.synchronize()
    eng.sync()
    ok2 = bool(torch.equal(out[:n], data))
    t2 = sum(a.elapsed_time(b) for a, b in evs) / len(evs) / 1e3
    alg2 = (float(n) + c_rand) / t2 / 1e9
    del data, slab, out
    torch.cuda.empty_cache()
    return {
        "workload": "BASELINE configs[1]: 1 GiB random bytes, LZ4 block decompress only, "
                    "64 KiB segments, HBM-resident",
        "decompress_gibs": round(n / t2 / GIB, 3), "avg_launch_ms": round(t2 * 1e3, 4),
        "roofline": {"bound": "hbm", "kernel": "lz4_decompress_kernel",
                     "achieved": round(alg2, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(alg2 / HBM_PEAK_GBS, 4),
                     "algorithmic_bytes_per_launch": float(n) + c_rand},
        "roundtrip_ok": ok2}


def host_threads():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        return os.cpu_count() or 1


def cpu_quota():
    """CPUs' worth of time this process's cgroup may use (cgroup v2 cpu.max), None if
    unlimited or unknown: the GPU box shares its host CPUs, so this can be far below the
    visible core count."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        return None


def stock_decode(eng, args):
    """GPU decode of streams the stock libraries produced on the host from the same input
    (compressed and uploaded outside the timed region; the decode is timed with HIP events
    and checked byte for byte).  Also yields the stock ratios of the headline input."""
    import numpy as np
    import torch
    import bitar_amd
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import stock_lib as S  # stock third-party codecs (baseline infrastructure)
    n = args.bytes
    th = baseline_threads()
    legs = (("lz4", S.LZ4, 1, 65536, args.kind, "liblz4 1.9.3 LZ4_compress_default"),
            ("deflate", S.DEFLATE, 1, 59460, args.kind,
             "zlib 1.2.11 raw DEFLATE level 1 (dynamic Huffman), the reference's codec "
             "(config.cc:83-105) at its 59460-B segments (app_common.h:39)"),
            ("zstd", S.ZSTD, 1, 65536, 2, "libzstd level 1 (Huffman literals, FSE tables)"))
    res, ratios = {}, {}
    for name, sc, level, seg, kind, desc in legs:
        data = eng.empty(n)
        eng.fill(kind, 0, data)
        host = data.cpu().numpy()
        slab_h, stride, sizes_h = S.compress(sc, host, seg, level, th)
        nseg = sizes_h.size
        C = float(sizes_h.astype(np.int64).sum())
        ratios[name] = round(n / C, 4)
        slab = torch.from_numpy(slab_h).to(f"cuda:{eng.device}")
        sizes = torch.from_numpy(sizes_h.view(np.int32)).to(f"cuda:{eng.device}")
        del slab_h, host
        out = eng.empty(nseg * seg)
        prod = eng.empty(nseg, dtype=torch.int32)
        stream = torch.cuda.current_stream()
        # (zlib level 1 writes dynamic-Huffman blocks: the DYNAMIC hint, HuffmanEncoding's
        # default, picks the inflater built for them)
        codec = codec_id("deflate_dyn" if name == "deflate" else name)
        evs = []
        for i in range(args.warmup + args.steps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            eng.decompress_slab_into(codec, slab, stride, sizes, nseg, seg, out, prod,
                                     capacity=nseg * seg)
            e1.record(stream)
            if i >= args.warmup:
                evs.append((e0, e1))
        torch.cuda.synchronize()
        try:
            eng.sync()
        except bitar_amd.BitarError as e:
            p = prod.cpu().numpy().view(np.uint32)
            bad = np.nonzero(p == 0xFFFFFFFF)[0]
            raise RuntimeError(f"stock {name} decode: {e}; {bad.size} failed segments, first "
                               f"{bad[:8].tolist()}") from e
        ok = bool(torch.equal(out[:n], data)) and int(prod.to(torch.int64).sum().item()) == n
        t = sum(a.elapsed_time(b) for a, b in evs) / len(evs) / 1e3
        alg = (n + C) / t / 1e9
        res[name] = {"stream": desc, "input_kind": kind, "segment_bytes": seg,
                     "stock_ratio": ratios[name], "decompress_gibs": round(n / t / GIB, 3),
                     "avg_launch_ms": round(t * 1e3, 4),
                     "roofline": {"bound": "hbm", "achieved": round(alg, 2),
                                  "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": round(alg / HBM_PEAK_GBS, 4),
                                  "algorithmic_bytes_per_launch": n + C},
                     "roundtrip_ok": ok}
        del data, slab, sizes, out, prod
        torch.cuda.empty_cache()
    return res, ratios


def ipc_sample(nbytes):
    """BASELINE configs[0]'s input: the first nbytes of an Arrow IPC stream of a synthetic
    Parquet-like table (seed 42: int64 uniform [0,1000), float64 N(0,1), dictionary
    strings), as demo_app's ReadTableBytes serializes a table (demo_app.cc:195-204)."""
    import numpy as np
    try:
        import pyarrow as pa
    except ImportError:  # pragma: no cover - pyarrow is in this image
        return None
    rng = np.random.default_rng(42)
    rows = max(1, nbytes // 12)
    words = np.array([f"value_{i:04d}" for i in range(500)])
    t = pa.table({"i": pa.array(rng.integers(0, 1000, rows, dtype=np.int64)),
                  "f": pa.array(rng.standard_normal(rows)),
                  "s": pa.DictionaryArray.from_arrays(
                      pa.array(rng.integers(0, 500, rows).astype(np.int32)),
                      pa.array(words))})
    sink = pa.BufferOutputStream()
    with pa.ipc.new_stream(sink, t.schema) as w:
        w.write_table(t)
    buf = np.frombuffer(sink.getvalue(), np.uint8)
    return buf[:nbytes].copy()


def baseline_threads():
    """Threads for the all-core CPU baseline: the CPUs this process may run on, capped by its
    cgroup CPU-time quota (the GPU box shows 256 CPUs but grants 16 cores' worth): more
    threads than the quota only thrash."""
    n = host_threads()
    q = cpu_quota()
    if q:
        n = min(n, max(1, int(-(-q // 1))))
    return n


def cpu_baseline(args):
    """The CPU baseline of BASELINE.md §2 on this host's cores, over a bounded sample of the
    same workload, best of kNumTests = 3 (apps/demo_app.h:45): stock liblz4 (the north-star
    codec, 64 KiB segments), zlib level-1 raw DEFLATE (the reference's codec, 59460-B
    segments) and libzstd level 1 (configs[4]'s codec, 64 KiB segments, kind-2 input), each
    on 1 core and on every core the process may use (`cores`); plus BASELINE configs[0] on 1
    core, and the oracle's C restatement of our LZ4 path ("port") beside them."""
    import numpy as np
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import oracle_lib as O  # the generator of the same input + the port (baseline leg only)
    import stock_lib as S
    nall = baseline_threads()
    n = args.cpu_sample
    data = O.fill(args.kind, 0, n)
    data2 = None

    def timed(sc, seg, level, sample, threads, reps=3, src=None):
        d = (data if src is None else src)[:sample]
        slab, stride, sizes = S.compress(sc, d, seg, level, threads)  # warm-up (+ pages)
        out = S.decompress(sc, slab, stride, sizes, sample, seg, threads)
        assert np.array_equal(out, d)
        bc = bd = 1e30
        for _ in range(reps):
            t0 = time.perf_counter()
            S.compress(sc, d, seg, level, threads, stride=stride)
            t1 = time.perf_counter()
            S.decompress(sc, slab, stride, sizes, sample, seg, threads, out=out)
            t2 = time.perf_counter()
            bc, bd = min(bc, t1 - t0), min(bd, t2 - t1)
        return {"roundtrip_gibs": round(sample / GIB / (bc + bd), 4),
                "compress_gibs": round(sample / GIB / bc, 4),
                "decompress_gibs": round(sample / GIB / bd, 4),
                "ratio": round(sample / float(sizes.astype(np.int64).sum()), 4),
                "sample_bytes": sample, "threads": threads}

    lz4_all = timed(S.LZ4, 65536, 1, n, nall)
    lz4_one = timed(S.LZ4, 65536, 1, min(n, 64 << 20), 1)
    # zlib-1 compresses ~0.15 GiB/s per core: smaller samples keep this leg ~10 s
    z_all = timed(S.DEFLATE, 59460, 1, min(n, max(16 << 20, nall * (8 << 20))), nall)
    z_one = timed(S.DEFLATE, 59460, 1, 16 << 20, 1)
    # libzstd level 1 on the configs[4] input (the kind-2 Arrow record batch)
    zs_n = min(n, max(64 << 20, nall * (16 << 20)))
    data2 = O.fill(2, 1000, zs_n)
    zs_all = timed(S.ZSTD, 65536, 1, zs_n, nall, src=data2)
    zs_one = timed(S.ZSTD, 65536, 1, min(zs_n, 32 << 20), 1, src=data2)
    # the port: the oracle's C restatement of this path (window-scan parse + LZ4 emitter,
    # LZ4 block decode), bit-exact with the GPU kernels
    pn = min(n, 16 << 20)
    stride = O.lz4_bound(65536) + 256 & ~255

    def port(threads):
        best_c = best_d = 1e30
        for _ in range(2):
            t0 = time.perf_counter()
            r, slab, sizes = O.compress_segments(O.CODEC_LZ4, data[:pn], 65536, stride, threads)
            t1 = time.perf_counter()
            assert r == 0
            blobs = [slab[i * stride:i * stride + sizes[i]] for i in range(sizes.size)]
            t2 = time.perf_counter()
            r, out, _ = O.decompress_segments(O.CODEC_LZ4, blobs, 65536, pn, threads)
            t3 = time.perf_counter()
            assert r == 0 and np.array_equal(out, data[:pn])
            best_c, best_d = min(best_c, t1 - t0), min(best_d, t3 - t2)
        return {"roundtrip_gibs": round(pn / GIB / (best_c + best_d), 4),
                "compress_gibs": round(pn / GIB / best_c, 4),
                "decompress_gibs": round(pn / GIB / best_d, 4),
                "ratio": round(pn / float(sizes.astype(np.int64).sum()), 4),
                "sample_bytes": pn, "threads": threads}

    cfg0 = None
    ipc = ipc_sample(1 << 20)
    if ipc is not None:
        c0 = {}
        for name, sc, seg in (("deflate_raw_l1_59460", S.DEFLATE, 59460),
                              ("lz4_64k", S.LZ4, 65536)):
            slab, stride0, sizes = S.compress(sc, ipc, seg, 1, 1)
            out = S.decompress(sc, slab, stride0, sizes, ipc.size, seg, 1)
            assert np.array_equal(out, ipc)
            reps = 20
            t0 = time.perf_counter()
            for _ in range(reps):
                S.compress(sc, ipc, seg, 1, 1, stride=stride0)
            t1 = time.perf_counter()
            for _ in range(reps):
                S.decompress(sc, slab, stride0, sizes, ipc.size, seg, 1, out=out)
            t2 = time.perf_counter()
            tc, td = (t1 - t0) / reps, (t2 - t1) / reps
            c0[name] = {"compress_gibs": round(ipc.size / GIB / tc, 4),
                        "decompress_gibs": round(ipc.size / GIB / td, 4),
                        "roundtrip_gibs": round(ipc.size / GIB / (tc + td), 4),
                        "ratio": round(ipc.size / float(sizes.astype(np.int64).sum()), 4),
                        "segments": int(sizes.size)}
        cfg0 = {"workload": "BASELINE configs[0]: 1 MiB Arrow IPC stream of a Parquet-like "
                            "table (seed 42), 1 host core", **c0}
    return {
        "value": lz4_all["roundtrip_gibs"],
        "unit": "GiB/s",
        "cores": nall,
        "kind": "stock",
        "kind_note": "BASELINE.md §2's CPU baseline is the stock library: the reference has no "
                     "software LZ4 path and its DEFLATE is a hardware engine, so no 'reference' "
                     "build exists; 'port' (the oracle's C restatement of this LZ4 path) is "
                     "timed below",
        "sample": f"{n >> 20} MiB of the same kind-{args.kind} input, 65536-B segments, stock "
                  f"liblz4 1.9.3 (LZ4_compress_default + LZ4_decompress_safe) on {nall} "
                  f"threads = this process's CPU set ({host_threads()} CPUs, os.cpu_count() "
                  f"{os.cpu_count()}) capped by its cgroup quota ({cpu_quota()} cores), best of 3",
        "lz4": {"all_cores": lz4_all, "one_core": lz4_one},
        "deflate_zlib1": {"all_cores": z_all, "one_core": z_one,
                          "note": "the reference's codec in software: zlib 1.2.11 raw DEFLATE "
                                  "level 1, 59460-B segments"},
        "zstd_libzstd1": {"all_cores": zs_all, "one_core": zs_one,
                          "note": "BASELINE configs[4]'s codec: libzstd level 1, 65536-B "
                                  "segments, kind-2 Arrow record-batch input"},
        "port": {"all_cores": port(nall), "one_core": port(1),
                 "note": "oracle/bitar_oracle.c: the CPU restatement of the GPU LZ4 path "
                         "(bit-exact), 16 MiB sample"},
        "configs0": cfg0,
        "os_cpu_count": os.cpu_count(),
        "affinity_cpus": host_threads(),
        "cpu_quota_cores": cpu_quota(),
    }


def frontend_legs(args, headline_ms):
    """The drop-in C++ API measured by bitar_amd/cpp/build/frontend_bench (a child process):
    CompressDevice::Compress + Decompress + Recycle on an HBM arrow::Buffer of the headline's
    size and input (reference apps/demo_app.cc:332-357), and the same round trip with
    host-resident (pinned) data, whose staging copies cross PCIe, beside the raw link rates."""
    import subprocess
    exe = os.path.join(HERE, "bitar_amd", "cpp", "build", "frontend_bench")
    if not os.path.exists(exe):
        return {"skipped": "bitar_amd/cpp/build/frontend_bench is not built"}, None
    cmd = [exe, "--bytes", str(args.bytes), "--seg", str(args.seg), "--kind", str(args.kind),
           "--steps", str(args.steps), "--warmup", str(args.warmup)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"failed": f"rc {p.returncode}: {p.stderr[-500:]}"}, None
    r = json.loads(lines[0])
    h = r["hbm"]
    fe = {"workload": r["workload"] + " (HBM-resident input and output)",
          "value": h["roundtrip_gibs"], "unit": "GiB/s", "ms_per_roundtrip": h["ms_per_roundtrip"],
          "compress_call_ms": h["compress_call_ms"], "decompress_call_ms": h["decompress_call_ms"],
          "recycle_call_ms": h["recycle_call_ms"], "compression_ratio": h["ratio"],
          "roundtrip_ok": r["roundtrip_ok"],
          # > 0: time the C++ front-end adds to the C-ABI headline step (host tables, slot
          # pool, the arrow::Buffer views, one stream sync per call)
          "overhead_vs_c_abi": round(h["ms_per_roundtrip"] / headline_ms - 1.0, 4)}
    hd = None
    if "host" in r:
        x = r["host"]
        hd = {"workload": "the same round trip with host-resident data: pinned HipHost "
                          "arrow::Buffer input (Compress stages it to HBM) and output "
                          "(Decompress stages it back) -- PCIe-inclusive, never the headline",
              "roundtrip_gibs": x["roundtrip_gibs"], "ms_per_roundtrip": x["ms_per_roundtrip"],
              "compress_call_ms": x["compress_call_ms"],
              "decompress_call_ms": x["decompress_call_ms"],
              "roundtrip_ok": r["host_roundtrip_ok"],
              "link_h2d_gibs": r["h2d_gibs"], "link_d2h_gibs": r["d2h_gibs"],
              "link_h2d_ms": r["h2d_ms"], "link_d2h_ms": r["d2h_ms"]}
    return fe, hd


def want(args, leg):
    if args.only is None:
        return True
    return leg in args.only.split(",")


def main():
    args = parse()
    from bitar_amd import launch
    if args.gpus > 1 and not launch.is_rank_process():
        # one process per GPU, started from this parent (which never touches the GPU)
        sys.exit(launch.spawn(args.gpus, os.path.abspath(__file__), sys.argv[1:]))
    import torch
    import torch.distributed as dist
    import bitar_amd

    world, rank, local = launch.rank_env()
    backend = launch.dist_backend()
    # a process group whenever a launcher started this rank (world 1 too: one-rank RCCL)
    use_dist = world > 1 or launch.is_rank_process()
    if use_dist:
        gpu = launch.rank_device(local, torch.cuda.device_count())
        torch.cuda.set_device(gpu)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{gpu}"))
        else:  # one-GPU rehearsal of the N-rank path (bitar_amd.launch.dist_backend)
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()
    eng = bitar_amd.Engine(dev, num_streams=max(1, args.streams))
    n, seg = args.bytes, args.seg
    r = run_job(eng, args.codec, args.kind, world * n, seg, 1, args.steps, args.warmup, world,
                rank)
    rb = zs = df = None
    if not args.no_recordbatch and want(args, "recordbatch"):
        rb = run_job(eng, "lz4", 2, args.record_bytes, 65536, max(1, args.streams),
                     args.steps, args.warmup, world, rank, seed=3)
    if args.codec != "zstd" and not args.no_zstd and want(args, "zstd"):
        zs = run_job(eng, "zstd", 2, world * n, seg, 1, args.steps, args.warmup, world, rank,
                     seed=1000)
    if args.codec != "deflate" and not args.no_deflate and want(args, "deflate"):
        df = run_job(eng, "deflate", args.kind, world * n, 59460, 1, args.steps, args.warmup,
                     world, rank, seed=2000)
    dd = None
    if args.codec != "deflate_dyn" and not args.no_deflate and want(args, "deflate_dyn"):
        # the reference's default frame: dynamic Huffman (config.h:151)
        dd = run_job(eng, "deflate_dyn", args.kind, world * n, 59460, 1, args.steps,
                     args.warmup, world, rank, seed=2000)
    ka = None
    if args.codec == "lz4" and args.kind != 2 and not args.no_lz4_arrow and want(args, "lz4_arrow"):
        # the Arrow record-batch input (kind 2) through the headline's LZ4 round trip, one
        # 1-GiB call per GPU (the harder, more representative LZ4 number)
        ka = run_job(eng, "lz4", 2, world * n, seg, 1, args.steps, args.warmup, world, rank,
                     seed=3)
    qp2 = None
    if args.codec == "lz4" and not args.no_qp2 and want(args, "qp2"):
        # the headline job split over two queue-pair streams (reference EvaluateAsync,
        # demo_app.cc:548-693): each half's decompress follows its compress on its stream, so
        # one half's compress overlaps the other's decompress (informational, not `value`)
        qp2 = run_job(eng, args.codec, args.kind, world * n, seg, 2, args.steps, args.warmup,
                      world, rank)
    lw = None
    if args.codec == "lz4" and not args.no_lz4_wide and want(args, "lz4_wide"):
        # the ratio operating point: the same job through the wide LZ4 parse
        lw = run_job(eng, "lz4_wide", args.kind, world * n, seg, 1, args.steps, args.warmup,
                     world, rank, seed=0)
    sec = stock = None
    if world == 1 and args.codec == "lz4":
        if not args.no_secondary and want(args, "secondary"):
            sec = random_decompress(eng, n, seg, args)
        if not args.no_stock and want(args, "stock"):
            stock = stock_decode(eng, args)
    if rank != 0:
        if use_dist:
            dist.destroy_process_group()
        return

    U = float(world * n)
    value = U * args.steps / r["elapsed"] / GIB
    roof, kernels = kernel_lines(args.codec, r, args.traffic_json)
    std = args.kind == 1 and args.codec == "lz4"
    res = {
        "metric": "GiB/s compress+decompress on 1-GiB Arrow buffer, 1/2/4/8 GPUs; % HBM roofline",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(r["elapsed"] / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (deterministic SplitMix64 generator, generated in HBM)",
        "config": {"workload": "LZ4 block compress + decompress round trip, 1 GiB per GPU, "
                               "64 KiB segments, Silesia-style mix (BASELINE configs[2])"
                               if std else f"{args.codec} round trip, kind {args.kind}, seg {seg}",
                   "bytes_per_gpu": n, "segment_bytes": seg,
                   "segments_per_gpu": r["local"]["nseg"],
                   "codec": CODEC_NAMES[args.codec],
                   "input_kind": args.kind,
                   "parallelism": (f"{world} ranks, round-robin batches of 256 segments, "
                                   + ("RCCL all-gather of sizes" if backend == "nccl" else
                                      f"{backend} all-gather of sizes (ranks sharing "
                                      f"{torch.cuda.device_count()} GPU(s): rehearsal)"))
                                  if use_dist else "1 GPU"},
        "compression_ratio": round(U / r["csize_total"], 4),
        "compress_gibs": round(r["local"]["nbytes"] / r["t_comp"] / GIB, 3),
        "decompress_gibs": round(r["local"]["nbytes"] / r["t_dec"] / GIB, 3),
        "roundtrip_ok": r["ok"],
        "roofline": roof,
        "kernels": kernels,
    }
    if world > 1:
        res["rank_spread"] = r["rank_spread"]
    if stock is not None:
        res["stock_ratio"] = {
            "ours_lz4": res["compression_ratio"] if std else None,
            "liblz4_default": stock[1]["lz4"],
            "zlib1_raw_deflate_59460": stock[1]["deflate"],
            "libzstd1_on_arrow_kind2": stock[1]["zstd"]}
    if rb is not None:
        s = leg_summary("lz4", rb, world, args.steps, args.traffic_json, leg="recordbatch", workload=
                        f"BASELINE configs[3]: {args.record_bytes >> 30} GiB Arrow record-batch "
                        f"job, 64 KiB chunks, round-robin batches of 256 chunks over {world} "
                        f"GPU(s), {args.streams} concurrent queue-pair streams per GPU, LZ4 "
                        f"compress + {'RCCL size all-gather + ' if use_dist and backend == 'nccl' else ''}decompress "
                        f"(total work fixed)")
        s["scaling"] = "strong"
        s["streams_per_gpu"] = args.streams
        res["recordbatch"] = s
    if sec is not None:
        res["secondary"] = sec
    if qp2 is not None:
        s = leg_summary(args.codec, qp2, world, args.steps, args.traffic_json, leg="headline",
                        workload="the headline job (same input, same work) split over 2 "
                                 "queue-pair streams per GPU: each half compresses then "
                                 "decompresses on its own stream, the halves overlapping")
        s["streams_per_gpu"] = 2
        res["headline_2qp"] = s
    if zs is not None:
        res["zstd"] = leg_summary(
            "zstd", zs, world, args.steps, args.traffic_json,
            "BASELINE configs[4] codec: level-1-class Zstd frame per 64 KiB segment "
            "(repeat-offset parse, Huffman literals, per-table FSE / RLE / predefined "
            "sequence codes), compress + decompress, 1 GiB Arrow record-batch buffer per GPU"
            + (", RCCL size all-gather" if use_dist and backend == "nccl" else ""))
    if df is not None:
        res["deflate"] = leg_summary(
            "deflate", df, world, args.steps, args.traffic_json,
            "the reference's codec: raw DEFLATE (fixed-Huffman blocks) per 59460-B segment, "
            "compress + decompress, same input and sharding as the headline")
    if dd is not None:
        res["deflate_dynamic"] = leg_summary(
            "deflate_dyn", dd, world, args.steps, args.traffic_json,
            "the reference's DEFAULT frame: raw DEFLATE with dynamic Huffman codes "
            "(HuffmanEncoding::DYNAMIC, config.h:151) per 59460-B segment, compress + "
            "decompress, same input and sharding as the headline")
    if ka is not None:
        res["lz4_arrow"] = leg_summary(
            "lz4", ka, world, args.steps, args.traffic_json,
            "the headline's LZ4 round trip on the Arrow record-batch input (kind 2: int64 / "
            "float64 / dictionary / string columns), 1 GiB per GPU, 64 KiB segments, one "
            "call", leg="lz4_arrow")
    if lw is not None:
        res["lz4_wide"] = leg_summary(
            "lz4_wide", lw, world, args.steps, args.traffic_json,
            "the ratio operating point: the headline job through the wide LZ4 parse "
            "(BITAR_HIP_CODEC_LZ4_WIDE: 16 KiB history window, 4096-entry table; ordinary "
            "LZ4 blocks), compress + decompress")
        if stock is not None:
            res["lz4_wide"]["liblz4_default_ratio"] = stock[1]["lz4"]
            res["stock_ratio"]["ours_lz4_wide"] = res["lz4_wide"]["compression_ratio"]
    if stock is not None:
        res["stock_decode"] = stock[0]
    if world == 1 and args.codec == "lz4" and (args.only is None or want(args, "frontend")):
        res["frontend"], hd = frontend_legs(args, res["ms_per_step"])
        if hd is not None:
            res["h2d_d2h"] = hd
    if not args.no_cpu_baseline and world == 1 and args.codec == "lz4" and args.only is None:
        res["cpu_baseline"] = cpu_baseline(args)
    print(json.dumps(res), flush=True)
    if use_dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
