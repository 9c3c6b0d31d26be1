#!/usr/bin/env python3
"""bench.py -- the driver-facing benchmark of the MI355X segment codec engine.

Workload (BASELINE.json metric "GiB/s compress+decompress on 1-GiB Arrow buffer";
configs[2]): every rank owns a 1 GiB HBM-resident buffer of the Silesia-style mix
(kind 1), cut into 64 KiB segments (16384 per GiB).  One step = LZ4 compress
of the whole buffer into per-segment slots + (N > 1) the RCCL all-gather of the per-segment
compressed sizes that builds the global frame index + LZ4 decompress of every slot back into
a 1 GiB output.  value = bytes of uncompressed data round-tripped by all ranks / wall time.
Beside it: "secondary" (BASELINE configs[1], random bytes, LZ4 decompress only, N = 1),
"zstd" (BASELINE configs[5], Zstd frames on Arrow record-batch bodies, same sharding and
all-gather at every N) and "deflate" (the reference's own codec at its 59460-B segments).

Prints ONE JSON line (rank 0).  Launch: python bench.py [--gpus N --steps K --warmup W];
for N > 1 under torch.distributed.run (one process per GPU, RCCL).
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
    p.add_argument("--bytes", type=int, default=1 << 30, help="bytes per rank")
    p.add_argument("--seg", type=int, default=65536)
    p.add_argument("--kind", type=int, default=1, help="0 random, 1 mixed, 2 arrow")
    p.add_argument("--codec", default="lz4", choices=["lz4", "deflate", "zstd"])
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-sample", type=int, default=256 << 20)
    p.add_argument("--no-secondary", action="store_true",
                   help="skip the random-data decompress-only line (BASELINE configs[1])")
    p.add_argument("--no-zstd", action="store_true",
                   help="skip the Zstd round-trip line (BASELINE configs[5])")
    p.add_argument("--no-deflate", action="store_true",
                   help="skip the DEFLATE line (the reference's own codec, 59460-B segments)")
    p.add_argument("--traffic-json", default=os.path.join(HERE, "profiles", "traffic.json"))
    return p.parse_args()


def cpu_baseline(args):
    """The oracle's C LZ4 codec (a port: bitar has no software LZ4 path)
    timed on this host's cores over a bounded sample of the same workload."""
    import ctypes
    import numpy as np
    sys.path.insert(0, os.path.join(HERE, "tests"))
    import oracle_lib as O  # cpu_baseline leg only: the oracle is the CPU reference here
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    n = args.cpu_sample
    seg = args.seg
    data = O.fill(args.kind, 0, n)
    stride = O.lz4_bound(seg) + 64
    nseg = (n + seg - 1) // seg
    L = O.lib()
    slab = np.zeros(nseg * stride, np.uint8)
    sizes = np.zeros(nseg, np.uint32)
    out = np.zeros(nseg * seg, np.uint8)
    prod = np.zeros(nseg, np.uint32)
    nout = ctypes.c_uint32(0)
    total = ctypes.c_uint64(0)

    def comp():
        r = L.bo_compress(O.CODEC_LZ4, O._ptr(data), n, seg, O._ptr(slab), stride, O._ptr(sizes),
                          ctypes.byref(nout), threads)
        assert r == 0

    ptrs = None

    def decomp():
        r = L.bo_decompress(O.CODEC_LZ4, O._ptr(ptrs), O._ptr(sizes), nseg, seg, O._ptr(out),
                            nseg * seg, ctypes.byref(total), O._ptr(prod), threads)
        assert r == 0

    comp()
    ptrs = np.array([slab.ctypes.data + i * stride for i in range(nseg)], dtype=np.uint64)
    decomp()
    assert np.array_equal(out[:n], data)
    best_c = best_d = 1e30
    for _ in range(3):  # best of kNumTests = 3 (reference apps/demo_app.h:45)
        t0 = time.perf_counter(); comp(); t1 = time.perf_counter(); decomp()
        t2 = time.perf_counter()
        best_c, best_d = min(best_c, t1 - t0), min(best_d, t2 - t1)
    return {
        "value": round(n / GIB / (best_c + best_d), 4),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{n >> 20} MiB of the same kind-{args.kind} input, {seg}-B segments, "
                  f"oracle C LZ4 (window-scan parse) compress+decompress, best of 3",
        "compress_gibs": round(n / GIB / best_c, 4),
        "decompress_gibs": round(n / GIB / best_d, 4),
    }


KERNELS = {"lz4": ("lz4_compress_kernel", "lz4_decompress_kernel"),
           # decompress = inflate_lanes_kernel (lane per segment) + inflate_kernel in
           # defer-only mode; timed together
           "deflate": ("deflate_compress_kernel", "inflate_lanes_kernel"),
           # decompress = zstd_lanes_kernel (lane per segment) + zstd_decompress_kernel in
           # defer-only mode (an early exit per segment for our frames); timed together
           "zstd": ("zstd_compress_kernel", "zstd_lanes_kernel")}
CODEC_NAMES = {"lz4": "lz4-block", "deflate": "deflate-raw-fixed", "zstd": "zstd-frame"}


def roundtrip(eng, ctx, codec_name, kind, n, seg, steps, warmup, seed):
    """K timed steps of compress (+ RCCL size all-gather + frame index when world > 1) +
    decompress of an n-byte HBM-resident buffer; returns the rank's timings and sizes."""
    import torch
    import torch.distributed as dist
    import bitar_amd
    from bitar_amd import dist as bd
    world = ctx["world"]
    codec = {"lz4": bitar_amd.CODEC_LZ4, "deflate": bitar_amd.CODEC_DEFLATE,
             "zstd": bitar_amd.CODEC_ZSTD}[codec_name]
    nseg = (n + seg - 1) // seg
    stride = bitar_amd.slot_size(codec, seg)
    data = eng.empty(n)
    eng.fill(kind, seed, data)  # the rank's shard of the job (weak scaling)
    slab = eng.empty(nseg * stride)
    sizes = eng.empty(nseg, dtype=torch.int32)
    out = eng.empty(nseg * seg)
    prod = eng.empty(nseg, dtype=torch.int32)
    all_sizes = eng.empty(nseg * world, dtype=torch.int32) if world > 1 else None
    index = [None]
    stream = torch.cuda.current_stream()
    ev = []  # (compress start, compress end, decompress start, decompress end)

    def step(timed):
        if timed:
            e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            e[0].record(stream)
        eng.compress_into(codec, data, seg, slab, stride, sizes, n=n)
        if timed:
            e[1].record(stream)
        if world > 1:  # global frame index: per-segment sizes of every rank
            dist.all_gather_into_tensor(all_sizes, sizes)
            index[0] = bd.frame_index(all_sizes)  # rank-major = global segment order
        if timed:
            e[2].record(stream)
        eng.decompress_slab_into(codec, slab, stride, sizes, nseg, seg, out, prod,
                                 capacity=nseg * seg)
        if timed:
            e[3].record(stream)
            ev.append(e)

    for _ in range(warmup):
        step(False)
    eng.sync()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.sync()  # raises if any segment op failed

    # correctness of the timed output (byte equality of the round trip, demo_app.cc:534-543)
    ok = bool(torch.equal(out[:n], data)) and int(prod.to(torch.int64).sum().item()) == n
    csize = int(sizes.to(torch.int64).sum().item())
    if world > 1:
        dev = torch.cuda.current_device()
        t = torch.tensor([elapsed, 0.0 if ok else 1.0, float(csize)], device=f"cuda:{dev}",
                         dtype=torch.float64)
        mx = t.clone()
        dist.all_reduce(mx[:2], op=dist.ReduceOp.MAX)
        sm = t.clone()
        dist.all_reduce(sm[2:], op=dist.ReduceOp.SUM)
        elapsed = float(mx[0].item())
        ok = mx[1].item() == 0.0
        csize_total = int(sm[2].item())
        # the frame index every rank built from the all-gathered sizes spans the whole job
        ok = ok and int(index[0][-1].item()) == csize_total
    t_comp = sum(e[0].elapsed_time(e[1]) for e in ev) / len(ev) / 1e3  # seconds
    t_dec = sum(e[2].elapsed_time(e[3]) for e in ev) / len(ev) / 1e3
    del data, slab, out
    torch.cuda.empty_cache()
    return {"elapsed": elapsed, "ok": ok, "csize": csize, "t_comp": t_comp, "t_dec": t_dec,
            "nseg": nseg}


def kernel_lines(codec_name, r, n, traffic_json):
    """roofline of the dominant kernel + per-kernel averages (HIP events on the launch stream)."""
    U, C = float(n), float(r["csize"])
    comp_bytes = U + C + 4.0 * r["nseg"]   # algorithmic bytes of one compress launch
    dec_bytes = U + C                      # algorithmic bytes of one decompress launch
    kc, kd = KERNELS[codec_name]
    t_comp, t_dec = r["t_comp"], r["t_dec"]
    dominant = (kc, comp_bytes, t_comp) if t_comp >= t_dec else (kd, dec_bytes, t_dec)
    achieved = dominant[1] / dominant[2] / 1e9
    traffic = None
    try:
        with open(traffic_json) as f:
            traffic = json.load(f).get(dominant[0])
    except (OSError, ValueError):
        pass
    roof = {"bound": "hbm", "kernel": dominant[0], "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic, "algorithmic_bytes_per_launch": dominant[1],
            "avg_launch_ms": round(dominant[2] * 1e3, 4)}
    kernels = {kc: {"avg_ms": round(t_comp * 1e3, 4), "alg_GBs": round(comp_bytes / t_comp / 1e9, 2)},
               kd: {"avg_ms": round(t_dec * 1e3, 4), "alg_GBs": round(dec_bytes / t_dec / 1e9, 2)}}
    return roof, kernels


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    import bitar_amd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()
    eng = bitar_amd.Engine(dev)
    ctx = {"world": world, "rank": rank}
    n, seg = args.bytes, args.seg
    r = roundtrip(eng, ctx, args.codec, args.kind, n, seg, args.steps, args.warmup, rank)
    zs = None
    if args.codec != "zstd" and not args.no_zstd:
        # BASELINE configs[5]: Zstd level-1-class frames on Parquet-column-like buffers
        # (kind 2, Arrow record-batch bodies), same sharding and all-gather, every rank
        zs = roundtrip(eng, ctx, "zstd", 2, n, seg, args.steps, args.warmup, rank + 1000)
    df = None
    if args.codec != "deflate" and not args.no_deflate:
        # the reference's own segment codec (RTE_COMP_ALGO_DEFLATE, config.cc:83-105) at its
        # default segment size (59460 B, app_common.h:39), same input as the headline
        df = roundtrip(eng, ctx, "deflate", args.kind, n, 59460, args.steps, args.warmup,
                       rank + 2000)
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    U = float(n)
    C = float(r["csize"])
    value = world * U * args.steps / r["elapsed"] / GIB
    roof, kernels = kernel_lines(args.codec, r, n, args.traffic_json)
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
                   "bytes_per_gpu": n, "segment_bytes": seg, "segments_per_gpu": r["nseg"],
                   "codec": CODEC_NAMES[args.codec],
                   "input_kind": args.kind,
                   "parallelism": f"{world} independent shards (round-robin segments), "
                                  "RCCL all-gather of sizes" if world > 1 else "1 GPU"},
        "compression_ratio": round(U / C, 4),
        "compress_gibs": round(U / r["t_comp"] / GIB, 3),
        "decompress_gibs": round(U / r["t_dec"] / GIB, 3),
        "roundtrip_ok": r["ok"],
        "roofline": roof,
        "kernels": kernels,
    }
    if world == 1 and args.codec == "lz4" and not args.no_secondary:
        # BASELINE configs[1]: 1-GiB random-byte buffer, LZ4 decompress only (the HBM-bound
        # case of the same kernel), reported beside the headline round trip
        res["secondary"] = random_decompress(eng, n, seg, args)
    if zs is not None:
        zroof, zkern = kernel_lines("zstd", zs, n, args.traffic_json)
        res["zstd"] = {
            "workload": "BASELINE configs[5]: Zstd frame per 64 KiB segment (raw literals, "
                        "predefined FSE sequences), compress + RCCL size all-gather + "
                        "decompress, 1 GiB Arrow record-batch buffer per GPU",
            "value": round(world * U * args.steps / zs["elapsed"] / GIB, 3), "unit": "GiB/s",
            "ms_per_step": round(zs["elapsed"] / args.steps * 1e3, 4),
            "compression_ratio": round(U / zs["csize"], 4),
            "compress_gibs": round(U / zs["t_comp"] / GIB, 3),
            "decompress_gibs": round(U / zs["t_dec"] / GIB, 3),
            "roundtrip_ok": zs["ok"], "roofline": zroof, "kernels": zkern}
    if df is not None:
        droof, dkern = kernel_lines("deflate", df, n, args.traffic_json)
        res["deflate"] = {
            "workload": "the reference's codec: raw DEFLATE (fixed-Huffman blocks) per 59460-B "
                        "segment, compress + decompress, same input and sharding as the headline",
            "value": round(world * U * args.steps / df["elapsed"] / GIB, 3), "unit": "GiB/s",
            "ms_per_step": round(df["elapsed"] / args.steps * 1e3, 4),
            "compression_ratio": round(U / df["csize"], 4),
            "compress_gibs": round(U / df["t_comp"] / GIB, 3),
            "decompress_gibs": round(U / df["t_dec"] / GIB, 3),
            "roundtrip_ok": df["ok"], "roofline": droof, "kernels": dkern}
    if not args.no_cpu_baseline and world == 1 and args.codec == "lz4":
        res["cpu_baseline"] = cpu_baseline(args)
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def random_decompress(eng, n, seg, args):
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
    return {
        "workload": "BASELINE configs[1]: 1 GiB random bytes, LZ4 block decompress only, "
                    "64 KiB segments, HBM-resident",
        "decompress_gibs": round(n / t2 / GIB, 3), "avg_launch_ms": round(t2 * 1e3, 4),
        "roofline": {"bound": "hbm", "achieved": round(alg2, 2), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(alg2 / HBM_PEAK_GBS, 4),
                     "algorithmic_bytes_per_launch": float(n) + c_rand},
        "roundtrip_ok": ok2}


if __name__ == "__main__":
    main()
