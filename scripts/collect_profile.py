#!/usr/bin/env python3
"""Copy one gpu_bench.sh PROFILE=1 run (gpurun_out/) into profiles/<round>/ and derive the
per-launch HBM traffic that bench.py reports as roofline.traffic.

usage: python scripts/collect_profile.py TAG ROUND_DIR
  TAG        the TAG the GPU run used (gpurun_out/bench_TAG.json, prof_TAG/, pmc_TAG_*)
  ROUND_DIR  e.g. profiles/r01

Traffic per launch (MI355X_MICROARCH.md "HBM"): FETCH_SIZE and WRITE_SIZE are in KiB; on
gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane streaming reads, which is how
every bulk read of the wave-per-segment kernels is issued, so it is doubled (not for the
lane-per-segment zstd_lanes_kernel and inflate_lanes_kernel, whose reads are 8 B per lane); WRITE_SIZE is exact for
16-B-per-lane stores.  Each counter comes from its own --pmc pass; the value is averaged
over the kernel's launches in that pass.
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# FETCH_SIZE x2 for every kernel: calibrated on known byte counts in each access pattern
# these kernels use (scripts/calib/pmc_calib.hip -> profiles/r03/calibration.json): 16-B and
# 1-B coalesced reads and 8-B lane-owned read streams at 16 K concurrent streams all report
# exactly half their bytes (the counter tallies 128-B requests as 64 B).  Lane streams at
# 131 K / 2 M concurrent streams report 2.5x / 6.4x their bytes: real L2 over-fetch, kept.
# WRITE_SIZE is exact for 16-B and 1-B coalesced stores; 8-B lane-owned store streams
# report 1.7-9.5x their bytes (partial-line write-backs): real write amplification, kept.
FETCH_FACTOR = {}


def per_kernel(path, grid=None):
    agg = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if grid is not None and int(r["Grid_Size"]) != grid:
                continue
            name = r["Kernel_Name"].split("(")[0]
            if name.startswith("void "):  # templated kernels: "void ns::k<16u>"
                name = name[5:]
            if not name.startswith("bitar_hip::"):
                continue
            # one key per instantiation: lz4_decompress_kernel<false> and <true> are two
            # launches of one decompress call (the second mostly exits at once), so their
            # averages are SUMMED per call below, never averaged together
            key = name.split("::", 1)[-1]
            agg.setdefault(key, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def per_call(d):
    """{kernel base name: sum over its instantiations of their per-launch averages}"""
    out = {}
    for k, v in d.items():
        base = k.split("<")[0]
        out[base] = out.get(base, 0.0) + v
    return out


LEGS = ("headline", "zstd", "deflate", "deflate_dyn", "recordbatch", "lz4_arrow")
# legs whose kernels also run in the headline job of the same pass: only their own launches
# (by grid size) are averaged -- the record-batch job's parts are 8 GiB / 4 streams = 32768
# segments of 64 KiB, one 64-lane workgroup each
LEG_GRID = {"recordbatch": 32768 * 64}
# the kernels each leg is about (every pass also runs the headline's LZ4 kernels)
LEG_KERNELS = {"headline": ("lz4_",), "zstd": ("zstd_",),
               "deflate": ("deflate_compress", "inflate"),
               "deflate_dyn": ("deflate_dyn_", "inflate"), "recordbatch": ("lz4_",),
               "lz4_arrow": ("lz4_",)}


def main():
    tag, rdir = sys.argv[1], sys.argv[2]
    out = os.path.join(ROOT, "gpurun_out")
    rdir = os.path.join(ROOT, rdir)
    os.makedirs(rdir, exist_ok=True)
    shutil.copy(os.path.join(out, f"bench_{tag}.json"), os.path.join(rdir, "bench.json"))
    traffic, lines = {}, []
    for leg in LEGS:
        prof = os.path.join(out, f"prof_{tag}_{leg}", "trace_kernel_stats.csv")
        if not os.path.exists(prof):
            continue
        shutil.copy(prof, os.path.join(rdir, f"kernel_stats_{leg}.csv"))
        g = LEG_GRID.get(leg)
        fetch = per_call(per_kernel(os.path.join(out, f"pmc_{tag}_{leg}_FETCH_SIZE", "pmc_counter_collection.csv"), g))
        write = per_call(per_kernel(os.path.join(out, f"pmc_{tag}_{leg}_WRITE_SIZE", "pmc_counter_collection.csv"), g))
        for k in sorted(set(fetch) | set(write)):
            if not k.startswith(LEG_KERNELS[leg]):
                continue
            f_kib, w_kib = fetch.get(k, 0.0), write.get(k, 0.0)
            x = FETCH_FACTOR.get(k, 2.0)
            b = (x * f_kib + w_kib) * 1024.0
            traffic[f"{leg}/{k}"] = round(b)
            lines.append(f"{leg + '/' + k:40s} FETCH_SIZE {f_kib:14.1f} KiB (x{x:g} = "
                         f"{x * f_kib * 1024:.4g} B)  WRITE_SIZE {w_kib:14.1f} KiB  -> {b:.4g} B "
                         f"per launch")
    with open(os.path.join(rdir, "traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
    with open(os.path.join(ROOT, "profiles", "traffic.json"), "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
    with open(os.path.join(rdir, "pmc_summary.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
