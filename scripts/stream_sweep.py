"""Headline round trip (1 GiB kind 1, LZ4, 64 KiB segments) with the job split over K
queue-pair streams: GiB/s per K (timing experiment for DESIGN.md)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
import bitar_amd  # noqa: E402

eng = bitar_amd.Engine(0, num_streams=4)
n = 1 << 30
for rep in range(2):
    for k in (1, 2, 4):
        r = bench.run_job(eng, sys.argv[1] if len(sys.argv) > 1 else "lz4", 1, n, 65536, k,
                          20, 3, 1, 0)
        print(k, round(n * 20 / r["elapsed"] / 2**30, 2), "GiB/s", r["ok"],
              round(r["t_comp_span"] * 1e3, 3), round(r["t_dec_span"] * 1e3, 3), flush=True)
