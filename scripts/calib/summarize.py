"""Summarize the PMC calibration passes (scripts/gpu_calib.sh) into
profiles/<round>/calibration.json: per kernel and counter, the reported bytes over the bytes
the kernel actually moves.  usage: python scripts/calib/summarize.py profiles/r03"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
N = 1 << 30
PATTERN = {"read16": "16 B per lane, 1 KiB contiguous per wave instruction",
           "write16": "16 B per lane, 1 KiB contiguous per wave instruction",
           "read1": "1 B per lane, 64 B contiguous per wave instruction",
           "write1": "1 B per lane, 64 B contiguous per wave instruction",
           "read8_lane": "lane-owned sequential streams, 8 B per lane per load",
           "write8_lane": "lane-owned sequential streams, 8 B per lane per store"}
out = {}
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    path = os.path.join(ROOT, "gpurun_out", f"calib_{ctr}", "pmc_counter_collection.csv")
    seen = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0]
        if name not in PATTERN:
            continue
        key = f"{name} grid {r['Grid_Size']}"
        seen.setdefault(key, []).append(float(r["Counter_Value"]) * 1024.0)
    for key, v in sorted(seen.items()):
        kern = key.split()[0]
        moves = ("read" in kern) == (ctr == "FETCH_SIZE")
        if not moves:
            continue
        e = out.setdefault(key, {"pattern": PATTERN[kern], "bytes": N})
        e[ctr] = sum(v) / len(v)
        e[ctr + "_over_bytes"] = round(sum(v) / len(v) / N, 3)
rdir = os.path.join(ROOT, sys.argv[1])
os.makedirs(rdir, exist_ok=True)
with open(os.path.join(rdir, "calibration.json"), "w") as f:
    json.dump(out, f, indent=1, sort_keys=True)
for k, e in sorted(out.items()):
    print(f"{k:32s} {e['pattern']:55s} " + " ".join(f"{c} x{e[c + '_over_bytes']}" for c in ("FETCH_SIZE", "WRITE_SIZE") if c in e))
