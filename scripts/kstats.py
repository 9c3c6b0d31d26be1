#!/usr/bin/env python3
"""Per-kernel average duration from a rocprofv3 rocpd database (when no stats csv is written).
usage: python scripts/kstats.py <dir-or-db>"""
import glob
import sqlite3
import sys


def main():
    p = sys.argv[1]
    db = p if p.endswith(".db") else glob.glob(p + "/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    sym = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    dis = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    names = {r[0]: r[1] for r in c.execute(f"select id, kernel_name from {sym}")}
    agg = {}
    for kid, s, e in c.execute(f"select kernel_id, start, end from {dis}"):
        n = names.get(kid, str(kid)).split("(")[0].replace("void ", "")
        agg.setdefault(n, []).append((e - s) / 1e6)
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{sum(v) / len(v):9.3f} ms avg  x{len(v):3d}  {n}")


if __name__ == "__main__":
    main()
