"""Print the kernels of a rocprofv3 --kernel-trace csv as a timeline (start offset, duration,
stream), from the first kernel whose name contains FROM (default: the last occurrence).
usage: python scripts/timeline.py trace_kernel_trace.csv [FROM] [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
frm = sys.argv[2] if len(sys.argv) > 2 else None
n = int(sys.argv[3]) if len(sys.argv) > 3 else 30
start = 0
if frm:
    idx = [i for i, r in enumerate(rows) if frm in r["Kernel_Name"]]
    start = idx[-1] if idx else 0
t0 = int(rows[start]["Start_Timestamp"])
for r in rows[start:start + n]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("bitar_hip::", "")
    print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  q{r.get('Queue_Id', '?'):>3}  {name[:60]}")
