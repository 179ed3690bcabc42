"""Summarise a rocprofv3 kernel trace of scripts/band_cost.py: median duration
per kernel, and per call (a call starts at each rt_prepare_kernel, or at each
rt_tile_cert_kernel when the certificates are fused into one launch) the span
from its first kernel's start to its last kernel's end and the idle gaps
between its kernels.  Usage: trace_calls.py KERNEL_TRACE_CSV"""
import csv
import statistics
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "cg::" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
name = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "").replace("cg::", "")   # noqa: E731
by = {}
for r in rows:
    by.setdefault(name(r), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in by.items():
    print(f"  {k:32s} n={len(v):3d} median {statistics.median(v):8.1f} us")
first = "rt_prepare_kernel" if "rt_prepare_kernel" in by else "rt_tile_cert_kernel"
calls, cur = [], []
for r in rows:
    if name(r) == first and cur:
        calls.append(cur)
        cur = []
    cur.append(r)
if cur:
    calls.append(cur)
spans, gaps = [], []
for c in calls:
    s0 = int(c[0]["Start_Timestamp"])
    e = max(int(r["End_Timestamp"]) for r in c)
    spans.append((e - s0) / 1e3)
    g, end = 0, int(c[0]["End_Timestamp"])
    for r in c[1:]:
        g += max(0, int(r["Start_Timestamp"]) - end)
        end = max(end, int(r["End_Timestamp"]))
    gaps.append(g / 1e3)
if spans:
    print(f"  per call ({len(calls)}): device span median {statistics.median(spans):.1f} us, "
          f"idle gaps between its kernels median {statistics.median(gaps):.1f} us")
