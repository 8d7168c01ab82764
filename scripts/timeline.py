"""Print one window's kernel timeline and per-kernel averages from a rocprofv3 kernel trace."""
import csv
import collections
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/iter/trace/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
wb = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(("window_begin", "window_kernel"))]
a, b = wb[-8], wb[-7]
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"  {r['Kernel_Name'][:40]:40s} start {(s - t0) / 1e3:8.2f} dur {(e - s) / 1e3:8.2f}")
agg = collections.defaultdict(list)
for r in rows[wb[-21]:wb[-1]]:
    agg[r["Kernel_Name"].split("(")[0][:40]].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
per = (int(rows[wb[-1]]["Start_Timestamp"]) - int(rows[wb[-21]]["Start_Timestamp"])) / 20e3
print(f"window period over the last 20 windows: {per:.2f} us")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {k:40s} n={len(v):3d} avg {sum(v) / len(v):8.2f} us")
