"""Summarise gpurun_out/prof (scripts/profile.sh) into profiles/<round>_*:
kernel stats of both workloads, one config-2 window timeline, and nn_scan HBM traffic per launch
(FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM, plus WRITE_SIZE) at the 100k-node tree."""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "gpurun_out", "prof")
rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
OUT = os.path.join(ROOT, "profiles")


def rows(path):
    return sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))


def last_launches(path, name, k):
    by = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if not r["Kernel_Name"].startswith(name):
            continue
        d = int(r["Dispatch_Id"])
        by[d][r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(by)[-k:]
    return ids, by


shutil.copy(os.path.join(P, "trace", "run_kernel_stats.csv"), os.path.join(OUT, f"{rnd}_config2_kernel_stats.csv"))
shutil.copy(os.path.join(P, "trace3", "run_kernel_stats.csv"), os.path.join(OUT, f"{rnd}_config3_kernel_stats.csv"))

# one config-2 window (the last timed ones) and per-kernel averages over the last 20 windows
rs = rows(os.path.join(P, "trace", "run_kernel_trace.csv"))
wb = [i for i, r in enumerate(rs) if r["Kernel_Name"].startswith("window_begin")]
lines = ["config 2, 100k-node tree, K = 4096: one window (rocprofv3 kernel trace, us)"]
a, b = wb[-8], wb[-7]
t0 = int(rs[a]["Start_Timestamp"])
for r in rs[a:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    lines.append(f"  {r['Kernel_Name'][:34]:34s} start {(s - t0) / 1e3:8.2f}  dur {(e - s) / 1e3:8.2f}")
agg = collections.defaultdict(list)
for r in rs[wb[-21]:wb[-1]]:
    agg[r["Kernel_Name"][:34]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
per = (int(rs[wb[-1]]["Start_Timestamp"]) - int(rs[wb[-21]]["Start_Timestamp"])) / 20e3
lines.append(f"window period (last 20 windows, under the profiler): {per:.2f} us")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    lines.append(f"  {k:34s} n={len(v):3d} avg {sum(v) / len(v):8.2f} us")
rs3 = rows(os.path.join(P, "trace3", "run_kernel_trace.csv"))
ks = [i for i, r in enumerate(rs3) if r["Kernel_Name"].startswith("mq_sample_nn")]
agg3 = collections.defaultdict(list)
for r in rs3[ks[3]:ks[403]]:
    agg3[r["Kernel_Name"][:34]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
per3 = (int(rs3[ks[402]]["Start_Timestamp"]) - int(rs3[ks[3]]["Start_Timestamp"])) / 399e3
lines.append("")
lines.append("config 3, 8192 queries: one lockstep step (avg over 400 timed steps)")
lines.append(f"step period (under the profiler): {per3:.2f} us")
for k, v in sorted(agg3.items(), key=lambda kv: -sum(kv[1])):
    lines.append(f"  {k:34s} n={len(v):3d} avg {sum(v) / len(v):8.2f} us")
open(os.path.join(OUT, f"{rnd}_timeline.txt"), "w").write("\n".join(lines) + "\n")

# nn_scan traffic at 100k nodes (the last 20 launches of each counter pass)
fid, fby = last_launches(os.path.join(P, "fetch", "run_counter_collection.csv"), "nn_scan", 20)
wid, wby = last_launches(os.path.join(P, "write", "run_counter_collection.csv"), "nn_scan", 20)
fetch_kb = sum(fby[i]["FETCH_SIZE"] for i in fid) / len(fid)
write_kb = sum(wby[i]["WRITE_SIZE"] for i in wid) / len(wid)
traffic = {
    "kernel": "nn_scan",
    "tree_nodes": "~100k (the bench's timed windows)",
    "fetch_size_kb_per_launch": round(fetch_kb, 1),
    "write_size_kb_per_launch": round(write_kb, 1),
    "hbm_bytes_per_launch": int(2 * fetch_kb * 1024 + write_kb * 1024),
    "note": "FETCH_SIZE doubled (gfx950 tallies wide reads at half, MI355X_MICROARCH.md §HBM); "
            "nn_scan reads nodes with scalar loads, for which the correction is uncalibrated; "
            "WRITE_SIZE = the 64 per-chunk partials (12 B per sample and chunk)",
}
json.dump(traffic, open(os.path.join(OUT, "nn_scan_traffic.json"), "w"), indent=1)
print("\n".join(lines))
print(json.dumps(traffic, indent=1))
