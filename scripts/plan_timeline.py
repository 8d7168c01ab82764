#!/usr/bin/env python3
"""The last batch plan of a rocprofv3 kernel trace as an ordered dispatch list.

usage: plan_timeline.py TRACE_DIR > timeline.json

From the last cfb_depth_kernel (the plan's first launch) to the end of the trace: per dispatch
the kernel, its start offset and duration (µs), and the gap since the previous dispatch ended, so
the steer rounds' launches and their idle time can be read in order.
"""
import csv
import glob
import json
import sys


def main(d):
    paths = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not paths:
        sys.exit(f"no kernel trace under {d}")
    rows = list(csv.DictReader(open(paths[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "cfb_depth_kernel" in r["Kernel_Name"]]
    if not idx:
        sys.exit("no batch plan in the trace")
    seg = rows[idx[-1]:]
    t0 = int(seg[0]["Start_Timestamp"])
    prev_end = t0
    out = []
    for r in seg:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ppamd::", "")
        out.append({"k": name, "t_us": round((s - t0) / 1e3, 1), "dur_us": round((e - s) / 1e3, 1),
                    "gap_us": round((s - prev_end) / 1e3, 1), "wg": int(r.get("Grid_Size_X", 0) or 0)
                    // max(1, int(r.get("Workgroup_Size_X", 1) or 1))})
        prev_end = max(prev_end, e)
    json.dump({"span_us": round((prev_end - t0) / 1e3, 1), "dispatches": out}, sys.stdout, indent=0)


if __name__ == "__main__":
    main(sys.argv[1])
