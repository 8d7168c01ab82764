"""Per-kernel durations at the benched size from rocprofv3 kernel traces (scripts/gpu_trace.sh):
for each traced bench run, the average of the LAST n dispatches of every kernel — the profiled
pass of the bench (config 2: its 20 windows at the benched tree size; config 3/5: every step of
the profiled pass), not a whole-run average over growing trees — plus the wall span of those
dispatches.

  python scripts/trace_summary.py gpurun_out/<tag> NAME:LAST [NAME:LAST ...] > profiles/<file>.json

NAME is a traced run's directory (gpurun_out/<tag>/<NAME>/run_kernel_trace.csv); LAST the number
of trailing dispatches per kernel (0: all)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarise(path, last):
    rows = list(csv.DictReader(open(path)))
    per = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        if name.startswith("__amd_rocclr"):
            continue
        short = name.split("(")[0].replace("void ", "").replace("ppamd::", "")
        if int(r["Grid_Size_X"]) <= int(r["Workgroup_Size_X"]):
            short += " [1 workgroup]"  # window_kernel's drain / resolve-only launches
        per[short].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Grid_Size_X"]),
                           int(r["Workgroup_Size_X"]), int(r.get("Scratch_Size", 0) or 0),
                           int(r.get("VGPR_Count", 0) or 0), int(r.get("LDS_Block_Size", 0) or 0)))
    out = {}
    for k, v in per.items():
        v.sort()
        sel = v[-last:] if last else v
        d = [(e - s) / 1e3 for s, e, *_ in sel]
        out[k] = {
            "dispatches": len(sel),
            "avg_us": round(sum(d) / len(d), 3),
            "min_us": round(min(d), 3),
            "max_us": round(max(d), 3),
            "workgroups": sel[-1][2] // max(sel[-1][3], 1),
            "workgroup_size": sel[-1][3],
            "scratch_bytes_per_lane": sel[-1][4],
            "trace_vgpr_count": sel[-1][5],
            "lds_bytes": sel[-1][6],
        }
    return out


def main():
    root = sys.argv[1]
    res = {"source": "rocprofv3 --kernel-trace --stats (scripts/gpu_trace.sh), last N dispatches per kernel"}
    for spec in sys.argv[2:]:
        name, last = spec.split(":")
        paths = glob.glob(os.path.join(root, name, "**", "*kernel_trace.csv"), recursive=True)
        if not paths:
            continue
        entry = {"last_dispatches": int(last), "kernels": summarise(paths[0], int(last))}
        bench = os.path.join(root, name + ".json")
        if os.path.exists(bench):
            try:
                line = json.loads(open(bench).read().strip().splitlines()[-1])
                entry["bench_value"] = line.get("value")
                entry["bench_config"] = line.get("config")
                entry["lib_sha256_16"] = line.get("provenance", {}).get("lib_sha256_16")
            except (ValueError, IndexError):
                pass
        res[name] = entry
    json.dump(res, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
