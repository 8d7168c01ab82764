set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=r06i RUNS="c3|base|--workload config3 --no-cpu-baseline" bash scripts/gpu_trace_var.sh
python3 scripts/trace_summary.py gpurun_out/r06i c3:0 > gpurun_out/r06i/c3_all.json
python3 - <<'PY'
import csv, glob, json
from collections import defaultdict
p = glob.glob("gpurun_out/r06i/c3/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(p)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last batch plan: from the last cfb_depth_kernel to the end of the last cf_line_kernel
idx = [i for i, r in enumerate(rows) if "cfb_depth_kernel" in r["Kernel_Name"]]
start = idx[-1]
seg = rows[start:]
t0 = int(seg[0]["Start_Timestamp"])
per = defaultdict(lambda: [0, 0.0])
for r in seg:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("ppamd::", "")
    per[n][0] += 1
    per[n][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
end = max(int(r["End_Timestamp"]) for r in seg)
out = {"plan_span_us": (end - t0) / 1e3, "kernels": {k: {"n": v[0], "sum_us": round(v[1], 1)} for k, v in per.items()}}
json.dump(out, open("gpurun_out/r06i/c3_plan_breakdown.json", "w"), indent=1)
PY
find gpurun_out/r06i -name "*kernel_trace.csv" -delete
