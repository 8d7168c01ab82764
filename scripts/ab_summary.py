"""Summarise a gpu_runs.sh directory: per run the headline value, the records digest and (config
3) the batch plan's check_finish, grouped by (name, variant)."""
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]
rows = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    base = os.path.basename(f)[:-5]
    parts = base.rsplit("_", 2)
    if len(parts) != 3:
        continue
    try:
        L = [l for l in open(f) if l.strip().startswith("{")]
        j = json.loads(L[-1])
    except Exception:
        continue
    sub = j.get("config3") or {}
    plan = (sub.get("plan") or {}) if isinstance(sub, dict) else {}
    plan = plan or j.get("plan") or {}
    rows[(parts[0], parts[1])].append((j.get("value"), j.get("records_digest") or (sub or {}).get("records_digest"),
                                       plan.get("check_finish_ms"), j.get("lib_sha256_16")))
for (n, v), r in sorted(rows.items()):
    vals = " / ".join(f"{x[0] / 1e6:.2f}" for x in r)
    cf = " / ".join(str(x[2]) for x in r if x[2] is not None)
    print(f"{n:8s} {v:10s} {vals:24s} digest {r[0][1]} cf {cf} lib {r[0][3]}")
