"""Diagnostic: one check_finish_batch over every node of a single-tree plan (example_rrt's transit
scene, or bench6_open), with profiling on.  With the in-tree library the finish_* stats are
nodes / edges / walked points / arc points; with the `cftime` variant (scripts/variant_build.py,
PP_AMD_LIB) they are wall_clock64 ticks (10 ns) summed over waves: ancestor path, optimize,
finalize, and (the last) the longest wave's lifetime."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rs-pathplanning_amd"))
from pathplanning_amd import rrt, scenes  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "transit"
raw = scenes.transit() if which == "transit" else scenes.bench6_open()
sx, sy, syaw = raw["start"]
gx, gy, gyaw = raw["goal"]
p = rrt.RRT((sx, sy), syaw, (gx, gy), gyaw, raw["max_iter"], raw["step_size"],
            rrt.Space.from_raw(raw), seed=42, window=512, capacity=1 << 14)
p.extend(raw["max_iter"])
nodes = np.arange(1, p.tree_size(), dtype=np.int32)
p.check_finish_batch(nodes)
p.synchronize()
res = {}
for rep in range(2):
    p.reset_stats()
    p.set_profiling(rep == 1)
    p.synchronize()
    t0 = time.perf_counter()
    r = p.check_finish_batch(nodes)
    p.synchronize()
    res[f"wall_ms_{rep}"] = round(1e3 * (time.perf_counter() - t0), 3)
s = p.stats()
res.update({k: int(s[k]) for k in ("finish_nodes", "finish_edges", "finish_points",
                                    "finish_arc_points")})
res["finish_ms"] = s["finish_ms"]
res["nodes"] = len(nodes)
res["ok"] = int(np.sum(r["ok"]))
print(json.dumps({"scene": which, **res}))
