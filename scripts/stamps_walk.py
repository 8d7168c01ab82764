"""Diagnostic: the walk's load imbalance (a -DPP_STAMPS_WALK build in lib/<variant>/): per
steer_walk launch, the span, the mean wave lifetime and the longest one.  Config 3 (a query batch
of Q queries, default 1024 = one rank's shard at 8 GPUs) and config 2 at ~100k nodes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PP_AMD_LIB"] = os.path.join(ROOT, "rs-pathplanning_amd", "lib",
                                        sys.argv[1] if len(sys.argv) > 1 else "v_stamps_walk",
                                        "libpathplanning_amd.so")
sys.path.insert(0, os.path.join(ROOT, "rs-pathplanning_amd"))
from pathplanning_amd import rrt, scenes  # noqa: E402

raw = scenes.field512()
for Q in [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "1024,8192").split(",")]:
    starts, goals, seeds = scenes.config3_queries(raw, 0, Q)
    b = rrt.RRTBatch(starts, goals, 2000, raw["step_size"], rrt.Space.from_raw(raw), seeds)
    b.set_profiling(True)
    b.extend(2000)
    s = b.stats()["stamps"]
    n = max(s[3], 1)
    print("config3 Q=%d: %d walk launches: span %.2f us, mean wave %.2f us, longest wave %.2f us, "
          "longest task %.2f us" % (Q, s[3], s[0] / n / 100, s[1] / n / 100, s[2] / n / 100,
                                     s[4] / n / 100))
    print("  per chunk: %.2f items pass the bbox cull, %.2f the segment near test (%d chunks)"
          % (s[6] / max(s[5], 1), s[7] / max(s[5], 1), s[5]))
    b.close()
sx, sy, syaw = raw["start"]
gx, gy, gyaw = raw["goal"]
p = rrt.RRT((sx, sy), syaw, (gx, gy), gyaw, 0, raw["step_size"], rrt.Space.from_raw(raw),
            seed=42, capacity=1 << 18)
while p.tree_size() < 100000:
    p.extend(65536)
p.reset_stats()
p.extend(20 * 4096)
s = p.stats()["stamps"]
n = max(s[3], 1)
print("config2: %d walk launches: span %.2f us, mean wave %.2f us, longest wave %.2f us, "
      "longest task %.2f us" % (s[3], s[0] / n / 100, s[1] / n / 100, s[2] / n / 100, s[4] / n / 100))
print("  per chunk: %.2f items pass the bbox cull, %.2f the segment near test (%d chunks)"
      % (s[6] / max(s[5], 1), s[7] / max(s[5], 1), s[5]))
