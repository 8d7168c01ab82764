"""Diagnostic: resolve_kernel phase times (build with -DPP_STAMPS_RESOLVE into lib/stamps_resolve/).
Phases: 0 pending slots, 1 candidate lists + sort, 2 round passes, 3 publish."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PP_AMD_LIB"] = os.path.join(ROOT, "rs-pathplanning_amd", "lib", "stamps_resolve",
                                        "libpathplanning_amd.so")
sys.path.insert(0, os.path.join(ROOT, "rs-pathplanning_amd"))
from pathplanning_amd import rrt, scenes
raw = scenes.field512()
sx, sy, syaw = raw["start"]; gx, gy, gyaw = raw["goal"]
p = rrt.RRT((sx, sy), syaw, (gx, gy), gyaw, 0, raw["step_size"], rrt.Space.from_raw(raw), seed=42,
            capacity=1 << 18)
for target in (1000, 10000, 100000):
    while p.tree_size() < target:
        p.extend(4096)
    p.reset_stats()
    p.extend(20 * 4096)
    st = p.stats()
    s = st["stamps"]
    print(target, "resolve us/window: slots %.2f lists %.2f rounds %.2f publish %.2f  | "
          "rounds/window %.1f pending/window %.1f entries/window %.1f | repair_rounds %d repairs %d"
          % (s[0] / 20 / 100, s[1] / 20 / 100, s[2] / 20 / 100, s[3] / 20 / 100, s[4] / 20,
             s[5] / 20, s[6] / 20, st["repair_rounds"], st["repairs"]))
