"""Diagnostic: the window resolve's phase times (a -DPP_STAMPS_RESOLVE build in
lib/v_stamps_resolve/): pending slots, candidate lists + sort, round passes, publish, and the
commit, per window of 4096 at ~1k, 10k and 100k nodes (config 2)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PP_AMD_LIB"] = os.path.join(ROOT, "rs-pathplanning_amd", "lib", "v_stamps_resolve",
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
    w = max(st["windows"], 1)
    print(target, "resolve us/window: slots %.2f lists %.2f rounds %.2f publish %.2f commit %.2f | "
          "rounds/window %.1f pending/window %.1f entries/window %.1f | windows %d truncations %d "
          "repair_rounds %d repairs %d"
          % (s[0] / w / 100, s[1] / w / 100, s[2] / w / 100, s[3] / w / 100, s[7] / w / 100,
             s[4] / w, s[5] / w, s[6] / w, st["windows"], st["truncations"],
             st["repair_rounds"], st["repairs"]))
