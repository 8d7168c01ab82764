"""Diagnostic: grid pair search vs brute force (build with -DPP_PAIR_CHECK into lib/v_paircheck/)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PP_AMD_LIB"] = os.path.join(ROOT, "rs-pathplanning_amd", "lib", "v_paircheck", "libpathplanning_amd.so")
sys.path.insert(0, os.path.join(ROOT, "rs-pathplanning_amd"))
from pathplanning_amd import rrt, scenes
for name, raw, seed, win, n in (("bench6", scenes.bench6(), 1, 64, 400), ("field", scenes.field512(), 42, 4096, 40000)):
    sx, sy, syaw = raw["start"]; gx, gy, gyaw = raw["goal"]
    p = rrt.RRT((sx, sy), syaw, (gx, gy), gyaw, 0, raw["step_size"], rrt.Space.from_raw(raw), seed=seed, window=win)
    p.reset_stats()
    p.extend(n)
    print(name, p.stats()["stamps"])
