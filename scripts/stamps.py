"""Diagnostic: per-task phase times of steer_window (build with -DPP_STAMPS into lib/stamps/)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PP_AMD_LIB"] = os.path.join(ROOT, "rs-pathplanning_amd", "lib", "stamps", "libpathplanning_amd.so")
sys.path.insert(0, os.path.join(ROOT, "rs-pathplanning_amd"))
from pathplanning_amd import rrt, scenes
raw = scenes.field512()
sx, sy, syaw = raw["start"]; gx, gy, gyaw = raw["goal"]
p = rrt.RRT((sx, sy), syaw, (gx, gy), gyaw, 0, raw["step_size"], rrt.Space.from_raw(raw), seed=42, capacity=1 << 18)
for target in (10000, 100000):
    while p.tree_size() < target:
        p.extend(4096)
    p.reset_stats()
    p.extend(20 * 4096)
    st = p.stats()
    t = 20 * 4096
    s = st["stamps"]
    print(target, "per task us: total %.2f select %.2f chunk_rejects %.2f (of which bounds+reductions %.2f) chunks/task %.2f discs tested/task %.2f"
          % (s[0] / t / 100, s[1] / t / 100, s[2] / t / 100, s[4] / t / 100, s[3] / t, s[5] / t))
