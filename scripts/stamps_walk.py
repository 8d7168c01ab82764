"""Diagnostic: steer_walk phase times (build with -DPP_STAMPS_WALK into lib/v_stwalk/), config 2
at 100k nodes.  Per task: point generation, interpolation, collision; per workgroup: staging."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PP_AMD_LIB"] = os.path.join(ROOT, "rs-pathplanning_amd", "lib", "v_stwalk", "libpathplanning_amd.so")
sys.path.insert(0, os.path.join(ROOT, "rs-pathplanning_amd"))
from pathplanning_amd import rrt, scenes
raw = scenes.field512_grid() if "grid" in sys.argv else scenes.field512()
sx, sy, syaw = raw["start"]; gx, gy, gyaw = raw["goal"]
p = rrt.RRT((sx, sy), syaw, (gx, gy), gyaw, 0, raw["step_size"], rrt.Space.from_raw(raw), seed=42, capacity=1 << 18)
while p.tree_size() < 100000:
    p.extend(4096)
p.reset_stats()
p.extend(20 * 4096)
s = p.stats()["stamps"]
n = max(s[4], 1)
print("walk us per task: gen %.2f interp %.2f collide %.2f | chunks/task %.2f tasks %d | staging us/WG %.2f (%d WGs) | slowest task %.2f us"
      % (s[0] / n / 100, s[1] / n / 100, s[2] / n / 100, s[3] / n, n, s[5] / max(s[6], 1) / 100, s[6], s[7] / 100))
