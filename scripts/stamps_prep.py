"""Diagnostic: steer_prep phase times per wave-iteration (build with -DPP_STAMPS_PREP into
lib/v_stprep/).  Phases: 0 loads + frame change + 6 words, 1 selection + segment trig, 2 pd walk,
3 record store."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PP_AMD_LIB"] = os.path.join(ROOT, "rs-pathplanning_amd", "lib", "v_stprep", "libpathplanning_amd.so")
sys.path.insert(0, os.path.join(ROOT, "rs-pathplanning_amd"))
from pathplanning_amd import rrt, scenes
raw = scenes.field512()
sx, sy, syaw = raw["start"]; gx, gy, gyaw = raw["goal"]
p = rrt.RRT((sx, sy), syaw, (gx, gy), gyaw, 0, raw["step_size"], rrt.Space.from_raw(raw), seed=42, capacity=1 << 18)
while p.tree_size() < 100000:
    p.extend(4096)
p.reset_stats()
p.extend(20 * 4096)
s = p.stats()["stamps"]
n = max(s[4], 1)
print("prep us per wave-iteration: words %.2f select+trig %.2f walk %.2f store %.2f  (%d wave-iterations / 20 windows)"
      % (s[0] / n / 100, s[1] / n / 100, s[2] / n / 100, s[3] / n / 100, n))
