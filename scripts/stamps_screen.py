"""Diagnostic: the NN screen's phase times per wave (a -DPP_STAMPS_SCREEN build in
lib/v_stamps_screen/): samples + node range, first piece staged, screen loop, winning-block
re-evaluation, wave merge.  Config 2, 20 windows at ~100k nodes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PP_AMD_LIB"] = os.path.join(ROOT, "rs-pathplanning_amd", "lib",
                                        sys.argv[1] if len(sys.argv) > 1 else "v_stamps_screen",
                                        "libpathplanning_amd.so")
sys.path.insert(0, os.path.join(ROOT, "rs-pathplanning_amd"))
from pathplanning_amd import rrt, scenes  # noqa: E402

raw = scenes.field512()
sx, sy, syaw = raw["start"]
gx, gy, gyaw = raw["goal"]
p = rrt.RRT((sx, sy), syaw, (gx, gy), gyaw, 0, raw["step_size"], rrt.Space.from_raw(raw),
            seed=42, capacity=1 << 18)
for target in (10000, 100000):
    while p.tree_size() < target and p.iteration() < 60 * target:
        p.extend(4096)
    p.reset_stats()
    p.extend(20 * 4096)
    s = p.stats()["stamps"]
    w = max(s[3], 1)
    l0 = max(s[7], 1)
    print(target, "screen waves %d: samples+stage %.2f loop %.2f merge %.2f, max wave %.2f us | "
          "workgroup 0 (%d launches): resolve+commit %.2f samples %.2f us"
          % (s[3], s[0] / w / 100, s[1] / w / 100, s[2] / w / 100, s[4] / 100, s[7],
             s[5] / l0 / 100, s[6] / l0 / 100))
