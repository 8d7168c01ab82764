"""Diagnostic: nn_finalize phase times per workgroup (build with -DPP_STAMPS_FIN into
lib/v_stampsfin/).  Phases: 0 staging, 1 per-sample NN, 2 near-tie brute force, 3 pair search,
4 candidate append; 5 whole workgroup; 6 max workgroup; 7 workgroups."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PP_AMD_LIB"] = os.path.join(ROOT, "rs-pathplanning_amd", "lib", "v_stampsfin",
                                        "libpathplanning_amd.so")
sys.path.insert(0, os.path.join(ROOT, "rs-pathplanning_amd"))
from pathplanning_amd import rrt, scenes
raw = scenes.field512()
sx, sy, syaw = raw["start"]; gx, gy, gyaw = raw["goal"]
p = rrt.RRT((sx, sy), syaw, (gx, gy), gyaw, 0, raw["step_size"], rrt.Space.from_raw(raw), seed=42,
            capacity=1 << 18)
for target in ((100000,) if os.environ.get("PHASES") else (10000, 100000)):
    while p.tree_size() < target:
        p.extend(4096)
    p.reset_stats()
    p.extend(20 * 4096)
    s = p.stats()["stamps"]
    n0, n1 = max(s[1], 1), max(s[4], 1)
    print(target, "finalize workgroups/window: plain %.1f (avg %.2f us, max %.2f) | brute-force %.2f "
          "(avg %.2f us, max %.2f, of which brute force %.2f) | pair search avg %.2f us"
          % (s[1] / 20, s[0] / n0 / 100, s[2] / 100, s[4] / 20, s[3] / n1 / 100, s[5] / 100,
             s[6] / n1 / 100, s[7] / (s[1] + s[4]) / 100))
if os.environ.get("PHASES"):  # a -DPP_STAMPS_FIN -DPP_STAMPS_FIN_PHASES build
    p.reset_stats()
    p.extend(20 * 4096)
    s = p.stats()["stamps"]
    n = max(s[5], 1)
    print("phases per workgroup (us): staging %.2f, NN %.2f, brute force %.2f, pair search %.2f, "
          "append %.2f; max workgroup %.2f" % tuple([v / n / 100 for v in s[:5]] + [s[6] / 100]))
