"""Diagnostic: per window_kernel launch, the span from the first workgroup's start to the last
workgroup's end, the workgroups' start skew and workgroup 0's end (a -DPP_STAMPS_SPAN build in
lib/<variant>/), beside the HIP-event duration of the same launches.  Config 2 at ~100k nodes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PP_AMD_LIB"] = os.path.join(ROOT, "rs-pathplanning_amd", "lib",
                                        sys.argv[1] if len(sys.argv) > 1 else "v_stamps_span",
                                        "libpathplanning_amd.so")
sys.path.insert(0, os.path.join(ROOT, "rs-pathplanning_amd"))
from pathplanning_amd import rrt, scenes  # noqa: E402

raw = scenes.field512()
sx, sy, syaw = raw["start"]
gx, gy, gyaw = raw["goal"]
p = rrt.RRT((sx, sy), syaw, (gx, gy), gyaw, 0, raw["step_size"], rrt.Space.from_raw(raw),
            seed=42, capacity=1 << 18)
while p.tree_size() < 100000:
    p.extend(65536)
p.extend(4096 * 4)
p.set_profiling(True)
p.reset_stats()
p.stats()  # (a diagnostic build dumps and clears its per-workgroup sums here)
print("---- measured windows ----", file=sys.stderr, flush=True)
p.extend(20 * 4096)
st = p.stats()
s = st["stamps"]
n = max(s[3], 1)
print("launches %d: span %.2f us, start skew %.2f us, workgroup 0 end %.2f us, slowest screen "
      "workgroup %.2f us, mean %.2f us; HIP events %.2f us"
      % (s[3], s[0] / n / 100, s[1] / n / 100, s[2] / n / 100, s[4] / n / 100, s[5] / n / 100,
         1000 * st["nn_scan_ms"] / max(st["nn_scan_launches"], 1)))
