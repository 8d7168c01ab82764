"""Diagnostic (the `wdiag` variant library only, PP_AMD_LIB): the config-2 window walk's task
durations.  Grows the field512 tree past 100k nodes at K = 4096, then 20 windows with the
variant's counters reset: a log2 histogram of per-task walk_rec times (wall_clock64 ticks, 10 ns),
their sum and maximum, and the workgroups' spans (first task start to the workgroup's end)."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rs-pathplanning_amd"))
from pathplanning_amd import _ffi, rrt, scenes  # noqa: E402

raw = scenes.field512()
sx, sy, syaw = raw["start"]
gx, gy, gyaw = raw["goal"]
p = rrt.RRT((sx, sy), syaw, (gx, gy), gyaw, raw["max_iter"], raw["step_size"], rrt.Space.from_raw(raw),
            seed=42, window=4096, capacity=1 << 18)
while p.tree_size() < 100_000:
    p.extend(65536)
lib = _ffi.lib()
fn = lib.pp_variant_wdiag
fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
buf = (C.c_ulonglong * 32)()
assert fn(buf, 1) == 0
n0 = p.tree_size()
p.extend(20 * 4096)
assert fn(buf, 0) == 0
v = list(buf)
tick_us = 0.01
hist = {f"{(1 << b) * tick_us:.2f}-{(2 << b) * tick_us:.2f}us": v[b] for b in range(16) if v[b]}
print(json.dumps({"tree_nodes": n0, "tasks": v[18], "hist": hist,
                  "task_mean_us": round(v[16] / max(v[18], 1) * tick_us, 3),
                  "task_max_us": round(v[17] * tick_us, 3),
                  "wg_span_max_us": round(v[19] * tick_us, 3),
                  "wg_span_mean_us": round(v[20] / max(v[21], 1) * tick_us, 3),
                  "workgroups": v[21],
                  # (wdiag2 only) per-chunk phases summed over tasks: generator, interpolation,
                  # chunk test
                  "phase_us_per_task": [round(v[i] / max(v[18], 1) * tick_us, 3) for i in (22, 23, 24)]}))
