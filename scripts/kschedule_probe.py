"""Probe: config 3 with the per-query window changed during the run (pp_batch_set_window between
extend calls) — does a short window while the trees are small and a long one later beat one
fixed window?  Prints it/s per schedule for a Q-query batch (default: 1024, one rank's shard at
8 GPUs) and the per-query records digest, which must not depend on the schedule."""
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "rs-pathplanning_amd"))
from pathplanning_amd import rrt, scenes  # noqa: E402

Q = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
M = 2000
raw = scenes.field512()
space = rrt.Space.from_raw(raw)
starts, goals, seeds = scenes.config3_queries(raw, 0, Q)
SCHEDULES = {
    "fixed32": [(32, M)],
    "fixed16": [(16, M)],
    "8-32": [(8, 128), (16, 384), (32, M)],
    "16-32-64": [(16, 256), (32, 1024), (64, M)],
    "16-64": [(16, 512), (64, M)],
    "4-8-16-32-64": [(4, 32), (8, 128), (16, 384), (32, 1024), (64, M)],
    "8-16-32-64": [(8, 64), (16, 256), (32, 768), (64, M)],
}
for name, sched in SCHEDULES.items():
    best = None
    for rep in range(3):
        b = rrt.RRTBatch(starts, goals, M, raw["step_size"], space, seeds, window=sched[0][0])
        b.extend(1)
        b.close()
        b = rrt.RRTBatch(starts, goals, M, raw["step_size"], space, seeds, window=sched[0][0])
        t0 = time.perf_counter()
        done = 0
        for k, upto in sched:
            b.set_window(k)
            b.extend(upto - done)
            done = upto
        n, its = b.state()
        t = time.perf_counter() - t0
        dig = hashlib.sha256(np.ascontiguousarray(n).tobytes()).hexdigest()[:12]
        b.close()
        best = t if best is None else min(best, t)
    print(f"{name:16s} {Q * M / best / 1e6:8.1f} M it/s  nodes {int(n.sum())}  digest {dig}", flush=True)
