"""Probe: config 3's extend passes (PP_DEBUG=1 prints each pass's steps, window and the queries
still behind) and the batch rate, best of 3 after a warmup run, for Q in argv[1] (default
1024,8192)."""
import hashlib
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "rs-pathplanning_amd"))
from pathplanning_amd import rrt, scenes  # noqa: E402

raw = scenes.field512()
space = rrt.Space.from_raw(raw)
for Q in [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1024,8192").split(",")]:
    starts, goals, seeds = scenes.config3_queries(raw, 0, Q)
    best = None
    for rep in range(4):
        b = rrt.RRTBatch(starts, goals, 2000, raw["step_size"], space, seeds)
        t0 = time.perf_counter()
        b.extend(2000)
        t = time.perf_counter() - t0
        n, its = b.state()
        b.close()
        if rep:
            best = t if best is None else min(best, t)
    dig = hashlib.sha256(np.ascontiguousarray(n).tobytes()).hexdigest()[:12]
    print(f"Q={Q} topup={os.environ.get('PP_TOPUP_K', '-')}: {Q * 2000 / best / 1e6:.1f} M it/s, "
          f"nodes {int(n.sum())}, digest {dig}", flush=True)
