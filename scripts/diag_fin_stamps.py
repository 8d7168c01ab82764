"""nn_finalize phase stamps (a PP_FIN_STAMPS diagnostic build): run the config-2
bench against the variant library, then summarise gpurun_out/fin_stamps.txt — per workgroup the
wall-clock (100 MHz) stamps at: 0 entry, 1 after the appended-node staging barrier, 2 the chunk
partials loaded (max over waves), 3 the top-2 and margin test, 4 the winner's exact d2, 5 the
phase-1 barrier, 6 after the near-tie brute force, 7 the pair-search barrier, 8 the workgroup's
end; 9 the sampling workgroup's end.

  python scripts/diag_fin_stamps.py [gpurun_out/fin_stamps.txt] [min_nodes]"""
import sys

import numpy as np

SLOTS, WGS = 10, 512
path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/fin_stamps.txt"
min_nodes = int(sys.argv[2]) if len(sys.argv) > 2 else 90000
rows = []
for line in open(path):
    v = line.split()
    n, nw = int(v[0]), int(v[1])
    st = np.array([int(x) for x in v[2:]], dtype=np.int64).reshape(WGS, SLOTS)
    if n >= min_nodes:
        rows.append((n, st))
print(f"{len(rows)} launches at >= {min_nodes} nodes")
names = ["stage", "partials", "top2", "exact", "ph1_barrier", "neartie", "pairs", "end"]
agg = {k: [] for k in names}
spans, gen_end, plain_end = [], [], []
for n, st in rows:
    live = st[:, 8] > 0
    live &= st[:, 8] >= st[:, 0]
    t0 = st[live, 0].min()
    for i, k in enumerate(names):
        a, b = st[live, i], st[live, i + 1]
        agg[k].append(np.mean(b - a) * 10.0 / 1000)  # us
    ends = st[live, 8]
    gen = st[:, 9].max()
    spans.append((max(ends.max(), gen) - t0) * 0.01)
    plain_end.append((ends.max() - t0) * 0.01)
    gen_end.append((gen - t0) * 0.01)
for k in names:
    print(f"{k:12s} mean {np.mean(agg[k]):7.2f} us per workgroup")
print(f"launch span (entries to last end) {np.mean(spans):.2f} us; plain workgroups' last end "
      f"{np.mean(plain_end):.2f}; sampling workgroup end {np.mean(gen_end):.2f}")
n, st = rows[-1]
live = st[:, 8] > 0
t0 = st[live, 0].min()
print("last launch, entry offsets (us): min %.2f max %.2f; end offsets min %.2f max %.2f" % (
    0.0, (st[live, 0].max() - t0) * 0.01, (st[live, 8].min() - t0) * 0.01,
    (st[live, 8].max() - t0) * 0.01))
