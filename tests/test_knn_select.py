"""The RRT* kNN selection of star_knn (pp_kernels.hip) restated with numpy lanes and checked
against a plain sort: node i sits in lane i % 64; T = the k-th smallest lane minimum; every node
with d2 <= T is a candidate; the candidates sorted by (d2, index) start with the exact k nearest.
When there are more than 64 candidates the kernel falls back to k exclusion rounds, restated here
too.  CPU only (algorithm check; the HIP kernel is covered by tests/test_gpu_rrtstar.py)."""
import numpy as np


def select(d2, k):
    n = len(d2)
    lane_min = np.full(64, np.inf)
    for i in range(n):
        lane_min[i % 64] = min(lane_min[i % 64], d2[i])
    T = np.sort(lane_min)[k - 1]
    cand = [i for i in range(n) if d2[i] <= T]
    if len(cand) <= 64:
        return sorted(cand, key=lambda i: (d2[i], i))[:k], True
    out, pd, pi = [], -1.0, -1  # exclusion rounds: the lexicographic successor of the last winner
    for _ in range(k):
        best = None
        for i in range(n):
            if (d2[i] > pd or (d2[i] == pd and i > pi)) and (best is None or (d2[i], i) < (d2[best], best)):
                best = i
        out.append(best)
        pd, pi = d2[best], best
    return out, False


def exact(d2, k):
    return sorted(range(len(d2)), key=lambda i: (d2[i], i))[:k]


def test_knn_select_random_and_ties():
    rng = np.random.default_rng(7)
    paths = {True: 0, False: 0}
    for trial in range(300):
        n = int(rng.integers(1, 2049))
        k = int(min(n, rng.integers(1, 64)))
        if trial % 3 == 0:  # integer lattice: many exact ties in d2
            pts = rng.integers(0, 12, size=(n, 2)).astype(np.float64)
            q = rng.integers(0, 12, size=2).astype(np.float64)
        else:
            pts = rng.uniform(0, 512, size=(n, 2))
            q = rng.uniform(0, 512, size=2)
        d2 = (q[0] - pts[:, 0]) ** 2 + (q[1] - pts[:, 1]) ** 2
        got, fast = select(d2, k)
        paths[fast] += 1
        assert got == exact(d2, k), (n, k, trial)
    assert paths[True] > 0 and paths[False] > 0  # both the sort path and the fallback ran
