"""The lane-parallel `pd += d` generator of steer_walk (pp_kernels.hip, walk_rec) restated with
numpy lanes and checked against the serial walk of generate_local_course (dubins.rs:239-259):
same points, same segment split, same values bit for bit.  CPU only (algorithm check; the HIP
kernel itself is covered by the GPU parity tests)."""
import math
import struct
from fractions import Fraction

import numpy as np


def serial_walk(L, step):
    pts = []
    ll = 0.0
    for i in range(3):
        d = step if L[i] > 0.0 else -step
        pd = (-d - ll) if (i >= 1 and L[i - 1] * L[i] > 0.0) else (d - ll)
        while abs(pd) <= abs(L[i]):
            pts.append((i, pd))
            pd += d
        ll = L[i] - pd - d
    return pts


def _sign_exp(x):
    """the top 12 bits of an f64 (sign and exponent): equal ones share one ulp"""
    return struct.unpack("<Q", struct.pack("<d", x))[0] >> 52


def closed_form(pd, d, pos, aL):
    """walk_rec's closed form of a chunk pass: when w1 - w0 == w2 - w1 (=: delta), lane l's value
    is w0 + (l - pos) * delta (one exact fma), valid while every value up to the first one past
    |L| keeps w0's sign and exponent; None when the pass must take the serial chain"""
    w1 = pd + d
    w2 = w1 + d
    if (w1 - pd) != (w2 - w1):
        return None
    delta = w1 - pd
    v = np.full(64, pd)
    for lane in range(pos, 64):
        v[lane] = float(Fraction(pd) + (lane - pos) * Fraction(delta))  # representable: exact
    fail = [lane for lane in range(pos, 64) if not abs(v[lane]) <= aL]
    last = fail[0] if fail else 63
    if any(_sign_exp(float(v[lane])) != _sign_exp(pd) for lane in range(pos, last + 1)):
        return None
    return v


def lane_walk(L, step, stored=63, use_closed_form=False, stats=None):
    """chunk 0 from a serial prefix of `stored` points (steer_prep), then 63-lane chunks"""
    pts = []
    # steer_prep: serial walk of the first `stored` points, keeping the state there
    seg, ll = 0, 0.0
    d = step if L[0] > 0.0 else -step
    pd = d - 0.0
    while seg < 3:
        if abs(pd) <= abs(L[seg]):
            if len(pts) >= stored:
                break
            pts.append((seg, pd))
            pd += d
        else:
            ll = L[seg] - pd - d
            seg += 1
            if seg < 3:
                dn = step if L[seg] > 0.0 else -step
                pd = (-dn - ll) if (L[seg - 1] * L[seg] > 0.0) else (dn - ll)
                d = dn
    if seg >= 3:
        return pts
    lanes = np.arange(64)
    while seg < 3:  # steer_walk chunks
        pos = 1
        while pos <= 63 and seg < 3:
            Ls = L[seg]
            kk = lanes - pos
            v = closed_form(pd, d, pos, abs(Ls)) if use_closed_form else None
            if stats is not None:
                stats[v is not None] += 1
            if v is None:
                v = np.full(64, pd)
                for u in range(63 - pos):
                    v = np.where(u < kk, v + d, v)
            bad = (lanes >= pos) & ~(np.abs(v) <= abs(Ls))
            m = int(np.argmax(bad)) if bad.any() else 64
            for lane in range(pos, min(m, 64)):
                pts.append((seg, float(v[lane])))
            if m <= 63:
                pend = float(v[m])
                ll = Ls - pend - d
                seg += 1
                if seg < 3:
                    dn = step if L[seg] > 0.0 else -step
                    pd = (-dn - ll) if (Ls * L[seg] > 0.0) else (dn - ll)
                    d = dn
                pos = m
            else:
                pd = float(v[63]) + d
                pos = 64
    return pts


def test_lane_walk_equals_serial_walk():
    rng = np.random.default_rng(7)
    cases = [
        ([0.0, 0.0, 0.0], 0.1), ([2 * math.pi, 0.0, 0.0], 0.1), ([-3.0, 5.0, -0.05], 0.1),
        ([0.05, -0.05, 0.05], 0.1), ([12.3, 45.6, 7.8], 0.1), ([1e-12, 30.0, -1e-12], 0.3),
        ([6.3, 6.3, 6.3], 0.01),
    ]
    for _ in range(300):
        L = [float(v) for v in rng.uniform(-30, 30, 3) * rng.choice([0.0, 0.01, 1.0], 3)]
        cases.append((L, float(rng.choice([0.01, 0.05, 0.1, 0.3, 0.37]))))
    for L, step in cases:
        a = serial_walk(L, step)
        b = lane_walk(L, step)
        assert len(a) == len(b), (L, step)
        assert all(x[0] == y[0] and x[1] == y[1] for x, y in zip(a, b)), (L, step)


def test_closed_form_passes_equal_serial_walk():
    """the closed-form chunk passes (walk_rec, f64 fma) give the serial walk's values bit for bit,
    and most passes of long segments take them"""
    rng = np.random.default_rng(11)
    cases = [([150.0, 0.0, 0.0], 0.1), ([-175.3, 3.0, 96.0], 0.1), ([63.99, 64.2, -0.3], 0.1),
             ([1.0, -1.0, 1.0], 0.1), ([0.5, 300.0, 2.0], 0.37), ([127.9, -128.1, 255.9], 0.1)]
    for _ in range(120):
        L = [float(v) for v in rng.uniform(-200, 200, 3) * rng.choice([0.0, 0.01, 1.0], 3)]
        cases.append((L, float(rng.choice([0.01, 0.05, 0.1, 0.3, 0.37]))))
    stats = [0, 0]
    for L, step in cases:
        a = serial_walk(L, step)
        b = lane_walk(L, step, use_closed_form=True, stats=stats)
        assert len(a) == len(b), (L, step)
        assert all(x[0] == y[0] and x[1] == y[1] for x, y in zip(a, b)), (L, step)
    assert stats[1] > 4 * stats[0], stats  # the closed form serves most passes
