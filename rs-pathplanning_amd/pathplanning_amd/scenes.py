"""Synthetic scenes (host-side input data, no GPU needed).

* ``bench6`` — the reference's only fully specified scene, ``benches/all.rs:8-42`` (config 1).
* ``field512`` — BASELINE.json config 2/3/4: 1024 random discs on a 512x512 rectangle.

* ``transit`` / ``load_json`` — the example's JSON scene format (examples/rrt/src/main.rs:13-45):
  polygon bounds and polygon obstacles (§8f row 3, polygon mode).
* ``bench6_polygons`` — bench6 with its obstacles as ``create_circle`` polygons (rrt.rs:43-60).

A raw scene is a plain dict: ``bounds`` (x0, y0, x1, y1) of the un-shrunk rectangle, ``robot``
(width, height, max_steer) as in ``Robot::new`` (rrt.rs:25), ``circles`` (M, 3) array of
(cx, cy, r) as built by ``create_circle`` (rrt.rs:43), ``start``/``goal`` (x, y, yaw),
``max_iter`` and ``step_size`` as passed to ``RRT::new`` (rrt.rs:335-343).  A polygon scene
adds ``bounds_polygon`` (the bounds ring, (N, 2)) and ``obstacle_polygons`` (a list of (M_i, 2)
rings); its ``bounds`` is the ring's bbox and ``circles`` is empty.
"""
from __future__ import annotations

import math
import struct

import numpy as np

_M64 = (1 << 64) - 1


def rng_u64(seed: int, ctr: int) -> int:
    """SplitMix64 output ``ctr`` of the stream ``seed`` — the build's seeded replacement for
    ``rand::thread_rng`` (rrt.rs:140).  Mirrors pp_rng_u64 in the C-ABI."""
    z = (seed + (ctr + 1) * 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def gen_range(seed: int, ctr: int, low: float, high: float) -> float:
    """rand 0.7 ``gen_range(low, high)`` for f64 (UniformFloat::sample_single) on the seeded
    stream: 52 random bits under exponent 0 → [1, 2) → minus 1 → ``* scale + low``."""
    bits = (rng_u64(seed, ctr) >> 12) | 0x3FF0000000000000
    value0_1 = struct.unpack("<d", struct.pack("<Q", bits))[0] - 1.0
    scale = high - low
    while True:
        res = value0_1 * scale + low
        if res < high:
            return res
        scale = math.nextafter(scale, 0.0)


def to_radians(deg: float) -> float:
    """Rust ``f64::to_radians``: ``self * (PI / 180.0)``."""
    return deg * (math.pi / 180.0)


def bench6() -> dict:
    """benches/all.rs:8-42 (config 1)."""
    circles = np.array(
        [[5.0, 5.0, 1.0], [3.0, 6.0, 2.0], [3.0, 8.0, 2.0], [3.0, 10.0, 2.0],
         [7.0, 5.0, 2.0], [9.0, 5.0, 2.0]], dtype=np.float64)
    return {
        "name": "bench6",
        "bounds": (-6.0, -6.0, 15.0, 15.0),
        "robot": (1.0, 1.0, 0.8),
        "circles": circles,
        "start": (-5.0, -5.0, to_radians(-45.0)),
        "goal": (6.0, 10.0, to_radians(45.0)),
        "max_iter": 8000,
        "step_size": 0.1,
    }


def bench6_open(start_yaw: float = math.pi / 4.0) -> dict:
    """bench6 with the start moved into open space, (-3, -3, start_yaw): the goal-connection
    scene.  At bench6's own start (-5, -5, -45 deg) every check_finish fails — optimize's chain
    of root copies (yaw atan2(0,0) = 0, rrt.rs:463-487) ends in a Dubins loop into the root that
    leaves the shrunken bounds — so plan() has nothing to return there."""
    raw = bench6()
    raw["name"] = "bench6_open"
    raw["start"] = (-3.0, -3.0, float(start_yaw))
    return raw


def field512(n_obstacles: int = 1024, seed: int = 1234, size: float = 512.0,
             r_lo: float = 2.0, r_hi: float = 8.0, robot_width: float = 1.0,
             turn_radius: float = 4.0, step_size: float = 0.1,
             start=(8.0, 8.0, 0.0), goal=(504.0, 504.0, math.pi / 2.0),
             max_iter: int = 2000) -> dict:
    """BASELINE.json config 2: ``n_obstacles`` discs, centres U(0, size), r ~ U(r_lo, r_hi) from
    the seeded stream ``seed`` (attempt a draws counters 3a, 3a+1, 3a+2).  Discs whose inflated
    radius (plus a 1.0 margin) covers the start or the goal are rejected and redrawn."""
    half = robot_width / 2.0
    circles = []
    a = 0
    while len(circles) < n_obstacles:
        cx = gen_range(seed, 3 * a, 0.0, size)
        cy = gen_range(seed, 3 * a + 1, 0.0, size)
        r = gen_range(seed, 3 * a + 2, r_lo, r_hi)
        a += 1
        lim = r + half + 1.0
        bad = False
        for (px, py, _) in (start, goal):
            dx, dy = cx - px, cy - py
            if dx * dx + dy * dy <= lim * lim:
                bad = True
        if not bad:
            circles.append((cx, cy, r))
    return {
        "name": f"field{int(size)}_m{n_obstacles}_s{seed}",
        "bounds": (0.0, 0.0, size, size),
        "robot": (robot_width, robot_width, turn_radius),
        "circles": np.array(circles, dtype=np.float64).reshape(-1, 3),
        "start": tuple(start),
        "goal": tuple(goal),
        "max_iter": max_iter,
        "step_size": step_size,
    }


def config5_field() -> dict:
    """BASELINE config 5 (RRT*, build-defined): 10240 discs, centres U(0, 2048), r ~ U(1, 4) from
    stream 1234 (coverage ~7%: the crate's node-at-the-sample RRT accepts ~0.2% of long edges in
    a denser 10k field, too few for rewiring to matter), R = 4.0, step 0.1; the RRT* queries use
    Steer eta = 16."""
    return field512(n_obstacles=10240, size=2048.0, r_lo=1.0, r_hi=4.0,
                    start=(8.0, 8.0, 0.0), goal=(2040.0, 2040.0, math.pi / 2.0))


CONFIG5_ETA = 16.0


def query_endpoints(raw: dict, q: int, seed_base: int = 0):
    """Config 3: start/goal of query ``q`` drawn from free space by the seeded stream q.
    Rejection-samples points whose inflated-disc clearance is > 1.0; yaw U(-pi, pi)."""
    x0, y0, x1, y1 = raw["bounds"]
    half = raw["robot"][0] / 2.0
    circ = raw["circles"]

    def free(x, y):
        d2 = (circ[:, 0] - x) ** 2 + (circ[:, 1] - y) ** 2
        lim = circ[:, 2] + half + 1.0
        return bool(np.all(d2 > lim * lim))

    out = []
    ctr = 0
    s = seed_base + q
    while len(out) < 2:
        x = gen_range(s, ctr, x0 + half + 1.0, x1 - half - 1.0)
        y = gen_range(s, ctr + 1, y0 + half + 1.0, y1 - half - 1.0)
        yaw = gen_range(s, ctr + 2, -math.pi, math.pi)
        ctr += 3
        if free(x, y):
            out.append((x, y, yaw))
    return out[0], out[1]


def config3_queries(raw: dict, first: int, count: int, seed_base: int = 42):
    """BASELINE config 3: query q (q in [first, first + count)) samples with stream seed_base + q;
    its start and goal are the first two free poses of stream q — attempt a draws x, y, yaw from
    counters 3a, 3a+1, 3a+2 over the shrunken bounds; a pose is free when it is at least 1.0
    outside every inflated disc.  Returns (starts[count, 3], goals[count, 3], seeds[count])."""
    half = raw["robot"][0] / 2.0
    x0, y0, x1, y1 = raw["bounds"]
    minx, miny, maxx, maxy = x0 + half, y0 + half, x1 - half, y1 - half
    circ = np.asarray(raw["circles"], dtype=np.float64).reshape(-1, 3)
    cx, cy = circ[:, 0], circ[:, 1]
    lim2 = (circ[:, 2] + half + 1.0) ** 2
    starts = np.zeros((count, 3))
    goals = np.zeros((count, 3))
    for i in range(count):
        q = first + i
        poses = []
        a = 0
        while len(poses) < 2:
            x = gen_range(q, 3 * a, minx, maxx)
            y = gen_range(q, 3 * a + 1, miny, maxy)
            yaw = gen_range(q, 3 * a + 2, -math.pi, math.pi)
            a += 1
            if len(cx) == 0 or np.all((cx - x) ** 2 + (cy - y) ** 2 > lim2):
                poses.append((x, y, yaw))
        starts[i], goals[i] = poses
    seeds = np.arange(first, first + count, dtype=np.uint64) + np.uint64(seed_base)
    return starts, goals, seeds


def rasterize(raw: dict, w: int = 512, h: int = 512, x0: float = 0.0, y0: float = 0.0,
              cell: float = 1.0):
    """BASELINE config 4: the scene's discs rasterised into a w x h grid — cell (i, j) occupied
    when its centre (x0 + (i + 0.5) cell, y0 + (j + 0.5) cell) lies inside an inflated disc
    (dx*dx + dy*dy <= (r + width/2)^2) — bit-packed as uint32[h, ceil(w/32)], bit i % 32 of word
    i // 32.  Returns (bits, w, x0, y0, cell)."""
    half = raw["robot"][0] / 2.0
    circ = np.asarray(raw["circles"], dtype=np.float64).reshape(-1, 3)
    xs = x0 + (np.arange(w) + 0.5) * cell
    ys = y0 + (np.arange(h) + 0.5) * cell
    occ = np.zeros((h, w), dtype=bool)
    for cx, cy, r in circ:
        reff = r + half
        ix = np.nonzero(np.abs(xs - cx) <= reff + cell)[0]
        iy = np.nonzero(np.abs(ys - cy) <= reff + cell)[0]
        if len(ix) == 0 or len(iy) == 0:
            continue
        dx = xs[ix][None, :] - cx
        dy = ys[iy][:, None] - cy
        occ[np.ix_(iy, ix)] |= dx * dx + dy * dy <= reff * reff
    words = (w + 31) // 32
    padded = np.zeros((h, words * 32), dtype=bool)
    padded[:, :w] = occ
    bits = np.packbits(padded.reshape(h, words, 32)[:, :, ::-1], axis=2).view(">u4")
    return bits.reshape(h, words).astype(np.uint32), w, x0, y0, cell


def field512_grid() -> dict:
    """BASELINE config 4: field512 with its discs replaced by the 512 x 512 unit-cell raster."""
    raw = field512()
    raw["name"] = "field512_grid"
    raw["grid"] = rasterize(raw)
    return raw


# ------------------------------------------------------------------ polygon scenes (§8f row 3)
def ring(points) -> np.ndarray:
    """A polygon ring as (N, 2) f64 without the closing repeat (geo closes rings itself; the
    C ABI drops an exact repeat of the first vertex too)."""
    r = np.asarray(points, dtype=np.float64).reshape(-1, 2)
    if len(r) > 1 and r[0, 0] == r[-1, 0] and r[0, 1] == r[-1, 1]:
        r = r[:-1]
    return np.ascontiguousarray(r)


def create_circle_polygon(center, radius: float) -> np.ndarray:
    """``create_circle`` (rrt.rs:43-60) as the polygon the crate builds (pp_create_circle): n =
    ceil(2 pi r / 1.0) chords, vertices i = 0..=n at angle 2 pi / n * i (the last one repeats the
    first up to rounding), in the Rust expression's evaluation order.  (N + 1, 2) array."""
    import ctypes as C

    from . import _ffi

    n = C.c_int(0)
    L = _ffi.lib()
    _ffi.check(L.pp_create_circle(float(center[0]), float(center[1]), float(radius), None, 0,
                                  C.byref(n)))
    xy = np.zeros(2 * n.value)
    _ffi.check(L.pp_create_circle(float(center[0]), float(center[1]), float(radius),
                                  xy.ctypes.data_as(C.POINTER(C.c_double)), n.value, C.byref(n)))
    return xy.reshape(-1, 2)


def polygon_scene(bounds, obstacles, robot, start, goal, max_iter=8000, step_size=0.1,
                  name="polygons") -> dict:
    """A raw polygon scene: ``Space::new(Polygon(bounds), robot, obstacles)`` (rrt.rs:81-122)."""
    b = ring(bounds)
    obs = [ring(o) for o in obstacles]
    return {
        "name": name,
        "bounds": (float(b[:, 0].min()), float(b[:, 1].min()), float(b[:, 0].max()),
                   float(b[:, 1].max())),
        "bounds_polygon": b,
        "obstacle_polygons": obs,
        "robot": tuple(float(v) for v in robot),
        "circles": np.zeros((0, 3)),
        "start": tuple(float(v) for v in start),
        "goal": tuple(float(v) for v in goal),
        "max_iter": int(max_iter),
        "step_size": float(step_size),
    }


def load_json(src, name: str = "json") -> dict:
    """The example's scene file (examples/rrt/src/main.rs:13-45): ``{bounds: [[x, y]...],
    obstacles: [[[x, y]...]...], path, start: [x, y, yaw], goal: [x, y, yaw]}`` with the
    example's ``Robot::new(1.8, 3.0, 0.8)``, ``max_iter`` 8000 and step 0.1
    (main.rs:47, 58-66).  ``src``: a path or an already parsed dict."""
    import json

    conf = src if isinstance(src, dict) else json.load(open(src))
    return polygon_scene(conf["bounds"], conf["obstacles"], (1.8, 3.0, 0.8), conf["start"],
                         conf["goal"], 8000, 0.1, name=name)


def load_path(path: str) -> np.ndarray:
    """A ``cac.path`` file as examples/rrt/convert.py reads it: whitespace-separated x y per
    line, divided by 100.  Returns (N, 2)."""
    out = []
    with open(path) as f:
        for line in f:
            n = line.split()
            if len(n) >= 2:
                out.append((float(n[0]) / 100.0, float(n[1]) / 100.0))
    return np.array(out, dtype=np.float64).reshape(-1, 2)


def bench6_polygons() -> dict:
    """bench6 (benches/all.rs:8-42) with the obstacles as the crate's own ``create_circle``
    polygons and the bounds rectangle as a ring: the reference's scene in polygon mode."""
    raw = bench6()
    x0, y0, x1, y1 = raw["bounds"]
    obs = [create_circle_polygon((c[0], c[1]), c[2]) for c in raw["circles"]]
    # the ring in the bench's own vertex order (benches/all.rs:21-28)
    out = polygon_scene([(x0, y0), (x0, y1), (x1, y1), (x1, y0), (x0, y0)], obs, raw["robot"],
                        raw["start"], raw["goal"], raw["max_iter"], raw["step_size"],
                        name="bench6_polygons")
    return out


def bench6_polygons_open(start_yaw: float = math.pi / 4.0) -> dict:
    """bench6_polygons from bench6_open's start (-3, -3, start_yaw): the polygon-mode
    goal-connection scene (at bench6's own start nothing ever finishes, see bench6_open)."""
    raw = bench6_polygons()
    raw["name"] = "bench6_polygons_open"
    raw["start"] = (-3.0, -3.0, float(start_yaw))
    return raw


def transit(path: str | None = None) -> dict:
    """The example's own scene, examples/rrt/transit.debug.json (the data file ships with the
    package under data/, so the GPU box, which has no /root/reference, can load it)."""
    import os

    if path is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data",
                            "transit.debug.json")
    return load_json(path, name="transit")


def field512_polygons() -> dict:
    """config 2's field in polygon mode (§8f row 3 at scale): the same 1024 discs as the crate's
    own ``create_circle`` polygons (about 31 edges each, ~32k edges) and the 512 x 512 bounds as a
    ring, so Space::verify runs the polygon-buffer tests (Q10p) instead of the analytic discs."""
    raw = field512()
    x0, y0, x1, y1 = raw["bounds"]
    obs = [create_circle_polygon((c[0], c[1]), c[2]) for c in raw["circles"]]
    return polygon_scene([(x0, y0), (x1, y0), (x1, y1), (x0, y1)], obs, raw["robot"],
                         raw["start"], raw["goal"], raw["max_iter"], raw["step_size"],
                         name="field512_polygons")
