"""TEST INFRASTRUCTURE ONLY — second, independent restatement of the reference hot path.

A pure-Python restatement of tsturzl/rs-pathplanning's ``src/dubins.rs`` and of the sequential
spec of ``src/rrt.rs``'s extend loop.  It exists to generate the golden fixtures under
``tests/golden/`` (see ``tests/golden/gen_golden.py``) and to cross-check the C oracle
(``oracle/pp_oracle.c``); nothing in the product imports it.

Python's ``math`` module calls the platform libm for sin/cos/atan2/acos exactly as Rust's ``f64``
methods do (``hypot`` goes through libm via ctypes, see below), and CPython evaluates ``a * b + c`` without FMA contraction, so this restatement and
the C oracle are expected to agree bit for bit.  Parity against the Rust crate itself is
**unpinned** (no toolchain, no reference goldens: SURVEY.md K3/K7).

Build-defined deviations are the same as the C oracle's header lists (Q7-Q10, Q10p).
"""
from __future__ import annotations

import ctypes
import ctypes.util
import math
import struct

import numpy as np

# Rust's f64::hypot calls libm hypot (std's cmath shim); CPython's math.hypot is its own
# algorithm (vector_norm) and differs from glibc by an ulp on some inputs, so call libm directly.
_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
_libm.hypot.argtypes = [ctypes.c_double, ctypes.c_double]
_libm.hypot.restype = ctypes.c_double
libm_hypot = _libm.hypot

PI = math.pi  # == std::f64::consts::PI
TWO_PI = 2.0 * PI

L, S, R = 0, 1, 2
WORD_NAMES = ["LSL", "RSR", "LSR", "RSL", "RLR", "LRL"]
WORD_MODES = [(L, S, L), (R, S, R), (L, S, R), (R, S, L), (R, L, R), (L, R, L)]


def fmodr(x, y):  # dubins.rs:14-16
    q = x / y
    # f64::floor passes NaN / inf through (math.floor raises): a NaN pose gives NaN words, which
    # never win `bcost > cost` (dubins.rs:354), so the steer is None as in Rust
    return x - y * (math.floor(q) if math.isfinite(q) else q)


def mod2pi(theta):  # dubins.rs:18-20
    return fmodr(theta, TWO_PI)


def pi_2_pi(angle):  # dubins.rs:22-24 (Rust % == C fmod, truncated)
    return math.fmod(angle + PI, TWO_PI) - PI


def lsl(alpha, beta, d):  # dubins.rs:27-48
    sa, sb, ca, cb = math.sin(alpha), math.sin(beta), math.cos(alpha), math.cos(beta)
    c_ab = math.cos(alpha - beta)
    tmp0 = d + sa - sb
    p_squared = 2.0 + (d * d) - (2.0 * c_ab) + (2.0 * d * (sa - sb))
    if p_squared < 0.0:
        return None
    tmp1 = math.atan2(cb - ca, tmp0)
    return (mod2pi(-alpha + tmp1), math.sqrt(p_squared), mod2pi(beta - tmp1))


def rsr(alpha, beta, d):  # dubins.rs:51-71
    sa, sb, ca, cb = math.sin(alpha), math.sin(beta), math.cos(alpha), math.cos(beta)
    c_ab = math.cos(alpha - beta)
    tmp0 = d - sa + sb
    p_squared = 2.0 + (d * d) - (2.0 * c_ab) + (2.0 * d * (sb - sa))
    if p_squared < 0.0:
        return None
    tmp1 = math.atan2(ca - cb, tmp0)
    return (mod2pi(alpha - tmp1), math.sqrt(p_squared), mod2pi(-beta + tmp1))


def lsr(alpha, beta, d):  # dubins.rs:74-92
    sa, sb, ca, cb = math.sin(alpha), math.sin(beta), math.cos(alpha), math.cos(beta)
    c_ab = math.cos(alpha - beta)
    p_squared = -2.0 + (d * d) + (2.0 * c_ab) + (2.0 * d * (sa + sb))
    if p_squared < 0.0:
        return None
    p = math.sqrt(p_squared)
    tmp = math.atan2(-ca - cb, d + sa + sb) - math.atan2(-2.0, p)
    return (mod2pi(-alpha + tmp), p, mod2pi(-mod2pi(beta) + tmp))


def rsl(alpha, beta, d):  # dubins.rs:95-113
    sa, sb, ca, cb = math.sin(alpha), math.sin(beta), math.cos(alpha), math.cos(beta)
    c_ab = math.cos(alpha - beta)
    p_squared = -2.0 + (d * d) + (2.0 * c_ab) - (2.0 * d * (sa + sb))
    if p_squared < 0.0:
        return None
    p = math.sqrt(p_squared)
    tmp = math.atan2(ca + cb, d - sa - sb) - math.atan2(2.0, p)
    return (mod2pi(alpha - tmp), p, mod2pi(beta - tmp))


def rlr(alpha, beta, d):  # dubins.rs:116-133
    sa, sb, ca, cb = math.sin(alpha), math.sin(beta), math.cos(alpha), math.cos(beta)
    c_ab = math.cos(alpha - beta)
    tmp_rlr = (6.0 - d * d + 2.0 * c_ab + 2.0 * d * (sa - sb)) / 8.0
    if abs(tmp_rlr) > 1.0:
        return None
    p = mod2pi(2.0 * PI - math.acos(tmp_rlr))
    t = mod2pi(alpha - math.atan2(ca - cb, d - sa + sb) + mod2pi(p / 2.0))
    q = mod2pi(alpha - beta - t + mod2pi(p))
    return (t, p, q)


def lrl(alpha, beta, d):  # dubins.rs:136-153
    sa, sb, ca, cb = math.sin(alpha), math.sin(beta), math.cos(alpha), math.cos(beta)
    c_ab = math.cos(alpha - beta)
    tmp_lrl = (6.0 - d * d + 2.0 * c_ab + 2.0 * d * (-sa + sb)) / 8.0
    if abs(tmp_lrl) > 1.0:
        return None
    p = mod2pi(2.0 * PI - math.acos(tmp_lrl))
    t = mod2pi(-alpha - math.atan2(ca - cb, d + sa - sb) + p / 2.0)
    q = mod2pi(mod2pi(beta) - alpha - t + mod2pi(p))
    return (t, p, q)


ALL_PLANNERS = [lsl, rsr, lsr, rsl, rlr, lrl]  # dubins.rs:291


def _interpolate(ind, length, mode, c, ox, oy, oyaw, px, py, pyaw):  # dubins.rs:155-198
    if mode == S:
        px[ind] = ox + length / c * math.cos(oyaw)
        py[ind] = oy + length / c * math.sin(oyaw)
        pyaw[ind] = oyaw
    else:
        ldx = math.sin(length) / c
        if mode == L:
            ldy = (1.0 - math.cos(length)) / c
        else:
            ldy = (1.0 - math.cos(length)) / -c
        gdx = math.cos(-oyaw) * ldx + math.sin(-oyaw) * ldy
        gdy = -math.sin(-oyaw) * ldx + math.cos(-oyaw) * ldy
        px[ind] = ox + gdx
        py[ind] = oy + gdy
    if mode == L:
        pyaw[ind] = oyaw + length
    elif mode == R:
        pyaw[ind] = oyaw - length


def _generate_local_course(lengths, modes, c, step, px, py, pyaw):  # dubins.rs:200-289
    ind = 1
    ll = 0.0
    for i in range(3):
        m, l = modes[i], lengths[i]
        d = step if l > 0.0 else -step
        ox, oy, oyaw = px[ind], py[ind], pyaw[ind]
        ind -= 1
        if i >= 1 and (lengths[i - 1] * lengths[i]) > 0.0:
            pd = -d - ll
        else:
            pd = d - ll
        while abs(pd) <= abs(l):
            ind += 1
            _interpolate(ind, pd, m, c, ox, oy, oyaw, px, py, pyaw)
            pd += d
        ll = l - pd - d
        ind += 1
        _interpolate(ind, l, m, c, ox, oy, oyaw, px, py, pyaw)
    # trailing-zero trim (dubins.rs:281-288): pops every trailing 0.0 and one more element
    last = px[-1]
    while len(px) >= 1 and last == 0.0:
        last = px[-1]
        px.pop()
        py.pop()
        pyaw.pop()


def dubins_path_planning_from_origin(dx, dy, eyaw, c, step):  # dubins.rs:326-399
    hyp = libm_hypot(dx, dy)
    d = hyp * c
    theta = mod2pi(math.atan2(dy, dx))
    alpha = mod2pi(-theta)
    beta = mod2pi(eyaw - theta)
    bcost = math.inf
    best = None
    for i, f in enumerate(ALL_PLANNERS):
        r = f(alpha, beta, d)
        if r is not None:
            cost = abs(r[0]) + abs(r[1]) + abs(r[2])
            if bcost > cost:
                best, bcost = (i, r), cost
    if best is None:
        return None
    word, lengths = best
    total = 0.0
    for v in lengths:
        total += v
    n_point = int(math.trunc(total / step)) + 3 + 4
    px, py, pyaw = [0.0] * n_point, [0.0] * n_point, [0.0] * n_point
    _generate_local_course(lengths, WORD_MODES[word], c, step, px, py, pyaw)
    return px, py, pyaw, word, bcost


def dubins_path_planning(sx, sy, syaw, ex, ey, eyaw, turn_radius, step_size):  # dubins.rs:401-428
    exr = ex - sx
    eyr = ey - sy
    c = 1.0 / turn_radius
    lex = math.cos(syaw) * exr + math.sin(syaw) * eyr
    ley = -(math.sin(syaw)) * exr + math.cos(syaw) * eyr
    leyaw = eyaw - syaw
    r = dubins_path_planning_from_origin(lex, ley, leyaw, c, step_size)
    if r is None:
        return None
    lpx, lpy, lpyaw, word, cost = r
    cs, sn = math.cos(-syaw), math.sin(-syaw)
    px = [cs * x + sn * y + sx for x, y in zip(lpx, lpy)]
    py = [-sn * x + cs * y + sy for x, y in zip(lpx, lpy)]
    pyaw = [pi_2_pi(v + syaw) for v in lpyaw]
    return px, py, pyaw, word, cost


# ---------------------------------------------------------------- seeded sampling (Q7)
_M64 = (1 << 64) - 1


def rng_u64(seed, ctr):
    z = (seed + (ctr + 1) * 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def gen_range(seed, ctr, low, high):
    bits = (rng_u64(seed, ctr) >> 12) | 0x3FF0000000000000
    value1_2 = struct.unpack("<d", struct.pack("<Q", bits))[0]
    value0_1 = value1_2 - 1.0
    scale = high - low
    while True:
        res = value0_1 * scale + low
        if res < high:
            return res
        scale = math.nextafter(scale, 0.0)


# ------------------------------------------------------- sequential RRT extend (small cases)
def _seg_hits_any(xs, ys, cx, cy, r2):
    """vectorised restatement of the segment-vs-disc test (same op order as the C oracle)."""
    ax, ay = xs[:-1, None], ys[:-1, None]
    bx, by = xs[1:, None], ys[1:, None]
    vx, vy = bx - ax, by - ay
    wx, wy = cx[None, :] - ax, cy[None, :] - ay
    l2 = vx * vx + vy * vy
    with np.errstate(divide="ignore", invalid="ignore"):
        t = (wx * vx + wy * vy) / l2
    t = np.where(l2 > 0.0, t, 0.0)
    t = np.where(t < 0.0, 0.0, np.where(t > 1.0, 1.0, t))
    ex, ey = wx - t * vx, wy - t * vy
    return bool(np.any(ex * ex + ey * ey <= r2[None, :]))


def _seg_point_d2(ax, ay, bx, by, cx, cy):
    """squared distance from c to the closed segment a-b (broadcasting; same op order as C)"""
    vx, vy = bx - ax, by - ay
    wx, wy = cx - ax, cy - ay
    l2 = vx * vx + vy * vy
    with np.errstate(divide="ignore", invalid="ignore"):
        t = (wx * vx + wy * vy) / l2
    t = np.where(l2 > 0.0, t, 0.0)
    t = np.where(t < 0.0, 0.0, np.where(t > 1.0, 1.0, t))
    ex, ey = wx - t * vx, wy - t * vy
    return ex * ex + ey * ey


def _ray_crosses(px, py, xi, yi, xj, yj):
    """even-odd step: edge (xi, yi)-(xj, yj) crosses the ray from (px, py) toward +x"""
    with np.errstate(divide="ignore", invalid="ignore"):
        xc = (xj - xi) * (py - yi) / (yj - yi) + xi
    return ((yi > py) != (yj > py)) & (px < xc)


def _polygon_verify(scene, xs, ys):
    """Q10p (polygon scenes): points in the eroded bounds ring, segments clear of the obstacle
    edge buffers (cross or within h), point 0 outside every obstacle polygon."""
    h2 = scene["h2"]
    bvx, bvy = scene["bvx"], scene["bvy"]
    bjx, bjy = np.roll(bvx, -1), np.roll(bvy, -1)
    px, py = xs[:, None], ys[:, None]
    inside = np.sum(_ray_crosses(px, py, bvx[None, :], bvy[None, :], bjx[None, :], bjy[None, :]),
                    axis=1) % 2 == 1
    near = np.any(_seg_point_d2(bvx[None, :], bvy[None, :], bjx[None, :], bjy[None, :], px, py) < h2,
                  axis=1)
    if not np.all(inside & ~near):
        return False
    ex0, ey0, ex1, ey1 = scene["ex0"], scene["ey0"], scene["ex1"], scene["ey1"]
    if len(ex0) == 0:
        return True
    if len(xs) == 1:
        ax, ay, bx, by = xs[:, None], ys[:, None], xs[:, None], ys[:, None]
    else:
        ax, ay, bx, by = xs[:-1, None], ys[:-1, None], xs[1:, None], ys[1:, None]
    e0x, e0y, e1x, e1y = ex0[None, :], ey0[None, :], ex1[None, :], ey1[None, :]
    d1 = (e1x - e0x) * (ay - e0y) - (e1y - e0y) * (ax - e0x)
    d2 = (e1x - e0x) * (by - e0y) - (e1y - e0y) * (bx - e0x)
    d3 = (bx - ax) * (e0y - ay) - (by - ay) * (e0x - ax)
    d4 = (bx - ax) * (e1y - ay) - (by - ay) * (e1x - ax)
    cross = (((d1 > 0.0) & (d2 < 0.0)) | ((d1 < 0.0) & (d2 > 0.0))) & \
            (((d3 > 0.0) & (d4 < 0.0)) | ((d3 < 0.0) & (d4 > 0.0)))
    hit = cross | (_seg_point_d2(e0x, e0y, e1x, e1y, ax, ay) <= h2) | \
        (_seg_point_d2(e0x, e0y, e1x, e1y, bx, by) <= h2) | \
        (_seg_point_d2(ax, ay, bx, by, e0x, e0y) <= h2) | \
        (_seg_point_d2(ax, ay, bx, by, e1x, e1y) <= h2)
    if np.any(hit):
        return False
    c = _ray_crosses(xs[0], ys[0], ex0, ey0, ex1, ey1).astype(np.int64)
    per_poly = np.bincount(scene["epoly"], weights=c)
    return not np.any(per_poly.astype(np.int64) % 2 == 1)


def verify_line(scene, xs, ys):  # rrt.rs:124-137 (Q10)
    xs = np.asarray(xs, dtype=np.float64)
    ys = np.asarray(ys, dtype=np.float64)
    if len(xs) == 0:
        return True
    if np.any(xs < scene["minx"]) or np.any(xs > scene["maxx"]):
        return False
    if np.any(ys < scene["miny"]) or np.any(ys > scene["maxy"]):
        return False
    if scene.get("bvx") is not None:  # polygon scene (Q10p)
        return _polygon_verify(scene, xs, ys)
    if scene.get("grid") is not None:  # config 4: every point in a free cell
        bits, w, gx0, gy0, cell = scene["grid"]
        inv = 1.0 / cell
        for x, y in zip(xs, ys):
            fx, fy = math.floor((x - gx0) * inv), math.floor((y - gy0) * inv)
            if not (0 <= fx < w and 0 <= fy < bits.shape[0]):
                return False
            if (int(bits[fy, fx >> 5]) >> (fx & 31)) & 1:
                return False
        return True
    cx, cy, r2 = scene["cx"], scene["cy"], scene["r2"]
    if len(cx) == 0:
        return True
    if len(xs) == 1:
        xs = np.concatenate([xs, xs])
        ys = np.concatenate([ys, ys])
    return not _seg_hits_any(xs, ys, cx, cy, r2)


def rrt_extend(scene, tree, seed, it0, n_iter):
    """Sequential spec of plan_one's extend (rrt.rs:583-589), incremental verify.

    ``tree`` is a dict of python lists x, y, yaw, parent (root first).  Returns per-iteration
    (nearest, accepted) logs.
    """
    R, step = scene["turn_radius"], scene["step_size"]
    log = []
    for k in range(n_iter):
        it = it0 + k
        x = gen_range(seed, 2 * it, scene["minx"], scene["maxx"])
        y = gen_range(seed, 2 * it + 1, scene["miny"], scene["maxy"])
        best, bd = -1, math.inf
        for i, (nx, ny) in enumerate(zip(tree["x"], tree["y"])):
            dx, dy = x - nx, y - ny
            d2 = dx * dx + dy * dy
            if d2 < bd:
                best, bd = i, d2
        p = best
        yaw = math.atan2(tree["y"][p] - y, tree["x"][p] - x)  # rrt.rs:267-271
        r = dubins_path_planning(x, y, yaw, tree["x"][p], tree["y"][p], tree["yaw"][p], R, step)
        if r is None:
            xs, ys = [x], [y]
        else:
            xs, ys = list(r[0]), list(r[1])
        xs.append(tree["x"][p])
        ys.append(tree["y"][p])
        ok = verify_line(scene, xs, ys)
        if ok:
            tree["x"].append(x)
            tree["y"].append(y)
            tree["yaw"].append(yaw)
            tree["parent"].append(p)
        log.append((p, int(ok)))
    return log


# ------------------------------------------- check_finish / optimize / finalize (small cases)
class PNode:
    """rrt.rs:161-214: a point, an optional parent and the yaw toward it (or the given yaw)."""
    __slots__ = ("x", "y", "yaw", "parent")

    def __init__(self, x, y, yaw, parent):
        self.x, self.y, self.yaw, self.parent = x, y, yaw, parent

    @staticmethod
    def new(x, y, parent):  # Node::new, compute_yaw (rrt.rs:169-175, 267-271)
        return PNode(x, y, math.atan2(parent.y - y, parent.x - x), parent)

    def iter_to_root(self):  # NodeIter (rrt.rs:253-265)
        n = self
        while n is not None:
            yield n
            n = n.parent


def tree_nodes(tree):
    """PNode objects for a tree dict (x, y, yaw, parent lists, root first)."""
    nodes = []
    for i in range(len(tree["x"])):
        p = tree["parent"][i]
        nodes.append(PNode(tree["x"][i], tree["y"][i], tree["yaw"][i], nodes[p] if p >= 0 else None))
    return nodes


def line_to_origin(node, R, step):  # rrt.rs:291-321, sequential order
    xs, ys = [], []
    for n in node.iter_to_root():
        if n.parent is None:
            xs.append(n.x)
            ys.append(n.y)
            continue
        r = dubins_path_planning(n.x, n.y, n.yaw, n.parent.x, n.parent.y, n.parent.yaw, R, step)
        if r is None:
            xs.append(n.x)
            ys.append(n.y)
        else:
            xs.extend(r[0])
            ys.extend(r[1])
    return xs, ys


def optimize(scene, node, i, chain):  # rrt.rs:463-487, full line_to_origin verify
    if i >= 16:
        return None
    R, step = scene["turn_radius"], scene["step_size"]
    for to in reversed(list(node.iter_to_root())):
        new = PNode.new(node.x, node.y, to)
        if verify_line(scene, *line_to_origin(new, R, step)):
            chain.append(to)
            t = optimize(scene, to, i + 1, chain)
            return PNode.new(node.x, node.y, t) if t is not None else new
    return None


def finalize(scene, goal, goal_yaw=None):  # rrt.rs:489-540
    """goal_yaw: the planner's goal yaw, which optimize_from_goal gives the new goal node when
    optimize succeeds (rrt.rs:494-498); default: the goal node's own (check_finish: the same)."""
    R, step = scene["turn_radius"], scene["step_size"]
    chain = []
    if goal.parent is not None:
        n = optimize(scene, goal.parent, 0, chain)
        if n is not None:
            goal = PNode(goal.x, goal.y, goal.yaw if goal_yaw is None else goal_yaw, n)
    xs, ys = [], []
    for n in goal.iter_to_root():
        if n.parent is None:
            continue
        r = dubins_path_planning(n.x, n.y, n.yaw, n.parent.x, n.parent.y, n.parent.yaw, R, step)
        if r is None:
            raise RuntimeError("Should plan dubins curve")  # rrt.rs:529
        xs.extend(r[0])
        ys.extend(r[1])
    xs.reverse()
    ys.reverse()
    return xs, ys, chain


def line_length(xs, ys):  # geo EuclideanLength: sum of hypot over consecutive points
    s = 0.0
    for i in range(len(xs) - 1):
        s += libm_hypot(xs[i + 1] - xs[i], ys[i + 1] - ys[i])
    return s


def check_finish(scene, node, goal, goal_yaw):  # rrt.rs:428-438
    """(ok, xs, ys, length, chain) — chain = optimize's chosen ancestors (PNode objects)."""
    g = PNode(goal[0], goal[1], goal_yaw, node)  # Node::new_goal
    xs, ys, chain = finalize(scene, g)
    ok = verify_line(scene, xs, ys)
    return ok, xs, ys, line_length(xs, ys), chain
