"""TEST INFRASTRUCTURE ONLY — ctypes front-end of the C oracle (oracle/pp_oracle.c).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import this
module, and only as the checker (or the timed CPU baseline).  The product path
(``rs-pathplanning_amd/``) never imports, links or executes anything under ``oracle/``.

Parity status: unpinned against the Rust crate (it cannot be built or run here, and it ships no
golden vectors — SURVEY.md K3/K7); pinned against the independent pure-Python restatement
(oracle/dubins_py.py) through tests/golden/.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
_lock = threading.Lock()
_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH) or (
        os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "pp_oracle.c"))
    ):
        subprocess.run(["make", "-s", "-C", HERE, "-B" if force else "all"], check=True)
    return LIB_PATH


class Scene(C.Structure):
    _fields_ = [
        ("minx", C.c_double), ("maxx", C.c_double), ("miny", C.c_double), ("maxy", C.c_double),
        ("m", C.c_int),
        ("cx", C.POINTER(C.c_double)), ("cy", C.POINTER(C.c_double)), ("r2", C.POINTER(C.c_double)),
        ("turn_radius", C.c_double), ("step_size", C.c_double),
        ("bits", C.POINTER(C.c_uint32)), ("bw", C.c_int), ("bh", C.c_int), ("bwords", C.c_int),
        ("bx0", C.c_double), ("by0", C.c_double), ("binv", C.c_double),
        ("nbv", C.c_int), ("bvx", C.POINTER(C.c_double)), ("bvy", C.POINTER(C.c_double)),
        ("ne", C.c_int), ("ex0", C.POINTER(C.c_double)), ("ey0", C.POINTER(C.c_double)),
        ("ex1", C.POINTER(C.c_double)), ("ey1", C.POINTER(C.c_double)),
        ("epoly", C.POINTER(C.c_int)), ("h2", C.c_double),
    ]


class Tree(C.Structure):
    _fields_ = [
        ("x", C.POINTER(C.c_double)), ("y", C.POINTER(C.c_double)),
        ("yaw", C.POINTER(C.c_double)), ("parent", C.POINTER(C.c_int32)),
        ("cap", C.c_int), ("n", C.c_int),
    ]


def lib():
    global _lib
    with _lock:
        if _lib is None:
            build()
            L = C.CDLL(LIB_PATH)
            dp = C.POINTER(C.c_double)
            L.orc_dubins.argtypes = [dp, dp, dp, dp, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), dp]
            L.orc_dubins.restype = C.c_int
            L.orc_dubins_n_point.argtypes = [dp]
            L.orc_dubins_n_point.restype = C.c_int
            L.orc_rng_u64.argtypes = [C.c_uint64, C.c_uint64]
            L.orc_rng_u64.restype = C.c_uint64
            L.orc_gen_range.argtypes = [C.c_uint64, C.c_uint64, C.c_double, C.c_double]
            L.orc_gen_range.restype = C.c_double
            L.orc_mod2pi.argtypes = [C.c_double]
            L.orc_mod2pi.restype = C.c_double
            L.orc_pi_2_pi.argtypes = [C.c_double]
            L.orc_pi_2_pi.restype = C.c_double
            L.orc_verify_line.argtypes = [C.POINTER(Scene), dp, dp, C.c_int]
            L.orc_verify_line.restype = C.c_int
            L.orc_nearest.argtypes = [dp, dp, C.c_int, C.c_double, C.c_double, dp]
            L.orc_nearest.restype = C.c_int
            L.orc_rrt_extend.argtypes = [C.POINTER(Scene), C.POINTER(Tree), C.c_uint64, C.c_int64,
                                         C.c_int64, C.c_int, C.POINTER(C.c_int32), C.POINTER(C.c_int8)]
            L.orc_rrt_extend.restype = C.c_int64
            L.orc_rrt_extend_samples.argtypes = [C.POINTER(Scene), C.POINTER(Tree), dp, dp,
                                                 C.c_int64, C.c_int, C.POINTER(C.c_int32), dp,
                                                 C.POINTER(C.c_int8)]
            L.orc_rrt_extend_samples.restype = C.c_int64
            L.orc_verify_candidate.argtypes = [C.POINTER(Scene), C.POINTER(Tree), C.c_double,
                                               C.c_double, C.c_int, C.c_int, dp]
            L.orc_verify_candidate.restype = C.c_int
            ip = C.POINTER(C.c_int)
            L.orc_check_finish.argtypes = [C.POINTER(Scene), C.POINTER(Tree), C.c_int, C.c_double,
                                           C.c_double, C.c_double, C.c_int, dp, dp, C.c_int, ip,
                                           dp, ip, ip]
            L.orc_check_finish.restype = C.c_int
            L.orc_line_length.argtypes = [dp, dp, C.c_int]
            L.orc_line_length.restype = C.c_double
            L.orc_plan.argtypes = [C.POINTER(Scene), C.POINTER(Tree), C.c_uint64, C.c_int64,
                                   C.c_int64, C.c_double, C.c_double, C.c_double, C.c_int, ip, dp,
                                   C.POINTER(C.c_int32)]
            L.orc_plan.restype = C.c_int64
            L.orc_extend_replicas.argtypes = [C.POINTER(Scene), C.POINTER(Tree),
                                              C.POINTER(C.c_uint64), C.c_int, C.c_int64,
                                              C.c_int64, C.c_int, C.c_int]
            L.orc_extend_replicas.restype = C.c_int64
            L.orc_queries.argtypes = [C.POINTER(Scene), dp, C.POINTER(C.c_uint64), C.c_int,
                                      C.c_int64, C.c_int, C.c_int]
            L.orc_queries.restype = C.c_int64
            L.orc_star_k.argtypes = [C.c_int, C.c_int]
            L.orc_star_k.restype = C.c_int
            L.orc_star_extend.argtypes = [C.POINTER(Scene), C.POINTER(Tree), dp, dp, C.c_uint64,
                                          C.c_int64, C.c_int64, C.c_int, C.c_double,
                                          C.POINTER(C.c_int64), C.POINTER(C.c_int32),
                                          C.POINTER(C.c_int8)]
            L.orc_star_extend.restype = C.c_int64
            L.orc_star_queries.argtypes = [C.POINTER(Scene), dp, C.POINTER(C.c_uint64), C.c_int,
                                           C.c_int64, C.c_int, C.c_double, C.c_int,
                                           C.POINTER(C.c_int64)]
            L.orc_star_queries.restype = C.c_int64
            _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


# ------------------------------------------------------------------------------ dubins
def dubins(sx, sy, syaw, ex, ey, eyaw, turn_radius, step_size):
    """dubins_path_planning (dubins.rs:401-428): (px, py, pyaw, word, cost) or None."""
    L = lib()
    conf = np.array([sx, sy, syaw, ex, ey, eyaw, turn_radius, step_size], dtype=np.float64)
    cap = L.orc_dubins_n_point(_dp(conf))
    if cap <= 0:
        return None
    px, py, pyaw = (np.zeros(cap) for _ in range(3))
    n, word, cost = C.c_int(0), C.c_int(-1), C.c_double(0.0)
    r = L.orc_dubins(_dp(conf), _dp(px), _dp(py), _dp(pyaw), cap, C.byref(n), C.byref(word), C.byref(cost))
    if r < 0:
        raise RuntimeError("orc_dubins failed")
    if r == 0:
        return None
    k = n.value
    return px[:k].copy(), py[:k].copy(), pyaw[:k].copy(), word.value, cost.value


def gen_range(seed, ctr, low, high):
    return lib().orc_gen_range(seed, ctr, low, high)


def rng_u64(seed, ctr):
    return lib().orc_rng_u64(seed, ctr)


def mod2pi(x):
    return lib().orc_mod2pi(x)


def pi_2_pi(x):
    return lib().orc_pi_2_pi(x)


# ------------------------------------------------------------------------------- scene
def _ring(points):
    """polygon ring (N, 2) without an exact closing repeat of the first vertex"""
    r = np.asarray(points, dtype=np.float64).reshape(-1, 2)
    if len(r) > 1 and r[0, 0] == r[-1, 0] and r[0, 1] == r[-1, 1]:
        r = r[:-1]
    return np.ascontiguousarray(r)


class OracleScene:
    """Space::new (rrt.rs:81-122) restated for the oracle: bounds rectangle shrunk by width/2,
    discs inflated by width/2 (Q10).  Polygon mode (Q10p): ``polygons=(bounds_ring,
    [obstacle rings])`` — the sampling box is the ring's bbox shrunk by width/2, the obstacles
    are edge lists with exact Minkowski buffers."""

    def __init__(self, bounds, width, circles, turn_radius, step_size, grid=None, polygons=None):
        half = width / 2.0
        if polygons is not None:
            bring = _ring(polygons[0])
            bounds = (bring[:, 0].min(), bring[:, 1].min(), bring[:, 0].max(), bring[:, 1].max())
        x0, y0, x1, y1 = bounds
        self.minx, self.miny, self.maxx, self.maxy = x0 + half, y0 + half, x1 - half, y1 - half
        circ = np.asarray(circles, dtype=np.float64).reshape(-1, 3)
        self.cx = np.ascontiguousarray(circ[:, 0])
        self.cy = np.ascontiguousarray(circ[:, 1])
        reff = circ[:, 2] + half
        self.r2 = np.ascontiguousarray(reff * reff)
        self.turn_radius = float(turn_radius)
        self.step_size = float(step_size)
        self._c = Scene(self.minx, self.maxx, self.miny, self.maxy, len(self.cx), _dp(self.cx),
                        _dp(self.cy), _dp(self.r2), self.turn_radius, self.step_size)
        self.grid = None
        if grid is not None:
            bits, w, gx0, gy0, cell = grid
            self.bits = np.ascontiguousarray(bits, dtype=np.uint32)
            self.grid = (self.bits, int(w), float(gx0), float(gy0), float(cell))
            self._c.bits = self.bits.ctypes.data_as(C.POINTER(C.c_uint32))
            self._c.bw, self._c.bh, self._c.bwords = int(w), self.bits.shape[0], self.bits.shape[1]
            self._c.bx0, self._c.by0, self._c.binv = float(gx0), float(gy0), 1.0 / float(cell)
        self.polygons = None
        if polygons is not None:
            self.bvx = np.ascontiguousarray(bring[:, 0])
            self.bvy = np.ascontiguousarray(bring[:, 1])
            e0, e1, ep = [], [], []
            for k, o in enumerate(polygons[1]):
                r = _ring(o)
                if len(r) == 0:
                    continue
                e0.append(r)
                e1.append(np.roll(r, -1, axis=0))
                ep.append(np.full(len(r), k, dtype=np.int32))
            E0 = np.concatenate(e0) if e0 else np.zeros((0, 2))
            E1 = np.concatenate(e1) if e1 else np.zeros((0, 2))
            self.ex0, self.ey0 = np.ascontiguousarray(E0[:, 0]), np.ascontiguousarray(E0[:, 1])
            self.ex1, self.ey1 = np.ascontiguousarray(E1[:, 0]), np.ascontiguousarray(E1[:, 1])
            self.epoly = np.ascontiguousarray(np.concatenate(ep) if ep else np.zeros(0, np.int32))
            self.h2 = half * half
            self.polygons = (bring, [_ring(o) for o in polygons[1]])
            c = self._c
            c.nbv, c.bvx, c.bvy = len(self.bvx), _dp(self.bvx), _dp(self.bvy)
            c.ne = len(self.ex0)
            c.ex0, c.ey0, c.ex1, c.ey1 = _dp(self.ex0), _dp(self.ey0), _dp(self.ex1), _dp(self.ey1)
            c.epoly = self.epoly.ctypes.data_as(C.POINTER(C.c_int))
            c.h2 = self.h2

    @classmethod
    def from_raw(cls, raw):
        polys = None
        if "bounds_polygon" in raw:
            polys = (raw["bounds_polygon"], raw["obstacle_polygons"])
        return cls(raw["bounds"], raw["robot"][0], raw["circles"], raw["robot"][2], raw["step_size"],
                   grid=raw.get("grid"), polygons=polys)

    def as_dict(self):
        d = {"minx": self.minx, "maxx": self.maxx, "miny": self.miny, "maxy": self.maxy,
             "cx": self.cx, "cy": self.cy, "r2": self.r2, "turn_radius": self.turn_radius,
             "step_size": self.step_size, "grid": self.grid}
        if self.polygons is not None:
            d.update(bvx=self.bvx, bvy=self.bvy, ex0=self.ex0, ey0=self.ey0, ex1=self.ex1,
                     ey1=self.ey1, epoly=self.epoly, h2=self.h2)
        return d

    def verify_line(self, xs, ys):
        xs = np.ascontiguousarray(xs, dtype=np.float64)
        ys = np.ascontiguousarray(ys, dtype=np.float64)
        return bool(lib().orc_verify_line(C.byref(self._c), _dp(xs), _dp(ys), len(xs)))


class OracleTree:
    """SoA f64 tree, root first (RRT::new, rrt.rs:335-355)."""

    def __init__(self, start, cap):
        self.x = np.zeros(cap)
        self.y = np.zeros(cap)
        self.yaw = np.zeros(cap)
        self.parent = np.full(cap, -1, dtype=np.int32)
        self.x[0], self.y[0], self.yaw[0] = start
        self._c = Tree(_dp(self.x), _dp(self.y), _dp(self.yaw),
                       self.parent.ctypes.data_as(C.POINTER(C.c_int32)), cap, 1)

    @property
    def n(self):
        return self._c.n

    def arrays(self):
        n = self.n
        return self.x[:n].copy(), self.y[:n].copy(), self.yaw[:n].copy(), self.parent[:n].copy()


def rrt_extend(scene: OracleScene, tree: OracleTree, seed: int, it0: int, n_iter: int,
               full_reverify: bool = False):
    """Sequential extend for iterations [it0, it0+n_iter).  Returns (accepted, log_nn, log_acc)."""
    log_nn = np.zeros(n_iter, dtype=np.int32)
    log_acc = np.zeros(n_iter, dtype=np.int8)
    acc = lib().orc_rrt_extend(C.byref(scene._c), C.byref(tree._c), seed, it0, n_iter,
                               int(full_reverify), log_nn.ctypes.data_as(C.POINTER(C.c_int32)),
                               log_acc.ctypes.data_as(C.POINTER(C.c_int8)))
    if acc < 0:
        raise RuntimeError("orc_rrt_extend failed (capacity?)")
    return acc, log_nn, log_acc


def rrt_extend_samples(scene: OracleScene, tree: OracleTree, sx, sy, full_reverify: bool = False):
    """Sequential extend over caller-drawn samples (the host-owned RNG of pp_rrt_extend_samples).
    Returns (accepted, log_nn, log_yaw, log_acc)."""
    sx = np.ascontiguousarray(sx, dtype=np.float64)
    sy = np.ascontiguousarray(sy, dtype=np.float64)
    n = len(sx)
    log_nn = np.zeros(n, dtype=np.int32)
    log_yaw = np.zeros(n)
    log_acc = np.zeros(n, dtype=np.int8)
    acc = lib().orc_rrt_extend_samples(C.byref(scene._c), C.byref(tree._c), _dp(sx), _dp(sy), n,
                                       int(full_reverify),
                                       log_nn.ctypes.data_as(C.POINTER(C.c_int32)), _dp(log_yaw),
                                       log_acc.ctypes.data_as(C.POINTER(C.c_int8)))
    if acc < 0:
        raise RuntimeError("orc_rrt_extend_samples failed (capacity?)")
    return acc, log_nn, log_yaw, log_acc


def nearest(X, Y, qx, qy):
    X = np.ascontiguousarray(X, dtype=np.float64)
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    d2 = C.c_double(0)
    i = lib().orc_nearest(_dp(X), _dp(Y), len(X), qx, qy, C.byref(d2))
    return i, d2.value


def verify_candidate(scene: OracleScene, tree: OracleTree, x, y, parent, full_reverify=False):
    yaw = C.c_double(0)
    ok = lib().orc_verify_candidate(C.byref(scene._c), C.byref(tree._c), x, y, parent,
                                    int(full_reverify), C.byref(yaw))
    if ok < 0:
        raise RuntimeError("orc_verify_candidate failed")
    return bool(ok), yaw.value


def check_finish(scene: OracleScene, tree: OracleTree, node: int, goal, goal_yaw,
                 full_reverify=False):
    """RRT::check_finish (rrt.rs:428-438) for tree node `node`: None, or a dict with the finalized
    line (rrt.rs:503-540), its euclidean_length and optimize's chosen ancestors per level."""
    L = lib()
    gx, gy = goal
    n, ln, nch = C.c_int(0), C.c_double(0), C.c_int(0)
    chain = np.full(16, -1, dtype=np.int32)
    ip = C.POINTER(C.c_int)
    r = L.orc_check_finish(C.byref(scene._c), C.byref(tree._c), node, gx, gy, goal_yaw,
                           int(full_reverify), None, None, 0, C.byref(n), C.byref(ln),
                           chain.ctypes.data_as(ip), C.byref(nch))
    if r < 0:
        raise RuntimeError(f"orc_check_finish failed ({r})")
    out = {"ok": bool(r), "n": n.value, "length": ln.value, "chain": chain[:nch.value].tolist()}
    if r == 1:
        cap = max(n.value, 1)
        x, y = np.zeros(cap), np.zeros(cap)
        r2 = L.orc_check_finish(C.byref(scene._c), C.byref(tree._c), node, gx, gy, goal_yaw,
                                int(full_reverify), _dp(x), _dp(y), cap, C.byref(n), C.byref(ln),
                                None, None)
        assert r2 == 1
        out["x"], out["y"] = x[:n.value], y[:n.value]
    return out


def line_length(xs, ys):
    xs = np.ascontiguousarray(xs, dtype=np.float64)
    ys = np.ascontiguousarray(ys, dtype=np.float64)
    return lib().orc_line_length(_dp(xs), _dp(ys), len(xs))


def plan(scene: OracleScene, tree: OracleTree, seed: int, it0: int, n_iter: int, goal, goal_yaw,
         full_reverify=False):
    """RRT::plan (rrt.rs:599-619), sequential spec: extend + check_finish on every accepted node.
    Returns (accepted, best_node (-1: no finish), best_length, finish log per iteration
    (-1 not accepted, 0 None, 1 Some))."""
    bn, bl = C.c_int(-1), C.c_double(0)
    log = np.zeros(n_iter, dtype=np.int32)
    acc = lib().orc_plan(C.byref(scene._c), C.byref(tree._c), seed, it0, n_iter, goal[0], goal[1],
                         goal_yaw, int(full_reverify), C.byref(bn), C.byref(bl),
                         log.ctypes.data_as(C.POINTER(C.c_int32)))
    if acc < 0:
        raise RuntimeError(f"orc_plan failed ({acc})")
    return acc, bn.value, bl.value, log


def extend_replicas(scene: OracleScene, tree: OracleTree, seeds, it0: int, n_iter: int,
                    threads: int, full_reverify: bool = False) -> int:
    """len(seeds) independent continuations of ``tree`` (iterations [it0, it0 + n_iter), replica r
    with seeds[r]) on ``threads`` host threads (the multi-core CPU baseline).  Returns the nodes
    accepted over all replicas; ``tree`` is not modified."""
    seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
    r = lib().orc_extend_replicas(C.byref(scene._c), C.byref(tree._c),
                                  seeds.ctypes.data_as(C.POINTER(C.c_uint64)), len(seeds), it0,
                                  n_iter, int(full_reverify), int(threads))
    if r < 0:
        raise RuntimeError("orc_extend_replicas failed")
    return r


def queries(scene: OracleScene, starts, seeds, max_iter: int, threads: int,
            full_reverify: bool = False) -> int:
    """Independent queries (start starts[q], stream seeds[q], max_iter iterations each) on
    ``threads`` host threads.  Returns the nodes accepted over all queries."""
    starts = np.ascontiguousarray(starts, dtype=np.float64).reshape(-1, 3)
    seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
    r = lib().orc_queries(C.byref(scene._c), _dp(starts), seeds.ctypes.data_as(C.POINTER(C.c_uint64)),
                          len(seeds), max_iter, int(full_reverify), int(threads))
    if r < 0:
        raise RuntimeError("orc_queries failed")
    return r


# ------------------------------------------------------ RRT* (config 5, build-defined)
class OracleStarTree(OracleTree):
    """OracleTree plus the RRT* node costs and edge costs (root cost 0)."""

    def __init__(self, start, cap):
        super().__init__(start, cap)
        self.cost = np.zeros(cap)
        self.elen = np.zeros(cap)

    def star_arrays(self):
        n = self.n
        return self.arrays() + (self.cost[:n].copy(), self.elen[:n].copy())


def star_k(k_fixed: int, n: int) -> int:
    return lib().orc_star_k(int(k_fixed), int(n))


def star_extend(scene: OracleScene, tree: OracleStarTree, seed: int, it0: int, n_iter: int,
                k_fixed: int = 0, eta: float = 0.0):
    """RRT* iterations [it0, it0 + n_iter) (orc_star_extend).  Returns (accepted, rewires,
    log_nn, log_acc)."""
    log_nn = np.zeros(n_iter, dtype=np.int32)
    log_acc = np.zeros(n_iter, dtype=np.int8)
    rw = C.c_int64(0)
    acc = lib().orc_star_extend(C.byref(scene._c), C.byref(tree._c), _dp(tree.cost),
                                _dp(tree.elen), seed, it0, n_iter, int(k_fixed), float(eta),
                                C.byref(rw),
                                log_nn.ctypes.data_as(C.POINTER(C.c_int32)),
                                log_acc.ctypes.data_as(C.POINTER(C.c_int8)))
    if acc < 0:
        raise RuntimeError("orc_star_extend failed (capacity?)")
    return acc, rw.value, log_nn, log_acc


def star_queries(scene: OracleScene, starts, seeds, max_iter: int, k_fixed: int, eta: float,
                 threads: int):
    """Independent RRT* queries on ``threads`` host threads.  Returns (accepted, rewires)."""
    starts = np.ascontiguousarray(starts, dtype=np.float64).reshape(-1, 3)
    seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
    rw = C.c_int64(0)
    r = lib().orc_star_queries(C.byref(scene._c), _dp(starts),
                               seeds.ctypes.data_as(C.POINTER(C.c_uint64)), len(seeds), max_iter,
                               int(k_fixed), float(eta), int(threads), C.byref(rw))
    if r < 0:
        raise RuntimeError("orc_star_queries failed")
    return r, rw.value
