"""``pathplanning::rrt`` (src/rrt.rs) with the extend hot path on the GPU.

Same names and argument meaning as the crate: ``Robot``, ``create_circle``, ``Space``, ``Node``,
``RRT`` with ``get_nearest_node``, ``get_random_node``, ``verify_node``, ``plan_one`` and the
batched ``extend``.  Build-defined differences: obstacles are analytic discs
and the bounds an axis-aligned rectangle (Q10), sampling is a seeded stream (Q7), iterations run
with the sequential semantics of one rayon thread (Q8), the nearest neighbour is exact (Q9).
Polygon scenes (the example's JSON format) use exact Minkowski buffers in place of geo-offset
(Q10p).  ``plan()`` runs the goal connection (``check_finish``, ``optimize``, ``finalize``).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _ffi, scenes


class Robot:  # rrt.rs:16-40
    def __init__(self, width: float, height: float, max_steer: float):
        self.width = float(width)
        self.height = float(height)
        self.max_steer = float(max_steer)  # used as the Dubins turn radius (rrt.rs:37-39 → 424)

    def get_width(self) -> float:
        return self.width

    def get_steer(self) -> float:
        return self.max_steer


@dataclass(frozen=True)
class Circle:
    """Analytic stand-in for ``create_circle``'s polygon (rrt.rs:43-60)."""
    cx: float
    cy: float
    r: float


def create_circle(center, radius: float) -> Circle:  # rrt.rs:43
    return Circle(float(center[0]), float(center[1]), float(radius))


def _rect_of(bounds):
    """(x0, y0, x1, y1) when ``bounds`` is a 4-tuple or an axis-aligned rectangle ring, else None."""
    b = np.asarray(bounds, dtype=np.float64)
    if b.shape == (4,):
        return tuple(b)
    b = scenes.ring(b)
    if len(b) != 4:
        return None
    xs, ys = b[:, 0], b[:, 1]
    x0, x1, y0, y1 = xs.min(), xs.max(), ys.min(), ys.max()
    if not np.all(((xs == x0) | (xs == x1)) & ((ys == y0) | (ys == y1))):
        return None
    return (x0, y0, x1, y1)


class Space:  # rrt.rs:70-159
    """``Space::new(bounds, robot, obstacles)``.

    Disc mode (configs 1-4): ``bounds`` an axis-aligned rectangle (4-tuple or ring) and every
    obstacle a ``Circle`` — analytic discs (Q10).  Polygon mode (§8f row 3, Q10p): any obstacle
    given as a polygon ring ((M, 2) array-like) or non-rectangular bounds; ``Circle`` obstacles
    then become the crate's ``create_circle`` polygons.  ``grid`` (config 4, build-defined): an
    occupancy grid ``(bits uint32[h, ceil(w/32)], w, x0, y0, cell)`` that replaces the discs —
    every point of a line must lie in a free cell (pp_space_set_grid)."""

    def __init__(self, bounds, robot: Robot, obstacle_list, grid=None):
        self.robot = robot
        self.grid = grid
        obs = list(obstacle_list)
        rect = _rect_of(bounds)
        self.polygon_mode = rect is None or any(not isinstance(o, Circle) for o in obs)
        half = robot.get_width() / 2.0  # rrt.rs:82
        if self.polygon_mode:
            if grid is not None:
                raise ValueError("an occupancy grid replaces disc obstacles, not polygons")
            b = np.asarray(bounds, dtype=np.float64)
            if b.shape == (4,):
                x0, y0, x1, y1 = b
                b = [(x0, y0), (x1, y0), (x1, y1), (x0, y1)]
            self.bounds_polygon = scenes.ring(b)
            self.obstacle_polygons = [
                scenes.create_circle_polygon((o.cx, o.cy), o.r) if isinstance(o, Circle)
                else scenes.ring(o) for o in obs]
            bp = self.bounds_polygon
            self.raw_bounds = (bp[:, 0].min(), bp[:, 1].min(), bp[:, 0].max(), bp[:, 1].max())
            self.circles = np.zeros((0, 3))
        else:
            self.raw_bounds = rect
            self.circles = np.array([[o.cx, o.cy, o.r] for o in obs],
                                    dtype=np.float64).reshape(-1, 3)
        x0, y0, x1, y1 = self.raw_bounds
        self.minx, self.miny, self.maxx, self.maxy = x0 + half, y0 + half, x1 - half, y1 - half
        self._ctx = None

    @classmethod
    def from_raw(cls, raw: dict) -> "Space":
        if "bounds_polygon" in raw:
            return cls(raw["bounds_polygon"], Robot(*raw["robot"]), raw["obstacle_polygons"])
        return cls(raw["bounds"], Robot(*raw["robot"]),
                   [create_circle((c[0], c[1]), c[2]) for c in raw["circles"]],
                   grid=raw.get("grid"))

    def get_steer(self) -> float:
        return self.robot.get_steer()

    def get_bounds(self):
        """bbox of the shrunken bounds (minx, maxx, miny, maxy) — what rand_point samples."""
        return (self.minx, self.maxx, self.miny, self.maxy)

    def get_obs(self):
        """Disc mode: the inflated discs (cx, cy, r + width/2) (rrt.rs:108-111, 152-154).
        Polygon mode: the obstacle rings before buffering (the buffer is analytic, Q10p)."""
        if self.polygon_mode:
            return [p.copy() for p in self.obstacle_polygons]
        half = self.robot.get_width() / 2.0
        c = self.circles.copy()
        c[:, 2] += half
        return c

    def verify_batch(self, lines, ctx: _ffi.Context | None = None):
        """``Space::verify`` (rrt.rs:124-137) of many polylines (each (n, 2)) on the GPU: bool
        array.  Uses ``ctx`` (the scene is uploaded into it) or a context of its own."""
        if ctx is None:
            if self._ctx is None:
                self._ctx = _ffi.Context(0)
                self._upload(self._ctx)
            ctx = self._ctx
        else:
            self._upload(ctx)
        pts = [np.asarray(l, dtype=np.float64).reshape(-1, 2) for l in lines]
        off = np.zeros(len(pts) + 1, dtype=np.int64)
        off[1:] = np.cumsum([len(p) for p in pts])
        allp = np.concatenate(pts) if pts and off[-1] > 0 else np.zeros((1, 2))
        x = np.ascontiguousarray(allp[:, 0])
        y = np.ascontiguousarray(allp[:, 1])
        ok = np.zeros(len(pts), dtype=np.uint8)
        dp = C.POINTER(C.c_double)
        _ffi.check(_ffi.lib().pp_space_verify_batch(
            ctx.handle, x.ctypes.data_as(dp), y.ctypes.data_as(dp),
            off.ctypes.data_as(C.POINTER(C.c_int64)), len(pts),
            ok.ctypes.data_as(C.POINTER(C.c_uint8))))
        return ok.astype(bool)

    def verify(self, line, ctx: _ffi.Context | None = None) -> bool:
        """``Space::verify(&LineString) -> bool`` (rrt.rs:124-137)."""
        return bool(self.verify_batch([line], ctx)[0])

    def _upload(self, ctx: _ffi.Context):
        dp = C.POINTER(C.c_double)
        if self.polygon_mode:
            b = np.ascontiguousarray(self.bounds_polygon.reshape(-1))
            rings = self.obstacle_polygons
            off = np.zeros(len(rings) + 1, dtype=np.int32)
            off[1:] = np.cumsum([len(r) for r in rings])
            o = np.ascontiguousarray(np.concatenate(rings).reshape(-1)) if rings else np.zeros(2)
            _ffi.check(_ffi.lib().pp_space_new_polygons(
                ctx.handle, b.ctypes.data_as(dp), len(self.bounds_polygon), o.ctypes.data_as(dp),
                off.ctypes.data_as(C.POINTER(C.c_int32)), len(rings), self.robot.width,
                self.robot.height, self.robot.max_steer))
            return
        c = np.ascontiguousarray(self.circles)
        cx, cy, r = (np.ascontiguousarray(c[:, k]) for k in range(3))
        x0, y0, x1, y1 = self.raw_bounds
        _ffi.check(_ffi.lib().pp_space_new(
            ctx.handle, x0, y0, x1, y1, self.robot.width, self.robot.height,
            self.robot.max_steer, cx.ctypes.data_as(dp), cy.ctypes.data_as(dp),
            r.ctypes.data_as(dp), len(cx)))
        if self.grid is not None:
            bits, w, gx0, gy0, cell = self.grid
            bits = np.ascontiguousarray(bits, dtype=np.uint32)
            _ffi.check(_ffi.lib().pp_space_set_grid(
                ctx.handle, bits.ctypes.data_as(C.POINTER(C.c_uint32)), int(w), bits.shape[0],
                float(gx0), float(gy0), float(cell)))


@dataclass
class Node:  # rrt.rs:161-214 (a view of one tree row)
    index: int
    x: float
    y: float
    yaw: float
    parent: int  # -1 for the root

    def get_point(self):
        return (self.x, self.y)

    def get_yaw(self):
        return self.yaw


class RRT:  # rrt.rs:325-620
    """``RRT::new(start, start_yaw, goal, goal_yaw, max_iter, step_size, space)`` (rrt.rs:335).

    Extra keyword arguments: ``seed`` (sampling stream), ``device`` (GPU ordinal), ``window``
    (candidates evaluated per speculative GPU batch; results do not depend on it), ``capacity``
    (initial node capacity, grown on demand)."""

    def __init__(self, start, start_yaw, goal, goal_yaw, max_iter, step_size, space: Space,
                 seed: int = 0, device: int = 0, window: int = 4096, capacity: int = 1 << 16,
                 ctx: _ffi.Context | None = None):
        self.ctx = ctx or _ffi.Context(device)
        self.space = space
        self.goal = (float(goal[0]), float(goal[1]))
        self.goal_yaw = float(goal_yaw)
        self.max_iter = int(max_iter)
        self.step_size = float(step_size)
        self.seed = int(seed)
        space._upload(self.ctx)
        _ffi.check(_ffi.lib().pp_rrt_set_window(self.ctx.handle, int(window)))
        _ffi.check(_ffi.lib().pp_rrt_new(
            self.ctx.handle, float(start[0]), float(start[1]), float(start_yaw), self.goal[0],
            self.goal[1], self.goal_yaw, self.max_iter, self.step_size, self.seed, int(capacity)))

    # ---------------------------------------------------------------- hot path
    def extend(self, n_iter: int) -> int:
        """``n_iter`` × plan_one's extend (rrt.rs:583-589); returns the nodes inserted."""
        acc = C.c_int64(0)
        _ffi.check(_ffi.lib().pp_rrt_extend(self.ctx.handle, int(n_iter), C.byref(acc)))
        return acc.value

    def extend_samples(self, sx, sy, record: bool = True):
        """plan_one's extend (rrt.rs:583-589) over caller-drawn samples: iteration it + i takes
        (sx[i], sy[i]) as its rand_point (rrt.rs:139-146) — the host owns the RNG.  Returns the
        nodes inserted, or with ``record`` (nearest int32[k], yaw f64[k], ok bool[k]): per sample
        the nearest node of the tree as it stood (Node::new's parent), its yaw and whether it was
        inserted.  ``record=False`` lets the obstacle pre-test settle samples without their
        nearest node (faster)."""
        sx = np.ascontiguousarray(sx, dtype=np.float64)
        sy = np.ascontiguousarray(sy, dtype=np.float64)
        k = len(sx)
        if len(sy) != k:
            raise ValueError("sx and sy differ in length")
        acc = C.c_int64(0)
        dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
        if not record:
            _ffi.check(_ffi.lib().pp_rrt_extend_samples(
                self.ctx.handle, sx.ctypes.data_as(dp), sy.ctypes.data_as(dp), k, None, None, None,
                C.byref(acc)))
            return acc.value
        nearest = np.zeros(k, dtype=np.int32)
        yaw = np.zeros(k)
        ok = np.zeros(k, dtype=np.uint8)
        _ffi.check(_ffi.lib().pp_rrt_extend_samples(
            self.ctx.handle, sx.ctypes.data_as(dp), sy.ctypes.data_as(dp), k,
            nearest.ctypes.data_as(ip), yaw.ctypes.data_as(dp),
            ok.ctypes.data_as(C.POINTER(C.c_uint8)), C.byref(acc)))
        return nearest, yaw, ok.astype(bool)

    def tree_import(self, x, y, yaw, parent):
        """Replace the tree by host-owned nodes (root first, parent -1 for the root, otherwise an
        earlier node); the iteration counter, scene and goal stay."""
        x, y, yaw = (np.ascontiguousarray(a, dtype=np.float64) for a in (x, y, yaw))
        parent = np.ascontiguousarray(parent, dtype=np.int32)
        if not (len(x) == len(y) == len(yaw) == len(parent)):
            raise ValueError("tree arrays differ in length")
        dp = C.POINTER(C.c_double)
        _ffi.check(_ffi.lib().pp_rrt_tree_import(
            self.ctx.handle, x.ctypes.data_as(dp), y.ctypes.data_as(dp), yaw.ctypes.data_as(dp),
            parent.ctypes.data_as(C.POINTER(C.c_int32)), len(x)))

    def plan_one(self) -> bool:
        """plan_one's extend (rrt.rs:583-589): True when the node was inserted."""
        acc = C.c_int32(0)
        _ffi.check(_ffi.lib().pp_rrt_plan_one(self.ctx.handle, C.byref(acc)))
        return bool(acc.value)

    def set_window(self, k: int):
        _ffi.check(_ffi.lib().pp_rrt_set_window(self.ctx.handle, int(k)))

    # ---------------------------------------------------------------- queries
    def tree_size(self) -> int:
        n = C.c_int64(0)
        _ffi.check(_ffi.lib().pp_rrt_tree_size(self.ctx.handle, C.byref(n)))
        return n.value

    def iteration(self) -> int:
        it = C.c_int64(0)
        _ffi.check(_ffi.lib().pp_rrt_iteration(self.ctx.handle, C.byref(it)))
        return it.value

    def tree(self):
        """(x, y, yaw, parent) arrays, root first."""
        n = self.tree_size()
        x, y, yaw = np.zeros(n), np.zeros(n), np.zeros(n)
        par = np.zeros(n, dtype=np.int32)
        out = C.c_int64(0)
        dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
        _ffi.check(_ffi.lib().pp_rrt_tree_export(
            self.ctx.handle, x.ctypes.data_as(dp), y.ctypes.data_as(dp), yaw.ctypes.data_as(dp),
            par.ctypes.data_as(ip), n, C.byref(out)))
        return x, y, yaw, par

    def node(self, i: int) -> Node:
        x, y, yaw, par = self.tree()
        return Node(i, x[i], y[i], yaw[i], int(par[i]))

    def get_nearest_node_batch(self, qx, qy):
        """RRT::get_nearest_node (rrt.rs:378-391) for many points: (index, d2) arrays."""
        qx = np.ascontiguousarray(qx, dtype=np.float64)
        qy = np.ascontiguousarray(qy, dtype=np.float64)
        k = len(qx)
        idx = np.zeros(k, dtype=np.int32)
        d2 = np.zeros(k)
        dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
        _ffi.check(_ffi.lib().pp_rrt_get_nearest_node_batch(
            self.ctx.handle, qx.ctypes.data_as(dp), qy.ctypes.data_as(dp), k,
            idx.ctypes.data_as(ip), d2.ctypes.data_as(dp)))
        return idx, d2

    def get_nearest_node(self, point) -> int:
        idx, _ = self.get_nearest_node_batch([point[0]], [point[1]])
        return int(idx[0])

    def get_random_node(self, it: int | None = None):
        """rrt.rs:406-412: (x, y, nearest index, yaw) of iteration ``it``'s sample (default: the
        next iteration) — does not advance the planner."""
        it = self.iteration() if it is None else int(it)
        x0, x1, y0, y1 = self.space.get_bounds()
        x = _ffi.lib().pp_gen_range(self.seed, 2 * it, x0, x1)
        y = _ffi.lib().pp_gen_range(self.seed, 2 * it + 1, y0, y1)
        p = self.get_nearest_node((x, y))
        tx, ty, _, _ = self.tree()
        return x, y, p, float(np.arctan2(ty[p] - y, tx[p] - x))

    def verify_node_batch(self, x, y, parent):
        """verify_node(Node::new(point, tree[parent])) (rrt.rs:169-175, 414-426): (ok, yaw)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.ascontiguousarray(y, dtype=np.float64)
        parent = np.ascontiguousarray(parent, dtype=np.int32)
        k = len(x)
        ok = np.zeros(k, dtype=np.uint8)
        yaw = np.zeros(k)
        dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
        _ffi.check(_ffi.lib().pp_rrt_verify_node_batch(
            self.ctx.handle, x.ctypes.data_as(dp), y.ctypes.data_as(dp),
            parent.ctypes.data_as(ip), k, ok.ctypes.data_as(C.POINTER(C.c_uint8)),
            yaw.ctypes.data_as(dp)))
        return ok.astype(bool), yaw

    def verify_node(self, x, y, parent) -> bool:
        ok, _ = self.verify_node_batch([x], [y], [parent])
        return bool(ok[0])

    def line_to_origin(self, node: int):
        """line_to_origin (rrt.rs:291-321) of tree node ``node``: the (n, 2) polyline node -> root
        (each edge steered on the GPU with R = Robot.max_steer and the planner's step)."""
        n = C.c_int64(0)
        _ffi.check(_ffi.lib().pp_rrt_line_to_origin(self.ctx.handle, int(node), None, None, 0,
                                                    C.byref(n)))
        x, y = np.zeros(max(n.value, 1)), np.zeros(max(n.value, 1))
        dp = C.POINTER(C.c_double)
        _ffi.check(_ffi.lib().pp_rrt_line_to_origin(self.ctx.handle, int(node),
                                                    x.ctypes.data_as(dp), y.ctypes.data_as(dp),
                                                    n.value, C.byref(n)))
        return np.stack([x[:n.value], y[:n.value]], axis=1)

    # ---------------------------------------------------------------- goal connection
    def optimize(self, node: int, i: int = 0):
        """RRT::optimize(node, i) (rrt.rs:463-487): None, or the list of tree nodes the returned
        chain of copies connects to, level by level (the last one is the tree node it ends at)."""
        chain = np.zeros(16, dtype=np.int32)
        n = C.c_int(0)
        _ffi.check(_ffi.lib().pp_rrt_optimize(self.ctx.handle, int(node), int(i),
                                              chain.ctypes.data_as(C.POINTER(C.c_int32)),
                                              C.byref(n)))
        return None if n.value == 0 else chain[:n.value].tolist()

    def finalize(self, goal, goal_yaw: float, parent: int):
        """RRT::finalize (rrt.rs:489-540) of the goal node Node::new_goal(goal, parent, goal_yaw):
        ((n, 2) line, verified) — the line whether or not it verifies."""
        n = C.c_int64(0)
        ok = C.c_uint8(0)
        gx, gy = goal
        L = _ffi.lib()
        _ffi.check(L.pp_rrt_finalize(self.ctx.handle, float(gx), float(gy), float(goal_yaw),
                                     int(parent), None, None, 0, C.byref(n), C.byref(ok)))
        x, y = np.zeros(max(n.value, 1)), np.zeros(max(n.value, 1))
        dp = C.POINTER(C.c_double)
        _ffi.check(L.pp_rrt_finalize(self.ctx.handle, float(gx), float(gy), float(goal_yaw),
                                     int(parent), x.ctypes.data_as(dp), y.ctypes.data_as(dp),
                                     n.value, C.byref(n), C.byref(ok)))
        return np.stack([x[:n.value], y[:n.value]], axis=1), bool(ok.value)

    def check_finish_batch(self, nodes, with_length: bool = True):
        """RRT::check_finish (rrt.rs:428-438) for many tree nodes: dict of arrays ``ok``,
        ``length`` / ``n_points`` (verified lines only) and ``chain`` (rows of
        [levels, edges, optimize's chosen ancestor per level...])."""
        nodes = np.ascontiguousarray(nodes, dtype=np.int32)
        k = len(nodes)
        ok = np.zeros(k, dtype=np.uint8)
        length = np.zeros(k)
        npts = np.zeros(k, dtype=np.int32)
        chain = np.zeros((k, _ffi.PP_CF_CHAIN), dtype=np.int32)
        dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
        _ffi.check(_ffi.lib().pp_rrt_check_finish_batch(
            self.ctx.handle, nodes.ctypes.data_as(ip), k, ok.ctypes.data_as(C.POINTER(C.c_uint8)),
            length.ctypes.data_as(dp) if with_length else None,
            npts.ctypes.data_as(ip) if with_length else None, chain.ctypes.data_as(ip)))
        return {"ok": ok.astype(bool), "length": length, "n_points": npts, "chain": chain}

    def check_finish(self, node: int):
        """RRT::check_finish for one tree node: the finalized line as an (n, 2) array (root side
        first, rrt.rs:538), or None when it does not verify."""
        ok = C.c_uint8(0)
        n, ln = C.c_int64(0), C.c_double(0)
        _ffi.check(_ffi.lib().pp_rrt_check_finish(self.ctx.handle, int(node), C.byref(ok), None,
                                                  None, 0, C.byref(n), C.byref(ln)))
        if not ok.value:
            return None
        cap = n.value
        x, y = np.zeros(max(cap, 1)), np.zeros(max(cap, 1))
        dp = C.POINTER(C.c_double)
        _ffi.check(_ffi.lib().pp_rrt_check_finish(
            self.ctx.handle, int(node), C.byref(ok), x.ctypes.data_as(dp), y.ctypes.data_as(dp),
            cap, C.byref(n), C.byref(ln)))
        return np.stack([x[:n.value], y[:n.value]], axis=1)

    def plan(self, n_iter: int | None = None):
        """RRT::plan (rrt.rs:599-619), sequential spec: ``n_iter`` (default max_iter) plan_one
        iterations, check_finish on every accepted node; the line with the minimum
        euclidean_length (first on ties) or None.  ``self.last_plan`` keeps (node, length,
        finishes)."""
        bn, bl, nf = C.c_int32(-1), C.c_double(0), C.c_int64(0)
        n_iter = self.max_iter if n_iter is None else int(n_iter)
        _ffi.check(_ffi.lib().pp_rrt_plan(self.ctx.handle, n_iter, C.byref(bn), C.byref(bl),
                                          C.byref(nf)))
        self.last_plan = (bn.value, bl.value, nf.value)
        if bn.value < 0:
            return None
        return self.check_finish(bn.value)

    # ---------------------------------------------------------------- instrumentation
    def stats(self) -> dict:
        s = _ffi.StatsC()
        _ffi.check(_ffi.lib().pp_rrt_get_stats(self.ctx.handle, C.byref(s), C.sizeof(s)))
        return s.as_dict()

    def reset_stats(self):
        _ffi.check(_ffi.lib().pp_rrt_reset_stats(self.ctx.handle))

    def set_profiling(self, on: bool):
        _ffi.check(_ffi.lib().pp_set_profiling(self.ctx.handle, int(bool(on))))

    def synchronize(self):
        _ffi.check(_ffi.lib().pp_synchronize(self.ctx.handle))

    def close(self):
        self.ctx.close()


class RRTBatch:
    """Many independent planners on one scene (BASELINE config 3): ``RRT::new`` per query
    (rrt.rs:335-355) with its own start, goal and sampling stream, advanced in lockstep — one
    plan_one extend iteration (rrt.rs:583-589) of every query per step — on one GPU.  ``window``:
    iterations per query evaluated speculatively per GPU step (a power of two <= 64, 0 =
    automatic: 32, halved while a step would hold more than 262144 tasks); every query's tree
    equals its sequential run."""

    def __init__(self, starts, goals, max_iter, step_size, space: Space, seeds, device: int = 0,
                 ctx: _ffi.Context | None = None, window: int = 0):
        self.ctx = ctx or _ffi.Context(device)
        self.space = space
        starts = np.ascontiguousarray(starts, dtype=np.float64).reshape(-1, 3)
        goals = np.ascontiguousarray(goals, dtype=np.float64).reshape(-1, 3)
        seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
        self.q = len(starts)
        self.max_iter = int(max_iter)
        space._upload(self.ctx)
        # iterations per query evaluated per GPU step (0: automatic); results do not depend on it
        _ffi.check(_ffi.lib().pp_batch_set_window(self.ctx.handle, int(window)))
        dp = C.POINTER(C.c_double)
        _ffi.check(_ffi.lib().pp_batch_new(
            self.ctx.handle, self.q, starts.ctypes.data_as(dp), goals.ctypes.data_as(dp),
            seeds.ctypes.data_as(C.POINTER(C.c_uint64)), self.max_iter, float(step_size)))

    def extend(self, n_steps: int):
        """n_steps lockstep steps; returns (iterations consumed, nodes inserted) over the batch."""
        it, acc = C.c_int64(0), C.c_int64(0)
        _ffi.check(_ffi.lib().pp_batch_extend(self.ctx.handle, int(n_steps), C.byref(it),
                                              C.byref(acc)))
        return it.value, acc.value

    def set_finish_schedule(self, rounds: bool = True, span0: int = 0, span: int = 0):
        """How plan() runs check_finish (identical results): steer rounds with span0 / span
        candidate edges per node in the first / later rounds (0 = default), or rounds=False:
        check_finish_kernel alone."""
        _ffi.check(_ffi.lib().pp_batch_set_finish_schedule(self.ctx.handle, int(bool(rounds)),
                                                           int(span0), int(span)))

    def set_window(self, k: int):
        """The window for the following extend calls (a power of two <= 64); the trees do not
        depend on it."""
        _ffi.check(_ffi.lib().pp_batch_set_window(self.ctx.handle, int(k)))

    def state(self, with_evals: bool = False):
        """(tree sizes int32[q], iterations int64[q]) [+ NN node-distance evals int64[q]]."""
        n = np.zeros(self.q, dtype=np.int32)
        it = np.zeros(self.q, dtype=np.int64)
        ev = np.zeros(self.q, dtype=np.int64)
        i64 = C.POINTER(C.c_int64)
        _ffi.check(_ffi.lib().pp_batch_state(self.ctx.handle,
                                             n.ctypes.data_as(C.POINTER(C.c_int32)),
                                             it.ctypes.data_as(i64), ev.ctypes.data_as(i64)))
        return (n, it, ev) if with_evals else (n, it)

    def stats(self) -> dict:
        s = _ffi.StatsC()
        _ffi.check(_ffi.lib().pp_rrt_get_stats(self.ctx.handle, C.byref(s), C.sizeof(s)))
        return s.as_dict()

    def set_profiling(self, on: bool):
        _ffi.check(_ffi.lib().pp_set_profiling(self.ctx.handle, int(bool(on))))

    def plan(self):
        """RRT::plan (rrt.rs:599-619) of every query on its tree as extended so far: check_finish
        of every node the query inserted, the first minimum euclidean_length.  dict of per-query
        arrays ``best_node`` (-1: None), ``length`` (inf: None), ``n_points`` (of the finalized
        line), ``n_finishes``; ``checked`` = the (query, node) pairs checked."""
        bn = np.zeros(self.q, dtype=np.int32)
        ln = np.zeros(self.q)
        npts = np.zeros(self.q, dtype=np.int32)
        nf = np.zeros(self.q, dtype=np.int32)
        chk = C.c_int64(0)
        ip = C.POINTER(C.c_int32)
        _ffi.check(_ffi.lib().pp_batch_plan(
            self.ctx.handle, bn.ctypes.data_as(ip), ln.ctypes.data_as(C.POINTER(C.c_double)),
            npts.ctypes.data_as(ip), nf.ctypes.data_as(ip), C.byref(chk)))
        return {"best_node": bn, "length": ln, "n_points": npts, "n_finishes": nf,
                "checked": chk.value}

    def tree(self, query: int, n: int | None = None):
        """(x, y, yaw, parent) of one query's tree, root first (``n``: its size, when known)."""
        n = int(self.state()[0][query]) if n is None else int(n)
        x, y, yaw = np.zeros(n), np.zeros(n), np.zeros(n)
        par = np.zeros(n, dtype=np.int32)
        out = C.c_int64(0)
        dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
        _ffi.check(_ffi.lib().pp_batch_tree_export(
            self.ctx.handle, int(query), x.ctypes.data_as(dp), y.ctypes.data_as(dp),
            yaw.ctypes.data_as(dp), par.ctypes.data_as(ip), n, C.byref(out)))
        return x, y, yaw, par

    def close(self):
        self.ctx.close()


class RRTStarBatch:
    """Independent k-nearest RRT* planners on one scene (BASELINE config 5), one RRT* iteration
    of every query per lockstep step on one GPU.  Build-defined — the reference has no RRT*
    (SURVEY.md §8f row 4): the crate's rand_point / exact NN / Node::new / verify_node / Dubins
    steer (rrt.rs:139-175, 378-426; dubins.rs:401-428) around Karaman & Frazzoli's choose-parent
    and rewire, edge cost = the crate's Dubins cost (dubins.rs:351-361).  ``k``: neighbours per
    insert (0 = ceil(2e ln n), at most 63); ``eta``: Steer distance (0 = the node sits at the
    sample, like the crate).  DESIGN.md §3.7; oracle: oracle/pp_oracle.c orc_star_extend."""

    def __init__(self, starts, max_iter, step_size, space: Space, seeds, k: int = 0,
                 eta: float = 0.0, device: int = 0, ctx: _ffi.Context | None = None):
        self.ctx = ctx or _ffi.Context(device)
        self.space = space
        starts = np.ascontiguousarray(starts, dtype=np.float64).reshape(-1, 3)
        seeds = np.ascontiguousarray(seeds, dtype=np.uint64)
        self.q = len(starts)
        self.max_iter = int(max_iter)
        space._upload(self.ctx)
        _ffi.check(_ffi.lib().pp_star_new(
            self.ctx.handle, self.q, starts.ctypes.data_as(C.POINTER(C.c_double)),
            seeds.ctypes.data_as(C.POINTER(C.c_uint64)), self.max_iter, float(step_size), int(k),
            float(eta)))

    def extend(self, n_steps: int):
        """n_steps lockstep steps; returns (iterations, nodes inserted, rewires) over the batch."""
        it, acc, rw = C.c_int64(0), C.c_int64(0), C.c_int64(0)
        _ffi.check(_ffi.lib().pp_star_extend(self.ctx.handle, int(n_steps), C.byref(it),
                                             C.byref(acc), C.byref(rw)))
        return it.value, acc.value, rw.value

    def state(self):
        """(tree sizes int32[q], iterations, NN node-distance evals, rewires: int64[q] each)"""
        n = np.zeros(self.q, dtype=np.int32)
        it, ev, rw = (np.zeros(self.q, dtype=np.int64) for _ in range(3))
        i64 = C.POINTER(C.c_int64)
        _ffi.check(_ffi.lib().pp_star_state(self.ctx.handle, n.ctypes.data_as(C.POINTER(C.c_int32)),
                                            it.ctypes.data_as(i64), ev.ctypes.data_as(i64),
                                            rw.ctypes.data_as(i64)))
        return n, it, ev, rw

    def set_profiling(self, on: bool):
        _ffi.check(_ffi.lib().pp_set_profiling(self.ctx.handle, int(bool(on))))

    def stats(self) -> dict:
        s = _ffi.StatsC()
        _ffi.check(_ffi.lib().pp_rrt_get_stats(self.ctx.handle, C.byref(s), C.sizeof(s)))
        return s.as_dict()

    def tree(self, query: int, n: int | None = None):
        """(x, y, yaw, parent, cost) of one query's tree, root first (``n``: its size, when
        known)."""
        n = int(self.state()[0][query]) if n is None else int(n)
        x, y, yaw, cost = np.zeros(n), np.zeros(n), np.zeros(n), np.zeros(n)
        par = np.zeros(n, dtype=np.int32)
        out = C.c_int64(0)
        dp, ip = C.POINTER(C.c_double), C.POINTER(C.c_int32)
        _ffi.check(_ffi.lib().pp_star_tree_export(
            self.ctx.handle, int(query), x.ctypes.data_as(dp), y.ctypes.data_as(dp),
            yaw.ctypes.data_as(dp), par.ctypes.data_as(ip), cost.ctypes.data_as(dp), n,
            C.byref(out)))
        return x, y, yaw, par, cost

    def close(self):
        self.ctx.close()
