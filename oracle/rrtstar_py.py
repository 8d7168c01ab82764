"""TEST INFRASTRUCTURE ONLY — pure-Python restatement of the build's RRT* (BASELINE config 5).

The reference has no RRT* (SURVEY.md §8d config 5, §8f row 4), so there is nothing to be in
parity with: this file and ``orc_star_extend`` in ``oracle/pp_oracle.c`` are two independent
restatements of the build-defined spec, checked against each other bit for bit
and through ``tests/golden/rrtstar_*.json``.  Parity against any reference: **unpinned** (none
exists).  The spec reuses the crate's pieces unchanged — ``Space::rand_point``
(rrt.rs:139-146), the exact NN (rrt.rs:378-391, Q9), ``Node::new`` / ``compute_yaw``
(rrt.rs:169-175, 267-271), ``dubins_path_planning`` (dubins.rs:401-428) and the incremental
``verify_node`` (rrt.rs:414-426) — around Karaman & Frazzoli's k-nearest RRT*:

* with ``eta > 0`` a sample farther than eta from its nearest node moves onto the chord at
  distance eta (Steer; eta = 0 keeps the crate's node-at-the-sample, Q5);
* the edge to the nearest node gates the insert (a feasible edge: Dubins steer Some and
  ``verify(edge ++ [parent])``);
* edge cost = the crate's Dubins cost (dubins.rs:351-361); node cost = cost(parent) + edge cost;
* choose parent: the first strict minimum over the nearest node, then the k nearest nodes of the
  new point (by (d2, index));
* rewire: for m in that order (m != parent), the edge m -> new keeps m's pose; when feasible and
  cost(new) + edge cost < cost(m), m's parent becomes new and its subtree's costs are recomputed.
"""
from __future__ import annotations

import math

from dubins_py import dubins_path_planning, gen_range, verify_line

K_MAX = 63
K_RRT = 2.0 * 2.718281828459045  # 2e: k(n) = ceil(2e ln n), the k-nearest RRT* schedule


def star_k(k_fixed, n):
    """neighbours of an insert into an n-node tree (orc_star_k)"""
    if k_fixed > 0:
        k = k_fixed
    else:
        v = math.ceil(K_RRT * math.log(float(n))) if n > 1 else 1.0
        k = 1 if v < 1.0 else (K_MAX if v > K_MAX else int(v))
    k = min(k, K_MAX)
    return min(k, n)


def star_edge(scene, x, y, yaw, px, py, pyaw):
    """(feasible, Dubins cost) of the edge child (x, y, yaw) -> parent pose"""
    r = dubins_path_planning(x, y, yaw, px, py, pyaw, scene["turn_radius"], scene["step_size"])
    if r is None:
        return False, math.inf
    xs, ys = list(r[0]), list(r[1])
    xs.append(px)
    ys.append(py)
    return bool(verify_line(scene, xs, ys)), r[4]


def _knn(tree, x, y, k):
    d = []
    for i, (nx, ny) in enumerate(zip(tree["x"], tree["y"])):
        dx, dy = x - nx, y - ny
        d.append((dx * dx + dy * dy, i))
    d.sort()
    return [i for _, i in d[:k]]


def _propagate(tree, m):
    par, cost, elen = tree["parent"], tree["cost"], tree["elen"]
    front = {m}
    while front:
        nxt = set()
        for i, p in enumerate(par):
            if p in front:
                cost[i] = cost[p] + elen[i]
                nxt.add(i)
        front = nxt


def star_extend(scene, tree, seed, it0, n_iter, k_fixed=0, eta=0.0):
    """RRT* iterations [it0, it0 + n_iter).  ``tree``: dict of lists x, y, yaw, parent, cost,
    elen (root first, root cost 0).  Returns the per-iteration (nearest, accepted) log and the
    rewire count."""
    X, Y, W, P, C, E = (tree[k] for k in ("x", "y", "yaw", "parent", "cost", "elen"))
    log, rewires = [], 0
    for kk in range(n_iter):
        it = it0 + kk
        x = gen_range(seed, 2 * it, scene["minx"], scene["maxx"])
        y = gen_range(seed, 2 * it + 1, scene["miny"], scene["maxy"])
        p, bd = -1, math.inf
        for i, (nx, ny) in enumerate(zip(X, Y)):
            dx, dy = x - nx, y - ny
            d2 = dx * dx + dy * dy
            if d2 < bd:
                p, bd = i, d2
        if eta > 0.0 and bd > eta * eta:  # Steer(x_nearest, x_rand)
            f = eta / math.sqrt(bd)
            x = X[p] + (x - X[p]) * f
            y = Y[p] + (y - Y[p]) * f
        yb = math.atan2(Y[p] - y, X[p] - x)
        ok, eb = star_edge(scene, x, y, yb, X[p], Y[p], W[p])
        if not ok:
            log.append((p, 0))
            continue
        near = _knn(tree, x, y, star_k(k_fixed, len(X)))
        best, cb = p, C[p] + eb
        for q in near:
            if q == p:
                continue
            yq = math.atan2(Y[q] - y, X[q] - x)
            o, eq = star_edge(scene, x, y, yq, X[q], Y[q], W[q])
            if o:
                c = C[q] + eq
                if c < cb:
                    best, cb, yb, eb = q, c, yq, eq
        nw = len(X)
        X.append(x)
        Y.append(y)
        W.append(yb)
        P.append(best)
        C.append(cb)
        E.append(eb)
        for m in near:
            if m == best or not (cb < C[m]):
                continue
            o, em = star_edge(scene, X[m], Y[m], W[m], x, y, yb)
            if o and cb + em < C[m]:
                P[m] = nw
                E[m] = em
                C[m] = cb + em
                _propagate(tree, m)
                rewires += 1
        log.append((p, 1))
    return log, rewires


def new_tree(start):
    return {"x": [start[0]], "y": [start[1]], "yaw": [start[2]], "parent": [-1], "cost": [0.0],
            "elen": [0.0]}
