"""GPU parity, polygon mode: the example's JSON scene
(examples/rrt/transit.debug.json) and bench6 with its create_circle polygons, through the C ABI,
against the oracle and the golden fixtures.  Same tolerances as test_gpu_parity.py: node
coordinates, parents, accept flags and verdicts exact; yaw / line points within 1e-9."""
import math

import numpy as np
import pytest

from conftest import load_golden
from test_gpu_parity import ANG_TOL, PT_TOL, _assert_same_tree, _oracle_tree, _planner
from test_polygons_oracle import random_lines

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(pkg):
    c = pkg.Context(0)
    yield c
    c.close()


def _raw(name):
    from pathplanning_amd import scenes

    return {"transit": scenes.transit, "bench6_polygons": scenes.bench6_polygons,
            "bench6_polygons_open": scenes.bench6_polygons_open}[name]()


@pytest.mark.parametrize("idx", range(3))
@pytest.mark.parametrize("window", [64, 4096])
def test_polygon_golden_trees(pkg, ctx, idx, window):
    rec = load_golden("rrt_polygons.json")[idx]
    p = _planner(pkg, _raw(rec["scene"]), rec["seed"], window, ctx)
    p.extend(rec["n_iter"])
    _assert_same_tree(p.tree(), (np.array(rec["x"]), np.array(rec["y"]), np.array(rec["yaw"]),
                                 np.array(rec["parent"], dtype=np.int32)))


@pytest.mark.parametrize("window", [7, 4096])
def test_transit_full_run_any_window(pkg, ctx, oracle_mod, window):
    """the example's whole max_iter = 8000 run (examples/rrt/src/main.rs:58-66), any K"""
    raw = _raw("transit")
    n_iter = 8000 if window >= 256 else 2000
    exp, acc, _, _ = _oracle_tree(oracle_mod, raw, 3, n_iter)
    p = _planner(pkg, raw, 3, window, ctx)
    assert p.extend(n_iter) == acc
    _assert_same_tree(p.tree(), exp)


def test_polygon_check_finish_and_plan_golden(pkg, ctx):
    rec = load_golden("finish_polygons.json")[0]
    raw = _raw("bench6_polygons_open")
    p = _planner(pkg, raw, rec["seed"], 64, ctx)
    p.extend(rec["n_iter"])
    assert p.tree_size() == rec["n_nodes"]
    r = p.check_finish_batch(np.arange(1, rec["n_nodes"], dtype=np.int32))
    fin = rec["finish"]
    assert [bool(v) for v in r["ok"]] == [f["ok"] for f in fin]
    for i, f in enumerate(fin):
        levels = int(r["chain"][i, 0])
        assert r["chain"][i, 2:2 + levels].tolist() == f["chain"], f["node"]
        if f["ok"]:
            assert r["n_points"][i] == f["n"]
            assert abs(r["length"][i] - f["length"]) <= 1e-9 * f["length"]
    q = _planner(pkg, raw, rec["seed"], 4096, ctx)
    line = q.plan(rec["n_iter"])
    assert q.last_plan[0] == rec["best_node"]
    assert abs(q.last_plan[1] - rec["best_length"]) <= 1e-9 * rec["best_length"]
    assert np.max(np.abs(line[:, 0] - rec["best_x"])) <= PT_TOL
    assert np.max(np.abs(line[:, 1] - rec["best_y"])) <= PT_TOL


def test_transit_check_finish_vs_oracle(pkg, ctx, oracle_mod):
    """every node's check_finish verdict on the example scene (none finishes at this seed)"""
    raw = _raw("transit")
    p = _planner(pkg, raw, 42, 4096, ctx)
    p.extend(1500)
    sc = oracle_mod.OracleScene.from_raw(raw)
    (x, y, yaw, par), _, _, _ = _oracle_tree(oracle_mod, raw, 42, 1500)
    tr = oracle_mod.OracleTree(raw["start"], len(x) + 1)
    oracle_mod.rrt_extend(sc, tr, 42, 0, 1500)
    nodes = np.arange(1, p.tree_size(), 5, dtype=np.int32)
    r = p.check_finish_batch(nodes)
    exp = [oracle_mod.check_finish(sc, tr, int(n), raw["goal"][:2], raw["goal"][2])["ok"]
           for n in nodes]
    assert [bool(v) for v in r["ok"]] == exp


@pytest.mark.parametrize("scene", ["transit", "bench6_polygons", "field512", "field512_grid"])
def test_space_verify_batch_vs_oracle(pkg, ctx, oracle_mod, scene):
    """Space::verify (rrt.rs:124-137) of arbitrary polylines, every scene mode"""
    from pathplanning_amd import rrt, scenes

    raw = {"field512": scenes.field512, "field512_grid": scenes.field512_grid}.get(
        scene, lambda: _raw(scene))()
    sc = oracle_mod.OracleScene.from_raw(raw)
    lines = random_lines(sc, 3000, 5)
    lines.append(np.zeros((0, 2)))  # the empty line verifies
    long = np.stack([np.linspace(sc.minx, sc.maxx, 300), np.full(300, 0.5 * (sc.miny + sc.maxy))], 1)
    lines.append(long)  # > 4 chunks of 63 points
    got = rrt.Space.from_raw(raw).verify_batch(lines, ctx)
    exp = [sc.verify_line(l[:, 0], l[:, 1]) for l in lines]
    assert got.tolist() == exp
    assert 0 < sum(exp) < len(exp)


def test_polygon_verify_node_batch_vs_oracle(pkg, ctx, oracle_mod):
    raw = _raw("transit")
    p = _planner(pkg, raw, 42, 4096, ctx)
    p.extend(3000)
    x, y, yaw, par = p.tree()
    sc = oracle_mod.OracleScene.from_raw(raw)
    tr = oracle_mod.OracleTree(raw["start"], len(x) + 1)
    oracle_mod.rrt_extend(sc, tr, 42, 0, 3000)
    rng = np.random.default_rng(3)
    k = 2000
    qx = rng.uniform(sc.minx, sc.maxx, k)
    qy = rng.uniform(sc.miny, sc.maxy, k)
    parent = rng.integers(0, len(x), k).astype(np.int32)
    ok, qyaw = p.verify_node_batch(qx, qy, parent)
    for i in range(k):
        e, eyaw = oracle_mod.verify_candidate(sc, tr, qx[i], qy[i], int(parent[i]))
        assert bool(ok[i]) == e, i
        assert abs(qyaw[i] - eyaw) <= ANG_TOL


@pytest.mark.parametrize("scene", ["transit", "field512_polygons"])
def test_polygon_straight_segment_shortcut_vs_oracle(pkg, ctx, oracle_mod, scene):
    """The walk's analytic S segments in polygon mode (s_classify_poly: a sure hit rejects at
    once, a sure clearance keeps the segment's first and last point) must not change a verdict:
    candidates whose child -> parent line is tangent to an obstacle vertex's buffer disc (radius
    h + eps, eps from -1e-2 to 1e-2 and exactly 0), plus far parents (long S segments), against
    the oracle's full verify.  verify_node_batch runs the planners' walk (walk_rec)."""
    from pathplanning_amd import scenes

    raw = scenes.field512_polygons() if scene == "field512_polygons" else _raw(scene)
    p = _planner(pkg, raw, 8, 4096, ctx)
    p.extend(3000)
    x, y, yaw, par = p.tree()
    sc = oracle_mod.OracleScene.from_raw(raw)
    otr = oracle_mod.OracleTree(raw["start"], len(x) + 1)
    otr.x[:len(x)], otr.y[:len(x)], otr.yaw[:len(x)], otr.parent[:len(x)] = x, y, yaw, par
    otr._c.n = len(x)
    verts = np.concatenate([np.asarray(o, dtype=np.float64) for o in raw["obstacle_polygons"]])
    half = raw["robot"][0] / 2.0
    span = max(sc.maxx - sc.minx, sc.maxy - sc.miny)
    rng = np.random.default_rng(11)
    cx, cy, cp = [], [], []
    epss = [0.0, 1e-12, -1e-12, 1e-9, -1e-9, 1e-6, -1e-6, 1e-4, -1e-4, 1e-2, -1e-2]
    while len(cx) < 4000:
        i = int(rng.integers(0, len(x)))
        vx, vy = verts[int(rng.integers(0, len(verts)))]
        dist = math.hypot(vx - x[i], vy - y[i])
        rho = half + epss[len(cx) % len(epss)]
        if not (rho < dist < 0.25 * span):
            continue
        a = math.asin(rho / dist) * (1 if rng.random() < 0.5 else -1)
        b = math.atan2(vy - y[i], vx - x[i]) + a
        ln = dist * math.cos(a) + rng.uniform(0.01, 0.06) * span
        qx, qy = x[i] + ln * math.cos(b), y[i] + ln * math.sin(b)
        if sc.minx < qx < sc.maxx and sc.miny < qy < sc.maxy:
            cx.append(qx)
            cy.append(qy)
            cp.append(i)
    far = rng.integers(0, len(x), 2000)  # far parents: long S segments across the scene
    cx += list(rng.uniform(sc.minx, sc.maxx, 2000))
    cy += list(rng.uniform(sc.miny, sc.maxy, 2000))
    cp += list(far)
    cx, cy, cp = np.array(cx), np.array(cy), np.array(cp, dtype=np.int32)
    ok, _ = p.verify_node_batch(cx, cy, cp)
    bad = [i for i in range(len(cx))
           if bool(ok[i]) != oracle_mod.verify_candidate(sc, otr, cx[i], cy[i], int(cp[i]))[0]]
    assert not bad, (len(bad), bad[:10])
    assert 0 < int(np.sum(ok)) < len(ok)


def test_polygon_root_blocked(pkg, ctx, oracle_mod):
    """a start inside an obstacle polygon, away from its edges: every line_to_origin contains
    it, so nothing is ever inserted — window path, verify_node, check_finish and the batch"""
    from pathplanning_amd import rrt

    raw = dict(_raw("transit"))
    big = raw["obstacle_polygons"][2]
    c = big.mean(axis=0)
    raw["start"] = (float(c[0]), float(c[1]), 0.3)
    _, acc, _, _ = _oracle_tree(oracle_mod, raw, 1, 3000)
    assert acc == 0
    p = _planner(pkg, raw, 1, 4096, ctx)
    assert p.extend(3000) == 0 and p.tree_size() == 1 and p.iteration() == 3000
    ok, _ = p.verify_node_batch([raw["start"][0] + 0.05], [raw["start"][1]], [0])
    assert not ok[0]
    sc = oracle_mod.OracleScene.from_raw(raw)
    tr = oracle_mod.OracleTree(raw["start"], 2)
    r = p.check_finish_batch(np.array([0], dtype=np.int32))
    e = oracle_mod.check_finish(sc, tr, 0, raw["goal"][:2], raw["goal"][2])
    assert bool(r["ok"][0]) == e["ok"]
    # the batch: blocked and free queries side by side
    free = _raw("transit")["start"]
    starts = np.array([raw["start"], free, raw["start"], free], dtype=np.float64)
    seeds = np.array([5, 6, 7, 8], dtype=np.uint64)
    b = rrt.RRTBatch(starts, starts, 300, raw["step_size"], rrt.Space.from_raw(raw), seeds,
                     ctx=ctx)
    b.extend(300)
    n, its = b.state()
    assert (its == 300).all() and n[0] == 1 and n[2] == 1
    for q in (1, 3):
        exp_tr = oracle_mod.OracleTree(tuple(starts[q]), 400)
        oracle_mod.rrt_extend(sc, exp_tr, int(seeds[q]), 0, 300)
        _assert_same_tree(b.tree(q), exp_tr.arrays())


def test_polygon_batch_matches_independent_oracle_runs(pkg, ctx, oracle_mod):
    from pathplanning_amd import rrt

    raw = _raw("transit")
    sc = oracle_mod.OracleScene.from_raw(raw)
    rng = np.random.default_rng(9)
    starts = []
    while len(starts) < 21:
        x, y = rng.uniform(sc.minx, sc.maxx), rng.uniform(sc.miny, sc.maxy)
        if sc.verify_line([x], [y]):
            starts.append((x, y, rng.uniform(-math.pi, math.pi)))
    starts = np.array(starts)
    seeds = np.arange(100, 121, dtype=np.uint64)
    b = rrt.RRTBatch(starts, starts, 500, raw["step_size"], rrt.Space.from_raw(raw), seeds,
                     ctx=ctx)
    b.extend(500)
    for q in range(21):
        tr = oracle_mod.OracleTree(tuple(starts[q]), 600)
        oracle_mod.rrt_extend(sc, tr, int(seeds[q]), 0, 500)
        _assert_same_tree(b.tree(q), tr.arrays())


def test_field512_polygons_parity(pkg, ctx, oracle_mod):
    """bench.py --workload polygons at a testable size: config 2's field as ~32k create_circle
    polygon edges (the scene too big for the LDS image: the walk's global-memory path), K = 4096,
    15k iterations against the sequential oracle."""
    from pathplanning_amd import scenes

    raw = scenes.field512_polygons()
    exp, acc, _, _ = _oracle_tree(oracle_mod, raw, 42, 15000)
    assert acc > 1000
    p = _planner(pkg, raw, 42, 4096, ctx)
    assert p.extend(15000) == acc
    _assert_same_tree(p.tree(), exp)
