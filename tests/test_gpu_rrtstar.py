"""GPU parity of the RRT* query batch (BASELINE config 5, build-defined — DESIGN.md §3.7): the
HIP path through the C ABI (pp_star_*) against the C oracle (orc_star_extend) and the golden
fixtures of the pure-Python restatement.

Tolerances: node coordinates, parents, accept logs (tree sizes) and rewire counts EXACT; yaw
within 1e-9 absolute and node costs within 1e-9 relative (ocml vs glibc trig inside the Dubins
cost; a cost comparison could only flip on a 1e-15-wide tie, which these cases do not hit)."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

ANG_TOL = 1e-9
COST_RTOL = 1e-9


def _batch(pkg, raw, starts, seeds, max_iter, k, eta, ctx=None):
    from pathplanning_amd import rrt

    return rrt.RRTStarBatch(starts, max_iter, raw["step_size"], rrt.Space.from_raw(raw), seeds,
                            k=k, eta=eta, ctx=ctx)


def _oracle(oracle_mod, raw, start, seed, n_iter, k, eta):
    sc = oracle_mod.OracleScene.from_raw(raw)
    tr = oracle_mod.OracleStarTree(start, n_iter + 1)
    acc, rw, _, _ = oracle_mod.star_extend(sc, tr, seed, 0, n_iter, k, eta)
    return tr.star_arrays(), rw


def _assert_same(got, exp):
    x, y, yaw, par, cost = got
    ex, ey, eyaw, epar, ecost = exp[:5]
    assert len(x) == len(ex), (len(x), len(ex))
    assert np.array_equal(x, ex) and np.array_equal(y, ey)
    assert np.array_equal(par, epar)
    assert np.max(np.abs(yaw - eyaw), initial=0.0) <= ANG_TOL
    assert np.allclose(cost, ecost, rtol=COST_RTOL, atol=0.0)


@pytest.fixture(scope="module")
def ctx(pkg):
    c = pkg.Context(0)
    yield c
    c.close()


def test_star_golden(pkg, ctx):
    from pathplanning_amd import scenes

    for rec in load_golden("rrtstar.json"):
        raw = {"bench6_open": scenes.bench6_open, "bench6": scenes.bench6,
               "field2048_m10240_s1234": scenes.config5_field}[rec["scene"]]()
        b = _batch(pkg, raw, [rec["start"]], [rec["seed"]], rec["n_iter"], rec["k"], rec["eta"],
                   ctx=ctx)
        it, acc, rw = b.extend(rec["n_iter"])
        assert it == rec["n_iter"] and acc == len(rec["x"]) - 1 and rw == rec["rewires"]
        _assert_same(b.tree(0), (np.array(rec["x"]), np.array(rec["y"]), np.array(rec["yaw"]),
                                 np.array(rec["parent"]), np.array(rec["cost"])))


@pytest.mark.parametrize("k,eta", [(0, 0.0), (4, 0.0), (0, 2.0), (63, 1.0)])
def test_star_batch_vs_oracle_bench6(pkg, oracle_mod, ctx, k, eta):
    """several queries with their own streams, ragged step calls"""
    from pathplanning_amd import scenes

    raw = scenes.bench6_open()
    seeds = [0, 5, 11, 12]
    starts = [raw["start"], (-4.0, -4.5, 0.3), (-3.0, -3.0, 0.785), (2.0, -4.0, 1.2)]
    b = _batch(pkg, raw, starts, seeds, 400, k, eta, ctx=ctx)
    for n in (1, 37, 150, 1000):  # capped at max_iter
        b.extend(n)
    n_nodes, it, ev, rw = b.state()
    assert list(it) == [400] * 4
    for q in range(4):
        exp, erw = _oracle(oracle_mod, raw, starts[q], seeds[q], 400, k, eta)
        _assert_same(b.tree(q), exp)
        assert rw[q] == erw


def test_star_config5_field(pkg, oracle_mod, ctx):
    """the config-5 field (10240 discs, global-memory disc grid in the walk), Steer eta = 16"""
    from pathplanning_amd import scenes

    raw = scenes.config5_field()
    starts, _, seeds = scenes.config3_queries(raw, 0, 6)
    b = _batch(pkg, raw, starts, seeds, 300, 0, scenes.CONFIG5_ETA, ctx=ctx)
    b.extend(300)
    n_nodes, _, _, rw = b.state()
    tot_rw = 0
    for q in range(6):
        exp, erw = _oracle(oracle_mod, raw, tuple(starts[q]), int(seeds[q]), 300, 0,
                           scenes.CONFIG5_ETA)
        _assert_same(b.tree(q), exp)
        assert rw[q] == erw
        tot_rw += erw
    assert n_nodes.sum() > 6 * 100


def test_star_field512_rewires(pkg, oracle_mod, ctx):
    """config 2's field with Steer: long runs, many rewires and deep subtree propagations"""
    from pathplanning_amd import scenes

    raw = scenes.field512()
    starts, _, seeds = scenes.config3_queries(raw, 0, 4)
    b = _batch(pkg, raw, starts, seeds, 1500, 0, 12.0, ctx=ctx)
    b.extend(1500)
    _, _, _, rw = b.state()
    assert rw.sum() > 0
    for q in range(4):
        exp, erw = _oracle(oracle_mod, raw, tuple(starts[q]), int(seeds[q]), 1500, 0, 12.0)
        _assert_same(b.tree(q), exp)
        assert rw[q] == erw


def test_star_grid_and_polygons(pkg, oracle_mod, ctx):
    """the other scene modes: the config-4 occupancy grid and create_circle polygons"""
    from pathplanning_amd import scenes

    for raw, eta in ((scenes.field512_grid(), 10.0), (scenes.bench6_polygons_open(), 0.0)):
        starts = [raw["start"]]
        b = _batch(pkg, raw, starts, [3], 300, 0, eta, ctx=ctx)
        b.extend(300)
        exp, erw = _oracle(oracle_mod, raw, tuple(raw["start"]), 3, 300, 0, eta)
        _assert_same(b.tree(0), exp)
        assert b.state()[3][0] == erw


def test_star_errors(pkg, ctx):
    from pathplanning_amd import _ffi, rrt, scenes

    raw = scenes.bench6_open()
    with pytest.raises(_ffi.PPError):
        _batch(pkg, raw, [raw["start"]], [0], 10, 64, 0.0, ctx=ctx)  # k > 63
    with pytest.raises(_ffi.PPError):
        _batch(pkg, raw, [raw["start"]], [0], 10, 0, -1.0, ctx=ctx)  # eta < 0


def test_star_sub_batch_streams(pkg, oracle_mod, ctx):
    """>= 256 queries run as two sub-batches on two streams: every query still equals its own
    oracle run (spot-checked across both halves) and the totals equal the oracle's"""
    from pathplanning_amd import scenes

    raw = scenes.bench6_open()
    starts, _, seeds = scenes.config3_queries(raw, 0, 300)
    b = _batch(pkg, raw, starts, seeds, 80, 0, 0.0, ctx=ctx)
    b.extend(80)
    n, it, _, rw = b.state()
    assert (it == 80).all()
    for q in (0, 1, 149, 150, 151, 298, 299):
        exp, erw = _oracle(oracle_mod, raw, tuple(starts[q]), int(seeds[q]), 80, 0, 0.0)
        _assert_same(b.tree(q), exp)
        assert rw[q] == erw
    acc, rws = oracle_mod.star_queries(oracle_mod.OracleScene.from_raw(raw), starts, seeds, 80, 0,
                                       0.0, 8)
    assert int(n.sum()) - 300 == acc and int(rw.sum()) == rws


def test_star_large_tree_uncached_knn(pkg, oracle_mod, ctx):
    """a tree past the kNN's LDS distance cache (n > 2048 nodes): the exclusion rounds over global
    memory, plus k at its cap region"""
    from pathplanning_amd import scenes

    raw = scenes.bench6_open()
    b = _batch(pkg, raw, [raw["start"]], [21], 4000, 0, 0.0, ctx=ctx)
    b.extend(4000)
    n = int(b.state()[0][0])
    assert n > 2100
    exp, erw = _oracle(oracle_mod, raw, raw["start"], 21, 4000, 0, 0.0)
    _assert_same(b.tree(0), exp)
    assert b.state()[3][0] == erw


def test_star_split_fixed_at_new(pkg, oracle_mod, ctx, monkeypatch):
    """the sub-batch split is fixed at pp_star_new (the library reads no environment): a
    300-query batch runs its sub-batches with their own task counts"""
    from pathplanning_amd import scenes

    raw = scenes.bench6_open()
    starts, _, seeds = scenes.config3_queries(raw, 0, 300)
    b = _batch(pkg, raw, starts, seeds, 60, 0, 0.0, ctx=ctx)
    b.extend(60)
    n, it, _, rw = b.state()
    assert (it == 60).all()
    for q in (0, 149, 150, 299):
        exp, erw = _oracle(oracle_mod, raw, tuple(starts[q]), int(seeds[q]), 60, 0, 0.0)
        _assert_same(b.tree(q), exp)
        assert rw[q] == erw
