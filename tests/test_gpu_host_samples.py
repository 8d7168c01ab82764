"""The host-owned RNG and tree at the boundary (SURVEY.md §8(b) ``pp_extend_batch``):
``pp_rrt_extend_samples`` (plan_one's extend over caller-drawn samples, rrt.rs:139-146, 406-412,
583-589) and ``pp_rrt_tree_import`` (a host-owned tree, rrt.rs:583-589) against the oracle's
sequential run over the same samples (``orc_rrt_extend_samples``) and against ``pp_rrt_extend``.

Exact: node coordinates, parents, nearest indices, accept flags.  Within 1e-9: yaw (ocml vs
glibc atan2)."""
import numpy as np
import pytest

from test_gpu_parity import ANG_TOL, _assert_same_tree, _planner

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(pkg):
    c = pkg.Context(0)
    yield c
    c.close()


def _stream(pkg, raw, seed, it0, n):
    """Space::rand_point of iterations [it0, it0 + n) on the seeded stream, drawn by the HOST
    through pp_gen_range — what a Rust host keeping its own RNG would pass."""
    from pathplanning_amd import rrt

    x0, x1, y0, y1 = rrt.Space.from_raw(raw).get_bounds()
    L = pkg._ffi.lib()
    sx = np.array([L.pp_gen_range(seed, 2 * (it0 + k), x0, x1) for k in range(n)])
    sy = np.array([L.pp_gen_range(seed, 2 * (it0 + k) + 1, y0, y1) for k in range(n)])
    return sx, sy


def _oracle_samples(oracle_mod, raw, sx, sy, start_tree=None, cap=1 << 17):
    sc = oracle_mod.OracleScene.from_raw(raw)
    tr = oracle_mod.OracleTree(raw["start"], cap)
    if start_tree is not None:
        x, y, yaw, par = start_tree
        n = len(x)
        tr.x[:n], tr.y[:n], tr.yaw[:n], tr.parent[:n] = x, y, yaw, par
        tr._c.n = n
    acc, nn, yaw, ok = oracle_mod.rrt_extend_samples(sc, tr, sx, sy)
    return tr, acc, nn, yaw, ok


def _check_record(rec, nn, yaw, ok):
    g_nn, g_yaw, g_ok = rec
    assert np.array_equal(g_ok, ok.astype(bool)), np.flatnonzero(g_ok != ok.astype(bool))[:10]
    assert np.array_equal(g_nn, nn), np.flatnonzero(g_nn != nn)[:10]
    assert np.max(np.abs(g_yaw - yaw)) <= ANG_TOL


@pytest.mark.parametrize("window", [1, 7, 256, 4096])
def test_stream_samples_equal_extend_and_oracle(pkg, ctx, oracle_mod, window):
    """samples from pp_gen_range's stream reproduce pp_rrt_extend's tree and the oracle's run,
    with the per-iteration nearest node, yaw and verdict of the oracle's sequential spec"""
    from pathplanning_amd import scenes

    raw = scenes.bench6()
    n = 3000
    sx, sy = _stream(pkg, raw, 7, 0, n)
    p = _planner(pkg, raw, 7, window, ctx)
    rec = p.extend_samples(sx, sy)
    assert p.iteration() == n
    got = p.tree()
    tr, acc, nn, yaw, ok = _oracle_samples(oracle_mod, raw, sx, sy)
    _assert_same_tree(got, tr.arrays())
    _check_record(rec, nn, yaw, ok)
    assert int(rec[2].sum()) == acc == len(got[0]) - 1
    # the oracle's seeded run logs the same nearest nodes and verdicts
    otr = oracle_mod.OracleTree(raw["start"], 1 << 17)
    _, onn, oacc = oracle_mod.rrt_extend(oracle_mod.OracleScene.from_raw(raw), otr, 7, 0, n)
    assert np.array_equal(onn, nn) and np.array_equal(oacc, ok)
    q = _planner(pkg, raw, 7, window, ctx)
    assert q.extend(n) == acc
    _assert_same_tree(q.tree(), got)


@pytest.mark.parametrize("window", [64, 4096])
def test_arbitrary_samples_vs_oracle(pkg, ctx, oracle_mod, window):
    """samples that no seeded stream draws: clustered, repeated (a rejected sample drawn again,
    an accepted one landing exactly on its own node), exactly on existing nodes and on the root,
    outside the sampling box, and ragged call sizes"""
    from pathplanning_amd import scenes

    raw = scenes.field512()
    rng = np.random.default_rng(11)
    n = 6000
    sx = rng.uniform(0.0, 512.0, n)
    sy = rng.uniform(0.0, 512.0, n)
    sx[:1500] = 8.0 + rng.normal(0.0, 12.0, 1500)  # a cluster around the start: long windows cut
    sy[:1500] = 8.0 + rng.normal(0.0, 12.0, 1500)
    sx[2000:2100] = sx[1900:2000]  # repeats of earlier samples
    sy[2000:2100] = sy[1900:2000]
    sx[2100], sy[2100] = raw["start"][0], raw["start"][1]  # on the root
    sx[2200:2210] = -5.0  # outside the sampling box (verify rejects them)
    sx[2300:2310] = 600.0
    sx = sx.astype(np.float64)
    sy = sy.astype(np.float64)
    tr, acc, nn, yaw, ok = _oracle_samples(oracle_mod, raw, sx, sy)
    # samples exactly on accepted nodes (child on parent: the literal path's trim case)
    ox, oy, _, _ = tr.arrays()
    sx2 = np.concatenate([ox[1:200], rng.uniform(0.0, 512.0, 500)])
    sy2 = np.concatenate([oy[1:200], rng.uniform(0.0, 512.0, 500)])
    tr2, acc2, nn2, yaw2, ok2 = _oracle_samples(oracle_mod, raw, np.concatenate([sx, sx2]),
                                                 np.concatenate([sy, sy2]))
    p = _planner(pkg, raw, 0, window, ctx)
    recs = []
    for a, b in ((0, 1), (1, 1000), (1000, 1001), (1001, n)):  # ragged calls
        recs.append(p.extend_samples(sx[a:b], sy[a:b]))
    rec = tuple(np.concatenate([r[i] for r in recs]) for i in range(3))
    _assert_same_tree(p.tree(), tr.arrays())
    _check_record(rec, nn, yaw, ok)
    rec2 = p.extend_samples(sx2, sy2)
    _assert_same_tree(p.tree(), tr2.arrays())
    _check_record(rec2, nn2[n:], yaw2[n:], ok2[n:])
    assert p.iteration() == n + len(sx2)
    assert 0 < acc < n and int(ok2[n:].sum()) > 0


def test_record_off_keeps_the_pretest(pkg, ctx, oracle_mod):
    """without the per-sample record the obstacle pre-test settles blocked samples (no nearest
    node): the tree is the same"""
    from pathplanning_amd import scenes

    raw = scenes.field512()
    sx, sy = _stream(pkg, raw, 3, 0, 5000)
    p = _planner(pkg, raw, 3, 4096, ctx)
    p.reset_stats()
    acc = p.extend_samples(sx, sy, record=False)
    assert p.stats()["samples_blocked"] > 0
    q = _planner(pkg, raw, 3, 4096, ctx)
    q.reset_stats()
    rec = q.extend_samples(sx, sy)
    assert q.stats()["samples_blocked"] == 0
    assert acc == int(rec[2].sum())
    _assert_same_tree(p.tree(), q.tree())
    tr, _, _, _, _ = _oracle_samples(oracle_mod, raw, sx, sy)
    _assert_same_tree(p.tree(), tr.arrays())


@pytest.mark.parametrize("scene", ["transit", "field512_grid"])
def test_other_scene_modes(pkg, ctx, oracle_mod, scene):
    from pathplanning_amd import scenes

    raw = scenes.transit() if scene == "transit" else scenes.field512_grid()
    sx, sy = _stream(pkg, raw, 5, 0, 3000)
    p = _planner(pkg, raw, 5, 512, ctx)
    rec = p.extend_samples(sx, sy)
    tr, acc, nn, yaw, ok = _oracle_samples(oracle_mod, raw, sx, sy)
    _assert_same_tree(p.tree(), tr.arrays())
    _check_record(rec, nn, yaw, ok)
    assert acc > 0


def test_root_blocked_polygon(pkg, ctx, oracle_mod):
    """a root inside an obstacle: nothing is inserted, every sample still gets its nearest node
    (the root) and yaw"""
    from pathplanning_amd import scenes

    raw = dict(scenes.transit())
    c = raw["obstacle_polygons"][2].mean(axis=0)
    raw["start"] = (float(c[0]), float(c[1]), 0.3)
    sx, sy = _stream(pkg, raw, 1, 0, 500)
    p = _planner(pkg, raw, 1, 4096, ctx)
    nn_g, yaw_g, ok_g = p.extend_samples(sx, sy)
    _, acc, nn, yaw, ok = _oracle_samples(oracle_mod, raw, sx, sy)
    assert acc == 0 and not ok_g.any() and p.tree_size() == 1 and p.iteration() == 500
    assert np.array_equal(nn_g, nn) and np.max(np.abs(yaw_g - yaw)) <= ANG_TOL


@pytest.mark.parametrize("window", [7, 4096])
def test_import_then_extend_equals_extend(pkg, ctx, oracle_mod, window):
    """export -> import into a fresh planner -> extend equals one planner extending throughout,
    both over host samples and over the device's own stream"""
    from pathplanning_amd import scenes

    raw = scenes.field512()
    n1, n2 = 20000, 8000
    a = _planner(pkg, raw, 9, window, ctx)
    a.extend(n1)
    tree1 = a.tree()
    a.extend(n2)
    # host samples continue the stream at iteration n1
    sx, sy = _stream(pkg, raw, 9, n1, n2)
    b = _planner(pkg, raw, 9, window)
    b.tree_import(*tree1)
    assert b.tree_size() == len(tree1[0]) and b.iteration() == 0
    _assert_same_tree(b.tree(), tree1)
    rec = b.extend_samples(sx, sy)
    _assert_same_tree(b.tree(), a.tree())
    tr, acc, nn, yaw, ok = _oracle_samples(oracle_mod, raw, sx, sy, start_tree=tree1)
    _check_record(rec, nn, yaw, ok)
    # the device stream after an import continues from the planner's own counter (0 here)
    c = _planner(pkg, raw, 9, window)
    c.tree_import(*tree1)
    c.extend(3000)
    sc = oracle_mod.OracleScene.from_raw(raw)
    otr = oracle_mod.OracleTree(raw["start"], 1 << 17)
    x, y, yaw1, par = tree1
    k = len(x)
    otr.x[:k], otr.y[:k], otr.yaw[:k], otr.parent[:k] = x, y, yaw1, par
    otr._c.n = k
    oracle_mod.rrt_extend(sc, otr, 9, 0, 3000)
    _assert_same_tree(c.tree(), otr.arrays())
    b.close()
    c.close()


def test_chunked_call_equals_extend(pkg, ctx):
    """more samples than one device chunk (2^20): the chunks continue one sequential run"""
    from pathplanning_amd import scenes

    from pathplanning_amd import rrt

    raw = scenes.bench6()
    n = (1 << 20) + 4321
    x0, x1, y0, y1 = rrt.Space.from_raw(raw).get_bounds()
    L = pkg._ffi.lib()
    sx = np.fromiter((L.pp_gen_range(4, 2 * k, x0, x1) for k in range(n)), np.float64, n)
    sy = np.fromiter((L.pp_gen_range(4, 2 * k + 1, y0, y1) for k in range(n)), np.float64, n)
    p = _planner(pkg, raw, 4, 4096, ctx, capacity=1 << 20)
    nn, yaw, ok = p.extend_samples(sx, sy)
    q = _planner(pkg, raw, 4, 4096, ctx, capacity=1 << 20)
    acc = q.extend(n)
    assert acc == int(ok.sum())
    _assert_same_tree(p.tree(), q.tree())
    # the record of an accepted sample names its parent; the inserted nodes are the ok samples
    x, y, yaw_t, par = p.tree()
    idx = np.flatnonzero(ok)
    assert np.array_equal(x[1:], sx[idx]) and np.array_equal(y[1:], sy[idx])
    assert np.array_equal(par[1:], nn[idx]) and np.array_equal(yaw_t[1:], yaw[idx])


def test_bad_arguments(pkg, ctx):
    from pathplanning_amd import scenes

    raw = scenes.bench6()
    p = _planner(pkg, raw, 1, 64, ctx)
    with pytest.raises(pkg.PPError) as e:
        p.extend_samples(np.array([0.0, np.nan]), np.array([0.0, 1.0]))
    assert e.value.code == pkg._ffi.PP_ERR_INVALID_ARGUMENT
    assert p.iteration() == 0
    x, y, yaw, par = (np.array([0.0, 1.0]), np.array([0.0, 1.0]), np.zeros(2),
                      np.array([-1, 1], dtype=np.int32))  # a node its own parent
    with pytest.raises(pkg.PPError) as e:
        p.tree_import(x, y, yaw, par)
    assert e.value.code == pkg._ffi.PP_ERR_INVALID_ARGUMENT
    with pytest.raises(pkg.PPError):
        p.tree_import(x, y, yaw, np.array([0, 0], dtype=np.int32))  # no root
    assert p.tree_size() == 1
    # empty calls are no-ops
    assert p.extend_samples(np.zeros(0), np.zeros(0), record=False) == 0
    assert p.iteration() == 0
