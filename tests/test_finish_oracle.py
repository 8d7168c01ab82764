"""check_finish / optimize / finalize / plan (rrt.rs:428-619): the C
oracle against the golden fixtures made by the pure-Python restatement (full line_to_origin
verifies), plus the incremental-verify equivalence the HIP path relies on.  CPU only."""
import numpy as np
import pytest

from conftest import load_golden


def _scene_tree(oracle_mod, rec):
    from pathplanning_amd import scenes

    raw = scenes.bench6_open(rec["start"][2])
    sc = oracle_mod.OracleScene.from_raw(raw)
    tr = oracle_mod.OracleTree(raw["start"], 1 << 14)
    oracle_mod.rrt_extend(sc, tr, rec["seed"], 0, rec["n_iter"])
    return raw, sc, tr


@pytest.mark.parametrize("k", [0, 1])
def test_check_finish_golden(oracle_mod, k):
    rec = load_golden("finish_bench6_open.json")[k]
    raw, sc, tr = _scene_tree(oracle_mod, rec)
    assert tr.n == rec["n_nodes"]
    n_ok = 0
    for f in rec["finish"]:
        r = oracle_mod.check_finish(sc, tr, f["node"], raw["goal"][:2], raw["goal"][2])
        assert r["ok"] == f["ok"], f["node"]
        assert r["chain"] == f["chain"], f["node"]
        if f["ok"]:
            n_ok += 1
            assert r["n"] == f["n"] and r["length"] == f["length"], f["node"]
    assert n_ok > 20  # the scene exercises successful goal connections


@pytest.mark.parametrize("k", [0, 1])
def test_plan_golden(oracle_mod, k):
    rec = load_golden("finish_bench6_open.json")[k]
    from pathplanning_amd import scenes

    raw = scenes.bench6_open(rec["start"][2])
    sc = oracle_mod.OracleScene.from_raw(raw)
    tr = oracle_mod.OracleTree(raw["start"], 1 << 14)
    acc, bn, bl, log = oracle_mod.plan(sc, tr, rec["seed"], 0, rec["n_iter"], raw["goal"][:2],
                                       raw["goal"][2])
    assert acc == rec["n_nodes"] - 1
    assert bn == rec["best_node"] and bl == rec["best_length"]
    assert int((log == 1).sum()) == sum(f["ok"] for f in rec["finish"])
    r = oracle_mod.check_finish(sc, tr, bn, raw["goal"][:2], raw["goal"][2])
    assert np.array_equal(r["x"], rec["best_x"]) and np.array_equal(r["y"], rec["best_y"])
    assert oracle_mod.line_length(r["x"], r["y"]) == bl


def test_check_finish_incremental_equals_full(oracle_mod):
    """optimize's verify(line_to_origin(new)) ≡ verify(edge ++ [to])."""
    rec = load_golden("finish_bench6_open.json")[1]
    raw, sc, tr = _scene_tree(oracle_mod, rec)
    for node in range(1, tr.n, 2):
        a = oracle_mod.check_finish(sc, tr, node, raw["goal"][:2], raw["goal"][2])
        b = oracle_mod.check_finish(sc, tr, node, raw["goal"][:2], raw["goal"][2],
                                    full_reverify=True)
        assert (a["ok"], a["chain"], a["n"], a["length"]) == (b["ok"], b["chain"], b["n"],
                                                              b["length"])


def test_bench6_start_never_finishes(oracle_mod):
    """At bench6's own start the root-copy loop leaves the bounds."""
    from pathplanning_amd import scenes

    raw = scenes.bench6()
    sc = oracle_mod.OracleScene.from_raw(raw)
    tr = oracle_mod.OracleTree(raw["start"], 1 << 14)
    acc, bn, bl, log = oracle_mod.plan(sc, tr, 0, 0, 400, raw["goal"][:2], raw["goal"][2])
    assert acc > 50 and bn == -1 and not (log == 1).any()
    r = oracle_mod.check_finish(sc, tr, 1, raw["goal"][:2], raw["goal"][2])
    assert r["chain"][-1] == 0 and len(r["chain"]) == 16  # ... → root copies to the limit


def test_none_steers_nan_start_yaw(oracle_mod):
    """A None Dubins steer needs a non-finite pose (LSL's and RSR's p² differ only in the sign of
    one term, so one of them is >= 0 for finite inputs).  A NaN start yaw makes every edge into
    the root None: insertion takes it as the straight polyline [(x, y), root] (rrt.rs:313,
    line_to_origin), and finalize panics on it (rrt.rs:529).  Both restatements agree: the same
    tree, and check_finish of every node is the panic."""
    import dubins_py as dpy
    from pathplanning_amd import scenes

    raw = scenes.bench6_open(float("nan"))
    sc = oracle_mod.OracleScene.from_raw(raw)
    tr = oracle_mod.OracleTree(raw["start"], 1 << 12)
    oracle_mod.rrt_extend(sc, tr, 7, 0, 300)
    x, y, yaw, par = tr.arrays()
    ptree = {"x": [raw["start"][0]], "y": [raw["start"][1]], "yaw": [float("nan")], "parent": [-1]}
    dpy.rrt_extend(sc.as_dict(), ptree, 7, 0, 300)
    assert len(x) == len(ptree["x"]) > 50
    assert np.array_equal(x, ptree["x"]) and np.array_equal(y, ptree["y"])
    assert np.array_equal(par, ptree["parent"])
    assert int((par == 0).sum()) > 1  # several None edges into the root were inserted
    nodes = dpy.tree_nodes(ptree)
    for v in range(1, len(x), 7):
        with pytest.raises(RuntimeError):
            oracle_mod.check_finish(sc, tr, v, raw["goal"][:2], raw["goal"][2])
        with pytest.raises(RuntimeError):
            dpy.check_finish(sc.as_dict(), nodes[v], raw["goal"][:2], raw["goal"][2])
