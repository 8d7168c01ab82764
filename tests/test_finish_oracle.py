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
