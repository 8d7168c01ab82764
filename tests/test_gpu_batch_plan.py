"""GPU: RRT::plan of every query of a batch (pp_batch_plan; SURVEY.md §8e's per-query record
(ok, n_nodes, path_len, cost, iterations)) against the oracle's sequential plan of each query
(oracle/pp_oracle.c orc_plan: extend + check_finish on every accepted node, the first minimum
euclidean_length; rrt.rs:428-438, 591, 599-619).

Exact: the best node (per query) and the finish count.  The length within 1e-9 relative (geo
euclidean_length: a sum of hypot over points that ocml and glibc round differently in the last
bits) — except for the libm trim flips of DESIGN.md §2: optimize's same-position edges (a copy of
a node connecting to the node itself, rrt.rs:473-474: a Dubins loop back to its start) end on a
rounding residue whose exact 0.0 decides whether dubins.rs:281-288 pops one more point, and ocml
and glibc disagree on it in a few percent of configurations.  Such a query's line then differs
by exactly one point on an arc (|delta n| = 1, |delta length| = one chord 2R sin(step / 2)); the
test counts them (printed and, with PP_FLIP_REPORT_PLAN=<path>, written as JSON: profiles/) and
pins them near the committed measurement (FLIPS_MAX)."""
import json
import math
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPORT = {}
# one-point trim flips measured per case (profiles/r04_libm_flips_plan.json); the bound allows
# twice the measured count (at least 1): a regression that doubles the rate fails
FLIPS_MEASURED = {"bench6_open": 1, "field512": 0, "field512_128": 0}


def _bound(case):
    m = FLIPS_MEASURED[case]
    return None if m is None else max(1, 2 * m)


@pytest.fixture(scope="module")
def ctx(pkg):
    c = pkg.Context(0)
    yield c
    c.close()
    path = os.environ.get("PP_FLIP_REPORT_PLAN")
    if path and REPORT:
        with open(path, "w") as f:
            json.dump(REPORT, f, indent=1, sort_keys=True)


def _run(ctx, oracle_mod, raw, q0, nq, max_iter):
    from pathplanning_amd import rrt, scenes

    starts, goals, seeds = scenes.config3_queries(raw, q0, nq)
    b = rrt.RRTBatch(starts, goals, max_iter, raw["step_size"], rrt.Space.from_raw(raw), seeds,
                     ctx=ctx)
    b.extend(max_iter)
    got = b.plan()
    n = b.state()[0]
    sc = oracle_mod.OracleScene.from_raw(raw)
    exp = []
    for q in range(nq):
        tr = oracle_mod.OracleTree(tuple(starts[q]), max_iter + 1)
        acc, bn, bl, log = oracle_mod.plan(sc, tr, int(seeds[q]), 0, max_iter, goals[q][:2],
                                           goals[q][2])
        assert acc + 1 == n[q]
        npts = 0
        if bn >= 0:
            npts = oracle_mod.check_finish(sc, tr, bn, goals[q][:2], goals[q][2])["n"]
        exp.append((bn, bl, int((log == 1).sum()), npts))
    return got, exp, int(n.sum() - nq)


def _check(got, exp, checked, raw, case):
    assert got["checked"] == checked
    chord = 2.0 * raw["robot"][2] * math.sin(raw["step_size"] / 2.0)
    flips = 0
    finishing = 0
    for q, (bn, bl, nf, npts) in enumerate(exp):
        assert got["best_node"][q] == bn, q
        assert got["n_finishes"][q] == nf, q
        if bn < 0:
            assert math.isinf(got["length"][q]) and got["n_points"][q] == 0
            continue
        finishing += 1
        if abs(got["length"][q] - bl) <= 1e-9 * bl and got["n_points"][q] == npts:
            continue
        # a libm trim flip: one arc point more or less on a same-position edge
        flips += 1
        assert abs(int(got["n_points"][q]) - npts) == 1, q
        assert abs(abs(got["length"][q] - bl) - chord) <= 1e-6 * chord, q
    REPORT[case] = {"queries": len(exp), "queries_with_path": finishing, "one_point_flips": flips}
    print(f"plan {case}: {finishing} queries with a path, {flips} one-point libm trim flips")
    bound = _bound(case)
    assert flips <= (bound if bound is not None else max(1, finishing // 10))


def test_batch_plan_bench6_open(pkg, ctx, oracle_mod):
    """64 queries on the bench scene from the goal-connection start region (many finishes)"""
    from pathplanning_amd import scenes

    raw = scenes.bench6_open()
    got, exp, checked = _run(ctx, oracle_mod, raw, 0, 64, 300)
    assert sum(1 for e in exp if e[0] >= 0) >= 16  # the comparison covers real finishes
    _check(got, exp, checked, raw, "bench6_open")


def test_batch_plan_field512(pkg, ctx, oracle_mod):
    """config 3's own field and query recipe (the first 24 queries of the batch, 2000 iterations)"""
    from pathplanning_amd import scenes

    raw = scenes.field512()
    got, exp, checked = _run(ctx, oracle_mod, raw, 0, 24, 2000)
    _check(got, exp, checked, raw, "field512")


def test_batch_plan_before_extend_and_reuse(pkg, ctx, oracle_mod):
    """a fresh batch has only roots: nothing to check, every query None; planning twice gives the
    same answer"""
    from pathplanning_amd import rrt, scenes

    raw = scenes.bench6_open()
    starts, goals, seeds = scenes.config3_queries(raw, 0, 5)
    b = rrt.RRTBatch(starts, goals, 100, raw["step_size"], rrt.Space.from_raw(raw), seeds,
                     ctx=ctx)
    got = b.plan()
    assert got["checked"] == 0 and np.all(got["best_node"] == -1)
    b.extend(100)
    g1, g2 = b.plan(), b.plan()
    for k in ("best_node", "n_points", "n_finishes"):
        assert np.array_equal(g1[k], g2[k])
    assert np.array_equal(g1["length"], g2["length"])


def test_batch_plan_field512_128(pkg, ctx, oracle_mod):
    """config 3's recipe at 128 queries x 2000 iterations (~10k check_finish items in one launch:
    thousands of waves share optimize's memo) — every query's plan equals its
    sequential oracle plan"""
    from pathplanning_amd import scenes

    raw = scenes.field512()
    got, exp, checked = _run(ctx, oracle_mod, raw, 0, 128, 2000)
    assert checked >= 8192
    _check(got, exp, checked, raw, "field512_128")


def test_batch_plan_long_lines_tier2(pkg, ctx, oracle_mod):
    """lines past the line kernel's tier-1 capacity (6144 points: step 0.003 gives the config-3
    field's finishing lines 15-18k points) are handed to tier 2 (full capacity) and
    still equal the sequential oracle plan"""
    from pathplanning_amd import scenes

    raw = dict(scenes.field512())
    raw["step_size"] = 0.003
    got, exp, checked = _run(ctx, oracle_mod, raw, 0, 24, 2000)
    assert int((got["n_points"] > 6144).sum()) > 0  # tier 2 ran
    FLIPS_MEASURED.setdefault("field512_step0003", None)
    _check(got, exp, checked, raw, "field512_step0003")


def test_batch_plan_rounds_equal_one_kernel(pkg, ctx):
    """pp_batch_plan's steer rounds (phase A / B memo fill, lane-per-item assemble, DESIGN.md
    §3.3) against check_finish_kernel alone (pp_batch_set_finish_schedule rounds=0): the same
    best node, length (bit for bit), point count and finish count for every query of a
    512-query config-3 batch"""
    from pathplanning_amd import rrt, scenes

    raw = scenes.field512()
    starts, goals, seeds = scenes.config3_queries(raw, 0, 512)
    b = rrt.RRTBatch(starts, goals, 2000, raw["step_size"], rrt.Space.from_raw(raw), seeds,
                     ctx=ctx)
    b.extend(2000)
    out = []
    for rounds in (True, False):
        b.set_finish_schedule(rounds)
        out.append(b.plan())
    b.set_finish_schedule(True)
    a, k = out
    assert a["checked"] == k["checked"] > 0
    for key in ("best_node", "n_points", "n_finishes"):
        assert np.array_equal(a[key], k[key]), key
    assert np.array_equal(a["length"], k["length"])
    assert int((a["best_node"] >= 0).sum()) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("span0,span", [("1", "1"), ("4", "4"), ("1", "3")])
def test_batch_plan_span_schedules_agree(pkg, ctx, span0, span):
    """phase A's span schedule (pp_batch_set_finish_schedule span0 / span)
    changes which candidates are walked together, never a result: the same best nodes,
    lengths (bit for bit), point and finish counts as the default schedule on a 256-query
    config-3 batch"""
    from pathplanning_amd import rrt, scenes

    raw = scenes.field512()
    starts, goals, seeds = scenes.config3_queries(raw, 0, 256)
    b = rrt.RRTBatch(starts, goals, 2000, raw["step_size"], rrt.Space.from_raw(raw), seeds,
                     ctx=ctx)
    b.extend(2000)
    out = []
    for sched in ((0, 0), (int(span0), int(span))):
        b.set_finish_schedule(True, *sched)
        out.append(b.plan())
    b.set_finish_schedule(True)
    a, k = out
    assert a["checked"] == k["checked"] > 0
    for key in ("best_node", "n_points", "n_finishes", "length"):
        assert np.array_equal(a[key], k[key]), key


@pytest.mark.parametrize("rounds", [True, False])
def test_batch_plan_none_edges_panic(pkg, ctx, rounds):
    """A query whose start yaw is NaN makes every edge into its root a None steer; finalize panics
    on it (rrt.rs:529).  pp_batch_plan must return PP_ERR_REFERENCE_PANIC with the steer rounds
    (cfb_assemble's panic precedence: fnone of the goal edge, the phase-B memo, tnone_up of the
    tree edges) and with check_finish_kernel alone — for a batch of NaN-yaw queries and for a
    mixed batch in which the other queries' chains are ordinary (verified or rejected) — never a
    plain rejection.  The same batch without the NaN query plans without error."""
    from pathplanning_amd import _ffi, rrt, scenes

    raw = scenes.bench6_open()
    starts, goals, seeds = scenes.config3_queries(raw, 0, 24)
    starts = np.array(starts, dtype=np.float64).reshape(-1, 3)
    for nan_q in ([5], list(range(24))):
        st = starts.copy()
        st[nan_q, 2] = float("nan")
        b = rrt.RRTBatch(st, goals, 300, raw["step_size"], rrt.Space.from_raw(raw), seeds,
                         ctx=ctx)
        b.set_finish_schedule(rounds)
        b.extend(300)
        n, _ = b.state()
        assert int(n[nan_q[0]]) > 2  # the NaN query inserted nodes (straight root edges)
        with pytest.raises(_ffi.PPError) as e:
            b.plan()
        assert e.value.code == _ffi.PP_ERR_REFERENCE_PANIC, nan_q
        b.set_finish_schedule(True)
    b = rrt.RRTBatch(starts, goals, 300, raw["step_size"], rrt.Space.from_raw(raw), seeds,
                     ctx=ctx)
    b.set_finish_schedule(rounds)
    b.extend(300)
    res = b.plan()
    b.set_finish_schedule(True)
    assert res["checked"] > 0 and int((res["best_node"] >= 0).sum()) > 0
