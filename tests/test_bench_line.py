"""bench.py's output line is strict JSON (CPU, no GPU call).  Round 3's line carried
`"best_length": Infinity` (a plan with no finish) and the driver's parser rejected it; the line is
now sanitised and round-tripped through a parser that refuses every non-standard constant."""
import json
import math
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    sys.path.insert(0, ROOT)
    import bench

    return bench


def _refuse(tok):
    raise ValueError(tok)


def test_plan_without_finish_is_strict_json():
    bench = _bench()
    # a run_plan-shaped sub-result of a plan that never finished (p.last_plan = (-1, inf, 0))
    plan = {"value": 893000.0, "unit": "plan_one calls/s (with check_finish)",
            "best_node": -1, "best_length": math.inf, "finishes": 0, "line_points": 0,
            "roofline": {"frac": np.float64(0.0014), "traffic": None},
            "cpu_baseline": {"value": 597.0, "same_answer": np.bool_(True)}}
    line = {"metric": bench.METRIC, "value": 4.5e7, "example_rrt": plan,
            "plan": dict(plan, best_length=-math.inf), "config3": {"plan": {"mean_length": math.nan}},
            "list": [np.float32(1.5), float("nan"), np.int64(7)]}
    s = bench.line_json(line)
    back = json.loads(s, parse_constant=_refuse)
    assert back["example_rrt"]["best_length"] is None
    assert back["plan"]["best_length"] is None
    assert back["config3"]["plan"]["mean_length"] is None
    assert back["example_rrt"]["roofline"]["frac"] == pytest.approx(0.0014)
    assert back["example_rrt"]["cpu_baseline"]["same_answer"] is True
    assert back["list"] == [1.5, None, 7]
    assert "Infinity" not in s and "NaN" not in s


def test_plain_dumps_would_have_failed():
    """The failure mode itself: Python's default json.dumps writes Infinity, which a strict
    parser refuses — line_json must never let that through."""
    s = json.dumps({"best_length": math.inf})
    with pytest.raises(ValueError):
        json.loads(s, parse_constant=_refuse)
