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


def test_default_line_fits_the_driver_tail():
    """Rounds 3-4 printed 22-23 KB lines; the driver reads an ~8 KB stdout tail (stderr shares it)
    and parsed none of them.  The compact line built from round 4's full default record must be
    strict JSON of at most LINE_MAX (4 KB) and keep the contract's headline keys and every
    sub-result's value / frac / CPU value."""
    bench = _bench()
    with open(os.path.join(ROOT, "profiles", "r04_final_bench_default.json")) as f:
        full = json.load(f)
    assert len(json.dumps(full)) > 20000  # the failure mode this guards
    s = bench.compact_line(full, os.path.join(ROOT, "gpurun_out", "bench_detail.json"))
    assert len(s.encode()) <= bench.LINE_MAX <= 8192
    back = json.loads(s, parse_constant=_refuse)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert back[k] == full[k] or k == "config", k
    assert back["roofline"]["frac"] == full["roofline"]["frac"]
    assert {"bound", "achieved", "peak", "unit", "traffic"} <= set(back["roofline"])
    assert back["cpu_baseline"]["value"] == full["cpu_baseline"]["value"]
    assert back["cpu_baseline"]["cores"] == full["cpu_baseline"]["cores"]
    assert set(back["sub"]) == set(bench.SUB_KEYS)
    for k, v in back["sub"].items():
        assert v["value"] == full[k]["value"], k
        assert v["cpu"] == full[k]["cpu_baseline"]["value"], k
    assert back["sub"]["config3"]["records_digest"] == full["config3"]["records_digest"]
    assert back["sub"]["plan"]["same_answer"] is True
    assert back["detail"] == "gpurun_out/bench_detail.json"


def test_compact_line_sheds_fields_over_the_cap():
    """A line swollen by long error texts still fits: the least important fields go first."""
    bench = _bench()
    line = {"metric": bench.METRIC, "value": 1.0, "config": {"workload": "w" * 3000}}
    for k in bench.SUB_KEYS:
        line[k] = {"error": "E" * 5000}
    s = bench.compact_line(line)
    assert len(s.encode()) <= bench.LINE_MAX
    json.loads(s, parse_constant=_refuse)


def test_single_workload_line_keeps_the_multirank_keys():
    """test_gpu_multirank compares these keys between the 1-rank and 2-rank config-3 lines."""
    bench = _bench()
    with open(os.path.join(ROOT, "profiles", "r04_final_bench_config3.json")) as f:
        full = json.load(f)
    back = json.loads(bench.compact_line(full, None, with_subs=False), parse_constant=_refuse)
    for k in ("n_gpus", "iterations_total", "nodes_total", "records_digest"):
        assert back[k] == full[k], k
    assert back["config"]["queries_per_rank"] == full["config"]["queries_per_rank"]
    assert back["config"]["gather"] == full["config"]["gather"]
    assert "sub" not in back


def test_plain_dumps_would_have_failed():
    """The failure mode itself: Python's default json.dumps writes Infinity, which a strict
    parser refuses — line_json must never let that through."""
    s = json.dumps({"best_length": math.inf})
    with pytest.raises(ValueError):
        json.loads(s, parse_constant=_refuse)


def test_shard_line_carries_chain_and_nn_roofline():
    """A batch workload line (`--workload config3 --queries 1024`, an 8-GPU rank's shard) keeps
    its step chain and NN roofline in the compact line (they were in the detail
    file only); built from round 6's shard record."""
    bench = _bench()
    with open(os.path.join(ROOT, "profiles", "r06_bench_config3_shard1024_detail.json")) as f:
        full = json.load(f)
    s = bench.compact_line(full, None, with_subs=False)
    assert len(s.encode()) <= bench.LINE_MAX
    back = json.loads(s, parse_constant=_refuse)
    chain = back["step_chain_us"]
    assert set(chain) >= {"mq_sample_nn", "steer_prep", "steer_walk", "mq_insert"}
    assert "note" not in chain
    assert back["nn_roofline"]["kernel"].startswith("mq_sample_nn")
    assert back["passes"]["steps"] >= back["passes"]["ideal_steps"]
