"""Multi-rank bench path on the GPU box (SURVEY.md §4 last bullet, §8e): `bench.py --gpus 2`
starts two rank processes itself (both on device 0 of a one-GPU box), shards the query batch
contiguously, gathers the per-query records (query, iterations, nodes, tree digest) and must
report exactly the records of the one-rank run of the same query set."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args,
                        "--no-cpu-baseline", "--warmup", "2"],
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]  # rank 0 prints the only line
    # strict: the driver's parser refuses Infinity / NaN (round 3's line failed exactly so)
    return json.loads(lines[0], parse_constant=_refuse)


def _refuse(tok):
    raise ValueError(f"non-standard JSON constant {tok!r} in the bench line")


@pytest.mark.gpu
@pytest.mark.parametrize("workload,queries,max_iter", [("config3", 300, 300),
                                                       ("config5", 96, 150)])
def test_sharded_batch_equals_one_rank(workload, queries, max_iter):
    common = ["--workload", workload, "--queries", str(queries), "--max-iter", str(max_iter)]
    one = _bench(*common, "--gpus", "1")
    two = _bench(*common, "--gpus", "2")
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["queries_per_rank"] == queries // 2
    assert "gloo" in two["config"]["gather"] or "nccl" in two["config"]["gather"]
    assert two["iterations_total"] == one["iterations_total"] == queries * max_iter
    assert two["nodes_total"] == one["nodes_total"]
    # the gathered per-query records (query, iterations, nodes, tree digest) are identical
    assert two["records_digest"] == one["records_digest"]
