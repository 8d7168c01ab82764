"""The N>1 control plane of bench.py at world size 2 over gloo on the CPU: query sharding, the
max-time / sum reductions and the config-3 all_gather of per-query records, and
the self-launch of `bench.py --gpus N` (spawn_ranks).  The GPU compute is not involved (the
sharded-equals-single-rank check on the GPU is tests/test_gpu_multirank.py)."""
import os
import socket
import subprocess
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    import bench

    D = bench.Dist(bench.parse(["--gpus", str(world)]))
    assert (D.world, D.rank) == (world, rank)
    assert D.gather_backend == "gloo"  # no GPU here: the gather falls back to gloo
    a, b = bench.shard(10, world, rank)
    rec = np.stack([np.arange(a, b), np.full(b - a, 100 + rank), np.arange(a, b) * 2,
                    np.arange(a, b) * 7], 1)
    allrec = D.gather_records(rec.astype(np.int64))
    tmax = D.allreduce(1.0 + rank, "max")
    tsum = D.allreduce(b - a, "sum")
    D.barrier()
    out[rank] = (allrec.numpy().tolist(), tmax, tsum)
    D.close()


def test_world2_gather_and_reductions():
    world = 2
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    for rank in range(world):
        recs, tmax, tsum = res[rank]
        assert [row[0] for row in recs] == list(range(10))  # every query once, in order
        assert [row[1] for row in recs] == [100] * 5 + [101] * 5
        assert [row[3] for row in recs] == [7 * q for q in range(10)]
        assert tmax == 2.0 and tsum == 10


def test_shards_cover_every_query_once():
    import bench

    for total in (1, 7, 8192):
        for world in (1, 2, 3, 8):
            got = []
            for r in range(world):
                a, b = bench.shard(total, world, r)
                got.extend(range(a, b))
                assert abs((b - a) - total / world) < 1
            assert got == list(range(total))


def test_spawn_ranks_sets_the_rank_environment(tmp_path):
    """`bench.py --gpus 3` without WORLD_SIZE starts 3 children with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* set and returns the worst exit code (the parent never touches the
    GPU).  Checked with a stand-in script that records its environment."""
    probe = tmp_path / "probe.py"
    probe.write_text(
        "import json, os, sys\n"
        "keys = ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE', 'MASTER_ADDR')\n"
        f"open(os.path.join({str(tmp_path)!r}, 'r' + os.environ['RANK']), 'w').write("
        "json.dumps({k: os.environ[k] for k in keys}))\n"
        "sys.exit(3 if os.environ['RANK'] == '2' else 0)\n")
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); import bench, os; "
            f"bench.__file__ = {str(probe)!r}; sys.exit(bench.spawn_ranks(3))")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK")}
    rc = subprocess.run([sys.executable, "-c", code], env=env).returncode
    assert rc == 3
    import json

    for r in range(3):
        d = json.loads((tmp_path / f"r{r}").read_text())
        assert d == {"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": "3",
                     "LOCAL_WORLD_SIZE": "3", "MASTER_ADDR": "127.0.0.1"}
