"""The N>1 control plane of bench.py at world size 2 over gloo on the CPU: query sharding, the
max-time / sum reductions and the config-3 all_gather of per-query records.
The GPU compute is not involved (it is covered by the -m gpu tests)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import bench

    class A:
        pass

    dist, w, r, _ = bench.dist_setup(A(), "gloo")
    assert (w, r) == (world, rank)
    a, b = bench.shard(10, world, rank)
    rec = np.stack([np.arange(a, b), np.full(b - a, 100 + rank), np.arange(a, b) * 2], 1)
    allrec = bench.gather_records(dist, rec.astype(np.int64), "gloo")
    tmax = bench.allreduce_max(dist, 1.0 + rank)
    tsum = bench.allreduce_sum(dist, b - a)
    bench.barrier(dist)
    out[rank] = (allrec.numpy().tolist(), tmax, tsum)
    dist.destroy_process_group()


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
        assert tmax == 2.0 and tsum == 10
