"""RRT extend iterations/s (2D Dubins, 1k obstacles) — BASELINE.json config 2 on MI355X.

A step = one speculative window of K = 4096 extend iterations (sample, exact nearest neighbour,
Dubins steer, sampled-arc collision check, insert — plan_one minus check_finish) on a tree grown
beforehand to 100k nodes, with the sequential semantics of the reference (results independent
of K).  With --gpus N (torchrun), every rank grows its own independent replica tree on its own
GPU (seed 42 + rank): the path shards by planning query with no data-path collective, so scaling
is weak and `value` is the iterations of all ranks / the slowest rank's time.

Prints ONE JSON line (rank 0).  See DESIGN.md "Measurement" for the roofline accounting.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rs-pathplanning_amd"))

F32_VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md, Peak FP32 (vector), spec
HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md, HBM3E peak, spec
FLOP_PER_EVAL = 5             # dx, dy (2 sub), dx*dx (mul), + dy*dy (fma = 2)
BYTES_PER_EVAL = 8            # f32 x + f32 y of one SoA node


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", choices=("config2", "config3", "config4", "polygons",
                                           "config5"),
                    default="config2",
                    help="config2: one tree, K-candidate windows (default); config3: a batch of "
                         "independent queries sharded over the ranks; config4: config 2 with the "
                         "512x512 occupancy-grid collision; polygons: config 2 with its discs as "
                         "create_circle polygons (polygon mode, SURVEY §8f row 3); config5: a batch of "
                         "independent RRT* queries (k-nearest rewire) on a 10240-disc field")
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (config2: windows, default 20; config3: lockstep "
                         "iterations, default max_iter)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--queries", type=int, default=8192, help="config3: queries over all ranks")
    ap.add_argument("--batch-window", type=int, default=0,
                    help="config3: iterations per query evaluated speculatively per GPU step "
                         "(power of two <= 64; 0 = automatic: 16 up to 131072 tasks per step)")
    ap.add_argument("--max-iter", type=int, default=2000, help="config3: RRT.max_iter per query")
    ap.add_argument("--window", type=int, default=4096)
    ap.add_argument("--nodes", type=int, default=100_000, help="tree size before timing")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="bounded CPU-baseline sample per variant (rank 0, N=1 only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-size-sweep", action="store_true")
    return ap.parse_args()


def shard(total, world, rank):
    """Queries [a, b) of `rank`: contiguous, sizes differ by at most one."""
    base, extra = divmod(total, world)
    a = rank * base + min(rank, extra)
    return a, a + base + (1 if rank < extra else 0)


def dist_setup(args, backend="gloo"):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # control plane: barrier, max-time reduce, gather

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":  # RCCL over xGMI on the GPU box
            import torch

            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return dist, world, rank, local


def barrier(dist):
    if dist is not None:
        dist.barrier()


def allreduce_max(dist, v):
    if dist is None:
        return v
    import torch

    t = torch.tensor([float(v)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allreduce_sum(dist, v):
    if dist is None:
        return v
    import torch

    t = torch.tensor([float(v)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def make_planner(raw, seed, window, device):
    from pathplanning_amd import rrt

    sx, sy, syaw = raw["start"]
    gx, gy, gyaw = raw["goal"]
    return rrt.RRT((sx, sy), syaw, (gx, gy), gyaw, raw["max_iter"], raw["step_size"],
                   rrt.Space.from_raw(raw), seed=seed, window=window, device=device,
                   capacity=1 << 18)


def timed_windows(p, n_windows, window):
    p.synchronize()
    t0 = time.perf_counter()
    p.extend(n_windows * window)
    p.synchronize()
    return time.perf_counter() - t0


def auto_batch_window(q):
    """pp_batch_new's automatic window: 32 for at most 2048 queries, else the largest power of
    two <= 16 with q * K <= 131072."""
    if q <= 2048:
        return 32
    k = 1
    while k < 16 and q * k * 2 <= 131072:
        k *= 2
    return k


def host_threads():
    """The host cores the CPU baseline may use: OMP_NUM_THREADS (16 on the GPU box, its share of
    the machine), else all visible cores."""
    return max(1, int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1))


def cpu_baseline(raw, p, args):
    """The oracle restatement (oracle/, C) on the SAME workload: continue the GPU's 100k-node tree
    re-verifying the whole line to the root like the reference's verify_node (rrt.rs:414-426).
      1. one core, time-capped (a few seconds): the per-core rate, and the incremental-verify
         rate beside it;
      2. all host cores: one independent replica per thread (seed + r), each continuing the same
         tree for the per-core rate x cpu_seconds iterations — the CPU analogue of the GPU's
         replicas, timed on the wall clock."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (cpu_baseline leg: the oracle is the timed CPU port here)

    x, y, yaw, par = p.tree()
    it0 = p.iteration()
    sc = oracle.OracleScene.from_raw(raw)
    tr = oracle.OracleTree(raw["start"], len(x) + 1)
    n = len(x)
    tr.x[:n], tr.y[:n], tr.yaw[:n], tr.parent[:n] = x, y, yaw, par
    tr._c.n = n
    out = {}
    for name, full in (("full_reverify", True), ("incremental", False)):
        work = oracle.OracleTree(raw["start"], n + 200_000)
        work.x[:n], work.y[:n], work.yaw[:n], work.parent[:n] = x, y, yaw, par
        work._c.n = n
        done, chunk, t_used = 0, 1, 0.0
        while t_used < args.cpu_seconds / 3.0:
            t0 = time.perf_counter()
            oracle.rrt_extend(sc, work, args.seed, it0 + done, chunk, full_reverify=full)
            t_used += time.perf_counter() - t0
            done += chunk
            chunk = min(chunk * 2, 4096)
        out[name] = (done / t_used, done, t_used)
    threads = host_threads()
    per = max(16, int(out["full_reverify"][0] * args.cpu_seconds))
    seeds = [args.seed + 1000 + r for r in range(threads)]
    t0 = time.perf_counter()
    oracle.extend_replicas(sc, tr, seeds, it0, per, threads, full_reverify=True)
    t = time.perf_counter() - t0
    out["all_cores"] = (threads * per / t, threads * per, t, threads, per)
    return out


def cpu_baseline_queries(raw, starts, seeds, max_iter, seconds):
    """config 3's CPU baseline: the oracle (C) runs whole queries of the same batch — query q from
    its own start with its own seed, max_iter iterations each, the reference's full re-verify of
    the line to the root (rrt.rs:414-426) — first on one core (a few seconds: the per-query time),
    then a batch of them on all host cores, one query per thread at a time (wall clock)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (cpu_baseline leg: the oracle is the timed CPU port here)

    sc = oracle.OracleScene.from_raw(raw)
    done, t_used, nq = 0, 0.0, 0
    for q in range(len(seeds)):
        tr = oracle.OracleTree(tuple(starts[q]), max_iter + 1)
        t0 = time.perf_counter()
        oracle.rrt_extend(sc, tr, int(seeds[q]), 0, max_iter, full_reverify=True)
        t_used += time.perf_counter() - t0
        done += max_iter
        nq += 1
        if t_used >= seconds / 3.0:
            break
    one = (done / t_used, done, nq, t_used)
    threads = host_threads()
    per_query = t_used / nq
    qn = int(min(len(seeds), max(threads, threads * seconds / per_query)))
    t0 = time.perf_counter()
    oracle.queries(sc, starts[:qn], seeds[:qn], max_iter, threads, full_reverify=True)
    t = time.perf_counter() - t0
    return one, (qn * max_iter / t, qn * max_iter, qn, t, threads)


def load_traffic():
    """HBM bytes per nn_scan launch from the committed rocprofv3 PMC summary (or None)."""
    path = os.path.join(ROOT, "profiles", "nn_scan_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("hbm_bytes_per_launch")


def load_batch_traffic(workload):
    """HBM bytes per whole-batch NN launch of config 3 / 5 from the committed rocprofv3 PMC
    summary (scripts/traffic_summary.py), or None."""
    path = os.path.join(ROOT, "profiles", "batch_nn_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get(workload, {}).get("hbm_bytes_per_launch")


def gather_records(dist, rec, backend):
    """The config-3 result gather: every rank's per-query records to every rank (one
    all_gather; RCCL over xGMI when the backend is nccl).  rec: int64 [q_rank, 3]."""
    import torch

    if dist is None:
        return torch.from_numpy(rec)
    world = dist.get_world_size()
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else None
    n = torch.tensor([rec.shape[0]], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    mx = int(max(int(v.item()) for v in sizes))
    pad = torch.zeros((mx, 3), dtype=torch.int64, device=dev)
    pad[: rec.shape[0]] = torch.from_numpy(rec).to(pad.device)
    outs = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad)
    return torch.cat([o[: int(sz.item())].cpu() for o, sz in zip(outs, sizes)])


def main():
    args = parse()
    if args.workload == "config3":
        return main_config3(args)
    if args.workload == "config5":
        return main_config5(args)
    if args.steps is None:
        args.steps = 20
    dist, world, rank, local = dist_setup(args)
    from pathplanning_amd import scenes

    raw = {"config4": scenes.field512_grid, "polygons": scenes.field512_polygons}.get(
        args.workload, scenes.field512)()
    p = make_planner(raw, args.seed + rank, args.window, local)
    sweep = {}
    # grow the tree (untimed); on the way time a few windows at 1k and 10k nodes
    marks = [] if args.no_size_sweep else [1_000, 10_000]
    while p.tree_size() < args.nodes:
        if marks and p.tree_size() >= marks[0]:
            m = marks.pop(0)
            n0, it0 = p.tree_size(), p.iteration()
            dt = timed_windows(p, 5, args.window)
            sweep[str(m)] = {"iterations_per_s": (p.iteration() - it0) / dt, "tree_nodes": n0}
        p.extend(args.window)
    p.extend(args.warmup * args.window)
    p.synchronize()

    n_start = p.tree_size()
    p.reset_stats()
    barrier(dist)
    p.synchronize()
    t0 = time.perf_counter()
    p.extend(args.steps * args.window)  # the K steps back to back (windows enqueued without sync)
    p.synchronize()
    t_local = time.perf_counter() - t0
    barrier(dist)
    st = p.stats()
    t_max = allreduce_max(dist, t_local)
    iters_total = allreduce_sum(dist, st["iterations"])
    value = iters_total / t_max
    sweep[str(args.nodes)] = {"iterations_per_s": st["iterations"] / t_local, "tree_nodes": n_start}

    # profiled pass over the same workload (the next `steps` windows): HIP events on the planner's
    # stream around nn_scan and steer_window.  Kept out of the timed region above because every
    # event record adds a few microseconds of queue gap between the kernels.
    p.reset_stats()
    p.set_profiling(True)
    p.extend(args.steps * args.window)
    p.synchronize()
    p.set_profiling(False)
    sp = p.stats()

    # dominant kernel (nn_scan): algorithmic work per launch / average launch duration (HIP events)
    launches = max(sp["nn_scan_launches"], 1)
    avg_ms = sp["nn_scan_ms"] / launches
    evals_per_launch = sp["node_evals"] / launches
    achieved_tflops = evals_per_launch * FLOP_PER_EVAL / (avg_ms * 1e-3) / 1e12
    roofline = {
        "kernel": "window_kernel (NN screen; workgroup 0 resolves the previous window)",
        "bound": "valu",
        "achieved": round(achieved_tflops, 3),
        "peak": F32_VALU_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved_tflops / F32_VALU_PEAK_TFLOPS, 4),
        "traffic": load_traffic(),
        "avg_launch_ms": round(avg_ms, 5),
        "evals_per_launch": int(evals_per_launch),
        "algorithmic_hbm_view": {
            "bytes_per_eval": BYTES_PER_EVAL,
            "achieved_GBs": round(evals_per_launch * BYTES_PER_EVAL / (avg_ms * 1e-3) / 1e9, 1),
            "peak_GBs": HBM_PEAK_GBS,
            "note": "8 B/eval as if every eval read its node from HBM (SURVEY §8d); > peak means "
                    "the batch reuses each node across 256 samples per wave, so VALU is the bound",
        },
        "steer_avg_launch_ms": round(sp["steer_ms"] / max(sp["steer_launches"], 1), 5),
        "measured": f"HIP events on the planner stream, {sp['nn_scan_launches']} launches of the "
                    "profiled pass that follows the timed region (same workload)",
    }

    line = {
        "metric": "RRT extend iterations/sec (2D Dubins, 1k obstacles)",
        "value": round(value, 1),
        "unit": "iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * t_max / args.steps, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": {"config4": "config4: field512 rasterised to a 512x512 bit-packed "
                                    "occupancy grid (32 KB, point probes)",
                         "polygons": "polygons: field512's 1024 discs as create_circle polygons "
                                     f"({sum(len(o) for o in raw.get('obstacle_polygons', []))} "
                                     "edges, Minkowski buffers, SURVEY §8f row 3)"}.get(
                             args.workload, "config2: field512 (1024 discs r~U(2,8), 512x512)")
                        + f", R=4.0, step 0.1, K={args.window} candidates/window, tree grown to "
                        f"{args.nodes} nodes",
            "window": args.window,
            "tree_nodes_at_start": n_start,
            "obstacles": len(raw.get("obstacle_polygons", raw["circles"])),
            "parallelism": f"replicas{world}",
            "nn_screen_dtype": "f32 (exact f64 rescan of near-ties)",
        },
        "node_evals_per_s_per_gpu": round(st["node_evals"] / t_local, 1),
        "sizes": sweep,
        "stats": {k: st[k] for k in ("iterations", "accepted", "windows", "truncations",
                                     "repair_rounds", "repairs", "literal_repairs", "nn_flagged")},
        "roofline": roofline,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cb = cpu_baseline(raw, p, args)
        v, n, t = cb["full_reverify"]
        vi, ni, ti = cb["incremental"]
        va, na, ta, th, per = cb["all_cores"]
        line["cpu_baseline"] = {
            "value": round(va, 2), "unit": "iterations/s", "cores": th, "kind": "port",
            "sample": f"{th} independent replicas on {th} host threads, each continuing the same "
                      f"{n_start}-node tree for {per} iterations (seeds {args.seed + 1000}..), "
                      f"re-verifying the whole line to the root like rrt.rs:414-426; "
                      f"{na} iterations in {ta:.1f} s wall",
            "one_core": {"value": round(v, 2), "iterations": n, "seconds": round(t, 2)},
            "incremental_verify_one_core": {"value": round(vi, 2), "iterations": ni,
                                            "seconds": round(ti, 2)},
        }
    if rank == 0:
        print(json.dumps(line), flush=True)
    p.close()
    if dist is not None:
        dist.destroy_process_group()


def main_config3(args):
    """BASELINE config 3: `queries` independent planners on the config-2 field (query q: seed
    42 + q, start/goal from stream q), max_iter each, sharded contiguously over the ranks; a step
    = one lockstep extend iteration of every query of the rank.  Strong scaling: the total work is
    fixed, each rank runs queries/world of it; one all_gather of per-query records at the end."""
    import torch

    backend = "nccl" if (int(os.environ.get("WORLD_SIZE", "1")) > 1 and
                         torch.cuda.is_available()) else "gloo"
    dist, world, rank, local = dist_setup(args, backend)
    from pathplanning_amd import rrt, scenes

    raw = scenes.field512()
    space = rrt.Space.from_raw(raw)
    a, b = shard(args.queries, world, rank)
    starts, goals, seeds = scenes.config3_queries(raw, a, b - a)
    steps = args.max_iter if args.steps is None else args.steps
    batch = rrt.RRTBatch(starts, goals, args.max_iter, raw["step_size"], space, seeds,
                         device=local, window=args.batch_window)
    batch.extend(args.warmup)  # untimed warmup on a throwaway run
    batch.close()
    batch = rrt.RRTBatch(starts, goals, args.max_iter, raw["step_size"], space, seeds,
                         device=local, window=args.batch_window)
    barrier(dist)
    t0 = time.perf_counter()
    it_local, acc_local = batch.extend(steps)
    t_local = time.perf_counter() - t0
    barrier(dist)
    n, its, evals = batch.state(with_evals=True)
    rec = np.stack([np.arange(a, b, dtype=np.int64), its.astype(np.int64), n.astype(np.int64)], 1)
    allrec = gather_records(dist, rec, backend)
    t_max = allreduce_max(dist, t_local)
    iters_total = int(allrec[:, 1].sum())
    value = iters_total / t_max
    # profiled pass (same workload): HIP events around the batch NN kernel of every step
    batch.close()
    batch = rrt.RRTBatch(starts, goals, args.max_iter, raw["step_size"], space, seeds,
                         device=local, window=args.batch_window)
    batch.set_profiling(True)
    batch.extend(steps)
    sp = batch.stats()
    _, _, evals_p = batch.state(with_evals=True)
    nn_ms = sp["nn_scan_ms"] / max(sp["nn_scan_launches"], 1)
    evals_per_launch = float(evals_p.sum()) / max(sp["nn_scan_launches"], 1)
    bytes_per_eval = 16  # f64 x + f64 y of one SoA row (exact NN, no f32 screen here)
    achieved = evals_per_launch * bytes_per_eval / (nn_ms * 1e-3) / 1e9
    line = {
        "metric": "RRT extend iterations/sec (2D Dubins, 1k obstacles)",
        "value": round(value, 1),
        "unit": "iterations/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * t_max / steps, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": f"config3: {args.queries} independent queries on the config-2 field "
                        f"(query q: seed 42+q, start/goal from stream q), max_iter "
                        f"{args.max_iter}, sharded contiguously over {world} rank(s)",
            "queries": args.queries,
            "queries_per_rank": b - a,
            "parallelism": f"query-shard{world}",
            "window_per_query": args.batch_window or auto_batch_window(b - a),
            "gather": f"all_gather of per-query records ({backend})",
        },
        "iterations_total": iters_total,
        "nodes_total": int(allrec[:, 2].sum()),
        "roofline": {
            "kernel": "mq_sample_nn",
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": load_batch_traffic("config3") if args.queries == 8192 else None,
            "avg_launch_ms": round(nn_ms, 5),
            "evals_per_launch": int(evals_per_launch),
            "bytes_per_eval": bytes_per_eval,
            "measured": f"HIP events around mq_sample_nn, {sp['nn_scan_launches']} launches of "
                        "the profiled pass that follows the timed region (same workload)",
        },
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        (v, n, nq, t), (va, na, qa, ta, th) = cpu_baseline_queries(
            raw, starts, seeds, args.max_iter, args.cpu_seconds)
        line["cpu_baseline"] = {
            "value": round(va, 2), "unit": "iterations/s", "cores": th, "kind": "port",
            "sample": f"the first {qa} whole queries of the same batch ({na} iterations, max_iter "
                      f"{args.max_iter} each, full re-verify like rrt.rs:414-426) on {th} host "
                      f"threads, {ta:.1f} s wall",
            "one_core": {"value": round(v, 2), "queries": nq, "iterations": n,
                         "seconds": round(t, 2)},
        }
    if rank == 0:
        print(json.dumps(line), flush=True)
    batch.close()
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline_star(raw, starts, seeds, max_iter, eta, seconds):
    """config 5's CPU baseline: the RRT* oracle (C, orc_star_extend) on the same queries — query
    0 on one core in chunks of 100 iterations until seconds/3 (or max_iter), then `threads` whole
    queries of the batch, each for that many iterations, one per host thread (wall clock)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (cpu_baseline leg: the oracle is the timed CPU port here)

    sc = oracle.OracleScene.from_raw(raw)
    tr = oracle.OracleStarTree(tuple(starts[0]), max_iter + 1)
    done, t_used = 0, 0.0
    while done < max_iter and t_used < seconds / 3.0:
        n = min(100, max_iter - done)
        t0 = time.perf_counter()
        oracle.star_extend(sc, tr, int(seeds[0]), done, n, 0, eta)
        t_used += time.perf_counter() - t0
        done += n
    threads = min(host_threads(), len(seeds))
    t0 = time.perf_counter()
    oracle.star_queries(sc, starts[:threads], seeds[:threads], done, 0, eta, threads)
    t = time.perf_counter() - t0
    return (done / t_used, done, t_used), (threads * done / t, threads * done, threads, t, done)


def main_config5(args):
    """BASELINE config 5 (stretch; build-defined RRT*): `queries` independent
    k-nearest RRT* planners on a 10240-disc field (scenes.config5_field, Steer eta = 16, k =
    ceil(2e ln n)), max_iter each, sharded contiguously over the ranks like config 3; a step = one
    lockstep RRT* iteration of every query of the rank; one all_gather of records at the end."""
    import torch

    backend = "nccl" if (int(os.environ.get("WORLD_SIZE", "1")) > 1 and
                         torch.cuda.is_available()) else "gloo"
    dist, world, rank, local = dist_setup(args, backend)
    from pathplanning_amd import rrt, scenes

    raw = scenes.config5_field()
    eta = scenes.CONFIG5_ETA
    space = rrt.Space.from_raw(raw)
    a, b = shard(args.queries, world, rank)
    starts, _, seeds = scenes.config3_queries(raw, a, b - a)
    steps = args.max_iter if args.steps is None else args.steps

    def fresh():
        return rrt.RRTStarBatch(starts, args.max_iter, raw["step_size"], space, seeds, k=0,
                                eta=eta, device=local)

    batch = fresh()
    batch.extend(args.warmup)  # untimed warmup on a throwaway run
    batch.close()
    batch = fresh()
    barrier(dist)
    t0 = time.perf_counter()
    batch.extend(steps)
    t_local = time.perf_counter() - t0
    barrier(dist)
    n, its, evals, rw = batch.state()
    rec = np.stack([np.arange(a, b, dtype=np.int64), its.astype(np.int64), n.astype(np.int64)], 1)
    allrec = gather_records(dist, rec, backend)
    t_max = allreduce_max(dist, t_local)
    iters_total = int(allrec[:, 1].sum())
    rewires_total = int(allreduce_sum(dist, float(rw.sum())))
    value = iters_total / t_max
    # profiled pass (same workload): HIP events around star_sample (the exact NN) of every step
    batch.close()
    batch = fresh()
    batch.set_profiling(True)
    batch.extend(steps)
    sp = batch.stats()
    evals_p = batch.state()[2]
    nn_ms = sp["nn_scan_ms"] / max(sp["nn_scan_launches"], 1)
    evals_per_launch = float(evals_p.sum()) / max(sp["nn_scan_launches"], 1)
    bytes_per_eval = 16  # f64 x + f64 y of one SoA row
    achieved = evals_per_launch * bytes_per_eval / (nn_ms * 1e-3) / 1e9
    line = {
        "metric": "RRT* iterations/sec (SE(2) Dubins, k-nearest rewire, 10k obstacles)",
        "value": round(value, 1),
        "unit": "iterations/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * t_max / steps, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": f"config5 (stretch, build-defined RRT*): {args.queries} independent "
                        f"queries on {raw['name']} (10240 discs r~U(1,4) on 2048^2), Steer eta "
                        f"{eta}, k = ceil(2e ln n) <= 63, max_iter {args.max_iter}, sharded "
                        f"contiguously over {world} rank(s)",
            "queries": args.queries,
            "queries_per_rank": b - a,
            "parallelism": f"query-shard{world}",
            "gather": f"all_gather of per-query records ({backend})",
        },
        "iterations_total": iters_total,
        "nodes_total": int(allrec[:, 2].sum()),
        "rewires_total": rewires_total,
        "roofline": {
            "kernel": "star_sample (exact f64 NN)",
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": load_batch_traffic("config5") if args.queries == 8192 else None,
            "avg_launch_ms": round(nn_ms, 5),
            "evals_per_launch": int(evals_per_launch),
            "bytes_per_eval": bytes_per_eval,
            "measured": f"HIP events around star_sample, {sp['nn_scan_launches']} launches of "
                        "the profiled pass that follows the timed region (same workload)",
        },
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        (v, n1, t1), (va, na, th, ta, m) = cpu_baseline_star(raw, starts, seeds, args.max_iter,
                                                             eta, args.cpu_seconds)
        line["cpu_baseline"] = {
            "value": round(va, 2), "unit": "iterations/s", "cores": th, "kind": "port",
            "sample": f"the first {th} queries of the same batch, their first {m} RRT* "
                      f"iterations each ({na} iterations), on {th} host threads, {ta:.1f} s wall",
            "one_core": {"value": round(v, 2), "iterations": n1, "seconds": round(t1, 2)},
        }
    if rank == 0:
        print(json.dumps(line), flush=True)
    batch.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
