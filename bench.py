"""RRT extend iterations/s (2D Dubins, 1k obstacles) — BASELINE.json's metric on MI355X.

Headline (`value`): BASELINE config 2 — one tree grown to 100k nodes, a step = one speculative
window of K = 4096 extend iterations (sample, exact nearest neighbour, Dubins steer, sampled-arc
collision check, insert: plan_one minus check_finish, rrt.rs:583-589) with the sequential
semantics of the reference (results independent of K).  With N ranks every rank grows its own
replica tree on its own GPU (seed 42 + rank): weak scaling, `value` = all ranks' iterations / the
slowest rank's time.

Sub-results on the same line (the rows of SURVEY.md §8d the driver would not see otherwise):
  config3          8192 independent queries sharded contiguously over the N ranks (strong
                   scaling), one all_gather of per-query records over RCCL (nccl) when every rank
                   has its own GPU; `records_digest` is the same at every N when the sharded run
                   equals the 1-rank run
  config5          the RRT* query batch (build-defined, stretch), sharded the same way
  config4          config 2 on the 512x512 bit-packed occupancy grid (N = 1 only)
  polygons         config 2 with the 1024 discs as the crate's create_circle polygons (N = 1)
  config1          the reference's own bench scene (benches/all.rs:8-46), 8000 iterations, analytic
                   discs (N = 1 only)
  config1_polygons the same scene as the bench builds it: create_circle polygons (N = 1 only)
  plan             RRT::plan on bench6_open: extend + check_finish of every accepted node (N = 1)
  example_rrt      examples/rrt: RRT::plan on the example's own scene (transit.debug.json,
                   Robot::new(1.8, 3.0, 0.8), 8000 iterations) (N = 1 only)

`python bench.py --gpus N` without WORLD_SIZE starts N rank processes itself (before anything
touches the GPU); under torchrun it is one of them.  Rank 0 writes the full record to --detail
(gpurun_out/bench_detail.json) and prints ONE compact JSON line of at most LINE_MAX bytes (the
headline keys, the dominant kernel's roofline, the CPU baseline, one short record per sub-result).
See DESIGN.md §5 for the roofline accounting.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "rs-pathplanning_amd"))

F32_VALU_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md, Peak FP32 (vector), spec
# AMD Instinct MI355X datasheet, FP64 vector (spec).  MI355X_MICROARCH.md has no FP64 row.
FP64_VALU_PEAK_TFLOPS = 78.6
HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md, HBM3E peak, spec
CLOCK_GHZ = 2.4               # MI355X_MICROARCH.md, max clock
VALU_CYC = 2                  # cycles per wave64 VALU instruction on a SIMD-32 (MICROARCH: v_fma_f32)
FLOP_PER_EVAL = 5             # dx, dy (2 sub), dx*dx (mul), + dy*dy (fma = 2)
BYTES_PER_EVAL = 8            # f32 x + f32 y of one SoA node
# Algorithmic f64 work of one polyline point of the walk (dubins.rs:155-198 interpolate, 239-255
# the pd walk, 412-422 the world transform; rrt.rs:124-137 the bounds test), counted from the
# reference's expressions:
#   L/R point: sin + cos of the arc length (SINCOS_FLOP: a Cody-Waite reduction ~8 FLOP and two
#              degree-13/14 minimax polynomials ~32 FLOP, ocml's sincos), ldx = sin/c (1),
#              ldy = (1 - cos)/c (2), gdx / gdy = rotate by the segment origin (6), + origin (2)
#   S point:   x/y = origin + pd/c * cos/sin(origin yaw) (6)
#   both:      world transform (8: 4 mul, 4 add), pd += d (1), bounds (4 compares)
# The per-disc segment tests are not counted: the chunk cull passes < 1 disc per 63 points.
SINCOS_FLOP = 40
ARC_POINT_FLOP = SINCOS_FLOP + 11 + 8 + 1 + 4
LINE_POINT_FLOP = 6 + 8 + 1 + 4
METRIC = "RRT extend iterations/sec (2D Dubins, 1k obstacles)"
WORKLOADS = ("default", "config1", "config1_polygons", "config2", "config3", "config4",
             "polygons", "config5", "plan", "example_rrt")


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without WORLD_SIZE the bench starts them itself")
    ap.add_argument("--workload", choices=WORKLOADS, default="default",
                    help="default: config 2 + the sub-results; config2/config4/polygons: one tree, "
                         "K-candidate windows (config4: 512x512 occupancy grid; polygons: "
                         "create_circle polygons, SURVEY §8f row 3); config3: independent queries "
                         "sharded over the ranks; config5: RRT* query batch; config1 / "
                         "config1_polygons: the reference's bench scene; plan / example_rrt: "
                         "RRT::plan with check_finish")
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (windows for the one-tree workloads, default 20; lockstep "
                         "iterations for the batches, default max_iter)")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--queries", type=int, default=8192, help="config3/5: queries over all ranks")
    ap.add_argument("--batch-window", type=int, default=0,
                    help="config3: iterations per query evaluated speculatively per GPU step "
                         "(power of two <= 64; 0 = automatic)")
    ap.add_argument("--max-iter", type=int, default=2000, help="config3/5: RRT.max_iter per query")
    ap.add_argument("--window", type=int, default=4096)
    ap.add_argument("--nodes", type=int, default=100_000, help="tree size before timing")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="bounded CPU-baseline sample per variant (rank 0, N=1 only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-size-sweep", action="store_true")
    ap.add_argument("--no-sub", action="store_true", help="default workload: config 2 only")
    ap.add_argument("--pmc-run", action="store_true",
                    help="config3: no profiled plan pass (counter runs: the last walk dispatches "
                         "are then the profiled extend's)")
    ap.add_argument("--detail", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="where the full record goes (stdout gets the compact line)")
    ap.add_argument("--allow-variant-lib", action="store_true",
                    help="accept PP_AMD_LIB pointing at another build (experiments only)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------ ranks
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, timeout=1800):
    """`--gpus N` without a launcher: N child processes of this script with RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* set, started before this process touches the GPU (it never does).
    Returns the worst exit code; rank 0 prints the JSON line.  A rank that fails ends the run:
    the others are terminated (a peer stuck in a collective would wait for it forever)."""
    env0 = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
                WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n))
    procs = []
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    deadline = time.time() + timeout
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0:
                rc = rc or c
        if rc or time.time() > deadline:
            for p in live:
                p.terminate()
            for p in live:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
            rc = rc or 124
            break
        time.sleep(0.2)
    return rc


class Dist:
    """One process per GPU.  The data path never communicates; the control plane (barrier,
    max-time / sum reductions) runs over gloo and the per-query record gather over RCCL (nccl)
    when every local rank has a GPU of its own, else over gloo (ranks sharing one GPU: RCCL
    refuses two ranks on one device)."""

    def __init__(self, args):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(self.world)))
        if args.gpus > 1 and self.world != args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={self.world}")
        from pathplanning_amd import _ffi

        ndev = max(1, _ffi.device_count())
        self.device = self.local % ndev
        self.dist = None
        self.gather_backend = None
        if self.world > 1:
            import datetime

            import torch
            import torch.distributed as dist

            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            own_gpu = torch.cuda.is_available() and torch.cuda.device_count() >= local_world
            if own_gpu:
                torch.cuda.set_device(self.device)
                backend = "cpu:gloo,cuda:nccl"
                self.gather_backend = "nccl"
            else:
                backend = "gloo"
                self.gather_backend = "gloo"
            dist.init_process_group(backend=backend, rank=self.rank, world_size=self.world,
                                    timeout=datetime.timedelta(seconds=600))
            assert dist.get_world_size() == self.world
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            import torch

            self.dist.all_reduce(torch.zeros(1))  # on gloo: a CPU barrier that ignores devices

    def allreduce(self, v, op="max"):
        if self.dist is None:
            return v
        import torch

        t = torch.tensor([float(v)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX if op == "max" else self.dist.ReduceOp.SUM)
        return float(t.item())

    def gather_records(self, rec):
        """Every rank's per-query records (int64 [q_rank, C]) to every rank: one all_gather of
        the padded blocks (RCCL over xGMI when gather_backend is nccl).  An RCCL failure is not
        papered over: it raises, and the run ends (spawn_ranks stops the peers)."""
        import torch

        if self.dist is None:
            return torch.from_numpy(rec)
        dev = torch.device("cuda", self.device) if self.gather_backend == "nccl" else None
        n = torch.tensor([rec.shape[0]], dtype=torch.int64, device=dev)
        sizes = [torch.zeros_like(n) for _ in range(self.world)]
        self.dist.all_gather(sizes, n)
        mx = int(max(int(v.item()) for v in sizes))
        pad = torch.zeros((mx, rec.shape[1]), dtype=torch.int64, device=dev)
        pad[: rec.shape[0]] = torch.from_numpy(rec).to(pad.device)
        outs = [torch.zeros_like(pad) for _ in range(self.world)]
        self.dist.all_gather(outs, pad)
        return torch.cat([o[: int(sz.item())].cpu() for o, sz in zip(outs, sizes)])

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def shard(total, world, rank):
    """Queries [a, b) of `rank`: contiguous, sizes differ by at most one."""
    base, extra = divmod(total, world)
    a = rank * base + min(rank, extra)
    return a, a + base + (1 if rank < extra else 0)


# ------------------------------------------------------------------------------ provenance
def provenance(args):
    """The library this run measures: its sha256 and the flags __graft_entry__ builds it with.
    A PP_AMD_LIB override (a variant build) is refused unless --allow-variant-lib."""
    from pathplanning_amd import _ffi
    import __graft_entry__ as g

    if os.environ.get("PP_AMD_LIB") and not args.allow_variant_lib:
        raise SystemExit("PP_AMD_LIB is set: bench.py measures the in-tree build only "
                         "(--allow-variant-lib for experiments)")
    with open(_ffi.LIB_PATH, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()[:16]
    # PP_* variables in the environment (the library itself reads none; recorded for the record)
    knobs = {k: v for k, v in sorted(os.environ.items()) if k.startswith("PP_")}
    return {"lib": os.path.relpath(_ffi.LIB_PATH, ROOT), "lib_sha256_16": sha,
            "hipcc_flags": " ".join(g.HIPCC_FLAGS), "variant": bool(os.environ.get("PP_AMD_LIB")),
            "env_knobs": knobs}


def load_profile(name):
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        return json.load(f)


def host_threads():
    """The host cores the CPU baseline may use: OMP_NUM_THREADS (16 on the GPU box, its share of
    the machine), else all visible cores."""
    return max(1, int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1))


def host_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    vis = os.cpu_count() or 1
    return {"cpu_model": model, "nproc_visible": vis,
            "machine_share": f"{host_threads()} of {vis} visible cores "
                             f"({100.0 * host_threads() / vis:.1f}%: the GPU lease's "
                             f"OMP_NUM_THREADS share; single-core legs use 1)",
            "reference_crate": "not buildable here (Rust, no cargo/rustc, crates not vendored: "
                               "SURVEY.md K7); the CPU baseline is the build's C port (oracle/)"}


def device_free_bytes(device):
    """free device memory (hipMemGetInfo through torch, the process's one HIP runtime), or None"""
    try:
        import torch

        return int(torch.cuda.mem_get_info(device)[0])
    except Exception:
        return None


def oracle_mod():
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (cpu_baseline leg: the oracle is the timed CPU port here)

    return oracle


# ------------------------------------------------------------------------------ rooflines
def walk_flop(points, arc_points):
    """Algorithmic f64 FLOP of `points` walked polyline points, `arc_points` of them on L/R."""
    return arc_points * ARC_POINT_FLOP + (points - arc_points) * LINE_POINT_FLOP


def screen_roofline(sp, pmc):
    """window_kernel (the NN screen, dominant in config 2/4): algorithmic work per launch / the
    HIP-event average launch duration; plus the VALU instruction-issue bound from the committed
    PMC pass (VALU instructions per eval, profiles/window_kernel_pmc.json)."""
    launches = max(sp["nn_scan_launches"], 1)
    avg_ms = sp["nn_scan_ms"] / launches
    evals = sp["node_evals"] / launches
    achieved = evals * FLOP_PER_EVAL / (avg_ms * 1e-3) / 1e12
    r = {
        "kernel": "window_kernel (NN screen; workgroup 0 resolves the previous window)",
        "bound": "valu",
        "achieved": round(achieved, 3),
        "peak": F32_VALU_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved / F32_VALU_PEAK_TFLOPS, 4),
        "traffic": pmc.get("hbm_bytes_per_launch"),
        "avg_launch_ms": round(avg_ms, 5),
        "evals_per_launch": int(evals),
        "launches": int(sp["nn_scan_launches"]),
        "flop_per_eval": FLOP_PER_EVAL,
        "measured": f"HIP events on the planner stream, {sp['nn_scan_launches']} launches of the "
                    "profiled pass that follows the timed region (same workload)",
    }
    vpe = pmc.get("valu_insts_per_eval")
    if vpe:
        simds = 4 * pmc.get("screen_cus", 248)
        issue_us = evals * vpe / 64.0 * VALU_CYC / simds / (CLOCK_GHZ * 1e3)
        r["issue_bound"] = {
            "valu_insts_per_eval": vpe, "simds": simds,
            "issue_bound_us": round(issue_us, 2),
            "issue_frac": round(issue_us / (avg_ms * 1e3), 4),
            "pmc_valu_busy": pmc.get("valu_busy"),
            "note": "wave64 VALU instructions x 2 cycles (SIMD-32) / SIMDs / 2.4 GHz; the VALU "
                    "count per eval is the committed rocprofv3 SQ_INSTS_VALU pass",
        }
    return r


def fp64_roofline(kernel, ms, launches, points, arc_points, pmc=None, measured="", tasks=0):
    """A walk-type kernel (f64 Dubins interpolation + collision per polyline point): the
    algorithmic FLOP of the points it walked (walk_flop) / its HIP-event time against the FP64
    vector peak; the PMC VALU count per point (when a counter pass exists) beside it."""
    if not launches or not points or ms <= 0:
        return None
    avg_ms = ms / launches
    flop = walk_flop(points, arc_points) / launches
    achieved = flop / (avg_ms * 1e-3) / 1e12
    r = {"kernel": kernel, "bound": "fp64-valu", "achieved": round(achieved, 4),
         "peak": FP64_VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
         "frac": round(achieved / FP64_VALU_PEAK_TFLOPS, 5),
         "traffic": (pmc or {}).get("hbm_bytes_per_launch"),
         "avg_launch_ms": round(avg_ms, 5), "launches": int(launches),
         "points_per_launch": int(points / launches),
         "arc_points_per_launch": int(arc_points / launches),
         "flop_per_launch": int(flop),
         "flop_per_point": {"arc": ARC_POINT_FLOP, "line": LINE_POINT_FLOP,
                            "sincos": SINCOS_FLOP},
         "gpoints_per_s": round(points / launches / (avg_ms * 1e-3) / 1e9, 4),
         "peak_source": "AMD MI355X datasheet FP64 vector 78.6 TFLOP/s (spec; the guide has no "
                        "FP64 row)",
         "measured": measured}
    vpp = (pmc or {}).get("valu_insts_per_point")
    if vpp:
        simds = 4 * pmc.get("cus", 256)
        issue_peak = simds * CLOCK_GHZ * 1e9 / (vpp / 64.0 * VALU_CYC)
        r["issue"] = {"valu_insts_per_point": vpp,
                      "points_per_s_at_issue_rate": round(issue_peak / 1e9, 3),
                      "frac_of_issue_rate": round(points / launches / (avg_ms * 1e-3) / issue_peak, 4),
                      "note": "the measured VALU instruction count per point at one wave64 "
                              "instruction per 2 cycles per SIMD: the instruction-issue ceiling "
                              "of the code as compiled"}
    if tasks:
        # the walk's own unit: one (child, parent) edge per wave at a time, 63-point chunks
        tpl = tasks / launches
        r["tasks"] = {"tasks_per_launch": int(tpl), "points_per_task": round(points / tasks, 2),
                      "tasks_per_s": round(tpl / (avg_ms * 1e-3), 1),
                      "us_per_launch_per_1k_tasks": round(1e3 * avg_ms / max(tpl / 1e3, 1e-9), 3)}
        if vpp:
            r["tasks"]["valu_insts_per_task"] = round(vpp * points / tasks, 1)
    return r


def walk_roofline(sp, pmc, name):
    return fp64_roofline(f"steer_walk ({name})", sp["steer_ms"], sp["steer_launches"],
                         sp.get("walk_points", 0), sp.get("walk_arc_points", 0), pmc,
                         f"HIP events around steer_walk, {sp['steer_launches']} launches of the "
                         "profiled pass (the timed schedule's streams)",
                         tasks=sp.get("walk_tasks", 0))


def finish_roofline(sp):
    """check_finish (goal connection): the optimize candidates' and finalize's edges (steer +
    verify, the same per-point walk) against the FP64 peak.  pp_batch_plan runs it as steer
    rounds, pp_rrt_plan as check_finish_kernel; both end in cf_line_kernel."""
    r = fp64_roofline("check_finish", sp.get("finish_ms", 0.0),
                      sp.get("finish_launches", 0), sp.get("finish_points", 0),
                      sp.get("finish_arc_points", 0), None,
                      "HIP events around the whole check_finish (batch plan: the steer rounds, "
                      "their literal re-runs, assemble, check_finish_kernel on punted items and "
                      "cf_line_kernel; single plan: check_finish_kernel + cf_line_kernel) in a "
                      "profiled run of the same plan")
    if r:
        r["nodes"] = int(sp.get("finish_nodes", 0))
        r["edges"] = int(sp.get("finish_edges", 0))
        r["edges_per_node"] = round(sp.get("finish_edges", 0) / max(sp.get("finish_nodes", 1), 1), 2)
    return r


def window_chain(sp):
    """Per-window device time of each kernel of the window pipeline, µs."""
    w = max(sp["nn_scan_launches"], 1)
    return {"window_kernel": round(1e3 * sp["nn_scan_ms"] / w, 2),
            "nn_finalize": round(1e3 * sp["finalize_ms"] / w, 2),
            "steer_prep": round(1e3 * sp["prep_ms"] / w, 2),
            "steer_walk": round(1e3 * sp["steer_ms"] / w, 2),
            "windows": int(sp["nn_scan_launches"])}


# ------------------------------------------------------------------------- one tree (config 2/4)
def make_planner(raw, seed, window, device, capacity=1 << 18):
    from pathplanning_amd import rrt

    sx, sy, syaw = raw["start"]
    gx, gy, gyaw = raw["goal"]
    return rrt.RRT((sx, sy), syaw, (gx, gy), gyaw, raw["max_iter"], raw["step_size"],
                   rrt.Space.from_raw(raw), seed=seed, window=window, device=device,
                   capacity=capacity)


STAT_KEYS = ("iterations", "accepted", "windows", "truncations", "repair_rounds", "repairs",
             "literal_repairs", "nn_flagged", "samples_blocked")


def timed_windows(p, n_windows, window):
    p.synchronize()
    t0 = time.perf_counter()
    p.extend(n_windows * window)
    p.synchronize()
    return time.perf_counter() - t0


TREE_TAG = {"config2": "", "config4": "_config4", "polygons": "_polygons"}


def run_tree(args, D, raw, workload, with_cpu):
    """Config 2 / 4 / polygons: grow a tree to args.nodes (untimed; windows at ~1k and ~10k nodes
    timed on the way), W warmup windows, then `steps` windows timed back to back, then a profiled
    pass of as many windows (HIP events around every kernel)."""
    steps = args.steps or 20
    p = make_planner(raw, args.seed + D.rank, args.window, D.device)
    sweep = {}
    marks = [] if args.no_size_sweep else [1_000, 10_000]
    while p.tree_size() < args.nodes:
        if marks and p.tree_size() >= marks[0]:
            m = marks.pop(0)
            n0 = p.tree_size()
            p.reset_stats()
            dt = timed_windows(p, 5, args.window)
            st = p.stats()
            sweep[str(m)] = {"iterations_per_s": st["iterations"] / dt, "tree_nodes": n0,
                             "ms_per_window": round(1e3 * dt / max(st["windows"], 1), 4),
                             "stats": {k: st[k] for k in STAT_KEYS}}
        p.extend(args.window)
    p.extend(args.warmup * args.window)
    p.synchronize()
    n_start = p.tree_size()
    p.reset_stats()
    D.barrier()
    p.synchronize()
    t0 = time.perf_counter()
    p.extend(steps * args.window)  # the K steps back to back (windows enqueued without sync)
    p.synchronize()
    t_local = time.perf_counter() - t0
    D.barrier()
    st = p.stats()
    t_max = D.allreduce(t_local, "max")
    iters_total = D.allreduce(st["iterations"], "sum")
    sweep[str(args.nodes)] = {"iterations_per_s": st["iterations"] / t_local,
                              "tree_nodes": n_start,
                              "ms_per_window": round(1e3 * t_local / max(st["windows"], 1), 4),
                              "stats": {k: st[k] for k in STAT_KEYS}}
    p.reset_stats()
    p.set_profiling(True)
    p.extend(steps * args.window)
    p.synchronize()
    p.set_profiling(False)
    sp = p.stats()
    tag = TREE_TAG[workload]
    res = {
        "value": iters_total / t_max, "t_max": t_max, "steps": steps, "n_start": n_start,
        "node_evals_per_s_per_gpu": round(st["node_evals"] / t_local, 1),
        "sizes": sweep, "stats": {k: st[k] for k in STAT_KEYS},
        "roofline": screen_roofline(sp, load_profile(f"window_kernel_pmc{tag}.json")),
        "walk_roofline": walk_roofline(sp, load_profile(f"steer_walk_pmc{tag}.json"), workload),
        "window_chain_us": window_chain(sp),
    }
    if with_cpu:
        res["cpu_baseline"] = cpu_baseline_tree(raw, p, args)
    p.close()
    return res


def cpu_baseline_tree(raw, p, args):
    """The oracle restatement (oracle/, C) on the SAME workload: continue the GPU's tree
    re-verifying the whole line to the root like the reference's verify_node (rrt.rs:414-426):
    one core time-capped (plus the incremental-verify rate beside it), then one independent
    replica per host thread (seed + r) for the per-core rate x cpu_seconds iterations each."""
    oracle = oracle_mod()
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
    t0 = time.perf_counter()
    oracle.extend_replicas(sc, tr, [args.seed + 1000 + r for r in range(threads)], it0, per,
                           threads, full_reverify=True)
    t = time.perf_counter() - t0
    v, nn, tt = out["full_reverify"]
    vi, ni, ti = out["incremental"]
    return {
        "value": round(threads * per / t, 2), "unit": "iterations/s", "cores": threads,
        "kind": "port",
        "sample": f"{threads} independent replicas on {threads} host threads, each continuing the "
                  f"same {n}-node tree ({raw.get('name', 'scene')}) for {per} iterations (seeds "
                  f"{args.seed + 1000}..), re-verifying the whole line to the root like "
                  f"rrt.rs:414-426, exact brute-force NN (the crate's R-tree is rstar, not "
                  f"buildable here); {threads * per} iterations in {t:.1f} s wall",
        "one_core": {"value": round(v, 2), "iterations": nn, "seconds": round(tt, 2)},
        "incremental_verify_one_core": {"value": round(vi, 2), "iterations": ni,
                                        "seconds": round(ti, 2)},
        "host": host_info(),
    }


# --------------------------------------------------------------------- query batches (3 / 5)
def batch_digests(batch, star=False):
    """Per-query 64-bit digest of the tree (x, y bits and parents, root first): equal digests on
    every rank count mean the sharded run built exactly the 1-rank run's trees."""
    n = batch.state()[0]
    out = np.zeros(len(n), dtype=np.int64)
    for q in range(len(n)):
        t = batch.tree(q, int(n[q]))
        h = hashlib.blake2b(digest_size=8)
        h.update(np.ascontiguousarray(t[0]).tobytes())
        h.update(np.ascontiguousarray(t[1]).tobytes())
        h.update(np.ascontiguousarray(t[3]).tobytes())
        out[q] = np.frombuffer(h.digest(), dtype=np.int64)[0]
    return out


def run_batch(args, D, star, with_cpu):
    """Config 3 (star=False) / config 5 (star=True): args.queries independent planners, sharded
    contiguously over the ranks; a step = one lockstep iteration of every query of the rank; the
    timed region is the whole max_iter-step run of a fresh batch after an untimed warmup batch;
    then a profiled pass of the same run, on the same streams (HIP events around every kernel)."""
    from pathplanning_amd import rrt, scenes

    raw = scenes.config5_field() if star else scenes.field512()
    space = rrt.Space.from_raw(raw)
    a, b = shard(args.queries, D.world, D.rank)
    starts, goals, seeds = scenes.config3_queries(raw, a, b - a)
    steps = args.max_iter if args.steps is None else args.steps
    eta = scenes.CONFIG5_ETA

    def fresh():
        if star:
            return rrt.RRTStarBatch(starts, args.max_iter, raw["step_size"], space, seeds, k=0,
                                    eta=eta, device=D.device)
        return rrt.RRTBatch(starts, goals, args.max_iter, raw["step_size"], space, seeds,
                            device=D.device, window=args.batch_window)

    batch = fresh()
    batch.extend(args.warmup)  # untimed warmup on a throwaway run
    batch.close()
    batch = fresh()
    D.barrier()
    t0 = time.perf_counter()
    batch.extend(steps)
    t_local = time.perf_counter() - t0
    D.barrier()
    stt = batch.state()
    n, its = stt[0], stt[1]
    st_timed = batch.stats()
    dig = batch_digests(batch, star)
    cols = [np.arange(a, b, dtype=np.int64), its.astype(np.int64), n.astype(np.int64), dig]
    t_plan = None
    if not star:
        # RRT::plan of every query (check_finish of every accepted node, the first minimum
        # length): the per-query record of SURVEY §8e — (ok, n_nodes, path_len, cost, iterations)
        free0 = device_free_bytes(D.device)
        D.barrier()
        t0 = time.perf_counter()
        pr = batch.plan()
        t_plan_local = time.perf_counter() - t0
        D.barrier()
        # the plan's device reservations (its buffers stay with the batch's context)
        plan_reserved = None if free0 is None else free0 - device_free_bytes(D.device)
        t_plan = D.allreduce(t_plan_local, "max")
        cols += [(pr["best_node"] >= 0).astype(np.int64), pr["best_node"].astype(np.int64),
                 pr["n_points"].astype(np.int64), pr["length"].view(np.int64),
                 pr["n_finishes"].astype(np.int64)]
        checked = int(D.allreduce(pr["checked"], "sum"))
    rec = np.stack(cols, 1)
    allrec = D.gather_records(rec).numpy()
    t_max = D.allreduce(t_local, "max")
    iters_total = int(allrec[:, 1].sum())
    extra = {}
    if not star:
        ok = allrec[:, 4] == 1
        lens = allrec[ok, 7].view(np.float64)
        extra["plan"] = {
            "value": round(iters_total / (t_max + t_plan), 1),
            "unit": "plan_one calls/s (extend + check_finish of every accepted node)",
            "check_finish_ms": round(1e3 * t_plan, 3),
            "extend_ms": round(1e3 * t_max, 3),
            "nodes_checked": checked,
            "check_finish_per_s": round(checked / t_plan, 1) if t_plan > 0 else None,
            "queries_with_path": int(ok.sum()),
            "finishes_total": int(allrec[:, 8].sum()),
            "mean_length": round(float(lens.mean()), 4) if len(lens) else None,
            "device_reserved_mb": None if plan_reserved is None else round(plan_reserved / 2**20, 1),
            "record": "per query: (query, iterations, n_nodes, tree digest, ok, best node, "
                      "path points, length bits, finishes), gathered with the extend records",
        }
    if star:
        extra["rewires_total"] = int(D.allreduce(float(stt[3].sum()), "sum"))
    else:
        ideal = -(-steps // (args.batch_window or auto_batch_window(b - a)))
        extra["passes"] = {"steps": int(st_timed["batch_steps"]),
                           "host_passes": int(st_timed["batch_passes"]), "ideal_steps": ideal}
    # profiled pass (same workload, same streams): HIP events around every kernel of every step
    batch.close()
    batch = fresh()
    batch.set_profiling(True)
    batch.extend(steps)
    sp = batch.stats()
    evals_p = batch.state()[2] if star else batch.state(with_evals=True)[2]
    if not star and not args.pmc_run:
        batch.plan()
        extra["plan"]["roofline"] = finish_roofline(batch.stats())
    batch.close()
    wl = "config5" if star else "config3"
    # the counter passes were taken on one GPU: the whole 8192-query batch, and config 3's
    # 1024-query shard (an 8-GPU rank's share)
    pkey = wl if args.queries == 8192 else f"{wl}_q{args.queries}"
    pmc = load_profile("batch_pmc.json").get(pkey, {}) if D.world == 1 else {}
    evals_total = float(evals_p.sum())
    roof = walk_roofline(sp, pmc.get("steer_walk", {}), wl)
    nn_roof = lockstep_nn_roofline(sp, evals_total, star, pmc)
    res = {
        "value": round(iters_total / t_max, 1),
        "unit": "iterations/s",
        "n_gpus": D.world,
        "scaling": "strong",
        "ms_total": round(1e3 * t_max, 3),
        "steps": steps,
        "queries": args.queries,
        "queries_per_rank": b - a,
        "max_iter": args.max_iter,
        "parallelism": f"query-shard{D.world}",
        "gather": f"all_gather of per-query records ({D.gather_backend or 'none: one rank'})",
        "iterations_total": iters_total,
        "nodes_total": int(allrec[:, 2].sum()),
        "records_digest": hashlib.sha256(allrec.astype(np.int64).tobytes()).hexdigest()[:16],
        "roofline": roof,
        "nn_roofline": nn_roof,
        **extra,
    }
    if not star:
        launches = max(sp["nn_scan_launches"], 1)
        res["schedule"] = "lockstep (four launches per step, two sub-batch streams)"
        res["step_chain_us"] = {"mq_sample_nn": round(1e3 * sp["nn_scan_ms"] / launches, 2),
                                "steer_prep": round(1e3 * sp["prep_ms"] / launches, 2),
                                "steer_walk": round(1e3 * sp["steer_ms"] / launches, 2),
                                "mq_insert": round(1e3 * sp["insert_ms"] / launches, 2),
                                "launches_per_kernel": int(launches),
                                "note": "HIP-event stream spans per launch (the sub-batch streams "
                                        "overlap, so these include the other stream's kernels)"}
    if star:
        res["workload"] = (f"config5 (stretch, build-defined RRT*): {args.queries} queries on "
                           f"{raw['name']} (10240 discs r~U(1,4) on 2048^2), Steer eta {eta}, "
                           f"k = ceil(2e ln n) <= 63, max_iter {args.max_iter}")
    else:
        res["workload"] = (f"config3: {args.queries} independent queries on the config-2 field "
                           f"(query q: seed 42+q, start/goal from stream q), max_iter "
                           f"{args.max_iter}")
        res["window_per_query"] = args.batch_window or auto_batch_window(b - a)
    if with_cpu:
        res["cpu_baseline"] = (cpu_baseline_star(raw, starts, seeds, args.max_iter, eta,
                                                 args.cpu_seconds) if star else
                               cpu_baseline_queries(raw, starts, seeds, args.max_iter,
                                                    args.cpu_seconds))
        if not star:
            res["plan"]["cpu_baseline"] = cpu_baseline_batch_plan(
                raw, starts, goals, seeds, args.max_iter, args.cpu_seconds,
                allrec[:, 5], allrec[:, 7].view(np.float64))
    return res


def lockstep_nn_roofline(sp, evals_total, star, pmc):
    nn_ms = sp["nn_scan_ms"] / max(sp["nn_scan_launches"], 1)
    if nn_ms <= 0:
        return None
    evals_per_launch = evals_total / max(sp["nn_scan_launches"], 1)
    bytes_per_eval = 16  # f64 x + f64 y of one SoA row (exact NN)
    achieved = evals_per_launch * bytes_per_eval / (nn_ms * 1e-3) / 1e9
    nn_share = sp["nn_scan_ms"] / max(sp["nn_scan_ms"] + sp["steer_ms"], 1e-9)
    return {
        "kernel": "star_sample (exact f64 NN)" if star else "mq_sample_nn (exact f64 NN)",
        "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": pmc.get("nn", {}).get("hbm_bytes_per_launch"),
        "avg_launch_ms": round(nn_ms, 5), "evals_per_launch": int(evals_per_launch),
        "bytes_per_eval": bytes_per_eval,
        "share_of_nn_plus_walk_time": round(nn_share, 4),
    }


def cpu_baseline_batch_plan(raw, starts, goals, seeds, max_iter, seconds, best, length):
    """config 3's RRT::plan CPU baseline: the oracle's sequential plan (rrt.rs:599-619, full
    re-verify) of whole queries of the same batch, one after another on one core until
    `seconds` / 2; the answers are compared with the GPU's records."""
    oracle = oracle_mod()
    sc = oracle.OracleScene.from_raw(raw)
    done, t_used, same = 0, 0.0, True
    for q in range(len(seeds)):
        tr = oracle.OracleTree(tuple(starts[q]), max_iter + 1)
        t0 = time.perf_counter()
        _, bn, bl, _ = oracle.plan(sc, tr, int(seeds[q]), 0, max_iter, goals[q][:2], goals[q][2],
                                   full_reverify=True)
        t_used += time.perf_counter() - t0
        same &= bool(bn == best[q] and (bn < 0 or abs(bl - length[q]) <= 1e-9 * bl))
        done += 1
        if t_used >= seconds / 2.0:
            break
    return {"value": round(done * max_iter / t_used, 1),
            "unit": "plan_one calls/s (with check_finish)", "cores": 1, "kind": "port",
            "sample": f"the first {done} queries of the same batch planned in full (extend + "
                      f"check_finish, full re-verify), sequential on one core, "
                      f"{t_used:.1f} s",
            "same_answer": same, "host": host_info()}


def auto_batch_window(q):
    """pp_batch_new's automatic window (round 5): 32, halved while q * K > 262144 tasks."""
    k = 32
    while k > 1 and q * k > 262144:
        k //= 2
    return k


def cpu_baseline_queries(raw, starts, seeds, max_iter, seconds):
    """config 3's CPU baseline: the oracle (C) runs whole queries of the same batch (full
    re-verify of the line to the root, rrt.rs:414-426): first on one core (the per-query time),
    then a batch of them on all host threads, one query per thread at a time (wall clock)."""
    oracle = oracle_mod()
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
    threads = host_threads()
    qn = int(min(len(seeds), max(threads, threads * seconds / (t_used / nq))))
    t0 = time.perf_counter()
    oracle.queries(sc, starts[:qn], seeds[:qn], max_iter, threads, full_reverify=True)
    t = time.perf_counter() - t0
    return {"value": round(qn * max_iter / t, 2), "unit": "iterations/s", "cores": threads,
            "kind": "port",
            "sample": f"the first {qn} whole queries of the same batch ({qn * max_iter} "
                      f"iterations, max_iter {max_iter} each, full re-verify like "
                      f"rrt.rs:414-426) on {threads} host threads, {t:.1f} s wall",
            "one_core": {"value": round(done / t_used, 2), "queries": nq, "iterations": done,
                         "seconds": round(t_used, 2)},
            "host": host_info()}


def cpu_baseline_star(raw, starts, seeds, max_iter, eta, seconds):
    """config 5's CPU baseline: the RRT* oracle (C, orc_star_extend) on the same queries — query
    0 on one core in chunks of 100 iterations until seconds/3 (or max_iter), then `threads` whole
    queries of the batch, each for that many iterations, one per host thread (wall clock)."""
    oracle = oracle_mod()
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
    return {"value": round(threads * done / t, 2), "unit": "iterations/s", "cores": threads,
            "kind": "port",
            "sample": f"the first {threads} queries of the same batch, their first {done} RRT* "
                      f"iterations each ({threads * done} iterations), on {threads} host "
                      f"threads, {t:.1f} s wall",
            "one_core": {"value": round(done / t_used, 2), "iterations": done,
                         "seconds": round(t_used, 2)},
            "host": host_info()}


# ------------------------------------------------------ config 1, plan and the example (bench6)
def dominant_kernel(sp, pmc_tag="", walk_name="walk"):
    """The kernel of the window chain with the largest device time and its algorithmic roofline
    (a short run of small trees is latency-bound: the chain's 4 dependent launches per window)."""
    chain = window_chain(sp)
    times = {k: v for k, v in chain.items() if k != "windows"}
    dom = max(times, key=times.get)
    if dom == "window_kernel":
        r = screen_roofline(sp, {})
    else:
        r = walk_roofline(sp, {}, walk_name) or {}
        r = dict(r)
        if dom != "steer_walk":
            r["note"] = f"{dom} has the largest share; the walk's roofline is shown"
    r["dominant"] = dom
    r["window_chain_us"] = chain
    return r


def run_config1(args, D, with_cpu, polygons=False):
    """BASELINE config 1: the reference's only fully specified scene (benches/all.rs:8-42) —
    8000 plan_one extend iterations (plan_one minus check_finish, rrt.rs:583-589) of one query
    from a fresh tree.  GPU: the whole run per window size K (results identical for every K),
    then a profiled run at the best K; CPU: the C port's sequential run on one core with the
    reference's full re-verify.  polygons: the obstacles as the crate's create_circle polygons
    and the bounds as a ring, the way benches/all.rs:12-28 builds them (Q10p)."""
    from pathplanning_amd import scenes

    raw = scenes.bench6_polygons() if polygons else scenes.bench6()
    n_iter = raw["max_iter"]
    runs = {}
    for K in (32, 128, 512, 4096):
        best = None
        for rep in range(2):  # the first run of a K warms its buffers
            p = make_planner(raw, args.seed, K, D.device, capacity=1 << 14)
            p.synchronize()
            t0 = time.perf_counter()
            acc = p.extend(n_iter)
            p.synchronize()
            dt = time.perf_counter() - t0
            st = p.stats()
            p.close()
            if rep == 1:
                best = {"iterations_per_s": round(n_iter / dt, 1), "ms": round(1e3 * dt, 3),
                        "nodes": acc + 1, "stats": {k: st[k] for k in STAT_KEYS}}
        runs[str(K)] = best
    kbest = max(runs, key=lambda k: runs[k]["iterations_per_s"])
    p = make_planner(raw, args.seed, int(kbest), D.device, capacity=1 << 14)
    p.set_profiling(True)
    p.extend(n_iter)
    p.synchronize()
    sp = p.stats()
    p.close()
    name = "config1_polygons" if polygons else "config1"
    geom = ("create_circle polygons + ring bounds, exact Minkowski buffers (Q10p)" if polygons
            else "analytic discs r + w/2 (Q10)")
    res = {"value": runs[kbest]["iterations_per_s"], "unit": "iterations/s", "window": int(kbest),
           "workload": f"{name}: bench6 (benches/all.rs:8-42: 6 obstacles, R 0.8, step 0.1; "
                       f"{geom}), seed {args.seed}, {n_iter} iterations from the root",
           "per_window": runs,
           "roofline": dominant_kernel(sp, walk_name=name)}
    if with_cpu:
        oracle = oracle_mod()
        sc = oracle.OracleScene.from_raw(raw)
        tr = oracle.OracleTree(raw["start"], n_iter + 1)
        t0 = time.perf_counter()
        acc, _, _ = oracle.rrt_extend(sc, tr, args.seed, 0, n_iter, full_reverify=True)
        t = time.perf_counter() - t0
        res["cpu_baseline"] = {
            "value": round(n_iter / t, 1), "unit": "iterations/s", "cores": 1, "kind": "port",
            "sample": f"the same {n_iter} iterations (seed {args.seed}), sequential, full "
                      f"re-verify (rrt.rs:414-426), {t:.2f} s; {acc + 1} nodes like the GPU",
            "nodes": acc + 1}
    return res


def run_plan(args, D, with_cpu, example=False):
    """RRT::plan (rrt.rs:599-619), sequential spec: 8000 plan_one iterations with check_finish
    (optimize + finalize + verify, rrt.rs:428-540) on every accepted node, the first minimum
    euclidean_length.  GPU pp_rrt_plan (two runs, the second timed; then a profiled run for the
    check_finish_kernel roofline) against the C port's plan on one core.  example: the scene of
    examples/rrt (transit.debug.json, Robot::new(1.8, 3.0, 0.8), RRT::new(.., 8000, 0.1, ..),
    examples/rrt/src/main.rs:44-75) instead of bench6_open."""
    from pathplanning_amd import scenes

    raw = scenes.transit() if example else scenes.bench6_open()
    n_iter = raw["max_iter"]
    best = None
    for rep in range(2):
        p = make_planner(raw, args.seed, 512, D.device, capacity=1 << 14)
        p.synchronize()
        t0 = time.perf_counter()
        line = p.plan(n_iter)
        dt = time.perf_counter() - t0
        bn, bl, nf = p.last_plan
        # the check_finish share: the same nodes' check_finish batch on its own
        nodes = np.arange(1, p.tree_size(), dtype=np.int32)
        t1 = time.perf_counter()
        p.check_finish_batch(nodes)
        dcf = time.perf_counter() - t1
        p.close()
        best = {"plan_calls_per_s": round(n_iter / dt, 1), "ms": round(1e3 * dt, 3),
                "best_node": bn, "best_length": bl, "finishes": nf,
                "line_points": 0 if line is None else len(line),
                "check_finish_nodes": len(nodes),
                "check_finish_ms": round(1e3 * dcf, 3),
                "check_finish_per_s": round(len(nodes) / dcf, 1)}
    p = make_planner(raw, args.seed, 512, D.device, capacity=1 << 14)
    p.set_profiling(True)
    p.plan(n_iter)
    sp = p.stats()
    p.close()
    scene = ("examples/rrt: transit.debug.json (20-vertex bounds ring, 3 polygon obstacles), "
             "Robot(1.8, 3.0, 0.8)" if example else
             "bench6_open (bench6 scene, start (-3, -3, 45 deg))")
    res = {"value": best["plan_calls_per_s"], "unit": "plan_one calls/s (with check_finish)",
           "workload": f"{'example_rrt' if example else 'plan'}: {scene}, seed {args.seed}, "
                       f"RRT::plan with {n_iter} iterations", **best,
           "roofline": finish_roofline(sp),
           "extend_window_chain_us": window_chain(sp)}
    if with_cpu:
        oracle = oracle_mod()
        sc = oracle.OracleScene.from_raw(raw)
        tr = oracle.OracleTree(raw["start"], n_iter + 1)
        t0 = time.perf_counter()
        acc, obn, obl, _ = oracle.plan(sc, tr, args.seed, 0, n_iter, raw["goal"][:2],
                                       raw["goal"][2], full_reverify=True)
        t = time.perf_counter() - t0
        res["cpu_baseline"] = {
            "value": round(n_iter / t, 1), "unit": "plan_one calls/s", "cores": 1,
            "kind": "port",
            "sample": f"the same plan (seed {args.seed}, {n_iter} iterations, full re-verify), "
                      f"sequential, {t:.2f} s; best node {obn}, length {obl:.6f}",
            "same_answer": bool(obn == best["best_node"] and
                                (obn < 0 or abs(obl - best["best_length"])
                                 <= 1e-9 * max(1.0, abs(obl))))}
    return res


# ---------------------------------------------------------------------------------- main
def strict(v):
    """`v` with every non-finite float (a plan with no finish has length inf) mapped to None and
    numpy scalars to Python ones, so the line is RFC 8259 JSON (no Infinity / NaN tokens)."""
    if isinstance(v, dict):
        return {str(k): strict(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [strict(x) for x in v]
    if isinstance(v, np.generic):
        v = v.item()
    if isinstance(v, float) and not np.isfinite(v):
        return None
    return v


def _reject_constant(tok):
    raise ValueError(f"non-standard JSON constant {tok!r} in the bench line")


def line_json(line):
    """The one JSON line: strict (allow_nan=False), and checked by parsing it back with every
    non-standard constant refused — the driver's parser must read exactly this."""
    s = json.dumps(strict(line), allow_nan=False)
    json.loads(s, parse_constant=_reject_constant)
    return s


# The driver reads the LAST stdout line out of an ~8 KB tail that also holds stderr: rounds 3-4's
# 22-23 KB lines were never parsed.  The full record goes to a side file (--detail) and stdout gets
# a compact line of at most LINE_MAX bytes.
LINE_MAX = 4096
SUB_KEYS = ("config3", "config5", "config4", "polygons", "config1", "config1_polygons", "plan",
            "example_rrt")
SHORT_WL = {"config3": "8192 queries, field512, max_iter 2000, sharded (strong)",
            "config5": "RRT* 8192 queries, 10240 discs, max_iter 2000 (stretch)",
            "config4": "config2 on a 512x512 occupancy bitmap, 100k nodes",
            "polygons": "config2 with create_circle polygons, 100k nodes",
            "config1": "bench6 (benches/all.rs), 8000 iterations, discs",
            "config1_polygons": "bench6, 8000 iterations, create_circle polygons",
            "plan": "RRT::plan on bench6_open, 8000 iterations",
            "example_rrt": "examples/rrt RRT::plan (transit.debug.json), 8000 iterations"}


def _pick(d, keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def _short_roofline(r):
    out = _pick(r or {}, ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic",
                          "avg_launch_ms"))
    if isinstance(out.get("kernel"), str):
        out["kernel"] = out["kernel"].split(" (NN screen")[0][:40]
    return out or None


def _short_cpu(c, sample_len=120):
    if not isinstance(c, dict):
        return None
    out = _pick(c, ("value", "unit", "cores", "kind", "same_answer"))
    out["cores_visible"] = os.cpu_count()
    if isinstance(c.get("sample"), str):
        out["sample"] = c["sample"][:sample_len]
    return out


def _short_sub(name, r):
    if not isinstance(r, dict):
        return None
    if "error" in r:
        return {"error": str(r["error"])[:200]}
    roof = r.get("roofline") or {}
    s = {"value": r.get("value"), "unit": r.get("unit"), "workload": SHORT_WL.get(name, name),
         "frac": roof.get("frac"), "kernel": (roof.get("kernel") or "").split(" (")[0][:28] or None}
    cpu = r.get("cpu_baseline")
    if isinstance(cpu, dict):
        s["cpu"] = cpu.get("value")
        s["cpu_cores"] = cpu.get("cores")
        if "same_answer" in cpu:
            s["same_answer"] = cpu["same_answer"]
    for k in ("records_digest", "best_length", "check_finish_ms", "n_gpus"):
        if k in r:
            s[k] = r[k]
    if isinstance(r.get("plan"), dict):  # config 3's batch RRT::plan
        pl = r["plan"]
        s["plan"] = {"value": pl.get("value"), "check_finish_ms": pl.get("check_finish_ms"),
                     "device_reserved_mb": pl.get("device_reserved_mb"),
                     "cpu_same_answer": (pl.get("cpu_baseline") or {}).get("same_answer")}
    if isinstance(r.get("passes"), dict):
        s["steps"] = r["passes"].get("steps")
    return s


def compact_line(line, detail_path=None, with_subs=True):
    """The stdout line: the contract's headline keys, the dominant kernel's roofline, the CPU
    baseline and one short record per sub-result (value, roofline frac, CPU value, same answer /
    records digest); the rest of `line` is in the detail file.  Strict JSON, <= LINE_MAX bytes."""
    head = _pick(line, ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                        "higher_is_better", "scaling", "vs_baseline", "dtype", "data"))
    cfg = dict(line.get("config") or {})
    if isinstance(cfg.get("workload"), str):
        cfg["workload"] = cfg["workload"][:160]
    cfg.pop("nn_screen_dtype", None)
    head["config"] = cfg
    head["roofline"] = _short_roofline(line.get("roofline"))
    head["cpu_baseline"] = _short_cpu(line.get("cpu_baseline"))
    for k in ("node_evals_per_s_per_gpu", "records_digest", "iterations_total", "nodes_total",
              "rewires_total", "window_per_query", "passes", "best_length", "check_finish_ms",
              "same_answer"):
        if k in line:
            head[k] = line[k]
    if not with_subs and "records_digest" in line and isinstance(line.get("plan"), dict):
        pl = line["plan"]  # a config-3 line's batch RRT::plan
        head["plan"] = {"value": pl.get("value"), "check_finish_ms": pl.get("check_finish_ms"),
                        "device_reserved_mb": pl.get("device_reserved_mb"),
                        "frac": (pl.get("roofline") or {}).get("frac"),
                        "cpu_same_answer": (pl.get("cpu_baseline") or {}).get("same_answer")}
    if not with_subs:  # a batch workload line: its step chain and NN roofline
        sc = line.get("step_chain_us")
        if isinstance(sc, dict):
            head["step_chain_us"] = {k: v for k, v in sc.items() if k != "note"}
        if isinstance(line.get("nn_roofline"), dict):
            head["nn_roofline"] = _short_roofline(line["nn_roofline"])
    st = line.get("stats")
    if isinstance(st, dict) and st.get("iterations"):
        head["samples_blocked_frac"] = round(st.get("samples_blocked", 0) / st["iterations"], 4)
    wc = line.get("window_chain_us")
    if isinstance(wc, dict):
        head["window_chain_us"] = {k: v for k, v in wc.items() if k != "windows"}
    subs = {k: _short_sub(k, line[k]) for k in SUB_KEYS if with_subs and k in line}
    if subs:
        head["sub"] = subs
    if isinstance(line.get("strong_scaling"), dict):
        head["strong_scaling"] = _pick(line["strong_scaling"], ("workload", "value", "n_gpus",
                                                                 "records_digest"))
    prov = line.get("provenance") or {}
    head["lib_sha256_16"] = prov.get("lib_sha256_16")
    if detail_path:
        head["detail"] = os.path.relpath(detail_path, ROOT)
    s = line_json(head)
    # over the cap (long error texts, many sub-results): shed the least important fields first
    for drop in (("sub", "workload"), ("cpu_baseline", "sample"), ("sub", "kernel"),
                 ("config", "workload")):
        if len(s.encode()) <= LINE_MAX:
            break
        if drop[0] == "sub":
            for v in head.get("sub", {}).values():
                if isinstance(v, dict):
                    v.pop(drop[1], None)
        elif isinstance(head.get(drop[0]), dict):
            head[drop[0]].pop(drop[1], None)
        s = line_json(head)
    if len(s.encode()) > LINE_MAX:
        head.pop("sub", None)
        head["sub_dropped"] = "over the line cap: see the detail file"
        s = line_json(head)
    return s


def write_detail(path, s):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        f.write(s + "\n")


def tree_line(args, D, workload, raw, res):
    wl = {"config4": "config4: field512 rasterised to a 512x512 bit-packed occupancy grid "
                     "(32 KB, point probes)",
          "polygons": "polygons: field512's 1024 discs as create_circle polygons "
                      f"({sum(len(o) for o in raw.get('obstacle_polygons', []))} edges, "
                      "Minkowski buffers, SURVEY §8f row 3)"}.get(
        workload, "config2: field512 (1024 discs r~U(2,8), 512x512)")
    return {
        "metric": METRIC,
        "value": round(res["value"], 1),
        "unit": "iterations/s",
        "n_gpus": D.world,
        "steps": res["steps"],
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * res["t_max"] / res["steps"], 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": wl + f", R=4.0, step 0.1, K={args.window} candidates/window, tree grown "
                             f"to {args.nodes} nodes",
            "window": args.window,
            "tree_nodes_at_start": res["n_start"],
            "obstacles": len(raw.get("obstacle_polygons", raw["circles"])),
            "parallelism": f"replicas{D.world}",
            "nn_screen_dtype": "f32 (exact f64 rescan of near-ties)",
        },
        "node_evals_per_s_per_gpu": res["node_evals_per_s_per_gpu"],
        "sizes": res["sizes"],
        "stats": res["stats"],
        "roofline": res["roofline"],
        "walk_roofline": res["walk_roofline"],
        "window_chain_us": res["window_chain_us"],
        "cpu_baseline": res.get("cpu_baseline"),
    }


def batch_line(args, D, res, star):
    line = {
        "metric": ("RRT* iterations/sec (SE(2) Dubins, k-nearest rewire, 10k obstacles)" if star
                   else METRIC),
        "value": res["value"], "unit": "iterations/s", "n_gpus": D.world, "steps": res["steps"],
        "warmup": args.warmup, "ms_per_step": round(res["ms_total"] / res["steps"], 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": res["workload"], "queries": res["queries"],
                   "queries_per_rank": res["queries_per_rank"],
                   "parallelism": res["parallelism"], "gather": res["gather"]},
    }
    line.update({k: v for k, v in res.items() if k not in line and k not in (
        "workload", "queries", "queries_per_rank", "parallelism", "gather", "steps", "ms_total")})
    line.setdefault("cpu_baseline", None)
    return line


def sub(D, fn, *a):
    """A sub-result: its dict, or the error that stopped it (the headline line still prints).
    With several ranks a failure is raised instead: a rank that skipped a collective the others
    entered would leave them waiting (spawn_ranks then ends the run)."""
    try:
        return fn(*a)
    except Exception as e:  # noqa: BLE001 — reported in the line, never hidden
        if D.world > 1:
            raise
        return {"error": f"{type(e).__name__}: {e}"}


def tree_sub(args, D, raw, workload, cpu):
    ta = argparse.Namespace(**vars(args))
    ta.no_size_sweep = True
    res = {k: v for k, v in run_tree(ta, D, raw, workload, cpu).items()
           if k not in ("sizes", "t_max")}
    res.setdefault("unit", "iterations/s")
    return res


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(args.gpus)
    D = Dist(args)
    prov = provenance(args)
    cpu = D.rank == 0 and D.world == 1 and not args.no_cpu_baseline
    from pathplanning_amd import scenes

    wl = args.workload
    if wl in ("default", "config2", "config4", "polygons"):
        tw = "config2" if wl == "default" else wl
        raw = {"config4": scenes.field512_grid, "polygons": scenes.field512_polygons}.get(
            tw, scenes.field512)()
        line = tree_line(args, D, tw, raw, run_tree(args, D, raw, tw, cpu))
        if wl == "default" and not args.no_sub:
            sa = argparse.Namespace(**vars(args))
            sa.steps = None  # the batches run their whole max_iter
            line["config3"] = sub(D, run_batch, sa, D, False, cpu)
            line["config5"] = sub(D, run_batch, sa, D, True, cpu)
            if D.world == 1:
                line["config4"] = sub(D, tree_sub, args, D, scenes.field512_grid(), "config4", cpu)
                line["polygons"] = sub(D, tree_sub, args, D, scenes.field512_polygons(),
                                       "polygons", cpu)
                line["config1"] = sub(D, run_config1, args, D, cpu)
                line["config1_polygons"] = sub(D, run_config1, args, D, cpu, True)
                line["plan"] = sub(D, run_plan, args, D, cpu)
                line["example_rrt"] = sub(D, run_plan, args, D, cpu, True)
    elif wl in ("config3", "config5"):
        line = batch_line(args, D, run_batch(args, D, wl == "config5", cpu), wl == "config5")
    elif wl in ("config1", "config1_polygons"):
        res = run_config1(args, D, cpu, wl == "config1_polygons")
        line = {"metric": METRIC, "n_gpus": D.world, "steps": 1, "warmup": 1,
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
                "data": "synthetic", **res}
    else:  # plan / example_rrt
        res = run_plan(args, D, cpu, wl == "example_rrt")
        line = {"metric": "RRT::plan calls/sec (plan_one with check_finish)",
                "n_gpus": D.world, "steps": 1, "warmup": 1, "higher_is_better": True,
                "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
                **res}
    line["provenance"] = prov
    if wl == "default" and isinstance(line.get("config3"), dict) and "value" in line["config3"]:
        # `value` is config 2's replica (weak-scaling) rate; the sharded-query rate the north
        # star's 8-GPU target is quoted on sits beside it
        line["strong_scaling"] = {"workload": "config3", "value": line["config3"]["value"],
                                  "unit": "iterations/s", "n_gpus": D.world,
                                  "scaling": "strong",
                                  "records_digest": line["config3"].get("records_digest")}
    if D.rank == 0:
        detail = os.path.abspath(args.detail)
        write_detail(detail, line_json(line))
        print(compact_line(line, detail, wl == "default"), flush=True)
    D.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
