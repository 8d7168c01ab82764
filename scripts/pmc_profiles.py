"""Summarise scripts/gpu_pmc.sh (gpurun_out/<tag>/) into the committed counter profiles the
bench reads for its rooflines:

  profiles/window_kernel_pmc.json          config 2 NN screen: VALU instructions per eval, HBM bytes
  profiles/window_kernel_pmc_config4.json  the same on the occupancy-grid workload
  profiles/steer_walk_pmc.json             config 2 walk: VALU instructions per walked point, bytes
  profiles/steer_walk_pmc_config4.json
  profiles/batch_pmc.json                  config 3 / 5: steer_walk and the batch NN kernel

Only the profiled pass's dispatches count (the last N launches of the kernel, N from the bench line
of the same workload; a run's dispatch order is deterministic), the one-workgroup drain launches
of window_kernel excluded.  HBM bytes = FETCH_SIZE x 2 (the gfx950 correction of
MI355X_MICROARCH.md §HBM: wide reads tallied at half) + WRITE_SIZE, KB -> bytes."""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc2")
PROF = os.path.join(ROOT, "profiles")


def dispatches(job, kernel):
    path = None
    for d, _, files in os.walk(os.path.join(SRC, job)):
        for f in files:
            if f.endswith("counter_collection.csv"):
                path = os.path.join(d, f)
    if path is None:
        return []
    per = defaultdict(lambda: defaultdict(float))
    meta = {}
    for r in csv.DictReader(open(path)):
        if kernel not in r["Kernel_Name"]:
            continue
        if int(r["Grid_Size"]) <= int(r["Workgroup_Size"]):
            continue  # window_kernel's drain launch
        k = int(r["Dispatch_Id"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[k] = int(r["Grid_Size"]) // int(r["Workgroup_Size"])
    return [(k, meta[k], dict(per[k])) for k in sorted(per)]


def avg(job, kernel, last):
    ds = dispatches(job, kernel)[-last:]
    if not ds:
        return None, 0, 0
    keys = set().union(*(d[2] for d in ds))
    return {c: sum(d[2].get(c, 0.0) for d in ds) / len(ds) for c in keys}, len(ds), ds[-1][1]


def line(wl):
    """The workload's full bench record (--detail; the stdout line is the compact one)."""
    path = os.path.join(SRC, f"detail_{wl}.json")
    if not os.path.exists(path):
        path = os.path.join(SRC, f"bench_{wl}.json")
    with open(path) as f:
        return json.load(f)


def traffic(prefix, kernel, last):
    f, _, _ = avg(prefix + "_F", kernel, last)
    w, _, _ = avg(prefix + "_W", kernel, last)
    if not f or not w:
        return {}
    fk, wk = f.get("FETCH_SIZE", 0.0), w.get("WRITE_SIZE", 0.0)
    return {"fetch_size_kb_per_launch": round(fk, 1), "write_size_kb_per_launch": round(wk, 1),
            "hbm_bytes_per_launch": int(round((2 * fk + wk) * 1024))}


def sq(prefix, kernel, last, per_unit, unit):
    a, n, grid = avg(prefix + "_A", kernel, last)
    b, _, _ = avg(prefix + "_B", kernel, last)
    out = {"dispatches": n, "grid_workgroups": grid}
    if a:
        out["counters"] = {k: round(v, 1) for k, v in sorted(a.items())}
        out[f"valu_insts_per_{unit}"] = round(a["SQ_INSTS_VALU"] * 64.0 / per_unit, 4)
        out["valu_insts_per_wave"] = round(a["SQ_INSTS_VALU"] / max(a["SQ_WAVES"], 1), 1)
    if b:
        out["counters_b"] = {k: round(v, 1) for k, v in sorted(b.items())}
        wc = max(b["SQ_WAVE_CYCLES"], 1.0)
        out["valu_busy"] = round(b["SQ_ACTIVE_INST_VALU"] / wc, 4)
        out["wait_frac"] = round(b["SQ_WAIT_ANY"] / wc, 4)
        out["issue_stall_frac"] = round(b["SQ_WAIT_INST_ANY"] / wc, 4)
        out["lds_stall_frac"] = round(b["SQ_WAIT_INST_LDS"] / wc, 4)
    return out


def write(name, d):
    with open(os.path.join(PROF, name), "w") as f:
        json.dump(d, f, indent=1)
    print(name, json.dumps({k: v for k, v in d.items() if not k.startswith("counters")}))


NOTE = ("rocprofv3 --pmc passes (scripts/gpu_pmc.sh), the profiled pass's dispatches only; "
        "valu_insts_* = SQ_INSTS_VALU x 64 lanes per unit; valu_busy = SQ_ACTIVE_INST_VALU / "
        "SQ_WAVE_CYCLES (per wave), wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES; HBM bytes = "
        "FETCH_SIZE x 2 + WRITE_SIZE (MI355X_MICROARCH.md §HBM)")
for wl, tag in (("config2", ""), ("config4", "_config4")):
    if not os.path.exists(os.path.join(SRC, f"bench_{wl}.json")):
        continue
    L = line(wl)
    r, w = L["roofline"], L.get("walk_roofline") or {}
    pre = "c2" if wl == "config2" else "c4"
    d = sq(pre + "_win", "window_kernel", r["launches"], r["evals_per_launch"], "eval")
    d.update(traffic(pre + "_win", "window_kernel", r["launches"]))
    d.update(workload=wl, evals_per_launch=r["evals_per_launch"], note=NOTE,
             screen_cus=d.get("grid_workgroups", 249) - 1,
             lib_sha256_16=L.get("provenance", {}).get("lib_sha256_16"))
    write(f"window_kernel_pmc{tag}.json", d)
    if w:
        d = sq(pre + "_walk", "steer_walk", w["launches"], w["points_per_launch"], "point")
        d.update(traffic(pre + "_walk", "steer_walk", w["launches"]))
        d.update(workload=wl, points_per_launch=w["points_per_launch"], note=NOTE, cus=256,
                 lib_sha256_16=L.get("provenance", {}).get("lib_sha256_16"))
        write(f"steer_walk_pmc{tag}.json", d)
# (keys this pass did not measure keep their earlier record; each names its library)
_bp = os.path.join(PROF, "batch_pmc.json")
batch = json.load(open(_bp)) if os.path.exists(_bp) else {}
_new = False
for wl, pre, nn, key in (("config3", "c3", "mq_sample_nn", "config3"),
                         ("config3s", "c3s", "mq_sample_nn", "config3_q1024"),
                         ("config5", "c5", "star_sample", "config5")):
    if not os.path.exists(os.path.join(SRC, f"bench_{wl}.json")):
        continue
    _new = True
    L = line(wl)
    w, n = L["roofline"], L["nn_roofline"]
    d = sq(pre + "_walk", "steer_walk", w["launches"], w["points_per_launch"], "point")
    d.update(traffic(pre + "_walk", "steer_walk", w["launches"]))
    d.update(points_per_launch=w["points_per_launch"], cus=256, note=NOTE,
             lib_sha256_16=L.get("provenance", {}).get("lib_sha256_16"))
    nl = w["launches"] // (3 if wl == "config5" else 1)  # one NN launch per step
    batch[key] = {"steer_walk": d, "nn": dict(kernel=nn, **traffic(pre + "_nn", nn, nl))}
if _new:
    write("batch_pmc.json", batch)
