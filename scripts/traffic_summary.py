"""Summarise the batch-NN rocprofv3 counter passes of scripts/gpu_traffic_batch.sh into
profiles/batch_nn_traffic.json: HBM bytes per dispatch of mq_sample_nn (config 3) and star_sample
(config 5) = FETCH_SIZE x 2 (the gfx950 correction of MI355X_MICROARCH.md, HBM section; these
kernels load 8 B per lane, a width the guide leaves uncalibrated) + WRITE_SIZE."""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "traffic")


def per_dispatch(path, kernel):
    per = defaultdict(float)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
    v = list(per.values())
    return sum(v) / max(len(v), 1), len(v)


out = {}
for workload, kernel in (("config3", "mq_sample_nn"), ("config5", "star_sample")):
    f, nf = per_dispatch(os.path.join(SRC, f"{workload}_FETCH_SIZE", "run_counter_collection.csv"),
                         kernel)
    w, _ = per_dispatch(os.path.join(SRC, f"{workload}_WRITE_SIZE", "run_counter_collection.csv"),
                        kernel)
    out[workload] = {
        "kernel": kernel,
        "dispatches": nf,
        "fetch_size_kb_per_launch": round(f, 1),
        "write_size_kb_per_launch": round(w, 1),
        "hbm_bytes_per_launch": int(round((2 * f + w) * 1024)),
        "note": "whole-batch launches (PP_BATCH_STREAMS=1), averaged over every dispatch of the "
                "run (warmup, timed and profiled passes); FETCH_SIZE doubled per the guide's "
                "gfx950 correction, uncalibrated for 8-B loads",
    }
print(json.dumps(out, indent=1))
with open(os.path.join(ROOT, "profiles", "batch_nn_traffic.json"), "w") as fh:
    json.dump(out, fh, indent=1)
