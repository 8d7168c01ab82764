"""Per-kernel averages of the counters in gpurun_out/pmc over the last N dispatches of each kernel
(the timed 100k-node windows of the default bench)."""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
last = int(sys.argv[2]) if len(sys.argv) > 2 else 20
per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
for path in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("ppamd::", "")
        per[(k, int(r["Dispatch_Id"]), os.path.dirname(path))][r["Counter_Name"]] += float(r["Counter_Value"])
kern = defaultdict(list)
for (k, d, pth), c in per.items():
    kern[(k, pth)].append((d, c))
agg = defaultdict(lambda: defaultdict(list))
for (k, pth), lst in kern.items():
    lst.sort()
    for d, c in lst[-last:]:
        for name, v in c.items():
            agg[k][name].append(v)
for k in sorted(agg):
    a = {n: sum(v) / len(v) for n, v in agg[k].items()}
    print(k + ": " + "  ".join(f"{n}={a[n]:.0f}" for n in sorted(a)))
