"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/.../run_counter_collection.csv): the
average per dispatch of every counter for one kernel, plus derived clock / VALU-utilisation."""
import csv
import glob
import os
import sys
from collections import defaultdict

out, kern = sys.argv[1], sys.argv[2]
vals = defaultdict(list)
for path in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    per = defaultdict(float)
    for r in csv.DictReader(open(path)):
        if kern not in r["Kernel_Name"]:
            continue
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        vals[c].append(v)
avg = {c: sum(v) / len(v) for c, v in vals.items()}
for c in sorted(avg):
    print(f"{c:24s} {avg[c]:16.1f}  (n={len(vals[c])})")
try:
    print("VALU instr per wave      %.1f" % (avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"]))
    print("active VALU / busy (SQ)  %.3f" % (avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_BUSY_CYCLES"]))
    print("wait-any / wave-cycles   %.3f" % (avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"]))
    print("wait-inst / wave-cycles  %.3f" % (avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"]))
except KeyError as e:
    print("missing", e)
