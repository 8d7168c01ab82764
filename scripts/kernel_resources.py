"""Register / scratch / occupancy of every kernel of pp_kernels.hip for gfx950, from the
compiler's kernel-resource-usage remarks (no GPU needed): the spill check behind DESIGN.md §3.2.

  python scripts/kernel_resources.py [name-substring ...]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def resources(src=os.path.join(ROOT, "rs-pathplanning_amd", "csrc", "pp_kernels.hip")):
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                            "-ffp-contract=off", "-c", "--cuda-device-only",
                            "-Rpass-analysis=kernel-resource-usage", src, "-o",
                            os.path.join(d, "k.o")], capture_output=True, text=True, check=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        for key, tag in (("VGPRs", "vgpr"), ("SGPRs", "sgpr"),
                         (r"ScratchSize \[bytes/lane\]", "scratch"),
                         (r"Occupancy \[waves/SIMD\]", "occupancy")):
            m = re.search(key + r": (\d+)", line)
            if m and cur is not None:
                cur[tag] = int(m.group(1))
    names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows),
                           capture_output=True, text=True).stdout.splitlines()
    for r, n in zip(rows, names):
        r["name"] = n.replace("ppamd::", "").split("(")[0]
    return rows


if __name__ == "__main__":
    pats = sys.argv[1:]
    for r in resources():
        if not pats or any(p in r["name"] for p in pats):
            print(f"{r.get('vgpr', 0):4d} v {r.get('sgpr', 0):4d} s {r.get('scratch', 0):4d} B "
                  f"occ {r.get('occupancy', 0)}  {r['name']}")
