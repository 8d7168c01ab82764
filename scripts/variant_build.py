"""Build an A/B variant of the library from text substitutions on a copy of the sources (the
product sources are untouched): rs-pathplanning_amd/lib/<name>/libpathplanning_amd.so, for
scripts/gpu_ab.sh (VARIANTS=<name>).

  python scripts/variant_build.py NAME FILE 'old' 'new' [FILE 'old' 'new' ...]

Each substitution must match exactly once."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "rs-pathplanning_amd", "csrc")


def build(name, subs):
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge

    bdir = os.path.join(ROOT, "build", "variant_" + name)
    shutil.rmtree(bdir, ignore_errors=True)
    csrc = os.path.join(bdir, "pkg", "csrc")
    os.makedirs(csrc)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(bdir, "include"))
    for f in ge.SOURCES + ge.HEADERS:
        shutil.copy(os.path.join(SRC, f), csrc)
    for fname, a, b in subs:
        p = os.path.join(csrc, fname)
        s = open(p).read()
        assert s.count(a) == 1, (fname, a, s.count(a))
        open(p, "w").write(s.replace(a, b))
    out = os.path.join(ROOT, "rs-pathplanning_amd", "lib", name, "libpathplanning_amd.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = ["/opt/rocm/bin/hipcc", *ge.HIPCC_FLAGS, "-o", out] + [os.path.join(csrc, f) for f in ge.SOURCES]
    subprocess.run(cmd, check=True)
    print(out)


if __name__ == "__main__":
    args = sys.argv[2:]
    assert len(args) % 3 == 0, "FILE 'old' 'new' triples"
    build(sys.argv[1], [tuple(args[i:i + 3]) for i in range(0, len(args), 3)])
