"""Diagnostic build (never the product): per-workgroup timeline of every steer_walk launch.

  python scripts/diag_walk_timeline.py build    # -> rs-pathplanning_amd/lib/walktl/libpathplanning_amd.so
  PP_AMD_LIB=.../walktl/libpathplanning_amd.so PP_DIAG_OUT=out.bin python bench.py ... --allow-variant-lib
  python scripts/diag_walk_timeline.py report out.bin

Each walk workgroup writes one 64-byte record with plain vector stores into a device buffer (its
slot from one global atomic per workgroup): its entry, scene-staged and exit times on the 100 MHz
constant clock (s_memrealtime), its block index, grid, the sub-batch's DevState address, the task
count and how many tasks it walked.  pp_batch_extend appends the buffer to PP_DIAG_OUT per call.
The report splits the records into launches (per DevState, a repeated block index starts the next
launch) and prints, per launch size class, the launch span, the dispatch ramp (last workgroup
entry - first), the staging time, the task phase and where the last workgroup finished.
The patches are applied to a copy of the sources under build/; the product sources are untouched."""
import os
import shutil
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "rs-pathplanning_amd", "csrc")
OUTLIB = os.path.join(ROOT, "rs-pathplanning_amd", "lib", "walktl", "libpathplanning_amd.so")
BUILD = os.path.join(ROOT, "build", "walktl")
CAP = 1 << 19  # records

KERNEL_DECL = r"""
// ---- diagnostic timeline (scripts/diag_walk_timeline.py) ----
__device__ unsigned long long* g_tl;
__device__ unsigned int g_tl_n;
extern "C" void pptl_setup(void* buf) {
    const unsigned z = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tl), &buf, sizeof buf);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tl_n), &z, sizeof z);
}
extern "C" unsigned pptl_count() {
    unsigned n = 0;
    (void)hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_tl_n), sizeof n);
    return n;
}
"""

PATCHES_K = [
    ("extern __shared__ __attribute__((aligned(16))) char pp_smem[];",
     "extern __shared__ __attribute__((aligned(16))) char pp_smem[];\n" + KERNEL_DECL),
    ("""    const bool t0 = threadIdx.x == 0;
    if (kLds) stage_scene(sc);""",
     """    const bool t0 = threadIdx.x == 0;
    const unsigned long long tl_in = __builtin_amdgcn_s_memrealtime();
    if (kLds) stage_scene(sc);
    __syncthreads();
    const unsigned long long tl_st = __builtin_amdgcn_s_memrealtime();
    __shared__ int s_tl_tasks;
    if (t0) s_tl_tasks = 0;"""),
    ("""        ++ntasks;
        if (lane == 0) {
            if (al || t < W) {""",
     """        ++ntasks;
        if (lane == 0) atomicAdd(&s_tl_tasks, 1);
        if (lane == 0) {
            if (al || t < W) {"""),
    ("""    if (wg_points) {  // [b]: points, [kWalkTallySlots + b]: their arc points, [2 kWalkTallySlots + b]: tasks""",
     """    __syncthreads();
    if (g_tl && t0) {
        const unsigned slot = atomicAdd(&g_tl_n, 1u);
        if (slot < %d) {
            unsigned long long* r = g_tl + 8 * (size_t)slot;
            r[0] = tl_in;
            r[1] = tl_st;
            r[2] = __builtin_amdgcn_s_memrealtime();
            r[3] = (unsigned long long)blockIdx.x | ((unsigned long long)gridDim.x << 32);
            r[4] = (unsigned long long)(size_t)st;
            r[5] = (unsigned long long)(unsigned)total | ((unsigned long long)(unsigned)s_tl_tasks << 32);
            r[6] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);
            r[7] = 0;
        }
    }
    if (wg_points) {  // [b]: points, [kWalkTallySlots + b]: their arc points, [2 kWalkTallySlots + b]: tasks""" % CAP),
]

CAPI_TAIL = r"""
// ---- diagnostic dump (scripts/diag_walk_timeline.py) ----
extern "C" void pptl_setup(void* buf);
extern "C" unsigned pptl_count();
static void* g_tl_buf = nullptr;
extern "C" int pp_batch_extend(pp_ctx* ctx, int64_t n_steps, int64_t* n_iterations, int64_t* n_accepted) {
    const char* path = getenv("PP_DIAG_OUT");
    if (path) {
        if (!g_tl_buf) (void)hipMalloc(&g_tl_buf, (size_t)%d * 64);
        (void)hipDeviceSynchronize();
        pptl_setup(g_tl_buf);
        (void)hipDeviceSynchronize();
    }
    const int r = pp_batch_extend_impl(ctx, n_steps, n_iterations, n_accepted);
    if (path && g_tl_buf) {
        (void)hipDeviceSynchronize();
        unsigned n = pptl_count();
        if (n > %d) n = %d;
        std::vector<unsigned long long> h((size_t)n * 8);
        if (n) (void)hipMemcpy(h.data(), g_tl_buf, (size_t)n * 64, hipMemcpyDeviceToHost);
        FILE* f = fopen(path, "ab");
        if (f) {
            fwrite(&n, 4, 1, f);
            if (n) fwrite(h.data(), 64, n, f);
            fclose(f);
        }
        pptl_setup(nullptr);
        (void)hipDeviceSynchronize();
    }
    return r;
}
""" % (CAP, CAP, CAP)

PATCHES_C = [
    ("int pp_batch_extend(pp_ctx* ctx, int64_t n_steps, int64_t* n_iterations, int64_t* n_accepted) {",
     "static int pp_batch_extend_impl(pp_ctx* ctx, int64_t n_steps, int64_t* n_iterations, int64_t* n_accepted) {"),
]


def build():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge

    shutil.rmtree(BUILD, ignore_errors=True)
    csrc = os.path.join(BUILD, "pkg", "csrc")
    os.makedirs(csrc)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(BUILD, "include"))
    for f in ge.SOURCES + ge.HEADERS:
        shutil.copy(os.path.join(SRC, f), csrc)
    for name, patches, tail in (("pp_kernels.hip", PATCHES_K, ""), ("pp_capi.cpp", PATCHES_C, CAPI_TAIL)):
        p = os.path.join(csrc, name)
        s = open(p).read()
        for a, b in patches:
            assert s.count(a) == 1, (name, a[:60], s.count(a))
            s = s.replace(a, b)
        open(p, "w").write(s + tail)
    os.makedirs(os.path.dirname(OUTLIB), exist_ok=True)
    cmd = ["/opt/rocm/bin/hipcc", *ge.HIPCC_FLAGS, "-o", OUTLIB] + [os.path.join(csrc, f) for f in ge.SOURCES]
    subprocess.run(cmd, check=True)
    print(OUTLIB)


def load(path):
    calls = []
    with open(path, "rb") as f:
        while True:
            b = f.read(4)
            if len(b) < 4:
                break
            n = int(np.frombuffer(b, dtype=np.uint32)[0])
            a = np.frombuffer(f.read(n * 64), dtype=np.uint64).reshape(n, 8)
            calls.append(a)
    return calls


def launches(a):
    """split one call's records into launches: per DevState, in entry order, a repeated block
    index starts the next launch"""
    out = []
    for stv in np.unique(a[:, 4]):
        r = a[a[:, 4] == stv]
        r = r[np.argsort(r[:, 0], kind="stable")]
        seen, cur = set(), []
        for row in r:
            b = int(row[3] & 0xffffffff)
            if b in seen:
                out.append(np.array(cur))
                seen, cur = set(), []
            seen.add(b)
            cur.append(row)
        if cur:
            out.append(np.array(cur))
    out.sort(key=lambda x: int(x[:, 0].min()))
    return out


def report(path):
    for ci, a in enumerate(load(path)):
        if len(a) == 0:
            continue
        L = launches(a)
        print(f"call {ci}: {len(a)} workgroup records, {len(L)} launches")
        rows = []
        for x in L:
            t_in, t_st, t_end = x[:, 0].astype(np.int64), x[:, 1].astype(np.int64), x[:, 2].astype(np.int64)
            t0 = t_in.min()
            total = int(x[0, 5] & 0xffffffff)
            tasks = (x[:, 5] >> 32).astype(np.int64)
            last = int(np.argmax(t_end))
            rows.append(dict(total=total, wgs=len(x), span=(t_end.max() - t0) / 100.0,
                             ramp=(t_in.max() - t0) / 100.0, stage=float(np.mean(t_st - t_in)) / 100.0,
                             work_mean=float(np.mean(t_end - t_st)) / 100.0,
                             work_max=float(np.max(t_end - t_st)) / 100.0,
                             last_in=(t_in[last] - t0) / 100.0, last_tasks=int(tasks[last]),
                             tasks_max=int(tasks.max()), tasks_mean=float(tasks.mean())))
        # size classes by task count
        for lo, hi in ((0, 1), (1, 1000), (1000, 4000), (4000, 8000), (8000, 16000), (16000, 40000),
                       (40000, 1 << 30)):
            sel = [r for r in rows if lo <= r["total"] < hi]
            if not sel:
                continue
            m = {k: float(np.mean([r[k] for r in sel])) for k in sel[0]}
            print(f"  tasks [{lo}, {hi}): {len(sel)} launches; mean: tasks {m['total']:.0f}, wgs {m['wgs']:.0f}, "
                  f"span {m['span']:.1f} us, ramp {m['ramp']:.1f}, stage {m['stage']:.1f}, "
                  f"wg work mean {m['work_mean']:.1f} max {m['work_max']:.1f}, last wg entered at "
                  f"{m['last_in']:.1f} with {m['last_tasks']:.1f} tasks (wg max {m['tasks_max']:.1f}, "
                  f"mean {m['tasks_mean']:.1f})")


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        report(sys.argv[2])
