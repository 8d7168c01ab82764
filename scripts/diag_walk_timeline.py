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
REC = 24       # u64 words per record

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
    __shared__ unsigned s_tl_max, s_tl_wmin, s_tl_h[8], s_tl_hd[8];
    if (t0) {
        s_tl_tasks = 0;
        s_tl_max = 0;
        s_tl_wmin = 0xffffffffu;
        for (int i = 0; i < 8; ++i) s_tl_h[i] = s_tl_hd[i] = 0;
    }"""),
    ("""        const int t = al ? al[ti] : ti;
        const int s = walk_rec<kLds, kScene, kS>(""",
     """        const int t = al ? al[ti] : ti;
        const unsigned long long tl_t = __builtin_amdgcn_s_memrealtime();
        const int tl_np0 = npts;
        const int s = walk_rec<kLds, kScene, kS>("""),
    ("""        ++ntasks;
        if (lane == 0) {
            if (al || t < W) {""",
     """        ++ntasks;
        if (lane == 0) {
            atomicAdd(&s_tl_tasks, 1);
            const unsigned dur = (unsigned)(__builtin_amdgcn_s_memrealtime() - tl_t);
            atomicMax(&s_tl_max, dur);
            const int dp = npts - tl_np0;
            const int hb = dp <= 0 ? 0 : (dp <= 8 ? 1 : (dp <= 16 ? 2 : (dp <= 32 ? 3 : (dp <= 64 ? 4 : (dp <= 128 ? 5 : (dp <= 256 ? 6 : 7))))));
            atomicAdd(&s_tl_h[hb], 1u);
            atomicAdd(&s_tl_hd[hb], dur);
        }
        if (lane == 0) {
            if (al || t < W) {"""),
    ("""    if (wg_points) {  // [b]: points, [kWalkTallySlots + b]: their arc points, [2 kWalkTallySlots + b]: tasks""",
     """    if (lane == 0) atomicMin(&s_tl_wmin, (unsigned)(__builtin_amdgcn_s_memrealtime() - tl_st));
    __syncthreads();
    if (g_tl && t0) {
        const unsigned slot = atomicAdd(&g_tl_n, 1u);
        if (slot < %d) {
            unsigned long long* r = g_tl + REC_WORDS * (size_t)slot;
            for (int i = 0; i < 8; ++i) {
                r[8 + i] = s_tl_h[i];
                r[16 + i] = s_tl_hd[i];
            }
            r[0] = tl_in;
            r[1] = tl_st;
            r[2] = __builtin_amdgcn_s_memrealtime();
            r[3] = (unsigned long long)blockIdx.x | ((unsigned long long)gridDim.x << 32);
            r[4] = (unsigned long long)(size_t)st;
            r[5] = (unsigned long long)(unsigned)total | ((unsigned long long)(unsigned)s_tl_tasks << 32);
            r[6] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4);
            r[7] = (unsigned long long)s_tl_max | ((unsigned long long)s_tl_wmin << 32);
        }
    }
    if (wg_points) {  // [b]: points, [kWalkTallySlots + b]: their arc points, [2 kWalkTallySlots + b]: tasks""".replace("REC_WORDS", str(REC)) % CAP),
]

CAPI_TAIL = r"""
// ---- diagnostic dump (scripts/diag_walk_timeline.py) ----
extern "C" void pptl_setup(void* buf);
extern "C" unsigned pptl_count();
static void* g_tl_buf = nullptr;
static void tl_begin() {
    if (!getenv("PP_DIAG_OUT")) return;
    if (!g_tl_buf) (void)hipMalloc(&g_tl_buf, (size_t)CAPV * RECB);
    (void)hipDeviceSynchronize();
    pptl_setup(g_tl_buf);
    (void)hipDeviceSynchronize();
}
static void tl_end(unsigned tag) {
    const char* path = getenv("PP_DIAG_OUT");
    if (!path || !g_tl_buf) return;
    (void)hipDeviceSynchronize();
    unsigned n = pptl_count();
    if (n > CAPV) n = CAPV;
    std::vector<unsigned long long> h((size_t)n * RECW);
    if (n) (void)hipMemcpy(h.data(), g_tl_buf, (size_t)n * RECB, hipMemcpyDeviceToHost);
    FILE* f = fopen(path, "ab");
    if (f) {
        fwrite(&n, 4, 1, f);
        fwrite(&tag, 4, 1, f);
        if (n) fwrite(h.data(), RECB, n, f);
        fclose(f);
    }
    pptl_setup(nullptr);
    (void)hipDeviceSynchronize();
}
extern "C" int pp_batch_extend(pp_ctx* ctx, int64_t n_steps, int64_t* n_iterations, int64_t* n_accepted) {
    tl_begin();
    const int r = pp_batch_extend_impl(ctx, n_steps, n_iterations, n_accepted);
    tl_end(0);
    return r;
}
extern "C" int pp_batch_plan(pp_ctx* ctx, int32_t* best_node, double* length, int32_t* n_points,
                             int32_t* n_finishes, int64_t* n_checked) {
    tl_begin();
    const int r = pp_batch_plan_impl(ctx, best_node, length, n_points, n_finishes, n_checked);
    tl_end(1);
    return r;
}
""".replace("CAPV", str(CAP)).replace("RECB", str(REC * 8)).replace("RECW", str(REC))

PATCHES_C = [
    ("""int pp_batch_plan(pp_ctx* ctx, int32_t* best_node, double* length, int32_t* n_points,
                  int32_t* n_finishes, int64_t* n_checked) {""",
     """static int pp_batch_plan_impl(pp_ctx* ctx, int32_t* best_node, double* length, int32_t* n_points,
                  int32_t* n_finishes, int64_t* n_checked) {"""),
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
            tag = int(np.frombuffer(f.read(4), dtype=np.uint32)[0])
            a = np.frombuffer(f.read(n * REC * 8), dtype=np.uint64).reshape(n, REC)
            calls.append((tag, a))
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
    for ci, (tag, a) in enumerate(load(path)):
        if len(a) == 0:
            continue
        L = launches(a)
        print(f"call {ci} ({'batch_plan' if tag else 'batch_extend'}): {len(a)} workgroup records, {len(L)} launches")
        rows = []
        for x in L:
            t_in, t_st, t_end = x[:, 0].astype(np.int64), x[:, 1].astype(np.int64), x[:, 2].astype(np.int64)
            t0 = t_in.min()
            total = int(x[0, 5] & 0xffffffff)
            tasks = (x[:, 5] >> 32).astype(np.int64)
            last = int(np.argmax(t_end))
            tmax = (x[:, 7] & 0xffffffff).astype(np.int64)
            wmin = (x[:, 7] >> 32).astype(np.int64)
            hist = x[:, 8:16].sum(axis=0).astype(np.float64)
            hdur = x[:, 16:24].sum(axis=0).astype(np.float64)
            rows.append(dict(hist=hist, hdur=hdur, total=total, wgs=len(x), span=(t_end.max() - t0) / 100.0,
                             ramp=(t_in.max() - t0) / 100.0, stage=float(np.mean(t_st - t_in)) / 100.0,
                             work_mean=float(np.mean(t_end - t_st)) / 100.0,
                             work_max=float(np.max(t_end - t_st)) / 100.0,
                             last_in=(t_in[last] - t0) / 100.0, last_tasks=int(tasks[last]),
                             tasks_max=int(tasks.max()), tasks_mean=float(tasks.mean()),
                             task_max=float(tmax.max()) / 100.0, task_max_wg_mean=float(tmax.mean()) / 100.0,
                             last_task_max=tmax[last] / 100.0,
                             wave_spread=float(np.mean((t_end - t_st) - wmin)) / 100.0,
                             last_wave_spread=((t_end[last] - t_st[last]) - wmin[last]) / 100.0,
                             work_p50=float(np.percentile(t_end - t_st, 50)) / 100.0,
                             work_p90=float(np.percentile(t_end - t_st, 90)) / 100.0))
        # size classes by task count
        for lo, hi in ((0, 1), (1, 1000), (1000, 4000), (4000, 8000), (8000, 16000), (16000, 40000),
                       (40000, 1 << 30)):
            sel = [r for r in rows if lo <= r["total"] < hi]
            if not sel:
                continue
            m = {k: float(np.mean([r[k] for r in sel])) for k in sel[0] if k not in ("hist", "hdur")}
            h = np.sum([r["hist"] for r in sel], axis=0)
            hd = np.sum([r["hdur"] for r in sel], axis=0)
            print(f"  tasks [{lo}, {hi}): {len(sel)} launches; mean: tasks {m['total']:.0f}, wgs {m['wgs']:.0f}, "
                  f"span {m['span']:.1f} us, ramp {m['ramp']:.1f}, stage {m['stage']:.1f}, "
                  f"wg work mean {m['work_mean']:.1f} max {m['work_max']:.1f}, last wg entered at "
                  f"{m['last_in']:.1f} with {m['last_tasks']:.1f} tasks (wg max {m['tasks_max']:.1f}, "
                  f"mean {m['tasks_mean']:.1f})")
            print(f"      longest task {m['task_max']:.1f} us (per-wg longest, mean {m['task_max_wg_mean']:.1f}; "
                  f"the last wg's {m['last_task_max']:.1f}); wave exit spread in a wg {m['wave_spread']:.1f} "
                  f"(last wg {m['last_wave_spread']:.1f}); wg work p50 {m['work_p50']:.1f} p90 {m['work_p90']:.1f}")
            names = ["0", "1-8", "9-16", "17-32", "33-64", "65-128", "129-256", ">256"]
            tot, totd = max(h.sum(), 1), max(hd.sum(), 1)
            print("      points per task: " + "  ".join(
                f"{names[i]}: {h[i] / tot * 100:.1f}% of tasks, {hd[i] / totd * 100:.1f}% of task time, "
                f"{hd[i] / max(h[i], 1) / 100.0:.2f} us" for i in range(8) if h[i] > 0))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        report(sys.argv[2])
