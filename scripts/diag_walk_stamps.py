"""Diagnostic build (never the product): the library with clock stamps around every steer_walk task.

  python scripts/diag_walk_stamps.py build     # -> rs-pathplanning_amd/lib/walkdiag/libpathplanning_amd.so
  PP_AMD_LIB=.../walkdiag/libpathplanning_amd.so PP_DIAG_OUT=out.bin python bench.py ... --allow-variant-lib
  python scripts/diag_walk_stamps.py report out.bin

Each wave sums, in registers, its tasks' shader-clock cycles split into the PrepRec load, the
point generation + interpolation and chunk_rejects, plus a per-task cycle histogram, and adds them
to a 64-word device buffer with one non-returning atomic per word at its exit (so the stamps do
not serialise the walk).  pp_batch_extend / pp_rrt_extend dump the buffer per call.
The patches are applied to a copy of the sources under build/; the product sources are untouched."""
import os
import shutil
import struct
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "rs-pathplanning_amd", "csrc")
OUTLIB = os.path.join(ROOT, "rs-pathplanning_amd", "lib", "walkdiag", "libpathplanning_amd.so")
BUILD = os.path.join(ROOT, "build", "walkdiag")

KERNEL_DECL = r"""
// ---- diagnostic stamps (scripts/diag_walk_stamps.py) ----
__device__ unsigned long long* g_diag;
extern "C" void ppdiag_setup(void* buf, unsigned cap) {
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_diag), &buf, sizeof buf);
    (void)hipMemset(buf, 0, 128 * 8);
}
extern "C" unsigned ppdiag_count() { return 128; }
"""

# per-wave sums in registers, one fire-and-forget atomicAdd each at the wave's exit:
# [0] tasks [1] points [2] task cycles [3] rec-load cycles [4] interpolate cycles
# [5] chunk_rejects items cycles [6] chunks [7] wave span cycles (first task start .. exit)
# [30] generate cycles [31] chunk_rejects setup cycles (bounds, bbox, cells)
# [8..31] per-task cycle histogram, bin = floor(log2(cycles)) - 8; [32..63] chunks per task (31: more)
PATCHES_K = [
    ("extern __shared__ __attribute__((aligned(16))) char pp_smem[];",
     "extern __shared__ __attribute__((aligned(16))) char pp_smem[];\n" + KERNEL_DECL),
    ("""    const int ncx = cx1 - cx0 + 1, ncy = cy1 - cy0 + 1;
    if (ncx <= 0 || ncy <= 0) return false;""",
     """    const int ncx = cx1 - cx0 + 1, ncy = cy1 - cy0 + 1;
    if (g_diag && lane == 0) {
        const int nc = (ncx > 0 && ncy > 0) ? ncx * ncy : 0;
        atomicAdd(g_diag + 64 + (nc < 31 ? nc : 31), 1ull);
    }
    if (ncx <= 0 || ncy <= 0) return false;"""),
    ("""            if (items_reject(kk >= 0, kk)) return true;
            if (mb + 64 >= run) break;""",
     """            if (g_diag && lane == 0 && mb == 0) atomicAdd(g_diag + 96 + (run < 31 ? run : 31), 1ull);
            if (items_reject(kk >= 0, kk)) return true;
            if (mb + 64 >= run) break;"""),

    ("""__device__ __forceinline__ bool chunk_rejects(const SceneDev& sc, bool has, bool check_bounds,
                                              bool seg_valid, double qx, double qy) {""",
     """__device__ __forceinline__ bool chunk_rejects(const SceneDev& sc, bool has, bool check_bounds,
                                              bool seg_valid, double qx, double qy,
                                              long long* dgc = nullptr) {"""),
    ("""    auto items_reject = [&](bool valid, int kk) -> bool {""",
     """    if (dgc) {
        __builtin_amdgcn_s_waitcnt(0);
        dgc[0] = __builtin_amdgcn_s_memtime();
    }
    auto items_reject = [&](bool valid, int kk) -> bool {"""),
    ("""        const bool junction_here = done && cnt < 63;""",
     """        if (dg) {
            __builtin_amdgcn_s_waitcnt(0);
            const long long t = __builtin_amdgcn_s_memtime();
            dg[4] += t - dt0;
            dt0 = t;
        }
        const bool junction_here = done && cnt < 63;"""),
    ("""                                        int& npts, int& napts, bool junction = true) {
    const int lane = threadIdx.x & 63;
    const int state = p->state;
    const double x = p->x, y = p->y, px = p->px, py = p->py;""",
     """                                        int& npts, int& napts, bool junction = true,
                                        long long* dg = nullptr) {
    const int lane = threadIdx.x & 63;
    long long dt0 = dg ? __builtin_amdgcn_s_memtime() : 0;
    const int state = p->state;
    const double x = p->x, y = p->y, px = p->px, py = p->py;
    if (dg) {
        __builtin_amdgcn_s_waitcnt(0);
        const long long t = __builtin_amdgcn_s_memtime();
        dg[0] += t - dt0 + (state & 0);
        dt0 = t;
    }"""),
    ("""        const bool has = lane == 0 || isgrid || isj;
        const bool chk = isgrid || isj || (base == 0 && lane == 0);""",
     """        if (dg) {
            __builtin_amdgcn_s_waitcnt(0);
            const long long t = __builtin_amdgcn_s_memtime();
            dg[1] += t - dt0;
            dt0 = t;
            dg[3] += 1;
        }
        const bool has = lane == 0 || isgrid || isj;
        const bool chk = isgrid || isj || (base == 0 && lane == 0);"""),
    ("""        if (chunk_rejects<kLds, kScene>(sc, has, chk, has && lane >= 1, qx, qy)) return kReject;
        if (junction_here) break;""",
     """        long long dgc[1] = {0};
        const bool rj = chunk_rejects<kLds, kScene>(sc, has, chk, has && lane >= 1, qx, qy,
                                                    dg ? dgc : nullptr);
        if (dg) {
            const long long t = __builtin_amdgcn_s_memtime();
            if (dgc[0] > 0) {  // (0: returned before the items: bounds, or no cell)
                dg[5] += dgc[0] - dt0;
                dg[2] += t - dgc[0];
            } else {
                dg[5] += t - dt0;
            }
            dt0 = t;
        }
        if (rj) return kReject;
        if (junction_here) break;"""),
    ("""    __shared__ int s_next;
    const int G = (int)gridDim.x;
    if (threadIdx.x == 0) s_next = 0;
    __syncthreads();
    for (;;) {
        int k = 0;
        if (lane == 0) k = atomicAdd(&s_next, 1);
        const int t = (int)blockIdx.x + G * __builtin_amdgcn_readlane(k, 0);
        if (t >= total) break;
        const int s = walk_rec<kLds, kScene>(sc, rec + t, pdbuf + (size_t)t * kPdCap, gs, npts, napts);""",
     """    __shared__ int s_next;
    const int G = (int)gridDim.x;
    if (threadIdx.x == 0) s_next = 0;
    __syncthreads();
    long long dsum[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    int dh[24], dcn[32];
    for (int i = 0; i < 24; ++i) dh[i] = 0;
    for (int i = 0; i < 32; ++i) dcn[i] = 0;
    long long dfirst = -1;
    for (;;) {
        int k = 0;
        if (lane == 0) k = atomicAdd(&s_next, 1);
        const int t = (int)blockIdx.x + G * __builtin_amdgcn_readlane(k, 0);
        if (t >= total) break;
        const long long dc0 = __builtin_amdgcn_s_memtime();
        if (dfirst < 0) dfirst = dc0;
        const int dp0 = npts;
        long long dg[6] = {0, 0, 0, 0, 0, 0};
        const int s = walk_rec<kLds, kScene>(sc, rec + t, pdbuf + (size_t)t * kPdCap, gs, npts, napts,
                                             true, g_diag ? dg : nullptr);
        {
            const long long dc = __builtin_amdgcn_s_memtime() - dc0;
            dsum[0] += 1;
            dsum[1] += npts - dp0;
            dsum[2] += dc;
            dsum[3] += dg[0];
            dsum[4] += dg[1];
            dsum[5] += dg[2];
            dsum[6] += dg[3];
            dsum[8] += dg[4];
            dsum[9] += dg[5];
            int b = 63 - __builtin_clzll((unsigned long long)(dc | 1)) - 8;
            b = b < 0 ? 0 : (b > 21 ? 21 : b);
            for (int i = 0; i < 22; ++i) dh[i] += (i == b);
            const int ch = (int)(dg[3] < 31 ? dg[3] : 31);
            for (int i = 0; i < 32; ++i) dcn[i] += (i == ch);
        }"""),
    ("""    if (wg_points) {  // [b]: points, [kWalkTallySlots + b]: their arc points""",
     """    if (g_diag && lane == 0 && dsum[0] > 0) {
        dsum[7] = __builtin_amdgcn_s_memtime() - dfirst;
        for (int i = 0; i < 8; ++i) atomicAdd(g_diag + i, (unsigned long long)dsum[i]);
        atomicAdd(g_diag + 30, (unsigned long long)dsum[8]);
        atomicAdd(g_diag + 31, (unsigned long long)dsum[9]);
        for (int i = 0; i < 22; ++i)
            if (dh[i]) atomicAdd(g_diag + 8 + i, (unsigned long long)dh[i]);
        for (int i = 0; i < 32; ++i)
            if (dcn[i]) atomicAdd(g_diag + 32 + i, (unsigned long long)dcn[i]);
    }
    if (wg_points) {  // [b]: points, [kWalkTallySlots + b]: their arc points"""),
]

CAPI_TAIL = r"""
// ---- diagnostic dump (scripts/diag_walk_stamps.py) ----
extern "C" void ppdiag_setup(void* buf, unsigned cap);
static void* g_diag_buf = nullptr;
static void diag_begin() {
    if (!getenv("PP_DIAG_OUT")) return;
    if (!g_diag_buf) (void)hipMalloc(&g_diag_buf, 128 * 8);
    ppdiag_setup(g_diag_buf, 128);
    (void)hipDeviceSynchronize();
}
static void diag_end(const char* what) {
    const char* path = getenv("PP_DIAG_OUT");
    if (!path || !g_diag_buf) return;
    (void)hipDeviceSynchronize();
    unsigned long long h[128];
    (void)hipMemcpy(h, g_diag_buf, sizeof h, hipMemcpyDeviceToHost);
    FILE* f = fopen(path, "ab");
    if (!f) return;
    char tag[16] = {};
    strncpy(tag, what, 15);
    fwrite(tag, 1, 16, f);
    fwrite(h, 8, 128, f);
    fclose(f);
}
extern "C" int pp_batch_extend(pp_ctx* ctx, int64_t n_steps, int64_t* n_iterations, int64_t* n_accepted) {
    diag_begin();
    const int r = pp_batch_extend_impl(ctx, n_steps, n_iterations, n_accepted);
    diag_end("batch");
    return r;
}
extern "C" int pp_rrt_extend(pp_ctx* ctx, int64_t n_iter, int64_t* n_accepted) {
    diag_begin();
    const int r = pp_rrt_extend_impl(ctx, n_iter, n_accepted);
    diag_end("tree");
    return r;
}
"""

PATCHES_C = [
    ("int pp_batch_extend(pp_ctx* ctx, int64_t n_steps, int64_t* n_iterations, int64_t* n_accepted) {",
     "static int pp_batch_extend_impl(pp_ctx* ctx, int64_t n_steps, int64_t* n_iterations, int64_t* n_accepted) {"),
    ("int pp_rrt_extend(pp_ctx* ctx, int64_t n_iter, int64_t* n_accepted) {",
     "static int pp_rrt_extend_impl(pp_ctx* ctx, int64_t n_iter, int64_t* n_accepted) {"),
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
            assert s.count(a) == 1, (name, a[:60])
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
            tag = f.read(16)
            if len(tag) < 16:
                break
            a = np.frombuffer(f.read(128 * 8), dtype=np.uint64).astype(np.float64)
            calls.append((tag.rstrip(b"\0").decode(), a))
    return calls


def report(path):
    for ci, (tag, a) in enumerate(load(path)):
        n = a[0]
        if n == 0:
            continue
        cyc = a[2]
        print(f"call {ci} {tag}: tasks {n:.0f}  points/task {a[1] / n:.1f}  chunks/task {a[6] / n:.2f}  "
              f"cycles/task {cyc / n:.0f}  cycles/chunk {cyc / max(a[6], 1):.0f}")
        rest = cyc - a[3] - a[30] - a[4] - a[31] - a[5]
        print(f"  share of task cycles: rec load {a[3] / cyc:.3f}  generate {a[30] / cyc:.3f}  "
              f"interpolate {a[4] / cyc:.3f}  rejects setup (bounds, bbox, cells) {a[31] / cyc:.3f}  "
              f"items {a[5] / cyc:.3f}  other {rest / cyc:.3f}")
        print(f"  per task rec load {a[3] / n:.0f} cycles; wave busy share {cyc / max(a[7], 1):.3f}")
        h = a[8:30]
        tot = h.sum()
        print("  task cycles histogram: " + "  ".join(f"2^{i + 8}:{h[i] / tot * 100:.1f}%" for i in range(22) if h[i] > 0))
        ch = max(a[6], 1)
        print(f"  per chunk cycles: generate {a[30] / ch:.0f}, interpolate {a[4] / ch:.0f}, "
              f"rejects setup (bounds, bbox, cells) {a[31] / ch:.0f}, items {a[5] / ch:.0f}")
        c = a[32:64]
        print("  chunks per task: " + "  ".join(f"{i}:{int(c[i])}" for i in range(32) if c[i] > 0))
        c = a[64:96]
        print("  cells per chunk (all chunk_rejects calls): " + "  ".join(f"{i}:{int(c[i])}" for i in range(32) if c[i] > 0))
        c = a[96:128]
        print("  items listed per chunk (<= 64 cells): " + "  ".join(f"{i}:{int(c[i])}" for i in range(32) if c[i] > 0))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build()
    else:
        report(sys.argv[2])
