// pp_capi.cpp — host side of the MI355X RRT extend path: context, scene, device-resident tree and
// planner state, the window enqueue loop, and the C ABI (include/pathplanning_amd.h).
//
// Extend semantics: iteration it samples (x, y) from the seeded stream, takes
// the exact nearest node of the tree as it stands after iterations < it, steers child→parent with
// Dubins, verifies, inserts.  The GPU evaluates a window of K iterations against the tree
// snapshot at the window start, and a one-workgroup resolve kernel replays the window in order:
//   * sample j's true parent is the nearest of {snapshot NN} ∪ {accepted window samples i < j};
//     nn_finalize's pair search lists the i that are strictly nearer than the snapshot NN, so the parent is
//     the first accepted entry of that list in (d2, i) order, or the snapshot NN;
//   * the verdict for (j, parent) was precomputed for the snapshot NN and for every listed i
//     under i's own snapshot parent; only a parent that itself changed needs a repair steer.
// The result is identical to the one-at-a-time sequential spec for every K.  All planner state
// (it, n, counters) lives in device memory, so the host enqueues windows back to back and
// synchronises once per batch of windows.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include "../../include/pathplanning_amd.h"
#include "pp_device.h"
#include "pp_kernels.h"
#include "pp_scene.h"

using namespace ppamd;

namespace {

thread_local std::string g_err;

int set_err(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define PP_HIP(expr)                                                                         \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return set_err(PP_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

template <typename T>
struct DBuf {
    T* p = nullptr;
    size_t n = 0;
    hipError_t reserve(size_t count) {
        if (count <= n) return hipSuccess;
        release();
        hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(count, 1) * sizeof(T));
        if (e == hipSuccess) n = count;
        else p = nullptr;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
    ~DBuf() { release(); }
};

template <typename T>
struct HBuf {  // pinned host staging
    T* p = nullptr;
    size_t n = 0;
    hipError_t reserve(size_t count) {
        if (count <= n) return hipSuccess;
        release();
        hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), std::max<size_t>(count, 1) * sizeof(T),
                                     hipHostMallocDefault);
        if (e == hipSuccess) n = count;
        else p = nullptr;
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        n = 0;
    }
    ~HBuf() { release(); }
};

constexpr int kMaxBatch = 64;  // windows enqueued between two host synchronisations
constexpr int kInsideCells = 2048;  // the inside bitmap's cells per axis (point_blocked)
constexpr int kScreenPad = 64;  // f32 screen copies: the LDS-DMA reads whole float4s (<= 3 floats past)

}  // namespace

struct pp_ctx {
    int device = 0;
    hipStream_t stream = nullptr;

    // ---- scene (Space)
    bool has_scene = false;
    double minx = 0, maxx = 0, miny = 0, maxy = 0;
    double width = 0, height = 0, max_steer = 0;
    int m = 0;
    DBuf<double> d_cx, d_cy, d_r2, d_rcull;
    DBuf<int> d_goff, d_gitems;
    DBuf<uint4> d_img, d_gimg;  // LDS images (discs / occupancy bits), contiguous
    double gx0 = 0, gy0 = 0, ginv = 1;
    int gnx = 1, gny = 1;
    int lds_bytes = 0, lds_goff = 0, lds_items = 0, lds_cx = 0, lds_cy = 0, lds_r2 = 0, lds_d4 = 0;
    DBuf<float4> d_d4;
    // occupancy grid (config 4)
    bool has_grid = false;
    DBuf<uint32_t> d_bits;
    int bw = 0, bh = 0, bwords = 0, lds_bits_bytes = 0;
    double bx0 = 0, by0 = 0, binv = 1;
    // polygon mode (pp_space_new_polygons, Q10p): obstacle edges, bounds ring; host copies for
    // the point checks (root / query starts)
    // disc scenes: the inside bitmap (scene::inside_bitmap), the point_blocked pre-test
    DBuf<uint32_t> d_ibits;
    int ibn = 0;
    double ibx0 = 0.0, iby0 = 0.0, ibinv = 1.0;
    int ne = 0, nbv = 0;
    double h2 = 0.0;
    float cull_slack = 1.0e-3f;
    DBuf<double> d_ex0, d_ey0, d_ex1, d_ey1, d_bvx, d_bvy;
    DBuf<int> d_epoly;
    std::vector<double> h_ex0, h_ey0, h_ex1, h_ey1, h_bvx, h_bvy;
    std::vector<int> h_epoly;

    // ---- planner (RRT)
    bool has_rrt = false;
    double start[3] = {0, 0, 0}, goal[3] = {0, 0, 0};
    int64_t max_iter = 0;
    double step = 0.1;
    uint64_t seed = 0;
    int64_t it = 0;   // mirror of DevState.it (exact after every synchronisation)
    int64_t seq = 0;  // windows enqueued so far (their sequence numbers)
    int64_t n = 0;    // mirror of DevState.n
    int64_t cap = 0;  // tree capacity
    double eps_coord = 0.0;
    bool root_blocked = false;  // polygon mode: the root fails verify (nothing is ever inserted)
    DBuf<float> x32, y32;
    DBuf<double> X, Y, YAW;
    DBuf<int> PAR;
    DBuf<DevState> d_state, d_api_state;
    HBuf<DevState> h_state;
    // pp_rrt_extend_samples: the caller's samples and the per-iteration record (one chunk)
    DBuf<double> hs_x, hs_y, hs_yaw;
    DBuf<int> hs_par;
    DBuf<uint8_t> hs_ok;

    // ---- window buffers (sized for Kcap)
    int K = 4096;
    int Kcap = 0;
    DBuf<double> wsx, wsy, nn_d2, snap_yaw, snap_pose;
    DBuf<float> pbest, psecond, wsx32, wsy32;
    DBuf<int> perm, cofs, ipos;
    DBuf<float2> sxy;
    DBuf<double> sqb, ssx, ssy;
    DBuf<float2> ob;
    DBuf<int> pidx, nn_idx, cand_cnt, snap_status;
    DBuf<CandEntry> cand;
    DBuf<PrepRec> rec;   // per-task steer records
    DBuf<int> r_order, r_rep, pend, fin_par;
    DBuf<unsigned char> blk;   // [2 Kcap] window samples in an obstacle (point_blocked)
    DBuf<SceneDev> d_scene;    // the scene in device memory (samples_role, the literal paths)
    DBuf<SceneDev> cf_scene;   // check_finish_kernel's scene (its step may be a batch's)
    SceneDev cf_scene_host{};  // what cf_scene holds (the source of its last upload)
    bool cf_scene_ok = false;
    DBuf<double> r_repyaw;
    DBuf<double> lit_scratch;  // resolve: one literal buffer per wave
    // verify_node API
    DBuf<SteerTask> tasks;
    DBuf<int> task_status;
    DBuf<double> task_yaw;
    DBuf<double> api_lit_scratch;
    HBuf<SteerTask> h_tasks;
    // check_finish
    DBuf<int> cf_nodes, cf_ok, cf_npts, cf_chain, cf_etab, cf_err, cf_path, cf_items;
    DBuf<int> cf_lpath, cf_spill;  // cf_line_kernel's ancestor paths; tier 1's spill list
    DBuf<int> cf_memo;  // check_finish_kernel's optimize memo (CfBatch::ftab / gtab), per launch
    DBuf<double> cf_len, cf_pts;
    // ---- multi-query batch (config 3)
    bool has_batch = false;
    int mq_Q = 0, mq_cap = 0;
    int64_t mq_max_iter = 0;
    double mq_step = 0.1;
    DBuf<double> mq_x, mq_y, mq_yaw, mq_yawbuf;
    DBuf<int> mq_par, mq_n, mq_status, mq_err, mq_alist, mq_lstat;
    DBuf<int64_t> mq_it, mq_evals;
    DBuf<int64_t> mq_itprev;  // the lockstep NN's verdict cache (MqDev::it_prev)
    DBuf<uint64_t> mq_seed;
    DBuf<uint8_t> mq_blocked;
    bool mq_any_blocked = false;
    int mq_K = 1;                 // speculative window per query of the current batch
    int mq_K_user = 0;            // pp_batch_set_window (0: automatic)
    int mq_nsub = 1;              // sub-batches of the current batch (fixed at pp_batch_new)
    DBuf<int64_t> mq_target;      // [Q] iteration targets of the running pp_batch_extend
    DBuf<double> mq_nnd2;         // [Q * kMqMaxK]
    DBuf<SteerTask> mq_tasks, mq_ctask;
    DBuf<PrepRec> mq_rec;
    DBuf<DevState> mq_state;      // [3]: the whole batch, then one per sub-batch (mq_sub_args)
    hipStream_t sub_stream[4] = {};  // sub-batch streams 1.. (0 is `stream`), created on first use
    DBuf<SceneDev> mq_scene;      // the scene in device memory (point_blocked)
    hipEvent_t fork_ev = nullptr;
    std::vector<double> mq_goal;  // 3 per query (RRT::new's goal; pp_batch_plan)
    DBuf<double> mq_goal_d;       // [3Q] the goals on the device (pp_batch_plan)
    DBuf<int> mp_off, mp_qidx, mp_nodes, mp_ok, mp_npts, mp_best, mp_bpts, mp_nfin;
    DBuf<double> mp_len, mp_blen;
    // pp_batch_plan's check_finish in steer rounds (CfbArgs)
    DBuf<int> cfb_nodei;   // [4 (nitems + Q)]: depth, open, tfirst, tcnt
    DBuf<int> cfb_rows;    // [rows]: gclaim
    DBuf<unsigned char> cfb_rows8;  // [2 rows]: tnone, tnone_up
    DBuf<int> cfb_gotab, cfb_plist, cfb_tnode, cfb_status, cfb_misc, cfb_lit, cfb_dhist;
    DBuf<SteerTask> cfb_tasks;
    DBuf<StarTaskExt> cfb_ext;
    DBuf<PrepRec> cfb_rec;
    DBuf<unsigned char> cfb_none;
    DBuf<double> cfb_yaw;
    DBuf<DevState> cfb_state;
    DBuf<long long> cfb_pts;  // profiling: the rounds' walk point tallies
    int64_t cfb_nodes = 0, cfb_edges = 0, cfb_points = 0, cfb_arc = 0;  // profiling
    bool cf_rounds = true;  // pp_batch_plan in steer rounds (pp_batch_set_finish_schedule)
    int cfb_span0 = kCfbSpan, cfb_span = kCfbSpan;  // phase A candidates per node: first / later rounds

    // ---- RRT* query batch (BASELINE config 5, build-defined: DESIGN.md §3.7)
    bool has_star = false;
    int star_Q = 0, star_cap = 0, star_kfix = 0;
    int star_nsub = 1;  // sub-batches of the current RRT* batch (fixed at pp_star_new)
    int64_t star_max_iter = 0;
    double star_step = 0.1, star_eta = 0.0;
    DBuf<double> sr_x, sr_y, sr_yaw, sr_cost, sr_elen, sr_px, sr_py, sr_cb;
    DBuf<int> sr_par, sr_n, sr_mark, sr_stamp, sr_ksched, sr_pn, sr_near, sr_nnear, sr_bslot,
        sr_cslot, sr_err;
    DBuf<uint64_t> sr_cmask, sr_bmask, sr_seed;
    DBuf<int> lit_locks;  // literal scratch slot locks (api_lit_scratch), zeroed once
    DBuf<int64_t> sr_it, sr_evals, sr_target, sr_rew;
    DBuf<uint8_t> sr_blocked;
    bool sr_any_blocked = false;
    DBuf<DevState> sr_state;  // [3 * (1 + kMaxSub)]: rounds A, B, C of the batch, then per sub-batch
    DBuf<SteerTask> sr_tA, sr_tB, sr_tC;
    DBuf<StarTaskExt> sr_eB, sr_eC;
    DBuf<int> sr_sA, sr_sB, sr_sC;
    DBuf<double> sr_yA, sr_yB, sr_yC, sr_cA, sr_cB, sr_cC;
    DBuf<PrepRec> sr_rec;

    // ---- profiling
    bool prof = false;
    std::vector<hipEvent_t> ev;  // 4 per window or batch step, 8 per RRT* step
    double nn_scan_ms = 0.0, steer_ms = 0.0, finish_ms = 0.0, finalize_ms = 0.0, prep_ms = 0.0,
           insert_ms = 0.0;
    int64_t nn_scan_launches = 0, steer_launches = 0, finish_launches = 0;
    int64_t batch_steps = 0, batch_passes = 0;
    DBuf<long long> cf_tally;  // check_finish (profiling): nodes, edges, points, arc points
    DBuf<long long> wg_pts;  // walked polyline points per walk workgroup (profiling on)
    long long* prof_points() const { return prof ? wg_pts.p : nullptr; }
    // every counter of pp_stats that lives on the host or in the profiling tallies (not DevState)
    int reset_host_stats() {
        nn_scan_ms = steer_ms = finish_ms = finalize_ms = prep_ms = insert_ms = 0.0;
        nn_scan_launches = steer_launches = finish_launches = 0;
        batch_steps = batch_passes = 0;
        cfb_nodes = cfb_edges = cfb_points = cfb_arc = 0;
        if (wg_pts.p && hipMemsetAsync(wg_pts.p, 0, wg_pts.n * sizeof(long long), stream) != hipSuccess)
            return PP_ERR_HIP;
        if (cf_tally.p && hipMemsetAsync(cf_tally.p, 0, cf_tally.n * sizeof(long long), stream) != hipSuccess)
            return PP_ERR_HIP;
        return hipStreamSynchronize(stream) == hipSuccess ? PP_OK : PP_ERR_HIP;
    }

    ~pp_ctx() {
        for (auto& e : ev)
            if (e) (void)hipEventDestroy(e);
        if (fork_ev) (void)hipEventDestroy(fork_ev);
        for (auto& ss : sub_stream)
            if (ss) (void)hipStreamDestroy(ss);
        if (stream) (void)hipStreamDestroy(stream);
    }

    SceneDev scene_dev() const {
        SceneDev s;
        s.minx = minx;
        s.maxx = maxx;
        s.miny = miny;
        s.maxy = maxy;
        s.turn_radius = max_steer;
        s.step_size = step;
        s.m = m;
        s.cx = d_cx.p;
        s.cy = d_cy.p;
        s.r2 = d_r2.p;
        s.rcull = d_rcull.p;
        s.gx0 = gx0;
        s.gy0 = gy0;
        s.ginv = ginv;
        s.gcell = 1.0 / ginv;
        s.gnx = gnx;
        s.gny = gny;
        s.goff = d_goff.p;
        s.gitems = d_gitems.p;
        s.lds_bytes = lds_bytes;
        s.lds_goff = lds_goff;
        s.lds_items = lds_items;
        s.lds_cx = lds_cx;
        s.lds_cy = lds_cy;
        s.lds_r2 = lds_r2;
        s.d4 = d_d4.p;
        s.lds_d4 = lds_d4;
        s.bits = has_grid ? d_bits.p : nullptr;
        s.bw = bw;
        s.bh = bh;
        s.bwords = bwords;
        s.bx0 = bx0;
        s.by0 = by0;
        s.binv = binv;
        s.img = d_img.p;
        if (has_grid) {
            s.lds_bytes = lds_bits_bytes;
            s.img = d_gimg.p;
        }
        s.ne = ne;
        s.ex0 = d_ex0.p;
        s.ey0 = d_ey0.p;
        s.ex1 = d_ex1.p;
        s.ey1 = d_ey1.p;
        s.epoly = d_epoly.p;
        s.h2 = h2;
        s.nbv = nbv;
        s.bvx = d_bvx.p;
        s.bvy = d_bvy.p;
        s.cull_slack = cull_slack;
        s.root_blocked = root_blocked ? 1 : 0;
        s.ibits = ibn > 0 ? d_ibits.p : nullptr;
        s.ibn = ibn;
        s.ibwords = ibn / 32;
        s.ibx0 = ibx0;
        s.iby0 = iby0;
        s.ibinv = ibinv;
        return s;
    }
    // Space::verify of the one-point line [(x, y)] on the host, polygon mode (Q10p; the same
    // arithmetic as the kernels and the oracle): bounds, edge buffers, inside an obstacle
    bool point_ok(double x, double y) const {
        SceneDev s{};
        s.minx = minx;
        s.maxx = maxx;
        s.miny = miny;
        s.maxy = maxy;
        s.nbv = nbv;
        s.bvx = h_bvx.data();
        s.bvy = h_bvy.data();
        s.h2 = h2;
        if (!point_in_bounds(s, x, y)) return false;
        for (int k = 0; k < ne; ++k)
            if (seg_hits_edge(x, y, x, y, h_ex0[k], h_ey0[k], h_ex1[k], h_ey1[k], h2)) return false;
        return !in_obstacle(ne, h_ex0.data(), h_ey0.data(), h_ex1.data(), h_ey1.data(),
                            h_epoly.data(), x, y);
    }
    TreeDev tree_dev() const {
        TreeDev t;
        t.x32 = x32.p;
        t.y32 = y32.p;
        t.x = X.p;
        t.y = Y.p;
        t.yaw = YAW.p;
        t.parent = PAR.p;
        return t;
    }
    WindowArgs window_args(DevState* st) const {
        WindowArgs a;
        a.K = Kcap;
        a.Kcap = Kcap;
        a.seed = seed;
        a.eps_coord = eps_coord;
        a.st = st;
        a.sc = scene_dev();
        a.tr = tree_dev();
        a.wsx = wsx.p;
        a.wsy = wsy.p;
        a.wsx32 = wsx32.p;
        a.wsy32 = wsy32.p;
        a.perm = perm.p;
        a.cofs = cofs.p;
        a.sxy = sxy.p;
        a.sq = sqb.p;
        a.ssx = ssx.p;
        a.ssy = ssy.p;
        a.ob = ob.p;
        a.ipos = ipos.p;
        a.pbest = pbest.p;
        a.psecond = psecond.p;
        a.pidx = pidx.p;
        a.nn_idx = nn_idx.p;
        a.nn_d2 = nn_d2.p;
        a.cand_cnt = cand_cnt.p;
        a.cand = cand.p;
        a.snap_status = snap_status.p;
        a.snap_yaw = snap_yaw.p;
        a.snap_pose = snap_pose.p;
        a.rec = rec.p;
        a.pend = pend.p;
        a.fin_par = fin_par.p;
        a.rs.order = r_order.p;
        a.rs.rep = r_rep.p;
        a.rs.repyaw = r_repyaw.p;
        a.lit_scratch = lit_scratch.p;
        a.wg_points = prof_points();
        a.scp = d_scene.p;
        a.blk = d_scene.p ? blk.p : nullptr;
        return a;
    }
};

namespace {

int check_ctx(pp_ctx* c, bool need_scene, bool need_rrt) {
    if (!c) return set_err(PP_ERR_INVALID_ARGUMENT, "null context");
    if (need_scene && !c->has_scene) return set_err(PP_ERR_STATE, "pp_space_new has not been called");
    if (need_rrt && !c->has_rrt) return set_err(PP_ERR_STATE, "pp_rrt_new has not been called");
    PP_HIP(hipSetDevice(c->device));
    return PP_OK;
}

// The window pipeline is compiled for window sizes that are multiples of 256 (nn_scan sample
// blocks); any requested K runs inside a buffer of round_up(K, 256).
int ensure_window(pp_ctx* c, int K) {
    K = (K + 255) & ~255;
    if (K <= c->Kcap) return PP_OK;
    const size_t k = (size_t)K;
    PP_HIP(c->wsx.reserve(2 * k));  // double-buffered by window parity
    PP_HIP(c->wsy.reserve(2 * k));
    PP_HIP(c->wsx32.reserve(2 * k));
    PP_HIP(c->wsy32.reserve(2 * k));
    PP_HIP(c->perm.reserve(2 * k));
    PP_HIP(c->ipos.reserve(2 * k));
    PP_HIP(c->sxy.reserve(2 * k));
    PP_HIP(c->cofs.reserve(2 * 257));
    PP_HIP(c->sqb.reserve(2 * k));
    PP_HIP(c->ssx.reserve(2 * k));
    PP_HIP(c->ssy.reserve(2 * k));
    PP_HIP(c->ob.reserve(2 * (size_t)kMaxWindow / 256));
    PP_HIP(c->pbest.reserve(k * kMaxChunks));
    PP_HIP(c->psecond.reserve(k * kMaxChunks));
    PP_HIP(c->pidx.reserve(k * kMaxChunks));
    PP_HIP(c->nn_idx.reserve(k));
    PP_HIP(c->nn_d2.reserve(k));
    PP_HIP(c->cand_cnt.reserve(k));
    PP_HIP(c->cand.reserve(k * kCandCap));
    PP_HIP(c->rec.reserve(k + k * kCandCap));
    PP_HIP(c->snap_status.reserve(k));
    PP_HIP(c->snap_yaw.reserve(k));
    PP_HIP(c->snap_pose.reserve(3 * k));
    PP_HIP(c->r_order.reserve(k * kCandCap));
    PP_HIP(c->r_rep.reserve(k));
    PP_HIP(c->pend.reserve(k));
    PP_HIP(c->fin_par.reserve(k));
    PP_HIP(c->blk.reserve(2 * k));
    PP_HIP(hipMemsetAsync(c->cand_cnt.p, 0, k * sizeof(int), c->stream));
    PP_HIP(c->r_repyaw.reserve(k));
    PP_HIP(c->tasks.reserve(k));
    PP_HIP(c->task_status.reserve(k));
    PP_HIP(c->task_yaw.reserve(k));
    PP_HIP(c->h_tasks.reserve(k));
    PP_HIP(c->lit_scratch.reserve((size_t)(kResolveThreads / 64) * 3 * kLiteralCap));
    c->Kcap = K;
    return PP_OK;
}

template <typename T>
int grow_copy(pp_ctx* c, DBuf<T>& b, size_t old_n, size_t new_cap) {
    DBuf<T> nb;
    PP_HIP(nb.reserve(new_cap));
    if (old_n)
        PP_HIP(hipMemcpyAsync(nb.p, b.p, old_n * sizeof(T), hipMemcpyDeviceToDevice, c->stream));
    PP_HIP(hipStreamSynchronize(c->stream));
    std::swap(b.p, nb.p);
    std::swap(b.n, nb.n);
    return PP_OK;
}

int ensure_tree(pp_ctx* c, int64_t need) {
    if (need <= c->cap) return PP_OK;
    if (need > (int64_t)0x7fff0000) return set_err(PP_ERR_CAPACITY, "tree larger than 2^31 nodes");
    int64_t nc = std::max<int64_t>(need, c->cap * 2);
    nc = std::max<int64_t>(nc, 1024);
    int r;
    // the f32 screen copies get kScreenPad floats of slack: the screen's LDS-DMA reads whole
    // float4s, up to 3 floats past the last node
    if ((r = grow_copy(c, c->x32, c->n, nc + kScreenPad))) return r;
    if ((r = grow_copy(c, c->y32, c->n, nc + kScreenPad))) return r;
    if ((r = grow_copy(c, c->X, c->n, nc))) return r;
    if ((r = grow_copy(c, c->Y, c->n, nc))) return r;
    if ((r = grow_copy(c, c->YAW, c->n, nc))) return r;
    if ((r = grow_copy(c, c->PAR, c->n, nc))) return r;
    c->cap = nc;
    return PP_OK;
}

int ensure_events(pp_ctx* c, size_t count) {
    while (c->ev.size() < count) {
        hipEvent_t e;
        PP_HIP(hipEventCreate(&e));
        c->ev.push_back(e);
    }
    return PP_OK;
}

static_assert(PP_CF_CHAIN == kCfLevels + 2, "chain row layout");
constexpr int kCfBatch = 16384;     // nodes per check_finish launch
constexpr int kCfPtsCap = 1 << 16;  // line points per check_finish workgroup
static_assert(4 * kCfMaxEdges <= kCfPtsCap, "cf_line_kernel keeps 4 doubles per edge in the hypot buffer");
// cf_line_kernel in two tiers (CfLines): tier 1 runs every line on kCfLineGrid workgroups with
// room for kCfLinePts1 points and a kCfLinePath1-deep path each (3 x 6144 doubles: 144 KB; the
// config-3 plan's lines have ~2400 points), tier 2 the few longer or deeper ones at the full
// capacities (kCfPtsCap points, kCfMaxDepth) on kCfLineGrid2 workgroups (1.5 MB each).  Round 5
// gave every one of 2048 workgroups the full capacity: 3.2 GB.  1024 tier-1
// workgroups cost the config-3 plan ~0.5 ms of its 12.5 (one wave per line: the lines in flight
// are the workgroups), so the grid stays at 2048 (300 MB).
constexpr int kCfLineGrid = 2048;
constexpr int kCfLinePts1 = 6144;
constexpr int kCfLinePath1 = 1024;
constexpr int kCfLineGrid2 = 64;
constexpr int kCfSpillCap = 1 << 17;  // tier-1 lines handed to tier 2 per launch
static_assert(4 * (kCfLinePath1 + kCfLevels + 1) <= kCfLinePts1, "tier 1: 4 doubles per edge");
// phase A's task arrays (status, lists, SteerTask, StarTaskExt, yaw, None flag per task) are
// sized for span x (items + queries) tasks: a span that would need more than this is clamped (the
// spans change which candidates are walked together, never a result); the records (PrepRec,
// 256 B a task) are steered in chunks of kCfbRecChunk tasks
constexpr size_t kCfbTaskBudget = (size_t)512 << 20;
constexpr size_t kCfbRecChunk = (size_t)1 << 20;

// check_finish for nodes[0, k) (device pointer already filled); results on the device
// The goal of a check_finish_kernel launch: the planner's (check_finish), or a caller-built goal
// node (finalize), and the kernel mode / optimize's starting level.
struct CfGoal {
    double x, y, yaw, yaw_opt;
    int level0 = 0, mode = kCfCheck;
};

// Where a check_finish_kernel launch writes its per-node results (device pointers).
struct CfOut {
    int* ok;
    double* len;
    int* npts;
    int* chain;  // may be null
};

// cf_line_kernel's buffers for a launch of `wgs` tier-1 workgroups (CfLines).  spill == 0: one
// tier at the full capacities (a one-node call, whose line the host reads from workgroup 0's
// buffer); else tier 1 hands up to `spill` lines to tier 2.  The spill count is zeroed on the
// stream.
int cf_line_buffers(pp_ctx* c, int wgs, int spill, CfLines& L) {
    const bool two = spill > 0;
    const int pc1 = two ? kCfLinePts1 : kCfPtsCap, dc1 = two ? kCfLinePath1 : kCfMaxDepth;
    const int g2 = two ? std::min(kCfLineGrid2, wgs) : 0;
    const size_t e1 = 2 * (size_t)(dc1 + kCfLevels + 1), e2 = 2 * (size_t)kCfMaxEdges;
    PP_HIP(c->cf_pts.reserve((size_t)wgs * 3 * pc1 + (size_t)g2 * 3 * kCfPtsCap));
    PP_HIP(c->cf_etab.reserve((size_t)wgs * e1 + (size_t)g2 * e2));
    PP_HIP(c->cf_lpath.reserve((size_t)wgs * dc1 + (size_t)g2 * kCfMaxDepth));
    L.grid1 = wgs;
    L.t1 = CfLineBufs{c->cf_pts.p, pc1, c->cf_etab.p, c->cf_lpath.p, dc1, nullptr};
    if (two) {
        PP_HIP(c->cf_spill.reserve(1 + (size_t)spill * kCfItem));
        PP_HIP(hipMemsetAsync(c->cf_spill.p, 0, sizeof(int), c->stream));
        L.t1.spill = c->cf_spill.p;
        L.t1.spill_cap = spill;
        L.grid2 = g2;
        L.t2 = CfLineBufs{c->cf_pts.p + (size_t)wgs * 3 * pc1, kCfPtsCap,
                          c->cf_etab.p + (size_t)wgs * e1, c->cf_lpath.p + (size_t)wgs * dc1,
                          kCfMaxDepth, nullptr};
    }
    return PP_OK;
}

// check_finish_kernel over nodes[0, k) (device) with its error handling; the one-tree planner
// (cb.qidx null: the context's tree, goal g) or a query batch (cb)
int cf_run(pp_ctx* c, const TreeDev& tr, const int* nodes, int k, int want_line, int grid,
           const CfGoal& gg, const CfOut& o, const CfBatch& cb_in) {
    const CfGoal* g = &gg;
    PP_HIP(c->cf_err.reserve(2));  // [0] error bits, [1] the kernel's node counter
    // optimize's memo: two ints per tree row (the batch's Q * row_cap rows, or the tree's nodes),
    // zeroed for this launch
    CfBatch cb = cb_in;
    // (a batch's memo rows are compact: its items plus a root per query)
    const size_t rows = cb.qidx ? (cb.moff ? (size_t)k + c->mq_Q : (size_t)c->mq_Q * (size_t)cb.row_cap)
                                : (size_t)c->n;
    PP_HIP(c->cf_memo.reserve(2 * std::max<size_t>(rows, 1)));
    PP_HIP(hipMemsetAsync(c->cf_memo.p, 0, 2 * rows * sizeof(int), c->stream));
    cb.ftab = c->cf_memo.p;
    cb.gtab = c->cf_memo.p + rows;
    // the line buffers (per workgroup of the line kernel) only when lines are materialised: one
    // workgroup at the full capacities for a one-node call (the host reads workgroup 0's line),
    // else the two tiers
    const int wgs = std::min(grid, k);
    CfLines lines;
    if (want_line) {
        PP_HIP(c->cf_items.reserve(1 + (size_t)k * kCfItem));
        PP_HIP(hipMemsetAsync(c->cf_items.p, 0, sizeof(int), c->stream));
        int r = cf_line_buffers(c, wgs, wgs > 1 ? std::min(k, kCfSpillCap) : 0, lines);
        if (r) return r;
    }
    // the ancestor paths of check_finish_kernel's waves (kCfWaves per workgroup, at most
    // min(grid, k / kCfWaves) workgroups)
    PP_HIP(c->cf_path.reserve((size_t)std::min(grid, (k + kCfWaves - 1) / kCfWaves) * kCfWaves * kCfMaxDepth));
    PP_HIP(c->api_lit_scratch.reserve((size_t)kLiteralWaves * 3 * kLiteralCap));
    if (!c->lit_locks.p) {  // the literal scratch pool's slot locks (zero: free)
        PP_HIP(c->lit_locks.reserve(kLiteralWaves));
        PP_HIP(hipMemsetAsync(c->lit_locks.p, 0, kLiteralWaves * sizeof(int), c->stream));
    }
    PP_HIP(hipMemsetAsync(c->cf_err.p, 0, 2 * sizeof(int), c->stream));
    if (c->prof) {
        if (int r = ensure_events(c, 2)) return r;
        PP_HIP(hipEventRecord(c->ev[0], c->stream));
    }
    SceneDev sd = c->scene_dev();
    if (cb.qidx) sd.step_size = c->mq_step;  // a query batch's edges use the batch's step
    // check_finish_kernel reads the scene from device memory (a reference to the kernel-argument
    // struct would copy it to every lane's stack); uploaded when it changed.  The stream is
    // synchronised at the end of every cf_run, so the host copy is never overwritten in flight.
    if (!c->cf_scene_ok || std::memcmp(&c->cf_scene_host, &sd, sizeof sd) != 0) {
        if (!c->cf_scene.p) PP_HIP(c->cf_scene.reserve(1));
        c->cf_scene_host = sd;
        PP_HIP(hipMemcpyAsync(c->cf_scene.p, &c->cf_scene_host, sizeof sd,
                              hipMemcpyHostToDevice, c->stream));
        c->cf_scene_ok = true;
    }
    PP_HIP(launch_check_finish(c->stream, sd, c->cf_scene.p, tr, nodes, k, g->x, g->y,
                               g->yaw, g->yaw_opt, g->level0, g->mode, want_line, o.ok, o.len,
                               o.npts, o.chain, c->api_lit_scratch.p, c->lit_locks.p, lines,
                               c->cf_err.p, grid, c->prof ? c->cf_tally.p : nullptr, cb,
                               c->cf_path.p, want_line ? c->cf_items.p : nullptr));
    if (c->prof) PP_HIP(hipEventRecord(c->ev[1], c->stream));
    int err = 0;
    PP_HIP(hipMemcpyAsync(&err, c->cf_err.p, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    PP_HIP(hipStreamSynchronize(c->stream));
    if (c->prof) {
        float ms = 0.f;
        PP_HIP(hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
        c->finish_ms += ms;
        c->finish_launches += 1;
    }
    if (err & 2) return set_err(PP_ERR_REFERENCE_PANIC, "finalize: a Dubins edge has no feasible word (rrt.rs:529 panics)");
    if (err & 4) return set_err(PP_ERR_STEER_OVERFLOW, "generate_local_course would index past n_point");
    if (err & 1) return set_err(PP_ERR_CAPACITY, "tree deeper than the check_finish path capacity");
    if (err & 8) return set_err(PP_ERR_CAPACITY, "finalized line longer than the point capacity");
    return PP_OK;
}

// pp_batch_plan's check_finish in steer rounds (CfbArgs, pp_kernels.hip): phase A rounds fill
// ftab for every node, phase B the goal and copy edges, the assemble kernel decides every item
// whose verdicts are known, and check_finish_kernel runs the rest (literal paths, errors) with
// the memo filled.  The same results as cf_run over all items; polygon scenes and batches with
// a blocked root take cf_run.

int cf_run_rounds(pp_ctx* c, const TreeDev& tr, int total, const CfBatch& cb_in, const CfOut& o) {
    const int Q = c->mq_Q;
    const size_t nn = (size_t)total + Q;
    const size_t rows = nn;  // the compact memo rows (cb_in.moff): every item and root
    // phase A: <= span tasks per node; B: <= 2 per node.  The spans are clamped to the task budget
    // (at least 2: phase B's tasks)
    const size_t task_bytes = 3 * sizeof(int) + sizeof(SteerTask) + sizeof(StarTaskExt) +
                              sizeof(double) + 1;
    const int span_cap = (int)std::max<size_t>(2, kCfbTaskBudget / (task_bytes * std::max<size_t>(nn, 1)));
    const int span0 = std::min(c->cfb_span0, span_cap), span1 = std::min(c->cfb_span, span_cap);
    const size_t cap_tasks = std::max<size_t>((size_t)std::max({span0, span1, 2}) * nn, 1);
    hipStream_t st = c->stream;
    PP_HIP(c->cf_err.reserve(2));
    PP_HIP(c->cf_memo.reserve(2 * std::max<size_t>(rows, 1)));
    PP_HIP(c->cf_items.reserve(1 + (size_t)total * kCfItem));
    // cf_line_kernel's workgroups: one line at a time each — latency-bound, so more lines in
    // flight than check_finish_kernel's grid
    const int wgs = std::min(kCfLineGrid, total);
    CfLines lines;
    if (wgs > 0) {
        int r = cf_line_buffers(c, wgs, std::min(total, kCfSpillCap), lines);
        if (r) return r;
    }
    PP_HIP(c->api_lit_scratch.reserve((size_t)kLiteralWaves * 3 * kLiteralCap));
    if (!c->lit_locks.p) {
        PP_HIP(c->lit_locks.reserve(kLiteralWaves));
        PP_HIP(hipMemsetAsync(c->lit_locks.p, 0, kLiteralWaves * sizeof(int), st));
    }
    PP_HIP(c->cfb_nodei.reserve(4 * nn));
    PP_HIP(c->cfb_rows.reserve(std::max<size_t>(rows, 1)));
    PP_HIP(c->cfb_rows8.reserve(2 * std::max<size_t>(rows, 1)));
    PP_HIP(c->cfb_gotab.reserve(std::max(total, 1)));
    PP_HIP(c->cfb_plist.reserve(std::max(total, 1)));
    PP_HIP(c->cfb_tnode.reserve(cap_tasks));
    PP_HIP(c->cfb_status.reserve(cap_tasks));
    PP_HIP(c->cfb_lit.reserve(cap_tasks));
    PP_HIP(c->cfb_tasks.reserve(cap_tasks));
    PP_HIP(c->cfb_ext.reserve(cap_tasks));
    const size_t rec_cap = std::min(cap_tasks, kCfbRecChunk);
    PP_HIP(c->cfb_rec.reserve(rec_cap));
    PP_HIP(c->cfb_none.reserve(cap_tasks));
    PP_HIP(c->cfb_yaw.reserve(cap_tasks));
    PP_HIP(c->cfb_state.reserve(2));  // [0] the round's, [1] a chunk's
    PP_HIP(c->cfb_misc.reserve(4));
    PP_HIP(c->cfb_dhist.reserve(kCfbDepthBins));
    if (c->prof) PP_HIP(c->cfb_pts.reserve(3 * kWalkTallySlots));
    SceneDev sd = c->scene_dev();
    sd.step_size = c->mq_step;
    // the kernel's scene in device memory (cf_run's upload)
    if (!c->cf_scene_ok || std::memcmp(&c->cf_scene_host, &sd, sizeof sd) != 0) {
        if (!c->cf_scene.p) PP_HIP(c->cf_scene.reserve(1));
        c->cf_scene_host = sd;
        PP_HIP(hipMemcpyAsync(c->cf_scene.p, &c->cf_scene_host, sizeof sd, hipMemcpyHostToDevice, st));
        c->cf_scene_ok = true;
    }
    CfbArgs a;
    a.tr = tr;
    a.row_cap = cb_in.row_cap;
    a.nitems = total;
    a.Q = Q;
    a.qidx = cb_in.qidx;
    a.nodes = c->mp_nodes.p;
    a.goals = cb_in.goals;
    a.moff = cb_in.moff;
    a.ftab = c->cf_memo.p;
    a.gtab = c->cf_memo.p + rows;
    a.gotab = c->cfb_gotab.p;
    a.gclaim = c->cfb_rows.p;
    a.tnone = c->cfb_rows8.p;
    a.tnone_up = c->cfb_rows8.p + rows;
    a.depth = c->cfb_nodei.p;
    a.open = c->cfb_nodei.p + nn;
    a.tfirst = c->cfb_nodei.p + 2 * nn;
    a.tcnt = c->cfb_nodei.p + 3 * nn;
    a.tnode = c->cfb_tnode.p;
    a.tasks = c->cfb_tasks.p;
    a.ext = c->cfb_ext.p;
    a.rec = c->cfb_rec.p;
    a.none = c->cfb_none.p;
    a.status = c->cfb_status.p;
    a.yaw = c->cfb_yaw.p;
    a.st = c->cfb_state.p;
    a.maxdepth = c->cfb_misc.p;
    a.pcount = c->cfb_misc.p + 1;
    a.wsum = c->cfb_misc.p + 2;  // (the rounds' task counts: profiling)
    a.dhist = c->cfb_dhist.p;
    // per launch: memo, goal verdicts, claims, line items, error bits, counters, DevState
    PP_HIP(hipMemsetAsync(c->cf_memo.p, 0, 2 * rows * sizeof(int), st));
    PP_HIP(hipMemsetAsync(c->cfb_gotab.p, 0, (size_t)total * sizeof(int), st));
    PP_HIP(hipMemsetAsync(c->cfb_rows.p, 0, rows * sizeof(int), st));
    PP_HIP(hipMemsetAsync(c->cf_items.p, 0, sizeof(int), st));
    PP_HIP(hipMemsetAsync(c->cf_err.p, 0, 2 * sizeof(int), st));
    PP_HIP(hipMemsetAsync(c->cfb_misc.p, 0, 4 * sizeof(int), st));
    PP_HIP(hipMemsetAsync(c->cfb_dhist.p, 0, kCfbDepthBins * sizeof(int), st));
    PP_HIP(hipMemsetAsync(c->cfb_state.p, 0, 2 * sizeof(DevState), st));
    if (c->prof) PP_HIP(hipMemsetAsync(c->cfb_pts.p, 0, 3 * kWalkTallySlots * sizeof(long long), st));
    if (c->prof) {
        if (int r = ensure_events(c, 2)) return r;
        PP_HIP(hipEventRecord(c->ev[0], st));
    }
    PP_HIP(launch_cfb(st, sd, a, kCfbDepth, 0));
    int misc[4] = {0, 0, 0, 0};
    int dh[kCfbDepthBins];
    PP_HIP(hipMemcpyAsync(misc, c->cfb_misc.p, sizeof misc, hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(dh, c->cfb_dhist.p, sizeof dh, hipMemcpyDeviceToHost, st));
    PP_HIP(hipStreamSynchronize(st));
    // a bound on round (m0, span)'s tasks: a node of depth d emits min(span, d + 1 - m0) of them
    // (fewer once it settled); the last bin's nodes (that depth or more) count span each
    auto round_bound = [&](int m0, int span) -> size_t {
        size_t t = 0;
        for (int d = 0; d < kCfbDepthBins; ++d) {
            const int e = d == kCfbDepthBins - 1 ? span : std::min(span, d + 1 - m0);
            if (e > 0) t += (size_t)e * (size_t)dh[d];
        }
        return t;
    };
    // round r tests the candidates at depths m0 .. m0 + span - 1 of every open node: the first
    // round cfb_span0 of them, the later ones cfb_span
    long long* wpts = c->prof ? c->cfb_pts.p : nullptr;
    // a round's steer over its a.st->W (<= mt) tasks, rec_cap records at a time
    auto steer = [&](int mt, bool own_yaw) -> int {
        for (size_t base = 0; base < (size_t)mt; base += rec_cap) {
            const int cn = (int)std::min(rec_cap, (size_t)mt - base);
            CfbArgs ac = a;
            ac.st = c->cfb_state.p + 1;
            ac.tasks += base;
            ac.ext += base;
            ac.status += base;
            ac.yaw += base;
            PP_HIP(launch_cfb_chunk(st, a.st, ac.st, (int)base, cn, true, nullptr, nullptr));
            PP_HIP(launch_cfb_steer(st, sd, ac, cn, own_yaw, wpts));
            PP_HIP(launch_cfb_chunk(st, a.st, ac.st, (int)base, cn, false, ac.rec, a.none + base));
        }
        return PP_OK;
    };
    int rounds = 0;
    for (int m0 = 0; m0 <= misc[0]; ++rounds) {
        a.span = rounds == 0 ? span0 : span1;
        const int mt = (int)std::min<size_t>(cap_tasks, std::min<size_t>((size_t)a.span * nn,
                                                                         round_bound(m0, a.span)));
        PP_HIP(launch_cfb(st, sd, a, kCfbEmitA, m0));
        if (int r = steer(mt, false)) return r;
        PP_HIP(launch_cfb_literal(st, sd, a, mt, c->cfb_lit.p, c->cfb_misc.p + 3, c->api_lit_scratch.p));
        PP_HIP(launch_cfb(st, sd, a, kCfbConsumeA, m0));
        m0 += a.span;
    }
    PP_HIP(launch_cfb(st, sd, a, kCfbEmitB, 0));
    if (int r = steer((int)std::min<size_t>(cap_tasks, 2 * nn), true)) return r;
    PP_HIP(launch_cfb_literal(st, sd, a, (int)std::min<size_t>(cap_tasks, 2 * nn), c->cfb_lit.p,
                              c->cfb_misc.p + 3, c->api_lit_scratch.p));
    PP_HIP(launch_cfb(st, sd, a, kCfbStoreB, (int)std::min<size_t>(cap_tasks, 2 * nn)));
    PP_HIP(launch_cfb(st, sd, a, kCfbAssemble, 0, o.ok, o.len, o.npts, c->cf_err.p, c->cf_items.p,
                      c->cfb_plist.p));
    PP_HIP(hipMemcpyAsync(misc, c->cfb_misc.p, sizeof misc, hipMemcpyDeviceToHost, st));
    PP_HIP(hipStreamSynchronize(st));
    const int np = misc[1];
    CfBatch cb = cb_in;
    cb.ftab = a.ftab;
    cb.gtab = a.gtab;
    cb.gotab = a.gotab;
    // the items left (unknown verdicts) on check_finish_kernel, then every line item's points
    PP_HIP(c->cf_path.reserve((size_t)std::max(1, std::min(kCfGrid, (np + kCfWaves - 1) / kCfWaves)) *
                              kCfWaves * kCfMaxDepth));
    PP_HIP(launch_check_finish(st, sd, c->cf_scene.p, tr, c->mp_nodes.p, np, 0.0, 0.0, 0.0, 0.0, 0,
                               kCfCheck, 1, o.ok, o.len, o.npts, nullptr, c->api_lit_scratch.p,
                               c->lit_locks.p, lines, c->cf_err.p, kCfGrid,
                               c->prof ? c->cf_tally.p : nullptr, cb, c->cf_path.p, c->cf_items.p,
                               c->cfb_plist.p));
    if (c->prof) PP_HIP(hipEventRecord(c->ev[1], st));
    int err = 0;
    PP_HIP(hipMemcpyAsync(&err, c->cf_err.p, sizeof(int), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(misc, c->cfb_misc.p, sizeof misc, hipMemcpyDeviceToHost, st));
    PP_HIP(hipStreamSynchronize(st));
    if (c->prof) {
        float ms = 0.f;
        PP_HIP(hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
        c->finish_ms += ms;
        c->finish_launches += 1;
        c->cfb_nodes += total - np;
        c->cfb_edges += misc[2];
        std::vector<long long> v(3 * kWalkTallySlots);
        PP_HIP(hipMemcpy(v.data(), c->cfb_pts.p, v.size() * sizeof(long long), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < 2 * (size_t)kWalkTallySlots; ++i)
            (i < (size_t)kWalkTallySlots ? c->cfb_points : c->cfb_arc) += v[i];
    }
    if (err & 2) return set_err(PP_ERR_REFERENCE_PANIC, "finalize: a Dubins edge has no feasible word (rrt.rs:529 panics)");
    if (err & 4) return set_err(PP_ERR_STEER_OVERFLOW, "generate_local_course would index past n_point");
    if (err & 1) return set_err(PP_ERR_CAPACITY, "tree deeper than the check_finish path capacity");
    if (err & 8) return set_err(PP_ERR_CAPACITY, "finalized line longer than the point capacity");
    return PP_OK;
}

// check_finish of the one-tree planner for cf_nodes[0, k) into the context's cf_* buffers
int cf_launch(pp_ctx* c, int k, int want_line, int grid, const CfGoal* g = nullptr) {
    const CfGoal dflt{c->goal[0], c->goal[1], c->goal[2], c->goal[2]};
    PP_HIP(c->cf_ok.reserve(kCfBatch));
    PP_HIP(c->cf_len.reserve(kCfBatch));
    PP_HIP(c->cf_npts.reserve(kCfBatch));
    PP_HIP(c->cf_chain.reserve((size_t)kCfBatch * (kCfLevels + 2)));
    return cf_run(c, c->tree_dev(), c->cf_nodes.p, k, want_line, grid, g ? *g : dflt,
                  CfOut{c->cf_ok.p, c->cf_len.p, c->cf_npts.p, c->cf_chain.p}, CfBatch{});
}

MqArgs mq_args(pp_ctx* c) {
    MqArgs a;
    a.mq.Q = c->mq_Q;
    a.mq.cap = c->mq_cap;
    a.mq.max_iter = c->mq_max_iter;
    a.mq.x = c->mq_x.p;
    a.mq.y = c->mq_y.p;
    a.mq.yaw = c->mq_yaw.p;
    a.mq.parent = c->mq_par.p;
    a.mq.n = c->mq_n.p;
    a.mq.it = c->mq_it.p;
    a.mq.evals = c->mq_evals.p;
    a.mq.seed = c->mq_seed.p;
    a.mq.blocked = c->mq_any_blocked ? c->mq_blocked.p : nullptr;
    a.mq.K = c->mq_K;
    a.mq.target = c->mq_target.p;
    a.mq.nnd2 = c->mq_nnd2.p;
    a.mq.it_prev = c->mq_itprev.p;
    a.mq.status = c->mq_status.p;
    a.mq.alist = c->mq_alist.p;
    a.mq.ctask = c->mq_ctask.p;
    a.mq.lstat = c->mq_lstat.p;
    a.mq.tyaw = c->mq_yawbuf.p;
    a.sc = c->scene_dev();
    a.sc.step_size = c->mq_step;
    a.st = c->mq_state.p;
    a.tasks = c->mq_tasks.p;
    a.rec = c->mq_rec.p;
    a.status = c->mq_status.p;
    a.yaw = c->mq_yawbuf.p;
    a.lit_scratch = c->api_lit_scratch.p;
    a.lit_locks = c->lit_locks.p;
    a.err = c->mq_err.p;
    a.wg_points = c->prof_points();
    a.scp = c->mq_scene.p;  // (uploaded by pp_batch_extend)
    a.mq.st = a.st;
    return a;
}

// Sub-batch s of nsub (queries [Q*s/nsub, Q*(s+1)/nsub)): a view of the batch with offset
// per-query pointers and its own DevState, so the sub-batches run their lockstep steps on their
// own streams and one's small kernels overlap another's walk.  Results do not depend on the
// split: queries are independent.
constexpr int kMaxSub = 4;
constexpr size_t kLstatPad = 1024;  // >= the walk's grid (kWalkMaxWG)
// streams: 2 for the extend batch (2: 289M it/s at 8192 queries, 177M on a 1024-query shard; 3:
// 291M / 160M; 4: 244M / 109M), 3 for RRT* (11 kernels a step: 16.4M / 4.5M against 15.0M / 4.2M
// with 2; 4 streams collapse to 10.7M / 2.4M, the box runs 4 hardware queues per process)
int mq_nsub(int Q, int dflt = 2) {
    int n = Q >= 256 ? dflt : 1;
    return std::min(n, std::max(Q, 1));
}
MqArgs mq_sub_args(pp_ctx* c, int sub, int nsub) {
    MqArgs a = mq_args(c);
    const int Q = c->mq_Q, K = c->mq_K;
    const int q0 = (int)((int64_t)Q * sub / nsub), q1 = (int)((int64_t)Q * (sub + 1) / nsub);
    const size_t r0 = (size_t)q0 * c->mq_cap, t0 = (size_t)q0 * K;
    a.mq.Q = q1 - q0;
    a.mq.x += r0;
    a.mq.y += r0;
    a.mq.yaw += r0;
    a.mq.parent += r0;
    a.mq.n += q0;
    a.mq.it += q0;
    a.mq.evals += q0;
    a.mq.seed += q0;
    if (a.mq.blocked) a.mq.blocked += q0;
    a.mq.target += q0;
    a.mq.nnd2 += t0;
    if (a.mq.it_prev) a.mq.it_prev += q0;
    if (a.mq.status) a.mq.status += t0;
    if (a.mq.alist) a.mq.alist += t0;
    if (a.mq.ctask) a.mq.ctask += t0;
    // (a sub-batch's verdict array spans its tasks plus one walk grid: DevState::lper rounds up)
    if (a.mq.lstat) a.mq.lstat += t0 + (size_t)sub * kLstatPad;
    if (a.mq.tyaw) a.mq.tyaw += t0;
    a.st = c->mq_state.p + 1 + sub;
    a.mq.st = a.st;
    a.tasks += t0;
    a.rec += t0;
    a.status += t0;
    a.yaw += t0;
    return a;
}

// DevState 0: the whole batch; 1 + s: sub-batch s of mq_nsub
int mq_write_states(pp_ctx* c, hipStream_t st) {
    DevState ds[1 + kMaxSub] = {};
    const int Q = c->mq_Q, nsub = c->mq_nsub;
    // W counts the step's active tasks (mq_sample_nn lists them, the insert resets it): 0 here;
    // each state's list is its task region's part of mq_alist
    ds[0].alist = c->mq_alist.p;
    for (int s = 0; s < nsub; ++s)
        ds[1 + s].alist = c->mq_alist.p + (size_t)((int64_t)Q * s / nsub) * c->mq_K;
    PP_HIP(hipMemcpyAsync(c->mq_state.p, ds, sizeof ds, hipMemcpyHostToDevice, st));
    PP_HIP(hipStreamSynchronize(st));  // ds lives on this stack frame
    return PP_OK;
}

// per-step task buffers of the batch: K slots per query
int mq_reserve_tasks(pp_ctx* c, int q, int K) {
    const size_t tq = (size_t)q * K;
    PP_HIP(c->mq_tasks.reserve(tq));
    PP_HIP(c->mq_ctask.reserve(tq));
    PP_HIP(c->mq_status.reserve(tq));
    PP_HIP(c->mq_yawbuf.reserve(tq));
    PP_HIP(c->mq_rec.reserve(tq));
    PP_HIP(c->mq_nnd2.reserve(tq));
    PP_HIP(c->mq_alist.reserve(tq));
    PP_HIP(c->mq_lstat.reserve(tq + (size_t)kMaxSub * kLstatPad));
    return PP_OK;
}

// |X_near| of an insert into an n-node RRT* tree: k_fixed, or the k-nearest RRT* schedule
// ceil(2e ln n) (Karaman & Frazzoli), capped at kStarKMax and at n (orc_star_k restates it)
int star_k(int k_fixed, int n) {
    int k;
    if (k_fixed > 0) {
        k = k_fixed;
    } else {
        const double v = n > 1 ? std::ceil(2.0 * 2.718281828459045 * std::log((double)n)) : 1.0;
        k = v < 1.0 ? 1 : (v > kStarKMax ? kStarKMax : (int)v);
    }
    if (k > kStarKMax) k = kStarKMax;
    return k < n ? k : n;
}

StarArgs star_args(pp_ctx* c) {
    StarArgs a;
    StarDev& d = a.sd;
    d.mq.Q = c->star_Q;
    d.mq.cap = c->star_cap;
    d.mq.max_iter = c->star_max_iter;
    d.mq.x = c->sr_x.p;
    d.mq.y = c->sr_y.p;
    d.mq.yaw = c->sr_yaw.p;
    d.mq.parent = c->sr_par.p;
    d.mq.n = c->sr_n.p;
    d.mq.it = c->sr_it.p;
    d.mq.evals = c->sr_evals.p;
    d.mq.seed = c->sr_seed.p;
    d.mq.blocked = c->sr_any_blocked ? c->sr_blocked.p : nullptr;
    d.mq.K = 1;
    d.mq.target = c->sr_target.p;
    d.cost = c->sr_cost.p;
    d.elen = c->sr_elen.p;
    d.mark = c->sr_mark.p;
    d.stamp = c->sr_stamp.p;
    d.ksched = c->sr_ksched.p;
    d.eta = c->star_eta;
    d.px = c->sr_px.p;
    d.py = c->sr_py.p;
    d.pn = c->sr_pn.p;
    d.near = c->sr_near.p;
    d.nnear = c->sr_nnear.p;
    d.bslot = c->sr_bslot.p;
    d.cslot = c->sr_cslot.p;
    d.cmask = c->sr_cmask.p;
    d.bmask = c->sr_bmask.p;
    d.curv = 1.0 / c->max_steer;
    d.lit_locks = c->lit_locks.p;
    d.cb = c->sr_cb.p;
    d.rewires = c->sr_rew.p;
    d.stA = c->sr_state.p;
    d.stB = c->sr_state.p + 1;
    d.stC = c->sr_state.p + 2;
    a.sc = c->scene_dev();
    a.sc.step_size = c->star_step;
    a.tA = c->sr_tA.p;
    a.tB = c->sr_tB.p;
    a.tC = c->sr_tC.p;
    a.eB = c->sr_eB.p;
    a.eC = c->sr_eC.p;
    a.sA = c->sr_sA.p;
    a.sB = c->sr_sB.p;
    a.sC = c->sr_sC.p;
    a.yA = c->sr_yA.p;
    a.yB = c->sr_yB.p;
    a.yC = c->sr_yC.p;
    a.cA = c->sr_cA.p;
    a.cB = c->sr_cB.p;
    a.cC = c->sr_cC.p;
    a.rec = c->sr_rec.p;
    a.lit_scratch = c->api_lit_scratch.p;
    a.err = c->sr_err.p;
    a.wg_points = c->prof_points();
    return a;
}

// Sub-batch s of nsub of the RRT* batch (as mq_sub_args): offset per-query pointers, its own
// round states and task regions (rounds B / C: kStarKMax slots per query)
StarArgs star_sub_args(pp_ctx* c, int sub, int nsub) {
    StarArgs a = star_args(c);
    const int Q = c->star_Q;
    const int q0 = (int)((int64_t)Q * sub / nsub), q1 = (int)((int64_t)Q * (sub + 1) / nsub);
    const size_t r0 = (size_t)q0 * c->star_cap, b0 = (size_t)q0 * kStarKMax;
    StarDev& d = a.sd;
    d.mq.Q = q1 - q0;
    d.mq.x += r0;
    d.mq.y += r0;
    d.mq.yaw += r0;
    d.mq.parent += r0;
    d.mq.n += q0;
    d.mq.it += q0;
    d.mq.evals += q0;
    d.mq.seed += q0;
    if (d.mq.blocked) d.mq.blocked += q0;
    d.mq.target += q0;
    d.cost += r0;
    d.elen += r0;
    d.mark += r0;
    d.stamp += q0;
    d.px += q0;
    d.py += q0;
    d.pn += q0;
    d.near += b0;
    d.nnear += q0;
    d.bslot += q0;
    d.bmask += q0;
    d.cslot += q0;
    d.cmask += q0;
    d.cb += q0;
    d.rewires += q0;
    d.stA = c->sr_state.p + 3 * (1 + sub);
    d.stB = d.stA + 1;
    d.stC = d.stA + 2;
    a.tA += q0;
    a.sA += q0;
    a.yA += q0;
    a.cA += q0;
    a.tB += b0;
    a.tC += b0;
    a.eB += b0;
    a.eC += b0;
    a.sB += b0;
    a.sC += b0;
    a.yB += b0;
    a.yC += b0;
    a.cB += b0;
    a.cC += b0;
    a.rec += b0;
    return a;
}

int star_totals(pp_ctx* c, int64_t* it_sum, int64_t* n_sum, int64_t* rw_sum) {
    const int Q = c->star_Q;
    std::vector<int> hn(Q);
    std::vector<int64_t> hit(Q), hrw(Q);
    PP_HIP(hipMemcpyAsync(hn.data(), c->sr_n.p, Q * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    PP_HIP(hipMemcpyAsync(hit.data(), c->sr_it.p, Q * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
    PP_HIP(hipMemcpyAsync(hrw.data(), c->sr_rew.p, Q * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
    PP_HIP(hipStreamSynchronize(c->stream));
    int64_t a = 0, b = 0, w = 0;
    for (int i = 0; i < Q; ++i) {
        a += hit[i];
        b += hn[i];
        w += hrw[i];
    }
    *it_sum = a;
    *n_sum = b;
    *rw_sum = w;
    return PP_OK;
}

int mq_totals(pp_ctx* c, int64_t* it_sum, int64_t* n_sum) {
    std::vector<int> hn(c->mq_Q);
    std::vector<int64_t> hit(c->mq_Q);
    PP_HIP(hipMemcpyAsync(hn.data(), c->mq_n.p, c->mq_Q * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    PP_HIP(hipMemcpyAsync(hit.data(), c->mq_it.p, c->mq_Q * sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
    PP_HIP(hipStreamSynchronize(c->stream));
    int64_t a = 0, b = 0;
    for (int i = 0; i < c->mq_Q; ++i) {
        a += hit[i];
        b += hn[i];
    }
    *it_sum = a;
    *n_sum = b;
    return PP_OK;
}
}  // namespace

// ===================================================================================== C ABI

extern "C" {

int pp_abi_version(void) { return PP_ABI_VERSION; }

const char* pp_last_error(void) { return g_err.c_str(); }

int pp_device_count(int* n) {
    if (!n) return set_err(PP_ERR_INVALID_ARGUMENT, "null output");
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) c = 0;
    *n = c;
    return PP_OK;
}

int pp_create(int device, pp_ctx** out) {
    if (!out) return set_err(PP_ERR_INVALID_ARGUMENT, "null output");
    *out = nullptr;
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess || cnt <= 0)
        return set_err(PP_ERR_NO_DEVICE, "no HIP device visible (the product path has no CPU fallback)");
    if (device < 0 || device >= cnt) return set_err(PP_ERR_INVALID_ARGUMENT, "device index out of range");
    PP_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    PP_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return set_err(PP_ERR_NO_DEVICE, std::string("built for gfx950, device is ") + prop.gcnArchName);
    pp_ctx* c = new pp_ctx();
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = c->d_state.reserve(1);
    if (e == hipSuccess) e = c->d_api_state.reserve(1);
    if (e == hipSuccess) e = c->h_state.reserve(2);
    if (e != hipSuccess) {
        delete c;
        return set_err(PP_ERR_HIP, std::string("context setup: ") + hipGetErrorString(e));
    }
    *out = c;
    return PP_OK;
}

int pp_destroy(pp_ctx* ctx) {
    if (!ctx) return PP_OK;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    delete ctx;
    return PP_OK;
}

int pp_synchronize(pp_ctx* ctx) {
    int r = check_ctx(ctx, false, false);
    if (r) return r;
    PP_HIP(hipStreamSynchronize(ctx->stream));
    return PP_OK;
}

uint64_t pp_rng_u64(uint64_t seed, uint64_t ctr) { return rng_u64(seed, ctr); }

double pp_gen_range(uint64_t seed, uint64_t ctr, double low, double high) {
    return gen_range(seed, ctr, low, high);
}

double pp_mod2pi(double theta) { return mod2pi(theta); }

double pp_pi_2_pi(double angle) { return pi_2_pi(angle); }

int pp_dubins_path_planning_batch(pp_ctx* ctx, const pp_dubins_config* confs, int n, int cap,
                                  double* px, double* py, double* pyaw, int32_t* n_points,
                                  int32_t* word, double* cost) {
    int r = check_ctx(ctx, false, false);
    if (r) return r;
    if (n < 0 || cap <= 0 || (n > 0 && (!confs || !px || !py || !pyaw || !n_points || !word || !cost)))
        return set_err(PP_ERR_INVALID_ARGUMENT, "bad dubins batch arguments");
    if (n == 0) return PP_OK;
    for (int i = 0; i < n; ++i)
        if (!(confs[i].turn_radius > 0.0) || !(confs[i].step_size > 0.0))
            return set_err(PP_ERR_INVALID_ARGUMENT, "turn_radius and step_size must be > 0");
    static_assert(sizeof(pp_dubins_config) == 8 * sizeof(double), "DubinsConfig layout");
    const size_t nn = (size_t)n, tot = nn * (size_t)cap;
    DBuf<double> dconf, dpx, dpy, dpyaw, dcost;
    DBuf<int> dn, dword, dstat;
    PP_HIP(dconf.reserve(nn * 8));
    PP_HIP(dpx.reserve(tot));
    PP_HIP(dpy.reserve(tot));
    PP_HIP(dpyaw.reserve(tot));
    PP_HIP(dcost.reserve(nn));
    PP_HIP(dn.reserve(nn));
    PP_HIP(dword.reserve(nn));
    PP_HIP(dstat.reserve(nn));
    hipStream_t st = ctx->stream;
    PP_HIP(hipMemcpyAsync(dconf.p, confs, nn * 8 * sizeof(double), hipMemcpyHostToDevice, st));
    PP_HIP(launch_dubins_batch(st, dconf.p, n, cap, dpx.p, dpy.p, dpyaw.p, dn.p, dword.p, dcost.p, dstat.p));
    std::vector<int> stat(nn), nv(nn), wv(nn);
    PP_HIP(hipMemcpyAsync(px, dpx.p, tot * sizeof(double), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(py, dpy.p, tot * sizeof(double), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(pyaw, dpyaw.p, tot * sizeof(double), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(cost, dcost.p, nn * sizeof(double), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(nv.data(), dn.p, nn * sizeof(int), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(wv.data(), dword.p, nn * sizeof(int), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(stat.data(), dstat.p, nn * sizeof(int), hipMemcpyDeviceToHost, st));
    PP_HIP(hipStreamSynchronize(st));
    bool overflow = false;
    for (size_t i = 0; i < nn; ++i) {
        if (stat[i] == kSteerOverflow) {
            overflow = true;
            word[i] = -2;
            n_points[i] = 0;
        } else if (stat[i] == kSteerNone) {
            word[i] = -1;
            n_points[i] = 0;
        } else {
            word[i] = wv[i];
            n_points[i] = nv[i];
        }
    }
    if (overflow) return set_err(PP_ERR_CAPACITY, "a configuration needs more than cap points");
    return PP_OK;
}

int pp_dubins_path_planning_from_origin_batch(pp_ctx* ctx, const double* conf5, int n, int cap,
                                              double* px, double* py, double* pyaw,
                                              int32_t* n_points, int32_t* word, double* cost) {
    int r = check_ctx(ctx, false, false);
    if (r) return r;
    if (n < 0 || cap <= 0 || (n > 0 && (!conf5 || !px || !py || !pyaw || !n_points || !word || !cost)))
        return set_err(PP_ERR_INVALID_ARGUMENT, "bad dubins batch arguments");
    if (n == 0) return PP_OK;
    for (int i = 0; i < n; ++i)
        if (!(conf5[5 * i + 4] > 0.0))
            return set_err(PP_ERR_INVALID_ARGUMENT, "step_size must be > 0");
    const size_t nn = (size_t)n, tot = nn * (size_t)cap;
    DBuf<double> dconf, dpx, dpy, dpyaw, dcost;
    DBuf<int> dn, dword, dstat;
    PP_HIP(dconf.reserve(nn * 5));
    PP_HIP(dpx.reserve(tot));
    PP_HIP(dpy.reserve(tot));
    PP_HIP(dpyaw.reserve(tot));
    PP_HIP(dcost.reserve(nn));
    PP_HIP(dn.reserve(nn));
    PP_HIP(dword.reserve(nn));
    PP_HIP(dstat.reserve(nn));
    hipStream_t st = ctx->stream;
    PP_HIP(hipMemcpyAsync(dconf.p, conf5, nn * 5 * sizeof(double), hipMemcpyHostToDevice, st));
    PP_HIP(launch_dubins_origin(st, dconf.p, n, cap, dpx.p, dpy.p, dpyaw.p, dn.p, dword.p, dcost.p, dstat.p));
    std::vector<int> stat(nn), nv(nn), wv(nn);
    PP_HIP(hipMemcpyAsync(px, dpx.p, tot * sizeof(double), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(py, dpy.p, tot * sizeof(double), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(pyaw, dpyaw.p, tot * sizeof(double), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(cost, dcost.p, nn * sizeof(double), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(nv.data(), dn.p, nn * sizeof(int), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(wv.data(), dword.p, nn * sizeof(int), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(stat.data(), dstat.p, nn * sizeof(int), hipMemcpyDeviceToHost, st));
    PP_HIP(hipStreamSynchronize(st));
    bool overflow = false;
    for (size_t i = 0; i < nn; ++i) {
        if (stat[i] == kSteerOverflow) {
            overflow = true;
            word[i] = -2;
            n_points[i] = 0;
        } else if (stat[i] == kSteerNone) {
            word[i] = -1;
            n_points[i] = 0;
        } else {
            word[i] = wv[i];
            n_points[i] = nv[i];
        }
    }
    if (overflow) return set_err(PP_ERR_CAPACITY, "a configuration needs more than cap points");
    return PP_OK;
}

int pp_dubins_words_batch(pp_ctx* ctx, const double* abd, int n, double* tpq, int32_t* ok) {
    int r = check_ctx(ctx, false, false);
    if (r) return r;
    if (n < 0 || (n > 0 && (!abd || !tpq || !ok)))
        return set_err(PP_ERR_INVALID_ARGUMENT, "bad dubins words arguments");
    if (n == 0) return PP_OK;
    const size_t nn = (size_t)n;
    DBuf<double> dabd, dtpq;
    DBuf<int> dok;
    PP_HIP(dabd.reserve(3 * nn));
    PP_HIP(dtpq.reserve(18 * nn));
    PP_HIP(dok.reserve(6 * nn));
    hipStream_t st = ctx->stream;
    PP_HIP(hipMemcpyAsync(dabd.p, abd, 3 * nn * sizeof(double), hipMemcpyHostToDevice, st));
    PP_HIP(launch_dubins_words(st, dabd.p, n, dtpq.p, dok.p));
    static_assert(sizeof(int) == sizeof(int32_t), "ok words");
    PP_HIP(hipMemcpyAsync(tpq, dtpq.p, 18 * nn * sizeof(double), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(ok, dok.p, 6 * nn * sizeof(int), hipMemcpyDeviceToHost, st));
    PP_HIP(hipStreamSynchronize(st));
    return PP_OK;
}

int pp_create_circle(double cx, double cy, double radius, double* xy, int cap, int* n) {
    if (!n || !(radius > 0.0) || cap < 0 || (cap > 0 && !xy))
        return set_err(PP_ERR_INVALID_ARGUMENT, "bad create_circle arguments");
    // rrt.rs:43-60: circum = 2 PI r; n = ceil(circum / 1.0); vertices 0..(n + 1) as usize
    const double kPi = 3.14159265358979323846;
    const double circum = 2.0 * kPi * radius;
    const double nf = std::ceil(circum / 1.0);
    if (!(nf < 1.0e8)) return set_err(PP_ERR_INVALID_ARGUMENT, "radius too large");
    const int count = (int)(nf + 1.0);
    *n = count;
    if (cap < count) return cap == 0 ? PP_OK : set_err(PP_ERR_CAPACITY, "vertex buffer too small");
    for (int i = 0; i < count; ++i) {
        const double a = 2.0 * kPi / nf * (double)i;
        xy[2 * i] = std::cos(a) * radius + cx;
        xy[2 * i + 1] = std::sin(a) * radius + cy;
    }
    return PP_OK;
}

namespace {
static_assert(sizeof(scene::CullDisc) == sizeof(float4), "cull disc layout");

// upload the item grid (pp_scene.cpp) and its LDS image; set the context's grid fields
int upload_item_grid(pp_ctx* ctx, double minx, double maxx, double miny, double maxy,
                     const scene::Items& items) {
    const scene::ItemGrid g =
        scene::build_item_grid(minx, maxx, miny, maxy, items, scene::kLdsImage);
    const int m = (int)items.d4.size();
    PP_HIP(ctx->d_goff.reserve(g.goff.size()));
    PP_HIP(ctx->d_gitems.reserve(std::max<size_t>(g.gitems.size(), 1)));
    PP_HIP(hipMemcpy(ctx->d_goff.p, g.goff.data(), g.goff.size() * sizeof(int), hipMemcpyHostToDevice));
    if (!g.gitems.empty())
        PP_HIP(hipMemcpy(ctx->d_gitems.p, g.gitems.data(), g.gitems.size() * sizeof(int),
                         hipMemcpyHostToDevice));
    ctx->lds_bytes = g.lds_total;
    if (g.lds_total > 0) {
        PP_HIP(ctx->d_img.reserve((size_t)g.lds_total / 16));
        PP_HIP(hipMemcpy(ctx->d_img.p, g.image.data(), (size_t)g.lds_total, hipMemcpyHostToDevice));
    }
    ctx->lds_goff = g.o_goff;
    ctx->lds_items = g.o_items;
    ctx->lds_cx = ctx->lds_cy = ctx->lds_r2 = -1;
    ctx->lds_d4 = g.o_d4;
    ctx->gx0 = g.x0;
    ctx->gy0 = g.y0;
    ctx->ginv = g.ginv;
    ctx->gnx = g.gnx;
    ctx->gny = g.gny;
    PP_HIP(ctx->d_d4.reserve((size_t)std::max(m, 1)));
    if (m > 0)
        PP_HIP(hipMemcpy(ctx->d_d4.p, items.d4.data(), m * sizeof(float4), hipMemcpyHostToDevice));
    return PP_OK;
}

// reset the polygon-mode part of the scene (pp_space_new / pp_space_new_polygons)
void clear_polygons(pp_ctx* ctx) {
    ctx->ibn = 0;  // (pp_space_new builds its inside bitmap after this)
    ctx->ne = 0;
    ctx->nbv = 0;
    ctx->h_ex0.clear();
    ctx->h_ey0.clear();
    ctx->h_ex1.clear();
    ctx->h_ey1.clear();
    ctx->h_epoly.clear();
    ctx->h_bvx.clear();
    ctx->h_bvy.clear();
}
}  // namespace

int pp_space_new(pp_ctx* ctx, double x0, double y0, double x1, double y1, double robot_width,
                 double robot_height, double max_steer, const double* cx, const double* cy,
                 const double* r, int m) {
    int rc = check_ctx(ctx, false, false);
    if (rc) return rc;
    if (!(robot_width >= 0.0) || !(max_steer > 0.0))
        return set_err(PP_ERR_INVALID_ARGUMENT, "robot width must be >= 0 and max_steer > 0");
    scene::DiscScene ds;
    std::string err;
    if ((rc = scene::disc_scene(x0, y0, x1, y1, robot_width, cx, cy, r, m, &ds, &err)))
        return set_err(rc, err);
    const double half = robot_width / 2.0;
    if ((rc = upload_item_grid(ctx, ds.minx, ds.maxx, ds.miny, ds.maxy, ds.items))) return rc;
    const size_t mm = (size_t)std::max(m, 1);
    PP_HIP(ctx->d_cx.reserve(mm));
    PP_HIP(ctx->d_cy.reserve(mm));
    PP_HIP(ctx->d_r2.reserve(mm));
    PP_HIP(ctx->d_rcull.reserve(mm));
    if (m > 0) {
        PP_HIP(hipMemcpy(ctx->d_cx.p, cx, m * sizeof(double), hipMemcpyHostToDevice));
        PP_HIP(hipMemcpy(ctx->d_cy.p, cy, m * sizeof(double), hipMemcpyHostToDevice));
        PP_HIP(hipMemcpy(ctx->d_r2.p, ds.r2.data(), m * sizeof(double), hipMemcpyHostToDevice));
        PP_HIP(hipMemcpy(ctx->d_rcull.p, ds.rcull.data(), m * sizeof(double), hipMemcpyHostToDevice));
    }
    clear_polygons(ctx);
    {  // the inside bitmap: 2048^2 cells (512 KB, L2-resident)
        const scene::InsideBits ib =
            scene::inside_bitmap(ds.minx, ds.maxx, ds.miny, ds.maxy, cx, cy, ds.r2, kInsideCells);
        ctx->ibn = ib.n;
        if (ib.n > 0) {
            PP_HIP(ctx->d_ibits.reserve(ib.bits.size()));
            PP_HIP(hipMemcpy(ctx->d_ibits.p, ib.bits.data(), ib.bits.size() * sizeof(uint32_t),
                             hipMemcpyHostToDevice));
            ctx->ibx0 = ib.x0;
            ctx->iby0 = ib.y0;
            ctx->ibinv = ib.inv;
        }
    }
    ctx->h2 = half * half;
    ctx->cull_slack = scene::cull_slack_for(ds.items.mx);
    ctx->minx = ds.minx;
    ctx->maxx = ds.maxx;
    ctx->miny = ds.miny;
    ctx->maxy = ds.maxy;
    ctx->width = robot_width;
    ctx->height = robot_height;
    ctx->max_steer = max_steer;
    ctx->m = m;
    ctx->has_grid = false;
    ctx->has_scene = true;
    ctx->has_rrt = false;  // a planner belongs to one Space (RRT::new moves it in, rrt.rs:342)
    ctx->has_batch = false;
    return PP_OK;
}

int pp_space_new_polygons(pp_ctx* ctx, const double* bounds_xy, int nb, const double* obs_xy,
                          const int32_t* obs_off, int n_obs, double robot_width,
                          double robot_height, double max_steer) {
    int rc = check_ctx(ctx, false, false);
    if (rc) return rc;
    if (!bounds_xy || nb < 3 || n_obs < 0 || (n_obs > 0 && (!obs_xy || !obs_off)))
        return set_err(PP_ERR_INVALID_ARGUMENT, "bad polygon arrays (bounds need >= 3 vertices)");
    if (!(robot_width >= 0.0) || !(max_steer > 0.0))
        return set_err(PP_ERR_INVALID_ARGUMENT, "robot width must be >= 0 and max_steer > 0");
    scene::PolygonScene ps;
    std::string err;
    if ((rc = scene::polygon_scene(bounds_xy, nb, obs_xy, obs_off, n_obs, robot_width, &ps, &err)))
        return set_err(rc, err);
    const double half = robot_width / 2.0;
    if ((rc = upload_item_grid(ctx, ps.minx, ps.maxx, ps.miny, ps.maxy, ps.items))) return rc;
    const int ne = (int)ps.ex0.size();
    const size_t nn = (size_t)std::max(ne, 1);
    PP_HIP(ctx->d_ex0.reserve(nn));
    PP_HIP(ctx->d_ey0.reserve(nn));
    PP_HIP(ctx->d_ex1.reserve(nn));
    PP_HIP(ctx->d_ey1.reserve(nn));
    PP_HIP(ctx->d_epoly.reserve(nn));
    PP_HIP(ctx->d_bvx.reserve(ps.bvx.size()));
    PP_HIP(ctx->d_bvy.reserve(ps.bvy.size()));
    if (ne > 0) {
        PP_HIP(hipMemcpy(ctx->d_ex0.p, ps.ex0.data(), ne * sizeof(double), hipMemcpyHostToDevice));
        PP_HIP(hipMemcpy(ctx->d_ey0.p, ps.ey0.data(), ne * sizeof(double), hipMemcpyHostToDevice));
        PP_HIP(hipMemcpy(ctx->d_ex1.p, ps.ex1.data(), ne * sizeof(double), hipMemcpyHostToDevice));
        PP_HIP(hipMemcpy(ctx->d_ey1.p, ps.ey1.data(), ne * sizeof(double), hipMemcpyHostToDevice));
        PP_HIP(hipMemcpy(ctx->d_epoly.p, ps.epoly.data(), ne * sizeof(int), hipMemcpyHostToDevice));
    }
    PP_HIP(hipMemcpy(ctx->d_bvx.p, ps.bvx.data(), ps.bvx.size() * sizeof(double), hipMemcpyHostToDevice));
    PP_HIP(hipMemcpy(ctx->d_bvy.p, ps.bvy.data(), ps.bvy.size() * sizeof(double), hipMemcpyHostToDevice));
    ctx->h_ex0 = std::move(ps.ex0);
    ctx->h_ey0 = std::move(ps.ey0);
    ctx->h_ex1 = std::move(ps.ex1);
    ctx->h_ey1 = std::move(ps.ey1);
    ctx->h_epoly = std::move(ps.epoly);
    ctx->h_bvx = std::move(ps.bvx);
    ctx->h_bvy = std::move(ps.bvy);
    ctx->ne = ne;
    ctx->nbv = (int)ctx->h_bvx.size();
    ctx->h2 = half * half;
    ctx->cull_slack = scene::cull_slack_for(ps.items.mx);
    ctx->minx = ps.minx;
    ctx->maxx = ps.maxx;
    ctx->miny = ps.miny;
    ctx->maxy = ps.maxy;
    ctx->width = robot_width;
    ctx->height = robot_height;
    ctx->max_steer = max_steer;
    ctx->m = 0;
    ctx->has_grid = false;
    ctx->has_scene = true;
    ctx->has_rrt = false;
    ctx->has_batch = false;
    return PP_OK;
}

int pp_space_set_grid(pp_ctx* ctx, const uint32_t* bits, int w, int h, double x0, double y0,
                      double cell) {
    int rc = check_ctx(ctx, true, false);
    if (rc) return rc;
    if (!bits || w <= 0 || h <= 0 || w > (1 << 16) || h > (1 << 16) || !(cell > 0.0))
        return set_err(PP_ERR_INVALID_ARGUMENT, "bad occupancy grid");
    const int words = (w + 31) / 32;
    const size_t n = (size_t)words * h;
    PP_HIP(ctx->d_bits.reserve(n));
    PP_HIP(hipMemcpy(ctx->d_bits.p, bits, n * sizeof(uint32_t), hipMemcpyHostToDevice));
    ctx->bw = w;
    ctx->bh = h;
    ctx->bwords = words;
    ctx->bx0 = x0;
    ctx->by0 = y0;
    ctx->binv = 1.0 / cell;
    const size_t img_bytes = (n * sizeof(uint32_t) + 15) & ~(size_t)15;
    ctx->lds_bits_bytes = img_bytes <= 64 * 1024 ? (int)img_bytes : 0;
    if (ctx->lds_bits_bytes) {
        std::vector<uint32_t> img(img_bytes / 4, 0u);
        std::memcpy(img.data(), bits, n * sizeof(uint32_t));
        PP_HIP(ctx->d_gimg.reserve(img_bytes / 16));
        PP_HIP(hipMemcpy(ctx->d_gimg.p, img.data(), img_bytes, hipMemcpyHostToDevice));
    }
    ctx->has_grid = true;
    ctx->has_rrt = false;  // the planner's Space changed (rrt.rs:342)
    return PP_OK;
}

int pp_space_verify_batch(pp_ctx* ctx, const double* x, const double* y, const int64_t* off,
                          int k, uint8_t* ok) {
    int r = check_ctx(ctx, true, false);
    if (r) return r;
    if (k < 0 || (k > 0 && (!off || !ok))) return set_err(PP_ERR_INVALID_ARGUMENT, "bad arguments");
    if (k == 0) return PP_OK;
    if (off[0] != 0) return set_err(PP_ERR_INVALID_ARGUMENT, "off[0] must be 0");
    for (int i = 0; i < k; ++i)
        if (off[i + 1] < off[i]) return set_err(PP_ERR_INVALID_ARGUMENT, "off must be non-decreasing");
    const int64_t np = off[k];
    if (np > 0 && (!x || !y)) return set_err(PP_ERR_INVALID_ARGUMENT, "null points");
    hipStream_t st = ctx->stream;
    DBuf<double> dx, dy;
    DBuf<int64_t> doff;
    DBuf<uint8_t> dok;
    PP_HIP(dx.reserve((size_t)std::max<int64_t>(np, 1)));
    PP_HIP(dy.reserve((size_t)std::max<int64_t>(np, 1)));
    PP_HIP(doff.reserve((size_t)k + 1));
    PP_HIP(dok.reserve((size_t)k));
    if (np > 0) {
        PP_HIP(hipMemcpyAsync(dx.p, x, np * sizeof(double), hipMemcpyHostToDevice, st));
        PP_HIP(hipMemcpyAsync(dy.p, y, np * sizeof(double), hipMemcpyHostToDevice, st));
    }
    PP_HIP(hipMemcpyAsync(doff.p, off, ((size_t)k + 1) * sizeof(int64_t), hipMemcpyHostToDevice, st));
    PP_HIP(launch_verify_lines(st, ctx->scene_dev(), dx.p, dy.p, doff.p, k, dok.p));
    PP_HIP(hipMemcpyAsync(ok, dok.p, (size_t)k, hipMemcpyDeviceToHost, st));
    PP_HIP(hipStreamSynchronize(st));
    return PP_OK;
}

int pp_space_get_bounds(pp_ctx* ctx, double out[4]) {
    int r = check_ctx(ctx, true, false);
    if (r) return r;
    if (!out) return set_err(PP_ERR_INVALID_ARGUMENT, "null output");
    out[0] = ctx->minx;
    out[1] = ctx->maxx;
    out[2] = ctx->miny;
    out[3] = ctx->maxy;
    return PP_OK;
}

int pp_rrt_new(pp_ctx* ctx, double sx, double sy, double syaw, double gx, double gy, double gyaw,
               int64_t max_iter, double step_size, uint64_t seed, int64_t capacity) {
    int r = check_ctx(ctx, true, false);
    if (r) return r;
    if (!(step_size > 0.0) || max_iter < 0)
        return set_err(PP_ERR_INVALID_ARGUMENT, "step_size must be > 0 and max_iter >= 0");
    ctx->has_rrt = false;
    PP_HIP(hipStreamSynchronize(ctx->stream));
    ctx->n = 0;
    ctx->it = 0;
    ctx->start[0] = sx;
    ctx->start[1] = sy;
    ctx->start[2] = syaw;
    ctx->goal[0] = gx;
    ctx->goal[1] = gy;
    ctx->goal[2] = gyaw;
    ctx->max_iter = max_iter;
    ctx->step = step_size;
    ctx->seed = seed;
    if ((r = ctx->reset_host_stats())) return set_err(r, "resetting the statistics");
    if ((r = ensure_tree(ctx, std::max<int64_t>(capacity, 1024)))) return r;
    if ((r = ensure_window(ctx, ctx->K))) return r;
    // f32 screen tolerance: coordinates are rounded to f32 with error <= max|c| * 2^-24
    double mx = std::max({std::fabs(ctx->minx), std::fabs(ctx->maxx), std::fabs(ctx->miny),
                          std::fabs(ctx->maxy), std::fabs(sx), std::fabs(sy)});
    ctx->eps_coord = mx * std::ldexp(1.0, -23);
    // polygon mode: a root that fails verify fails every line_to_origin (it ends the line), so
    // nothing is ever inserted; the kernels' incremental verify assumes a free root (Q10p)
    ctx->root_blocked = (ctx->ne > 0 || ctx->nbv > 0) && !ctx->point_ok(sx, sy);
    // RRT::new inserts the root (rrt.rs:344-346)
    const float fx = (float)sx, fy = (float)sy;
    const int par = -1;
    PP_HIP(hipMemcpy(ctx->x32.p, &fx, sizeof(float), hipMemcpyHostToDevice));
    PP_HIP(hipMemcpy(ctx->y32.p, &fy, sizeof(float), hipMemcpyHostToDevice));
    PP_HIP(hipMemcpy(ctx->X.p, &sx, sizeof(double), hipMemcpyHostToDevice));
    PP_HIP(hipMemcpy(ctx->Y.p, &sy, sizeof(double), hipMemcpyHostToDevice));
    PP_HIP(hipMemcpy(ctx->YAW.p, &syaw, sizeof(double), hipMemcpyHostToDevice));
    PP_HIP(hipMemcpy(ctx->PAR.p, &par, sizeof(int), hipMemcpyHostToDevice));
    DevState s{};
    s.it = 0;
    s.n = 1;
    s.n_scan = 1;
    s.it_spec = 0;
    s.void_seq = -1;
    s.kdyn = kMinDynWindow;  // a young tree starts with short windows (the commit adapts them)
    PP_HIP(hipMemcpy(ctx->d_state.p, &s, sizeof(DevState), hipMemcpyHostToDevice));
    ctx->h_state.p[0] = s;
    ctx->n = 1;
    ctx->has_rrt = true;
    return PP_OK;
}

int pp_rrt_set_window(pp_ctx* ctx, int k) {
    if (!ctx) return set_err(PP_ERR_INVALID_ARGUMENT, "null context");
    if (k < 1 || k > kMaxWindow)
        return set_err(PP_ERR_INVALID_ARGUMENT, "window must be in [1, 4096] (resolve state lives in LDS)");
    ctx->K = k;
    return PP_OK;
}

}  // extern "C"

namespace {

// The extend loop behind pp_rrt_extend (src: null, the seeded stream) and pp_rrt_extend_samples
// (src: the caller's samples of the iterations [ctx->it, ctx->it + n_iter), on the device, and
// the per-iteration record).  eps: the f32 screen tolerance of this call (the samples' magnitude).
struct SampleSrc {
    const double* x;
    const double* y;
    SampleRec rec;
    bool pretest;  // the obstacle pre-test may settle a sample without its nearest node
};

#ifdef PP_FIN_STAMPS
// diagnostic builds: append the last nn_finalize launch's phase stamps (per workgroup) to
// gpurun_out/fin_stamps.txt, one line per batch of windows: tree size, windows, then the stamps
void dump_fin_stamps(int64_t n, int nw) {
    std::vector<unsigned long long> v(kFinStampSlots * kFinStampWGs);
    if (fin_stamps_copy(v.data(), v.size()) != hipSuccess) return;
    FILE* f = std::fopen("gpurun_out/fin_stamps.txt", "a");
    if (!f) return;
    std::fprintf(f, "%lld %d", (long long)n, nw);
    for (unsigned long long x : v) std::fprintf(f, " %llu", x);
    std::fprintf(f, "\n");
    std::fclose(f);
}
#endif

int rrt_extend_impl(pp_ctx* ctx, int64_t n_iter, int64_t* n_accepted, const SampleSrc* src,
                    double eps) {
    int r;
    if ((r = ensure_window(ctx, ctx->K))) return r;
    if (ctx->root_blocked) {  // every iteration rejects: only the iteration counters advance
        DevState& s = ctx->h_state.p[0];
        PP_HIP(hipMemcpy(&s, ctx->d_state.p, sizeof(DevState), hipMemcpyDeviceToHost));
        s.it += n_iter;
        s.it_spec = s.it;
        s.iterations += n_iter;
        s.node_evals += n_iter;  // the NN of every iteration scans the root
        PP_HIP(hipMemcpy(ctx->d_state.p, &s, sizeof(DevState), hipMemcpyHostToDevice));
        ctx->it = s.it;
        if (n_accepted) *n_accepted = 0;
        return PP_OK;
    }
    const int64_t target = ctx->it + n_iter;
    const int64_t n_before = ctx->n;
    hipStream_t st = ctx->stream;
    {  // the scene in device memory for samples_role's point_blocked pre-test
        if (!ctx->d_scene.p) PP_HIP(ctx->d_scene.reserve(1));
        const SceneDev sd = ctx->scene_dev();
        PP_HIP(hipMemcpy(ctx->d_scene.p, &sd, sizeof sd, hipMemcpyHostToDevice));
    }
    while (ctx->it < target) {
        const int K = ctx->K;
        // windows draw min(K, kdyn) samples (the device adapts kdyn): enough windows for that
        const int64_t Kd = std::max(1, std::min(K, ctx->h_state.p[0].kdyn > 0 ? ctx->h_state.p[0].kdyn : K));
        const int64_t nw64 = std::min<int64_t>((target - ctx->it + Kd - 1) / Kd, kMaxBatch);
        const int nw = (int)nw64;
        if ((r = ensure_tree(ctx, ctx->n + (int64_t)nw * K))) return r;
        WindowArgs a = ctx->window_args(ctx->d_state.p);
        a.K = K;
        a.target = target;
        a.eps_coord = eps;
        if (src) {
            a.hsx = src->x;
            a.hsy = src->y;
            a.hrec = src->rec;
            if (!src->pretest) a.blk = nullptr;
        }
        if (ctx->prof && (r = ensure_events(ctx, 5 * (size_t)nw))) return r;
        const int64_t windows_before = ctx->h_state.p[0].windows;
        // windows are pipelined: window w's kernel resolves and commits w - 1; the drain launch
        // commits the batch's last window before the host reads the state
        for (int w = 0; w < nw; ++w)
            PP_HIP(launch_window(st, a, ctx->prof ? &ctx->ev[5 * w] : nullptr, ctx->seq++, w > 0));
        PP_HIP(launch_drain(st, a, ctx->seq));
        PP_HIP(hipMemcpyAsync(ctx->h_state.p, ctx->d_state.p, sizeof(DevState), hipMemcpyDeviceToHost, st));
        PP_HIP(hipStreamSynchronize(st));
        const DevState& s = ctx->h_state.p[0];
        if (s.error)
            return set_err(PP_ERR_STEER_OVERFLOW,
                           "generate_local_course would index past n_point (the reference panics)");
        if (s.it <= ctx->it && nw > 0 && s.windows == windows_before)
            return set_err(PP_ERR_HIP, "extend made no progress");
        if (ctx->prof) {
            const int64_t active = std::min<int64_t>(s.windows - windows_before, nw);
            for (int64_t w = 0; w < active; ++w) {
                double* acc[4] = {&ctx->nn_scan_ms, &ctx->finalize_ms, &ctx->prep_ms, &ctx->steer_ms};
                for (int k = 0; k < 4; ++k) {
                    float ms = 0.f;
                    PP_HIP(hipEventElapsedTime(&ms, ctx->ev[5 * w + k], ctx->ev[5 * w + k + 1]));
                    *acc[k] += ms;
                }
            }
            ctx->nn_scan_launches += active;
            ctx->steer_launches += active;
        }
        ctx->it = s.it;
        ctx->n = s.n;
#ifdef PP_FIN_STAMPS
        dump_fin_stamps(ctx->n, nw);
#endif
    }
    if (n_accepted) *n_accepted = ctx->n - n_before;
    return PP_OK;
}

// pp_rrt_extend_samples' device buffers: samples and records of kHostChunk iterations at a time
constexpr int64_t kHostChunk = (int64_t)1 << 20;

}  // namespace

extern "C" {

int pp_rrt_extend(pp_ctx* ctx, int64_t n_iter, int64_t* n_accepted) {
    int r = check_ctx(ctx, true, true);
    if (r) return r;
    if (n_iter < 0) return set_err(PP_ERR_INVALID_ARGUMENT, "n_iter < 0");
    return rrt_extend_impl(ctx, n_iter, n_accepted, nullptr, ctx->eps_coord);
}

int pp_rrt_extend_samples(pp_ctx* ctx, const double* sx, const double* sy, int64_t k,
                          int32_t* nearest, double* yaw, uint8_t* ok, int64_t* n_accepted) {
    int r = check_ctx(ctx, true, true);
    if (r) return r;
    if (k < 0 || (k > 0 && (!sx || !sy)))
        return set_err(PP_ERR_INVALID_ARGUMENT, "bad extend_samples arguments");
    double mx = 0.0;
    for (int64_t i = 0; i < k; ++i) {
        if (!std::isfinite(sx[i]) || !std::isfinite(sy[i]))
            return set_err(PP_ERR_INVALID_ARGUMENT, "a sample is not finite");
        mx = std::max({mx, std::fabs(sx[i]), std::fabs(sy[i])});
    }
    // the f32 screen's tolerance covers the coordinates it rounds: nodes and these samples
    const double eps = std::max(ctx->eps_coord, mx * std::ldexp(1.0, -23));
    int64_t acc_all = 0;
    if (ctx->root_blocked) {  // nothing is ever inserted: the tree is fixed, every verdict false
        const int64_t n_before = ctx->n;
        for (int64_t b = 0; b < k && (nearest || yaw); b += ctx->Kcap) {
            const int nb = (int)std::min<int64_t>(ctx->Kcap, k - b);
            std::vector<int32_t> idx((size_t)nb);
            if ((r = pp_rrt_get_nearest_node_batch(ctx, sx + b, sy + b, nb, idx.data(), nullptr)))
                return r;
            std::vector<double> tx((size_t)n_before), ty((size_t)n_before);
            if (yaw) {
                PP_HIP(hipMemcpy(tx.data(), ctx->X.p, tx.size() * sizeof(double), hipMemcpyDeviceToHost));
                PP_HIP(hipMemcpy(ty.data(), ctx->Y.p, ty.size() * sizeof(double), hipMemcpyDeviceToHost));
            }
            for (int i = 0; i < nb; ++i) {
                if (nearest) nearest[b + i] = idx[(size_t)i];
                if (yaw) yaw[b + i] = std::atan2(ty[(size_t)idx[i]] - sy[b + i], tx[(size_t)idx[i]] - sx[b + i]);
            }
        }
        if (ok) std::memset(ok, 0, (size_t)k);
        if ((r = rrt_extend_impl(ctx, k, nullptr, nullptr, eps))) return r;
        if (n_accepted) *n_accepted = 0;
        return PP_OK;
    }
    for (int64_t b = 0; b < k; b += kHostChunk) {
        const int64_t nb = std::min(kHostChunk, k - b);
        const size_t z = (size_t)nb;
        PP_HIP(ctx->hs_x.reserve(z));
        PP_HIP(ctx->hs_y.reserve(z));
        if (nearest) PP_HIP(ctx->hs_par.reserve(z));
        if (yaw) PP_HIP(ctx->hs_yaw.reserve(z));
        if (ok) PP_HIP(ctx->hs_ok.reserve(z));
        hipStream_t st = ctx->stream;
        PP_HIP(hipMemcpyAsync(ctx->hs_x.p, sx + b, z * sizeof(double), hipMemcpyHostToDevice, st));
        PP_HIP(hipMemcpyAsync(ctx->hs_y.p, sy + b, z * sizeof(double), hipMemcpyHostToDevice, st));
        SampleSrc src{ctx->hs_x.p, ctx->hs_y.p,
                      SampleRec{ctx->it, nearest ? ctx->hs_par.p : nullptr,
                                yaw ? ctx->hs_yaw.p : nullptr, ok ? ctx->hs_ok.p : nullptr},
                      !nearest && !yaw};
        int64_t acc = 0;
        if ((r = rrt_extend_impl(ctx, nb, &acc, &src, eps))) return r;
        acc_all += acc;
        if (nearest)
            PP_HIP(hipMemcpyAsync(nearest + b, ctx->hs_par.p, z * sizeof(int), hipMemcpyDeviceToHost, st));
        if (yaw) PP_HIP(hipMemcpyAsync(yaw + b, ctx->hs_yaw.p, z * sizeof(double), hipMemcpyDeviceToHost, st));
        if (ok) PP_HIP(hipMemcpyAsync(ok + b, ctx->hs_ok.p, z, hipMemcpyDeviceToHost, st));
        PP_HIP(hipStreamSynchronize(st));
    }
    if (n_accepted) *n_accepted = acc_all;
    return PP_OK;
}

int pp_rrt_tree_import(pp_ctx* ctx, const double* x, const double* y, const double* yaw,
                       const int32_t* parent, int64_t n) {
    int r = check_ctx(ctx, true, true);
    if (r) return r;
    if (n < 1 || !x || !y || !yaw || !parent)
        return set_err(PP_ERR_INVALID_ARGUMENT, "a tree has at least its root");
    if (n > (int64_t)0x7fff0000) return set_err(PP_ERR_CAPACITY, "tree larger than 2^31 nodes");
    if (parent[0] != -1) return set_err(PP_ERR_INVALID_ARGUMENT, "node 0 must be the root (parent -1)");
    double mx = std::max({std::fabs(ctx->minx), std::fabs(ctx->maxx), std::fabs(ctx->miny),
                          std::fabs(ctx->maxy)});
    for (int64_t i = 0; i < n; ++i) {
        if (i > 0 && (parent[i] < 0 || parent[i] >= i))
            return set_err(PP_ERR_INVALID_ARGUMENT,
                           "parent[i] must be an earlier node (insertion order, rrt.rs:586-589)");
        if (!std::isfinite(x[i]) || !std::isfinite(y[i]) || !std::isfinite(yaw[i]))
            return set_err(PP_ERR_INVALID_ARGUMENT, "a node coordinate is not finite");
        mx = std::max({mx, std::fabs(x[i]), std::fabs(y[i])});
    }
    PP_HIP(hipStreamSynchronize(ctx->stream));
    if ((r = ensure_tree(ctx, n + 1024))) return r;
    const size_t z = (size_t)n;
    std::vector<float> fx(z), fy(z);
    for (size_t i = 0; i < z; ++i) {
        fx[i] = (float)x[i];
        fy[i] = (float)y[i];
    }
    PP_HIP(hipMemcpy(ctx->x32.p, fx.data(), z * sizeof(float), hipMemcpyHostToDevice));
    PP_HIP(hipMemcpy(ctx->y32.p, fy.data(), z * sizeof(float), hipMemcpyHostToDevice));
    PP_HIP(hipMemcpy(ctx->X.p, x, z * sizeof(double), hipMemcpyHostToDevice));
    PP_HIP(hipMemcpy(ctx->Y.p, y, z * sizeof(double), hipMemcpyHostToDevice));
    PP_HIP(hipMemcpy(ctx->YAW.p, yaw, z * sizeof(double), hipMemcpyHostToDevice));
    PP_HIP(hipMemcpy(ctx->PAR.p, parent, z * sizeof(int32_t), hipMemcpyHostToDevice));
    // the planner continues from this tree: its iteration counter and statistics stay
    DevState& s = ctx->h_state.p[0];
    PP_HIP(hipMemcpy(&s, ctx->d_state.p, sizeof(DevState), hipMemcpyDeviceToHost));
    s.n = (int)n;
    s.n_scan = (int)n;
    s.it_spec = s.it;
    s.void_seq = -1;
    s.kdyn = kMinDynWindow;
    PP_HIP(hipMemcpy(ctx->d_state.p, &s, sizeof(DevState), hipMemcpyHostToDevice));
    ctx->n = n;
    ctx->start[0] = x[0];
    ctx->start[1] = y[0];
    ctx->start[2] = yaw[0];
    ctx->eps_coord = mx * std::ldexp(1.0, -23);
    ctx->root_blocked = (ctx->ne > 0 || ctx->nbv > 0) && !ctx->point_ok(x[0], y[0]);
    return PP_OK;
}

int pp_rrt_plan_one(pp_ctx* ctx, int32_t* accepted) {
    int64_t acc = 0;
    int r = pp_rrt_extend(ctx, 1, &acc);
    if (r) return r;
    if (accepted) *accepted = (int32_t)acc;
    return PP_OK;
}

int pp_rrt_tree_size(pp_ctx* ctx, int64_t* n) {
    int r = check_ctx(ctx, true, true);
    if (r) return r;
    if (!n) return set_err(PP_ERR_INVALID_ARGUMENT, "null output");
    *n = ctx->n;
    return PP_OK;
}

int pp_rrt_iteration(pp_ctx* ctx, int64_t* it) {
    int r = check_ctx(ctx, true, true);
    if (r) return r;
    if (!it) return set_err(PP_ERR_INVALID_ARGUMENT, "null output");
    *it = ctx->it;
    return PP_OK;
}

int pp_rrt_tree_export(pp_ctx* ctx, double* x, double* y, double* yaw, int32_t* parent,
                       int64_t cap, int64_t* n) {
    int r = check_ctx(ctx, true, true);
    if (r) return r;
    if (n) *n = ctx->n;
    if (cap < ctx->n) return set_err(PP_ERR_CAPACITY, "export buffer smaller than the tree");
    const size_t k = (size_t)ctx->n;
    hipStream_t st = ctx->stream;
    if (x) PP_HIP(hipMemcpyAsync(x, ctx->X.p, k * sizeof(double), hipMemcpyDeviceToHost, st));
    if (y) PP_HIP(hipMemcpyAsync(y, ctx->Y.p, k * sizeof(double), hipMemcpyDeviceToHost, st));
    if (yaw) PP_HIP(hipMemcpyAsync(yaw, ctx->YAW.p, k * sizeof(double), hipMemcpyDeviceToHost, st));
    if (parent) PP_HIP(hipMemcpyAsync(parent, ctx->PAR.p, k * sizeof(int), hipMemcpyDeviceToHost, st));
    PP_HIP(hipStreamSynchronize(st));
    return PP_OK;
}

int pp_rrt_line_to_origin(pp_ctx* ctx, int32_t node, double* x, double* y, int64_t cap,
                          int64_t* n) {
    int r = check_ctx(ctx, true, true);
    if (r) return r;
    if (!n || node < 0 || node >= ctx->n || cap < 0 || (cap > 0 && (!x || !y)))
        return set_err(PP_ERR_INVALID_ARGUMENT, "bad line_to_origin arguments");
    // the path node -> root (NodeIter, rrt.rs:248-265): the tree's rows, read once
    const size_t nt = (size_t)ctx->n;
    std::vector<double> hx(nt), hy(nt), hyaw(nt);
    std::vector<int> hp(nt);
    hipStream_t st = ctx->stream;
    PP_HIP(hipMemcpyAsync(hx.data(), ctx->X.p, nt * sizeof(double), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(hy.data(), ctx->Y.p, nt * sizeof(double), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(hyaw.data(), ctx->YAW.p, nt * sizeof(double), hipMemcpyDeviceToHost, st));
    PP_HIP(hipMemcpyAsync(hp.data(), ctx->PAR.p, nt * sizeof(int), hipMemcpyDeviceToHost, st));
    PP_HIP(hipStreamSynchronize(st));
    std::vector<int> path;
    for (int v = node; v >= 0; v = hp[(size_t)v]) {
        if (path.size() > nt) return set_err(PP_ERR_STATE, "parent cycle in the tree");
        path.push_back(v);
    }
    // every edge child -> parent as dubins_path_planning(child pose, parent pose, R, step) on the
    // GPU (rrt.rs:297-311); the capacity bound of pp_dubins_path_planning_batch's callers
    const int ne = (int)path.size() - 1;
    std::vector<pp_dubins_config> conf((size_t)std::max(ne, 1));
    int pcap = 16;
    for (int e = 0; e < ne; ++e) {
        const int c = path[(size_t)e], p = path[(size_t)e + 1];
        conf[(size_t)e] = pp_dubins_config{hx[(size_t)c], hy[(size_t)c], hyaw[(size_t)c],
                                           hx[(size_t)p], hy[(size_t)p], hyaw[(size_t)p],
                                           ctx->max_steer, ctx->step};
        const double d = std::hypot(hx[(size_t)p] - hx[(size_t)c], hy[(size_t)p] - hy[(size_t)c]);
        pcap = std::max(pcap, (int)((6.0 * 3.14159265358979323846 + d / ctx->max_steer + 4.0) /
                                    ctx->step) + 16);
    }
    std::vector<double> px, py, pyaw, cost((size_t)std::max(ne, 1));
    std::vector<int32_t> np((size_t)std::max(ne, 1)), word((size_t)std::max(ne, 1));
    if (ne > 0) {
        px.resize((size_t)ne * pcap);
        py.resize((size_t)ne * pcap);
        pyaw.resize((size_t)ne * pcap);
        if ((r = pp_dubins_path_planning_batch(ctx, conf.data(), ne, pcap, px.data(), py.data(),
                                               pyaw.data(), np.data(), word.data(), cost.data())))
            return r;
    }
    int64_t w = 0;
    auto put = [&](double a, double b) {
        if (w < cap) {
            x[w] = a;
            y[w] = b;
        }
        ++w;
    };
    for (int e = 0; e < ne; ++e) {
        if (word[(size_t)e] < 0) {  // None: the child's own point (rrt.rs:313)
            put(hx[(size_t)path[(size_t)e]], hy[(size_t)path[(size_t)e]]);
            continue;
        }
        for (int k = 0; k < np[(size_t)e]; ++k) put(px[(size_t)e * pcap + k], py[(size_t)e * pcap + k]);
    }
    put(hx[(size_t)path.back()], hy[(size_t)path.back()]);  // the root (rrt.rs:316)
    *n = w;
    if (cap > 0 && w > cap) return set_err(PP_ERR_CAPACITY, "line buffer smaller than the line");
    return PP_OK;
}

int pp_rrt_get_nearest_node_batch(pp_ctx* ctx, const double* qx, const double* qy, int k,
                                  int32_t* idx, double* d2) {
    int r = check_ctx(ctx, true, true);
    if (r) return r;
    if (k < 0 || (k > 0 && (!qx || !qy || !idx))) return set_err(PP_ERR_INVALID_ARGUMENT, "bad arguments");
    hipStream_t st = ctx->stream;
    WindowArgs a = ctx->window_args(ctx->d_api_state.p);
    for (int b = 0; b < k; b += ctx->Kcap) {
        const int nb = std::min(ctx->Kcap, k - b);
        DevState* hs = &ctx->h_state.p[1];
        *hs = DevState{};
        hs->W = nb;
        hs->Wp[0] = nb;
        hs->n = (int)ctx->n;
        hs->nsp[0] = (int)ctx->n;
        hs->n_scan = (int)ctx->n;
        hs->void_seq = -1;
        PP_HIP(hipMemcpyAsync(ctx->d_api_state.p, hs, sizeof(DevState), hipMemcpyHostToDevice, st));
        PP_HIP(hipMemcpyAsync(ctx->wsx.p, qx + b, nb * sizeof(double), hipMemcpyHostToDevice, st));
        PP_HIP(hipMemcpyAsync(ctx->wsy.p, qy + b, nb * sizeof(double), hipMemcpyHostToDevice, st));
        PP_HIP(launch_nearest(st, a));
        PP_HIP(hipMemcpyAsync(idx + b, ctx->nn_idx.p, nb * sizeof(int), hipMemcpyDeviceToHost, st));
        if (d2) PP_HIP(hipMemcpyAsync(d2 + b, ctx->nn_d2.p, nb * sizeof(double), hipMemcpyDeviceToHost, st));
        PP_HIP(hipStreamSynchronize(st));
    }
    return PP_OK;
}

int pp_rrt_verify_node_batch(pp_ctx* ctx, const double* x, const double* y,
                             const int32_t* parent, int k, uint8_t* ok, double* yaw) {
    int r = check_ctx(ctx, true, true);
    if (r) return r;
    if (k < 0 || (k > 0 && (!x || !y || !parent || !ok))) return set_err(PP_ERR_INVALID_ARGUMENT, "bad arguments");
    for (int i = 0; i < k; ++i)
        if (parent[i] < 0 || parent[i] >= ctx->n)
            return set_err(PP_ERR_INVALID_ARGUMENT, "parent index outside the tree");
    hipStream_t st = ctx->stream;
    const SceneDev sc = ctx->scene_dev();
    const TreeDev tr = ctx->tree_dev();
    std::vector<int> status(ctx->Kcap);
    for (int b = 0; b < k; b += ctx->Kcap) {
        const int nb = std::min(ctx->Kcap, k - b);
        for (int pass = 0; pass < 2; ++pass) {
            int nt = 0;
            std::vector<int> which;
            for (int i = 0; i < nb; ++i) {
                if (pass == 1 && status[i] != kLiteral) continue;
                SteerTask tk;
                tk.x = x[b + i];
                tk.y = y[b + i];
                tk.px = tk.py = tk.pyaw = 0.0;
                tk.pnode = parent[b + i];
                tk.literal = pass;
                ctx->h_tasks.p[nt++] = tk;
                which.push_back(i);
            }
            if (nt == 0) break;
            if (pass == 1)
                PP_HIP(ctx->api_lit_scratch.reserve((size_t)kLiteralWaves * 3 * kLiteralCap));
            std::vector<int> stv(nt);
            std::vector<double> yv(nt);
            PP_HIP(hipMemcpyAsync(ctx->tasks.p, ctx->h_tasks.p, nt * sizeof(SteerTask), hipMemcpyHostToDevice, st));
            PP_HIP(launch_steer_tasks(st, sc, tr, ctx->tasks.p, nt, ctx->task_status.p,
                                      ctx->task_yaw.p, pass ? ctx->api_lit_scratch.p : nullptr));
            PP_HIP(hipMemcpyAsync(stv.data(), ctx->task_status.p, nt * sizeof(int), hipMemcpyDeviceToHost, st));
            PP_HIP(hipMemcpyAsync(yv.data(), ctx->task_yaw.p, nt * sizeof(double), hipMemcpyDeviceToHost, st));
            PP_HIP(hipStreamSynchronize(st));
            for (int t = 0; t < nt; ++t) {
                const int i = which[t];
                if (stv[t] == kError)
                    return set_err(PP_ERR_STEER_OVERFLOW, "generate_local_course would index past n_point");
                status[i] = stv[t];
                ok[b + i] = stv[t] == kAccept && !ctx->root_blocked ? 1 : 0;
                if (yaw) yaw[b + i] = yv[t];
            }
        }
    }
    return PP_OK;
}

int pp_rrt_check_finish_batch(pp_ctx* ctx, const int32_t* nodes, int k, uint8_t* ok,
                              double* length, int32_t* n_points, int32_t* chain) {
    int r = check_ctx(ctx, true, true);
    if (r) return r;
    if (k < 0 || (k > 0 && (!nodes || !ok))) return set_err(PP_ERR_INVALID_ARGUMENT, "bad arguments");
    for (int i = 0; i < k; ++i)
        if (nodes[i] < 0 || nodes[i] >= ctx->n)
            return set_err(PP_ERR_INVALID_ARGUMENT, "node index outside the tree");
    const int want_line = (length || n_points) ? 1 : 0;
    std::vector<int> okv, npv;
    PP_HIP(ctx->cf_nodes.reserve(kCfBatch));
    for (int b = 0; b < k; b += kCfBatch) {
        const int nb = std::min(kCfBatch, k - b);
        PP_HIP(hipMemcpyAsync(ctx->cf_nodes.p, nodes + b, nb * sizeof(int), hipMemcpyHostToDevice, ctx->stream));
        if ((r = cf_launch(ctx, nb, want_line, kCfGrid))) return r;
        okv.resize(nb);
        PP_HIP(hipMemcpy(okv.data(), ctx->cf_ok.p, nb * sizeof(int), hipMemcpyDeviceToHost));
        for (int i = 0; i < nb; ++i) ok[b + i] = (uint8_t)okv[i];
        if (length) PP_HIP(hipMemcpy(length + b, ctx->cf_len.p, nb * sizeof(double), hipMemcpyDeviceToHost));
        if (n_points) PP_HIP(hipMemcpy(n_points + b, ctx->cf_npts.p, nb * sizeof(int), hipMemcpyDeviceToHost));
        if (chain)
            PP_HIP(hipMemcpy(chain + (size_t)b * (kCfLevels + 2), ctx->cf_chain.p,
                             (size_t)nb * (kCfLevels + 2) * sizeof(int), hipMemcpyDeviceToHost));
    }
    return PP_OK;
}

int pp_rrt_check_finish(pp_ctx* ctx, int32_t node, uint8_t* ok, double* x, double* y,
                        int64_t cap, int64_t* n, double* length) {
    int r = check_ctx(ctx, true, true);
    if (r) return r;
    if (!ok || node < 0 || node >= ctx->n) return set_err(PP_ERR_INVALID_ARGUMENT, "bad arguments");
    PP_HIP(ctx->cf_nodes.reserve(kCfBatch));
    PP_HIP(hipMemcpyAsync(ctx->cf_nodes.p, &node, sizeof(int), hipMemcpyHostToDevice, ctx->stream));
    if ((r = cf_launch(ctx, 1, 1, 1))) return r;
    int okv = 0, np = 0, row[kCfLevels + 2];
    double len = 0.0;
    PP_HIP(hipMemcpy(&okv, ctx->cf_ok.p, sizeof(int), hipMemcpyDeviceToHost));
    PP_HIP(hipMemcpy(&np, ctx->cf_npts.p, sizeof(int), hipMemcpyDeviceToHost));
    PP_HIP(hipMemcpy(&len, ctx->cf_len.p, sizeof(double), hipMemcpyDeviceToHost));
    PP_HIP(hipMemcpy(row, ctx->cf_chain.p, sizeof(row), hipMemcpyDeviceToHost));
    *ok = (uint8_t)okv;
    if (length) *length = len;
    if (n) *n = okv ? np : 0;
    if (!okv || !(x && y)) return PP_OK;
    if (cap < np) return set_err(PP_ERR_CAPACITY, "line buffer smaller than the finalized line");
    const int E = row[1];
    std::vector<int> et(2 * (size_t)E);
    std::vector<double> hx(kCfPtsCap), hy(kCfPtsCap);
    PP_HIP(hipMemcpy(et.data(), ctx->cf_etab.p, et.size() * sizeof(int), hipMemcpyDeviceToHost));
    PP_HIP(hipMemcpy(hx.data(), ctx->cf_pts.p, kCfPtsCap * sizeof(double), hipMemcpyDeviceToHost));
    PP_HIP(hipMemcpy(hy.data(), ctx->cf_pts.p + kCfPtsCap, kCfPtsCap * sizeof(double), hipMemcpyDeviceToHost));
    int64_t w = 0;  // l.reverse() (rrt.rs:538)
    for (int e = E - 1; e >= 0; --e)
        for (int i = et[2 * e + 1] - 1; i >= 0; --i) {
            x[w] = hx[et[2 * e] + i];
            y[w] = hy[et[2 * e] + i];
            ++w;
        }
    if (n) *n = w;
    return PP_OK;
}

int pp_rrt_optimize(pp_ctx* ctx, int32_t node, int i, int32_t* chain, int* n_chain) {
    int r = check_ctx(ctx, true, true);
    if (r) return r;
    if (!n_chain || node < 0 || node >= ctx->n || i < 0)
        return set_err(PP_ERR_INVALID_ARGUMENT, "bad arguments");
    *n_chain = 0;
    if (i >= kCfLevels) return PP_OK;  // RECURSION_LIMIT (rrt.rs:464-466): None
    PP_HIP(ctx->cf_nodes.reserve(kCfBatch));
    PP_HIP(hipMemcpyAsync(ctx->cf_nodes.p, &node, sizeof(int), hipMemcpyHostToDevice, ctx->stream));
    CfGoal g{ctx->goal[0], ctx->goal[1], ctx->goal[2], ctx->goal[2]};
    g.level0 = i;
    g.mode = kCfOptimize;
    if ((r = cf_launch(ctx, 1, 0, 1, &g))) return r;
    int row[kCfLevels + 2];
    PP_HIP(hipMemcpy(row, ctx->cf_chain.p, sizeof(row), hipMemcpyDeviceToHost));
    *n_chain = row[0];
    if (chain)
        for (int l = 0; l < row[0]; ++l) chain[l] = row[2 + l];
    return PP_OK;
}

int pp_rrt_finalize(pp_ctx* ctx, double gx, double gy, double gyaw, int32_t parent, double* x,
                    double* y, int64_t cap, int64_t* n, uint8_t* verified) {
    int r = check_ctx(ctx, true, true);
    if (r) return r;
    if (!n || parent < 0 || parent >= ctx->n || !std::isfinite(gx) || !std::isfinite(gy))
        return set_err(PP_ERR_INVALID_ARGUMENT, "bad arguments");
    PP_HIP(ctx->cf_nodes.reserve(kCfBatch));
    PP_HIP(hipMemcpyAsync(ctx->cf_nodes.p, &parent, sizeof(int), hipMemcpyHostToDevice, ctx->stream));
    CfGoal g{gx, gy, gyaw, ctx->goal[2]};
    g.mode = kCfFinalize;
    if ((r = cf_launch(ctx, 1, 1, 1, &g))) return r;
    int okv = 0, np = 0, row[kCfLevels + 2];
    PP_HIP(hipMemcpy(&okv, ctx->cf_ok.p, sizeof(int), hipMemcpyDeviceToHost));
    PP_HIP(hipMemcpy(&np, ctx->cf_npts.p, sizeof(int), hipMemcpyDeviceToHost));
    PP_HIP(hipMemcpy(row, ctx->cf_chain.p, sizeof(row), hipMemcpyDeviceToHost));
    if (verified) *verified = (uint8_t)okv;
    *n = np;
    if (!(x && y) || cap == 0) return PP_OK;
    if (cap < np) return set_err(PP_ERR_CAPACITY, "line buffer smaller than the finalized line");
    const int E = row[1];
    std::vector<int> et(2 * (size_t)E);
    std::vector<double> hx(kCfPtsCap), hy(kCfPtsCap);
    PP_HIP(hipMemcpy(et.data(), ctx->cf_etab.p, et.size() * sizeof(int), hipMemcpyDeviceToHost));
    PP_HIP(hipMemcpy(hx.data(), ctx->cf_pts.p, kCfPtsCap * sizeof(double), hipMemcpyDeviceToHost));
    PP_HIP(hipMemcpy(hy.data(), ctx->cf_pts.p + kCfPtsCap, kCfPtsCap * sizeof(double), hipMemcpyDeviceToHost));
    int64_t w = 0;  // l.reverse() (rrt.rs:538)
    for (int e = E - 1; e >= 0; --e)
        for (int i = et[2 * e + 1] - 1; i >= 0; --i) {
            x[w] = hx[et[2 * e] + i];
            y[w] = hy[et[2 * e] + i];
            ++w;
        }
    *n = w;
    return PP_OK;
}

int pp_rrt_plan(pp_ctx* ctx, int64_t n_iter, int32_t* best_node, double* best_length,
                int64_t* n_finishes) {
    int r = check_ctx(ctx, true, true);
    if (r) return r;
    if (n_iter < 0 || !best_node) return set_err(PP_ERR_INVALID_ARGUMENT, "bad arguments");
    const int64_t n0 = ctx->n;
    int64_t acc = 0;
    if ((r = pp_rrt_extend(ctx, n_iter, &acc))) return r;
    const int64_t n1 = ctx->n;
    std::vector<int32_t> nodes;
    nodes.reserve((size_t)(n1 - n0));
    for (int64_t i = n0; i < n1; ++i) nodes.push_back((int32_t)i);
    std::vector<uint8_t> okv(nodes.size());
    std::vector<double> lens(nodes.size());
    if (!nodes.empty() &&
        (r = pp_rrt_check_finish_batch(ctx, nodes.data(), (int)nodes.size(), okv.data(),
                                       lens.data(), nullptr, nullptr)))
        return r;
    // min_by(euclidean_length) over the finishes in iteration order: the first minimum wins
    int32_t bn = -1;
    double bl = __builtin_inf();
    int64_t nf = 0;
    for (size_t i = 0; i < nodes.size(); ++i) {
        if (!okv[i]) continue;
        ++nf;
        if (lens[i] < bl) {
            bl = lens[i];
            bn = nodes[i];
        }
    }
    *best_node = bn;
    if (best_length) *best_length = bl;
    if (n_finishes) *n_finishes = nf;
    return PP_OK;
}

int pp_batch_new(pp_ctx* ctx, int q, const double* starts, const double* goals,
                 const uint64_t* seeds, int64_t max_iter, double step_size) {
    int r = check_ctx(ctx, true, false);
    if (r) return r;
    if (q <= 0 || !starts || !seeds || max_iter < 0 || max_iter > 0x7ffffff0 || !(step_size > 0.0))
        return set_err(PP_ERR_INVALID_ARGUMENT, "bad batch arguments");
    const int64_t cap64 = max_iter + 1;
    if ((int64_t)q * cap64 > ((int64_t)1 << 34)) return set_err(PP_ERR_CAPACITY, "batch too large");
    const size_t rows = (size_t)q * (size_t)cap64;
    ctx->has_batch = false;
    PP_HIP(ctx->mq_x.reserve(rows));
    PP_HIP(ctx->mq_y.reserve(rows));
    PP_HIP(ctx->mq_yaw.reserve(rows));
    PP_HIP(ctx->mq_par.reserve(rows));
    PP_HIP(ctx->mq_n.reserve(q));
    PP_HIP(ctx->mq_it.reserve(q));
    PP_HIP(ctx->mq_itprev.reserve(q));
    PP_HIP(ctx->mq_evals.reserve(q));
    PP_HIP(ctx->mq_seed.reserve(q));
    PP_HIP(ctx->mq_target.reserve(q));
    PP_HIP(ctx->mq_state.reserve(1 + kMaxSub));
    PP_HIP(ctx->mq_err.reserve(1));
    PP_HIP(ctx->api_lit_scratch.reserve((size_t)kLiteralWaves * 3 * kLiteralCap));
    if (!ctx->lit_locks.p) {
        PP_HIP(ctx->lit_locks.reserve(kLiteralWaves));
        PP_HIP(hipMemset(ctx->lit_locks.p, 0, kLiteralWaves * sizeof(int)));
    }
    ctx->mq_Q = q;
    ctx->mq_cap = (int)cap64;
    ctx->mq_max_iter = max_iter;
    ctx->mq_step = step_size;
    ctx->mq_goal.assign(goals ? goals : starts, (goals ? goals : starts) + 3 * (size_t)q);
    // RRT::new per query: the root (rrt.rs:344-346) in row 0 of each tree
    hipStream_t st = ctx->stream;
    DBuf<double> d_starts;
    PP_HIP(d_starts.reserve(3 * (size_t)q));
    PP_HIP(hipMemcpyAsync(d_starts.p, starts, 3 * (size_t)q * sizeof(double), hipMemcpyHostToDevice, st));
    PP_HIP(launch_mq_init(st, mq_args(ctx).mq, d_starts.p));
    PP_HIP(hipMemcpyAsync(ctx->mq_seed.p, seeds, q * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    // polygon mode: queries whose root fails verify never insert (see pp_rrt_new)
    ctx->mq_any_blocked = false;
    if (ctx->ne > 0 || ctx->nbv > 0) {
        std::vector<uint8_t> blk(q);
        for (int i = 0; i < q; ++i) {
            blk[i] = ctx->point_ok(starts[3 * i], starts[3 * i + 1]) ? 0 : 1;
            ctx->mq_any_blocked |= blk[i] != 0;
        }
        PP_HIP(ctx->mq_blocked.reserve(q));
        PP_HIP(hipMemcpy(ctx->mq_blocked.p, blk.data(), q, hipMemcpyHostToDevice));
    }
    // default window: 32 iterations per query and step while that stays within 262144 tasks.
    // With the active-task list (round 5) a cut window's re-drawn slots cost neither a prep nor a
    // walk, and longer windows pay on the full batch too: 8192 queries 684 M it/s at K = 16
    // against 712 M at 32; the 1024-query shard 274 M at 16, 339 M at 32 and 64
    // (gpurun_out/r05kw; rounds 1-4 measured 16 best for the full batch without the list)
    if (ctx->mq_K_user > 0) {
        ctx->mq_K = ctx->mq_K_user;
    } else {
        int K = kMqAutoK;
        while (K > 1 && (int64_t)q * K > 262144) K >>= 1;
        ctx->mq_K = K;
    }
    if ((r = mq_reserve_tasks(ctx, q, ctx->mq_K))) return r;
    // the verdict cache starts empty: it_prev far below any iteration (0x80.. bytes)
    PP_HIP(hipMemsetAsync(ctx->mq_itprev.p, 0x80, q * sizeof(int64_t), st));
    ctx->mq_nsub = mq_nsub(q);  // the sub-batch DevStates are written for this split
    if ((r = mq_write_states(ctx, st))) return r;
    PP_HIP(hipMemsetAsync(ctx->mq_err.p, 0, sizeof(int), st));
    PP_HIP(hipStreamSynchronize(st));
    if ((r = ctx->reset_host_stats())) return set_err(r, "resetting the statistics");
    ctx->has_batch = true;
    return PP_OK;
}


int pp_batch_set_window(pp_ctx* ctx, int k) {
    if (!ctx) return set_err(PP_ERR_INVALID_ARGUMENT, "null context");
    if (k < 0 || k > kMqMaxK || (k & (k - 1)))
        return set_err(PP_ERR_INVALID_ARGUMENT, "batch window must be 0 (automatic) or a power of two <= 64");
    ctx->mq_K_user = k;
    if (ctx->has_batch && k > 0) {  // applies from the next pp_batch_extend
        PP_HIP(hipStreamSynchronize(ctx->stream));
        int r = mq_reserve_tasks(ctx, ctx->mq_Q, k);
        if (r) return r;
        ctx->mq_K = k;
        // a new window length: the task region's layout changes, the verdict cache is void
        PP_HIP(hipMemsetAsync(ctx->mq_itprev.p, 0x80, ctx->mq_Q * sizeof(int64_t), ctx->stream));
        if ((r = mq_write_states(ctx, ctx->stream))) return r;
        PP_HIP(hipStreamSynchronize(ctx->stream));
    }
    return PP_OK;
}

int pp_batch_set_finish_schedule(pp_ctx* ctx, int rounds, int span0, int span) {
    if (!ctx) return set_err(PP_ERR_INVALID_ARGUMENT, "null context");
    if (rounds != 0 && rounds != 1) return set_err(PP_ERR_INVALID_ARGUMENT, "rounds must be 0 or 1");
    if (span0 < 0 || span0 > 16 || span < 0 || span > 16)
        return set_err(PP_ERR_INVALID_ARGUMENT, "span0 / span must be in [0, 16]");
    ctx->cf_rounds = rounds != 0;
    ctx->cfb_span0 = span0 ? span0 : kCfbSpan;
    ctx->cfb_span = span ? span : kCfbSpan;
    return PP_OK;
}

int pp_batch_extend(pp_ctx* ctx, int64_t n_steps, int64_t* n_iterations, int64_t* n_accepted) {
    int r = check_ctx(ctx, true, false);
    if (r) return r;
    if (!ctx->has_batch) return set_err(PP_ERR_STATE, "pp_batch_new has not been called");
    if (n_steps < 0) return set_err(PP_ERR_INVALID_ARGUMENT, "n_steps < 0");
    int64_t it0 = 0, n0 = 0, it1 = 0, n1 = 0;
    if ((n_iterations || n_accepted) && (r = mq_totals(ctx, &it0, &n0))) return r;
    {  // the batch's scene in device memory (point_blocked)
        if (!ctx->mq_scene.p) PP_HIP(ctx->mq_scene.reserve(1));
        const SceneDev sd = mq_args(ctx).sc;
        PP_HIP(hipMemcpy(ctx->mq_scene.p, &sd, sizeof sd, hipMemcpyHostToDevice));
    }
    MqArgs a = mq_args(ctx);
    const int K = ctx->mq_K, Q = ctx->mq_Q;
    // an earlier call's PP_ERR_STEER_OVERFLOW does not stick to this one
    PP_HIP(hipMemsetAsync(ctx->mq_err.p, 0, sizeof(int), ctx->stream));
    PP_HIP(launch_mq_target(ctx->stream, a.mq, n_steps, ctx->mq_target.p));
    // sub-batches on their own streams (profiled too: the events time the schedule that runs)
    const int nsub = ctx->mq_nsub;
    MqArgs sub[kMaxSub];
    hipStream_t sst[kMaxSub] = {ctx->stream};
    for (int i = 0; i < nsub && nsub > 1; ++i) {
        sub[i] = mq_sub_args(ctx, i, nsub);
        if (i > 0) {
            if (!ctx->sub_stream[i])
                PP_HIP(hipStreamCreateWithFlags(&ctx->sub_stream[i], hipStreamNonBlocking));
            sst[i] = ctx->sub_stream[i];
        }
    }
    if (nsub > 1) {  // fork after the target kernel
        if (!ctx->fork_ev) PP_HIP(hipEventCreateWithFlags(&ctx->fork_ev, hipEventDisableTiming));
        PP_HIP(hipEventRecord(ctx->fork_ev, ctx->stream));
        for (int i = 1; i < nsub; ++i) PP_HIP(hipStreamWaitEvent(sst[i], ctx->fork_ev, 0));
    }
    // every query advances n_steps iterations (to max_iter at most); a window advances up to K
    // of them, fewer when the in-order replay stops early, so the host tops the steps up until
    // every query has reached its target
    int64_t steps = (n_steps + K - 1) / K;
    std::vector<int64_t> hit(Q), htg(Q);
    for (int pass = 0; steps > 0; ++pass) {
        if (pass > 64 + n_steps) return set_err(PP_ERR_HIP, "batch extend made no progress");
        for (int64_t done = 0; done < steps;) {
            const int chunk = (int)std::min<int64_t>(steps - done, 256);
            if (ctx->prof && (r = ensure_events(ctx, 5 * (size_t)chunk * nsub))) return r;
            if (nsub > 1) {  // interleaved, so every stream always holds work
                for (int k = 0; k < chunk; ++k)
                    for (int i = 0; i < nsub; ++i) {
                        sub[i].ev = ctx->prof ? ctx->ev.data() + 5 * ((size_t)k * nsub + i) : nullptr;
                        PP_HIP(launch_mq_steps(sst[i], sub[i], 1));
                    }
            } else {
                a.ev = ctx->prof ? ctx->ev.data() : nullptr;
                PP_HIP(launch_mq_steps(ctx->stream, a, chunk));
            }
            if (ctx->prof) {  // events: before mq_sample_nn, after it, prep, walk and insert
                for (int i = 0; i < nsub; ++i) PP_HIP(hipStreamSynchronize(sst[i]));
                double* acc[4] = {&ctx->nn_scan_ms, &ctx->prep_ms, &ctx->steer_ms, &ctx->insert_ms};
                for (size_t e = 0; e < (size_t)chunk * nsub; ++e)
                    for (int k = 0; k < 4; ++k) {
                        float ms = 0.f;
                        PP_HIP(hipEventElapsedTime(&ms, ctx->ev[5 * e + k], ctx->ev[5 * e + k + 1]));
                        *acc[k] += ms;
                    }
                ctx->nn_scan_launches += (int64_t)chunk * nsub;
                ctx->steer_launches += (int64_t)chunk * nsub;
            }
            done += chunk;
        }
        for (int i = 1; i < nsub; ++i) {  // join: the host reads the counters on `stream`
            PP_HIP(hipEventRecord(ctx->fork_ev, sst[i]));
            PP_HIP(hipStreamWaitEvent(ctx->stream, ctx->fork_ev, 0));
        }
        PP_HIP(hipMemcpyAsync(hit.data(), ctx->mq_it.p, Q * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
        PP_HIP(hipMemcpyAsync(htg.data(), ctx->mq_target.p, Q * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
        int err = 0;
        PP_HIP(hipMemcpyAsync(&err, ctx->mq_err.p, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
        PP_HIP(hipStreamSynchronize(ctx->stream));
        if (err) return set_err(PP_ERR_STEER_OVERFLOW, "generate_local_course would index past n_point");
        ctx->batch_steps += steps;
        ctx->batch_passes += 1;
        steps = 0;  // the top-up pass: queries whose windows stopped early
        for (int q = 0; q < Q; ++q) steps = std::max(steps, (htg[q] - hit[q] + K - 1) / K);
    }
    if ((n_iterations || n_accepted) && (r = mq_totals(ctx, &it1, &n1))) return r;
    if (n_iterations) *n_iterations = it1 - it0;
    if (n_accepted) *n_accepted = n1 - n0;
    return PP_OK;
}

int pp_batch_state(pp_ctx* ctx, int32_t* n_nodes, int64_t* iterations, int64_t* node_evals) {
    int r = check_ctx(ctx, true, false);
    if (r) return r;
    if (!ctx->has_batch) return set_err(PP_ERR_STATE, "pp_batch_new has not been called");
    if (node_evals) PP_HIP(hipMemcpyAsync(node_evals, ctx->mq_evals.p, ctx->mq_Q * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    if (n_nodes) PP_HIP(hipMemcpyAsync(n_nodes, ctx->mq_n.p, ctx->mq_Q * sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    if (iterations) PP_HIP(hipMemcpyAsync(iterations, ctx->mq_it.p, ctx->mq_Q * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
    PP_HIP(hipStreamSynchronize(ctx->stream));
    return PP_OK;
}

int pp_batch_tree_export(pp_ctx* ctx, int query, double* x, double* y, double* yaw,
                         int32_t* parent, int64_t cap, int64_t* n) {
    int r = check_ctx(ctx, true, false);
    if (r) return r;
    if (!ctx->has_batch) return set_err(PP_ERR_STATE, "pp_batch_new has not been called");
    if (query < 0 || query >= ctx->mq_Q) return set_err(PP_ERR_INVALID_ARGUMENT, "query out of range");
    int nn = 0;
    PP_HIP(hipMemcpy(&nn, ctx->mq_n.p + query, sizeof(int), hipMemcpyDeviceToHost));
    if (n) *n = nn;
    if (cap < nn) return set_err(PP_ERR_CAPACITY, "export buffer smaller than the tree");
    const size_t o = (size_t)query * ctx->mq_cap;
    hipStream_t st = ctx->stream;
    if (x) PP_HIP(hipMemcpyAsync(x, ctx->mq_x.p + o, nn * sizeof(double), hipMemcpyDeviceToHost, st));
    if (y) PP_HIP(hipMemcpyAsync(y, ctx->mq_y.p + o, nn * sizeof(double), hipMemcpyDeviceToHost, st));
    if (yaw) PP_HIP(hipMemcpyAsync(yaw, ctx->mq_yaw.p + o, nn * sizeof(double), hipMemcpyDeviceToHost, st));
    if (parent) PP_HIP(hipMemcpyAsync(parent, ctx->mq_par.p + o, nn * sizeof(int), hipMemcpyDeviceToHost, st));
    PP_HIP(hipStreamSynchronize(st));
    return PP_OK;
}

int pp_batch_plan(pp_ctx* ctx, int32_t* best_node, double* length, int32_t* n_points,
                  int32_t* n_finishes, int64_t* n_checked) {
    int r = check_ctx(ctx, true, false);
    if (r) return r;
    if (!ctx->has_batch) return set_err(PP_ERR_STATE, "pp_batch_new has not been called");
    const int Q = ctx->mq_Q;
    hipStream_t st = ctx->stream;
    // the accepted nodes of every query (1 .. n_q - 1, rrt.rs:591), flattened
    std::vector<int> hn(Q), off((size_t)Q + 1, 0);
    PP_HIP(hipMemcpyAsync(hn.data(), ctx->mq_n.p, Q * sizeof(int), hipMemcpyDeviceToHost, st));
    PP_HIP(hipStreamSynchronize(st));
    int64_t total = 0;
    for (int q = 0; q < Q; ++q) {
        off[q] = (int)total;
        total += std::max(hn[q] - 1, 0);
        if (total > (int64_t)0x7fff0000) return set_err(PP_ERR_CAPACITY, "too many nodes to plan");
    }
    off[Q] = (int)total;
    if (n_checked) *n_checked = total;
    const size_t tk = (size_t)std::max<int64_t>(total, 1);
    PP_HIP(ctx->mp_off.reserve((size_t)Q + 1));
    PP_HIP(ctx->mp_qidx.reserve(tk));
    PP_HIP(ctx->mp_nodes.reserve(tk));
    PP_HIP(ctx->mp_ok.reserve(tk));
    PP_HIP(ctx->mp_npts.reserve(tk));
    PP_HIP(ctx->mp_len.reserve(tk));
    PP_HIP(ctx->mp_best.reserve(Q));
    PP_HIP(ctx->mp_bpts.reserve(Q));
    PP_HIP(ctx->mp_nfin.reserve(Q));
    PP_HIP(ctx->mp_blen.reserve(Q));
    PP_HIP(ctx->mq_goal_d.reserve(3 * (size_t)Q));
    PP_HIP(hipMemcpyAsync(ctx->mp_off.p, off.data(), off.size() * sizeof(int), hipMemcpyHostToDevice, st));
    PP_HIP(hipMemcpyAsync(ctx->mq_goal_d.p, ctx->mq_goal.data(), 3 * (size_t)Q * sizeof(double),
                          hipMemcpyHostToDevice, st));
    PP_HIP(launch_mq_plan_items(st, Q, ctx->mp_off.p, ctx->mp_qidx.p, ctx->mp_nodes.p));
    if (total > 0) {
        CfBatch cb;
        cb.qidx = ctx->mp_qidx.p;
        cb.row_cap = ctx->mq_cap;
        cb.goals = ctx->mq_goal_d.p;
        cb.blocked = ctx->mq_any_blocked ? ctx->mq_blocked.p : nullptr;
        cb.moff = ctx->mp_off.p;  // compact memo rows
        TreeDev tr{};  // the batch's SoA rows (query q: offset q * mq_cap, cb.row_cap)
        tr.x = ctx->mq_x.p;
        tr.y = ctx->mq_y.p;
        tr.yaw = ctx->mq_yaw.p;
        tr.parent = ctx->mq_par.p;
        const CfGoal g{0.0, 0.0, 0.0, 0.0};  // (per query: cb.goals)
        const CfOut out{ctx->mp_ok.p, ctx->mp_len.p, ctx->mp_npts.p, nullptr};
        // steer rounds unless polygon mode or a blocked root (check_finish_kernel handles those)
        const bool rounds = ctx->cf_rounds && !cb.blocked && ctx->ne == 0 && ctx->nbv == 0;
        if ((r = rounds ? cf_run_rounds(ctx, tr, (int)total, cb, out)
                        : cf_run(ctx, tr, ctx->mp_nodes.p, (int)total, 1, kCfGrid, g, out, cb)))
            return r;
    }
    PP_HIP(launch_mq_plan_reduce(st, Q, ctx->mp_off.p, ctx->mp_ok.p, ctx->mp_len.p, ctx->mp_npts.p,
                                 ctx->mp_best.p, ctx->mp_blen.p, ctx->mp_bpts.p, ctx->mp_nfin.p));
    if (best_node) PP_HIP(hipMemcpyAsync(best_node, ctx->mp_best.p, Q * sizeof(int), hipMemcpyDeviceToHost, st));
    if (length) PP_HIP(hipMemcpyAsync(length, ctx->mp_blen.p, Q * sizeof(double), hipMemcpyDeviceToHost, st));
    if (n_points) PP_HIP(hipMemcpyAsync(n_points, ctx->mp_bpts.p, Q * sizeof(int), hipMemcpyDeviceToHost, st));
    if (n_finishes) PP_HIP(hipMemcpyAsync(n_finishes, ctx->mp_nfin.p, Q * sizeof(int), hipMemcpyDeviceToHost, st));
    PP_HIP(hipStreamSynchronize(st));
    return PP_OK;
}

int pp_star_new(pp_ctx* ctx, int q, const double* starts, const uint64_t* seeds,
                int64_t max_iter, double step_size, int k, double eta) {
    int r = check_ctx(ctx, true, false);
    if (r) return r;
    if (q <= 0 || !starts || !seeds || max_iter < 0 || max_iter > 0x7ffffff0 ||
        !(step_size > 0.0) || k < 0 || k > kStarKMax || !(eta >= 0.0))
        return set_err(PP_ERR_INVALID_ARGUMENT, "bad RRT* batch arguments");
    const int64_t cap64 = max_iter + 1;
    if ((int64_t)q * cap64 > ((int64_t)1 << 34) || (int64_t)q * kStarKMax > 0x7fffffff)
        return set_err(PP_ERR_CAPACITY, "RRT* batch too large");
    const size_t rows = (size_t)q * (size_t)cap64, tb = (size_t)q * kStarKMax;
    ctx->has_star = false;
    PP_HIP(ctx->sr_x.reserve(rows));
    PP_HIP(ctx->sr_y.reserve(rows));
    PP_HIP(ctx->sr_yaw.reserve(rows));
    PP_HIP(ctx->sr_par.reserve(rows));
    PP_HIP(ctx->sr_cost.reserve(rows));
    PP_HIP(ctx->sr_elen.reserve(rows));
    PP_HIP(ctx->sr_mark.reserve(rows));
    PP_HIP(ctx->sr_ksched.reserve((size_t)cap64 + 1));
    for (auto* b : {&ctx->sr_n, &ctx->sr_stamp, &ctx->sr_pn, &ctx->sr_nnear, &ctx->sr_bslot,
                    &ctx->sr_cslot, &ctx->sr_sA})
        PP_HIP(b->reserve(q));
    for (auto* b : {&ctx->sr_px, &ctx->sr_py, &ctx->sr_cb, &ctx->sr_yA, &ctx->sr_cA})
        PP_HIP(b->reserve(q));
    for (auto* b : {&ctx->sr_it, &ctx->sr_evals, &ctx->sr_target, &ctx->sr_rew}) PP_HIP(b->reserve(q));
    PP_HIP(ctx->sr_seed.reserve(q));
    PP_HIP(ctx->sr_cmask.reserve(q));
    PP_HIP(ctx->sr_bmask.reserve(q));
    if (!ctx->lit_locks.p) {
        PP_HIP(ctx->lit_locks.reserve(kLiteralWaves));
        PP_HIP(hipMemset(ctx->lit_locks.p, 0, kLiteralWaves * sizeof(int)));
    }
    PP_HIP(ctx->sr_near.reserve(tb));
    PP_HIP(ctx->sr_tA.reserve(q));
    PP_HIP(ctx->sr_tB.reserve(tb));
    PP_HIP(ctx->sr_tC.reserve(tb));
    PP_HIP(ctx->sr_eB.reserve(tb));
    PP_HIP(ctx->sr_eC.reserve(tb));
    PP_HIP(ctx->sr_sB.reserve(tb));
    PP_HIP(ctx->sr_sC.reserve(tb));
    for (auto* b : {&ctx->sr_yB, &ctx->sr_yC, &ctx->sr_cB, &ctx->sr_cC}) PP_HIP(b->reserve(tb));
    PP_HIP(ctx->sr_rec.reserve(tb));
    PP_HIP(ctx->sr_state.reserve(3 * (1 + kMaxSub)));
    PP_HIP(ctx->sr_err.reserve(1));
    PP_HIP(ctx->api_lit_scratch.reserve((size_t)kLiteralWaves * 3 * kLiteralCap));
    ctx->star_Q = q;
    ctx->star_cap = (int)cap64;
    ctx->star_max_iter = max_iter;
    ctx->star_step = step_size;
    ctx->star_kfix = k;
    ctx->star_eta = eta;
    hipStream_t st = ctx->stream;
    std::vector<int> ks((size_t)cap64 + 1);
    for (int64_t n = 0; n <= cap64; ++n) ks[n] = star_k(k, (int)n);
    PP_HIP(hipMemcpy(ctx->sr_ksched.p, ks.data(), ks.size() * sizeof(int), hipMemcpyHostToDevice));
    PP_HIP(hipMemsetAsync(ctx->sr_mark.p, 0, rows * sizeof(int), st));
    // polygon mode: queries whose root fails verify never insert (see pp_rrt_new)
    ctx->sr_any_blocked = false;
    if (ctx->ne > 0 || ctx->nbv > 0) {
        std::vector<uint8_t> blk(q);
        for (int i = 0; i < q; ++i) {
            blk[i] = ctx->point_ok(starts[3 * i], starts[3 * i + 1]) ? 0 : 1;
            ctx->sr_any_blocked |= blk[i] != 0;
        }
        PP_HIP(ctx->sr_blocked.reserve(q));
        PP_HIP(hipMemcpy(ctx->sr_blocked.p, blk.data(), q, hipMemcpyHostToDevice));
    }
    DBuf<double> d_starts;
    PP_HIP(d_starts.reserve(3 * (size_t)q));
    PP_HIP(hipMemcpyAsync(d_starts.p, starts, 3 * (size_t)q * sizeof(double), hipMemcpyHostToDevice, st));
    PP_HIP(hipMemcpyAsync(ctx->sr_seed.p, seeds, q * sizeof(uint64_t), hipMemcpyHostToDevice, st));
    PP_HIP(launch_star_init(st, star_args(ctx), d_starts.p));
    DevState ds[3 * (1 + kMaxSub)] = {};
    ds[0].W = q;  // round A of the whole batch; sub-batch s: 3 * (1 + s)
    const int nsub = mq_nsub(q, 3);
    ctx->star_nsub = nsub;  // the sub-batch DevStates are written for this split
    for (int sb = 0; sb < nsub; ++sb)
        ds[3 * (1 + sb)].W = (int)((int64_t)q * (sb + 1) / nsub - (int64_t)q * sb / nsub);
    PP_HIP(hipMemcpyAsync(ctx->sr_state.p, ds, sizeof ds, hipMemcpyHostToDevice, st));
    PP_HIP(hipMemsetAsync(ctx->sr_err.p, 0, sizeof(int), st));
    PP_HIP(hipStreamSynchronize(st));
    if ((r = ctx->reset_host_stats())) return set_err(r, "resetting the statistics");
    ctx->has_star = true;
    return PP_OK;
}

int pp_star_extend(pp_ctx* ctx, int64_t n_steps, int64_t* n_iterations, int64_t* n_accepted,
                   int64_t* n_rewires) {
    int r = check_ctx(ctx, true, false);
    if (r) return r;
    if (!ctx->has_star) return set_err(PP_ERR_STATE, "pp_star_new has not been called");
    if (n_steps < 0) return set_err(PP_ERR_INVALID_ARGUMENT, "n_steps < 0");
    const bool tot = n_iterations || n_accepted || n_rewires;
    int64_t it0 = 0, n0 = 0, w0 = 0, it1 = 0, n1 = 0, w1 = 0;
    if (tot && (r = star_totals(ctx, &it0, &n0, &w0))) return r;
    StarArgs a = star_args(ctx);
    PP_HIP(hipMemsetAsync(ctx->sr_err.p, 0, sizeof(int), ctx->stream));  // per call, not sticky
    PP_HIP(launch_mq_target(ctx->stream, a.sd.mq, n_steps, ctx->sr_target.p));
    const int64_t steps = std::min<int64_t>(n_steps, ctx->star_max_iter);  // one iteration a step
    // sub-batches on their own streams, as pp_batch_extend (profiled too)
    const int nsub = ctx->star_nsub;
    StarArgs sub[kMaxSub];
    hipStream_t sst[kMaxSub] = {ctx->stream};
    for (int i = 0; i < nsub && nsub > 1; ++i) {
        sub[i] = star_sub_args(ctx, i, nsub);
        if (i > 0) {
            if (!ctx->sub_stream[i])
                PP_HIP(hipStreamCreateWithFlags(&ctx->sub_stream[i], hipStreamNonBlocking));
            sst[i] = ctx->sub_stream[i];
        }
    }
    if (nsub > 1) {  // fork after the target kernel
        if (!ctx->fork_ev) PP_HIP(hipEventCreateWithFlags(&ctx->fork_ev, hipEventDisableTiming));
        PP_HIP(hipEventRecord(ctx->fork_ev, ctx->stream));
        for (int i = 1; i < nsub; ++i) PP_HIP(hipStreamWaitEvent(sst[i], ctx->fork_ev, 0));
    }
    for (int64_t done = 0; done < steps;) {
        const int chunk = (int)std::min<int64_t>(steps - done, 256);
        if (ctx->prof && (r = ensure_events(ctx, 8 * (size_t)chunk * nsub))) return r;
        if (nsub > 1) {  // interleaved, so every stream always holds work
            for (int k = 0; k < chunk; ++k)
                for (int i = 0; i < nsub; ++i) {
                    sub[i].ev = ctx->prof ? ctx->ev.data() + 8 * ((size_t)k * nsub + i) : nullptr;
                    PP_HIP(launch_star_steps(sst[i], sub[i], 1));
                }
        } else {
            a.ev = ctx->prof ? ctx->ev.data() : nullptr;
            PP_HIP(launch_star_steps(ctx->stream, a, chunk));
        }
        if (ctx->prof) {  // events: around star_sample, then around each round's walk
            for (int i = 0; i < nsub; ++i) PP_HIP(hipStreamSynchronize(sst[i]));
            for (size_t e = 0; e < (size_t)chunk * nsub; ++e) {
                float ms = 0.f;
                PP_HIP(hipEventElapsedTime(&ms, ctx->ev[8 * e], ctx->ev[8 * e + 1]));
                ctx->nn_scan_ms += ms;
                for (int w = 1; w < 4; ++w) {
                    PP_HIP(hipEventElapsedTime(&ms, ctx->ev[8 * e + 2 * w], ctx->ev[8 * e + 2 * w + 1]));
                    ctx->steer_ms += ms;
                }
            }
            ctx->nn_scan_launches += (int64_t)chunk * nsub;
            ctx->steer_launches += 3 * (int64_t)chunk * nsub;
        }
        done += chunk;
    }
    for (int i = 1; i < nsub; ++i) {  // join
        PP_HIP(hipEventRecord(ctx->fork_ev, sst[i]));
        PP_HIP(hipStreamWaitEvent(ctx->stream, ctx->fork_ev, 0));
    }
    int err = 0;
    PP_HIP(hipMemcpyAsync(&err, ctx->sr_err.p, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
    PP_HIP(hipStreamSynchronize(ctx->stream));
    if (err) return set_err(PP_ERR_STEER_OVERFLOW, "generate_local_course would index past n_point");
    if (tot && (r = star_totals(ctx, &it1, &n1, &w1))) return r;
    if (n_iterations) *n_iterations = it1 - it0;
    if (n_accepted) *n_accepted = n1 - n0;
    if (n_rewires) *n_rewires = w1 - w0;
    return PP_OK;
}

int pp_star_state(pp_ctx* ctx, int32_t* n_nodes, int64_t* iterations, int64_t* node_evals,
                  int64_t* rewires) {
    int r = check_ctx(ctx, true, false);
    if (r) return r;
    if (!ctx->has_star) return set_err(PP_ERR_STATE, "pp_star_new has not been called");
    const int Q = ctx->star_Q;
    hipStream_t st = ctx->stream;
    if (n_nodes) PP_HIP(hipMemcpyAsync(n_nodes, ctx->sr_n.p, Q * sizeof(int), hipMemcpyDeviceToHost, st));
    if (iterations) PP_HIP(hipMemcpyAsync(iterations, ctx->sr_it.p, Q * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    if (node_evals) PP_HIP(hipMemcpyAsync(node_evals, ctx->sr_evals.p, Q * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    if (rewires) PP_HIP(hipMemcpyAsync(rewires, ctx->sr_rew.p, Q * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    PP_HIP(hipStreamSynchronize(st));
    return PP_OK;
}

int pp_star_tree_export(pp_ctx* ctx, int query, double* x, double* y, double* yaw,
                        int32_t* parent, double* cost, int64_t cap, int64_t* n) {
    int r = check_ctx(ctx, true, false);
    if (r) return r;
    if (!ctx->has_star) return set_err(PP_ERR_STATE, "pp_star_new has not been called");
    if (query < 0 || query >= ctx->star_Q) return set_err(PP_ERR_INVALID_ARGUMENT, "query out of range");
    int nn = 0;
    PP_HIP(hipMemcpy(&nn, ctx->sr_n.p + query, sizeof(int), hipMemcpyDeviceToHost));
    if (n) *n = nn;
    if (cap < nn) return set_err(PP_ERR_CAPACITY, "export buffer smaller than the tree");
    const size_t o = (size_t)query * ctx->star_cap;
    hipStream_t st = ctx->stream;
    if (x) PP_HIP(hipMemcpyAsync(x, ctx->sr_x.p + o, nn * sizeof(double), hipMemcpyDeviceToHost, st));
    if (y) PP_HIP(hipMemcpyAsync(y, ctx->sr_y.p + o, nn * sizeof(double), hipMemcpyDeviceToHost, st));
    if (yaw) PP_HIP(hipMemcpyAsync(yaw, ctx->sr_yaw.p + o, nn * sizeof(double), hipMemcpyDeviceToHost, st));
    if (parent) PP_HIP(hipMemcpyAsync(parent, ctx->sr_par.p + o, nn * sizeof(int), hipMemcpyDeviceToHost, st));
    if (cost) PP_HIP(hipMemcpyAsync(cost, ctx->sr_cost.p + o, nn * sizeof(double), hipMemcpyDeviceToHost, st));
    PP_HIP(hipStreamSynchronize(st));
    return PP_OK;
}

int pp_rrt_get_stats(pp_ctx* ctx, pp_stats* out, uint64_t out_size) {
    if (!ctx || !out) return set_err(PP_ERR_INVALID_ARGUMENT, "null argument");
    int r = check_ctx(ctx, false, false);
    if (r) return r;
    pp_stats s{};
    if (ctx->has_rrt) {
        PP_HIP(hipMemcpyAsync(ctx->h_state.p, ctx->d_state.p, sizeof(DevState), hipMemcpyDeviceToHost, ctx->stream));
        PP_HIP(hipStreamSynchronize(ctx->stream));
        const DevState& d = ctx->h_state.p[0];
        s.iterations = d.iterations;
        s.accepted = d.accepted;
        s.windows = d.windows;
        s.truncations = d.truncations;
        s.repair_rounds = d.repair_rounds;
        s.repairs = d.repairs;
        s.literal_repairs = d.literal_repairs;
        s.nn_flagged = d.nn_flagged;
        s.node_evals = d.node_evals;
        s.samples_evaluated = d.iterations;
        s.samples_blocked = d.blocked;
    }
    s.nn_scan_ms = ctx->nn_scan_ms;
    s.nn_scan_launches = ctx->nn_scan_launches;
    s.steer_ms = ctx->steer_ms;
    s.steer_launches = ctx->steer_launches;
    s.finalize_ms = ctx->finalize_ms;
    s.prep_ms = ctx->prep_ms;
    s.insert_ms = ctx->insert_ms;
    s.batch_steps = ctx->batch_steps;
    s.batch_passes = ctx->batch_passes;
    s.finish_ms = ctx->finish_ms;
    s.finish_launches = ctx->finish_launches;
    if (ctx->wg_pts.p) {  // profiling: the walk workgroups' point tallies
        std::vector<long long> v(ctx->wg_pts.n);
        PP_HIP(hipMemcpyAsync(v.data(), ctx->wg_pts.p, v.size() * sizeof(long long), hipMemcpyDeviceToHost, ctx->stream));
        PP_HIP(hipStreamSynchronize(ctx->stream));
        for (size_t i = 0; i < v.size(); ++i) {
            const size_t k = i / (size_t)kWalkTallySlots;  // points, arc points, tasks
            (k == 0 ? s.walk_points : k == 1 ? s.walk_arc_points : s.walk_tasks) += v[i];
        }
    }
    if (ctx->cf_tally.p) {
        long long t[4];
        PP_HIP(hipMemcpyAsync(t, ctx->cf_tally.p, sizeof t, hipMemcpyDeviceToHost, ctx->stream));
        PP_HIP(hipStreamSynchronize(ctx->stream));
        // (+ the batch plan's steer rounds: their nodes, edges and walked points)
        s.finish_nodes = t[0] + ctx->cfb_nodes;
        s.finish_edges = t[1] + ctx->cfb_edges;
        s.finish_points = t[2] + ctx->cfb_points;
        s.finish_arc_points = t[3] + ctx->cfb_arc;
    }
    std::memcpy(out, &s, (size_t)std::min<uint64_t>(out_size, sizeof s));
    return PP_OK;
}

int pp_rrt_reset_stats(pp_ctx* ctx) {
    int r = check_ctx(ctx, false, false);
    if (r) return r;
    if (ctx->has_rrt) {
        PP_HIP(hipMemcpyAsync(ctx->h_state.p, ctx->d_state.p, sizeof(DevState), hipMemcpyDeviceToHost, ctx->stream));
        PP_HIP(hipStreamSynchronize(ctx->stream));
        DevState d = ctx->h_state.p[0];
        d.iterations = d.accepted = d.windows = d.truncations = d.repair_rounds = d.repairs =
            d.literal_repairs = d.nn_flagged = d.node_evals = d.blocked = 0;
        ctx->h_state.p[0] = d;
        PP_HIP(hipMemcpyAsync(ctx->d_state.p, ctx->h_state.p, sizeof(DevState), hipMemcpyHostToDevice, ctx->stream));
        PP_HIP(hipStreamSynchronize(ctx->stream));
    }
    if ((r = ctx->reset_host_stats())) return set_err(r, "resetting the statistics");
    return PP_OK;
}

int pp_set_profiling(pp_ctx* ctx, int enabled) {
    int r = check_ctx(ctx, false, false);
    if (r) return r;
    if (enabled && !ctx->wg_pts.p) {  // one tally slot per walk workgroup (any walk grid)
        PP_HIP(ctx->wg_pts.reserve(3 * kWalkTallySlots));
        PP_HIP(hipMemsetAsync(ctx->wg_pts.p, 0, 3 * kWalkTallySlots * sizeof(long long), ctx->stream));
        PP_HIP(hipStreamSynchronize(ctx->stream));
    }
    if (enabled && !ctx->cf_tally.p) {
        PP_HIP(ctx->cf_tally.reserve(4));
        PP_HIP(hipMemsetAsync(ctx->cf_tally.p, 0, 4 * sizeof(long long), ctx->stream));
        PP_HIP(hipStreamSynchronize(ctx->stream));
    }
    ctx->prof = enabled != 0;
    return PP_OK;
}

}  // extern "C"
