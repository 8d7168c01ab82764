// pp_kernels.h — host-side launch wrappers of the HIP kernels (pp_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "pp_types.h"

namespace ppamd {

// Everything one window (or one nearest-neighbour batch) touches.  Buffers are sized for K.
struct WindowArgs {
    int K = 0;           // samples per window
    int Kcap = 0;        // buffer capacity per window (parity stride of wsx / wsy)
    int64_t target = 0;  // iteration the enqueued windows stop at
    uint64_t seed = 0;
    double eps_coord = 0.0;
    DevState* st = nullptr;
    SceneDev sc{};
    TreeDev tr{};
    double* wsx = nullptr;        // [2 * Kcap] samples, double-buffered by window parity
    double* wsy = nullptr;
    float* wsx32 = nullptr;       // [2 * Kcap] their f32 copies
    float* wsy32 = nullptr;
    int* perm = nullptr;          // [2 * Kcap] spatially sorted sample order (window_samples)
    int* cofs = nullptr;          // [2 * 257] start of each Morton cell in the sorted order
    float2* sxy = nullptr;        // [2 * Kcap] the samples in sorted order (f32)
    double* sq = nullptr;         // [2 * Kcap] |q - o|^2 about the screen block's centre
    double* ssx = nullptr;        // [2 * Kcap] the samples in sorted order (f64)
    double* ssy = nullptr;
    float2* ob = nullptr;         // [2 * kMaxWindow / 512] the screen blocks' centres
    int* ipos = nullptr;          // [2 * Kcap] sample -> sorted position
    float* pbest = nullptr;
    float* psecond = nullptr;
    int* pidx = nullptr;
    int* nn_idx = nullptr;
    double* nn_d2 = nullptr;
    int* cand_cnt = nullptr;
    CandEntry* cand = nullptr;
    int* snap_status = nullptr;
    double* snap_yaw = nullptr;
    double* snap_pose = nullptr;  // [3K] parent pose of each unflagged sample (nn_finalize)
    PrepRec* rec = nullptr;       // [K + K * kCandCap] per-task steer records
    int* pend = nullptr;          // [K] samples queued for the resolve's round passes
    int* fin_par = nullptr;       // [K] window parent of a resolved sample (kWinParent)
    ResolveScratch rs{};
    double* lit_scratch = nullptr;
    long long* wg_points = nullptr;  // profiling: walked points per walk workgroup (or null)
    const SceneDev* scp = nullptr;  // the scene in device memory (samples_role's point_blocked)
    unsigned char* blk = nullptr;   // [2 * Kcap] sample in an obstacle (null: no pre-test)
    // caller-drawn samples (pp_rrt_extend_samples): iteration it's sample is (hsx, hsy)[it -
    // hrec.base] instead of the seeded stream (null: the stream); hrec: the per-iteration record
    const double* hsx = nullptr;
    const double* hsy = nullptr;
    SampleRec hrec{0, nullptr, nullptr, nullptr};
};

// Enqueue window number `seq` on stream s: its window kernel also resolves and commits window
// seq - 1 when resolve_prev (the previous window of the same batch).  ev (optional) = 5 timing
// events: before the window kernel, then after it, nn_finalize, steer_prep and steer_walk.
hipError_t launch_window(hipStream_t s, const WindowArgs& a, hipEvent_t* ev, int64_t seq,
                         int resolve_prev);
// PP_FIN_STAMPS diagnostic builds: nn_finalize's wall-clock phase stamps per workgroup
constexpr int kFinStampSlots = 10, kFinStampWGs = 512;
#ifdef PP_FIN_STAMPS
hipError_t fin_stamps_copy(unsigned long long* out, size_t n);
#endif

// Resolve and commit the last enqueued window (seq_next - 1): ends a batch.
hipError_t launch_drain(hipStream_t s, const WindowArgs& a, int64_t seq_next);

// Exact nearest tree node of Wp[0] samples (wsx, wsy parity 0; nsp[0] = n): screen + finalize +
// rescan.
hipError_t launch_nearest(hipStream_t s, const WindowArgs& a);

// Space::verify (rrt.rs:124-137) of k polylines, line i = points [off[i], off[i + 1]) of X/Y;
// ok[i] = 1 when it verifies.
hipError_t launch_verify_lines(hipStream_t st, const SceneDev& sc, const double* X,
                               const double* Y, const int64_t* off, int k, uint8_t* ok);

hipError_t launch_steer_tasks(hipStream_t st, const SceneDev& sc, const TreeDev& tr,
                              const SteerTask* tasks, int n, int* out_status, double* out_yaw,
                              double* scratch);

// RRT::check_finish for k tree nodes (one wave per node, at most `grid` workgroups of kCfWaves
// waves; gpath: grid * kCfWaves * kCfMaxDepth ints, the waves' ancestor paths).  ok/len/npts per
// node; chain (optional) = k rows of [levels, edges, optimize's chosen ancestors...] with
// kCfLevels + 2 ints per row; want_line: materialise the lines of the verified finishes (length;
// points of line item i in workgroup i's pts/etab, items: 1 + k * kCfItem ints, items[0] zeroed
// before the launch).  err |= 1 depth > kCfMaxDepth, 2 finalize panic, 4 steer overflow, 8 point
// capacity.  tally (profiling, optional): += nodes, edges steered + verified, polyline points
// walked.
// check_finish_kernel modes: check_finish (rrt.rs:428-438), optimize alone (rrt.rs:463-487),
// finalize of a caller-built goal node (rrt.rs:489-540)
enum : int { kCfCheck = 0, kCfOptimize = 1, kCfFinalize = 2 };
// check_finish over a query batch (pp_batch_plan): item b = node nodes[b] of query qidx[b]
struct CfBatch {
    const int* qidx = nullptr;  // null: the one-tree planner
    int row_cap = 0;            // SoA rows per query
    const double* goals = nullptr;   // [3Q] goal x, y, yaw
    const uint8_t* blocked = nullptr;  // [Q] polygon mode: the root fails verify (may be null)
    // optimize's memo (rows as the tree's SoA: query q at q * row_cap; zeroed per launch, may be
    // null): ftab[v] = 0 unknown, 1 no candidate of v verifies, 2 + m (| 1 << 30 when that edge's
    // steer is None) — v's first verifying candidate root first is its depth-m ancestor; gtab[v] =
    // 0 unknown, else 1 + the verdict of finalize's copy edge from v (see check_finish_kernel)
    int* ftab = nullptr;
    int* gtab = nullptr;
    // the batch plan's goal-edge verdicts per item (0 unknown, else 1 + verdict; may be null)
    const int* gotab = nullptr;
    // compact memo rows (may be null: q * row_cap): query q's nodes at moff[q] + q, moff = the
    // exclusive scan of the queries' items (n_q - 1)
    const int* moff = nullptr;
};

// check_finish of a query batch in steer rounds (pp_batch_plan, see pp_kernels.hip): phase A
// fills ftab for every node, phase B the goal edges (gotab) and copy edges (gtab), the assemble
// kernel decides every item whose verdicts are all known and lists the others (plist, pcount)
// for check_finish_kernel.  Node b < nitems is item b, b - nitems < Q query's root.
constexpr int kCfbSpan = 2;  // phase A candidates per node and round (span A/B: DESIGN §3.3)
struct CfbArgs {
    TreeDev tr{};
    int row_cap = 0;
    int span = kCfbSpan;  // phase A candidates per node in the current round
    int nitems = 0, Q = 0;
    const int* qidx = nullptr;
    const int* nodes = nullptr;
    const double* goals = nullptr;
    const int* moff = nullptr;  // compact memo rows: query q's nodes at moff[q] + q
    int* ftab = nullptr;      // rows (the memo of CfBatch)
    int* gtab = nullptr;      // rows
    int* gotab = nullptr;     // [nitems]
    int* gclaim = nullptr;    // rows: copy edge claimed for phase B
    unsigned char* tnone = nullptr;     // rows: the node's own tree edge has a None steer
    unsigned char* tnone_up = nullptr;  // rows: any tree edge from the node down to the root has one
    int* depth = nullptr;     // [nitems + Q]
    int* open = nullptr;      // [nitems + Q] phase A: not settled yet
    int* tfirst = nullptr;    // [nitems + Q] the round's first task of the node
    int* tcnt = nullptr;      // [nitems + Q] ... and its count
    int* tnode = nullptr;     // [tasks] phase A: node b; phase B: item b, or -1 - row (copy edge)
    SteerTask* tasks = nullptr;
    StarTaskExt* ext = nullptr;
    PrepRec* rec = nullptr;   // (one chunk of the round's tasks at a time: launch_cfb_chunk)
    unsigned char* none = nullptr;  // per task: its steer was None (the record's kPrepNone)
    int* status = nullptr;
    double* yaw = nullptr;
    DevState* st = nullptr;   // st->W: the round's task count (ncomp 0)
    int* maxdepth = nullptr;
    int* pcount = nullptr;
    int* wsum = nullptr;      // (profiling) += every round's task count
    int* dhist = nullptr;     // [kCfbDepthBins] nodes per depth (the last bin: that depth or more)
};
constexpr int kCfbDepthBins = 64;
enum : int { kCfbDepth = 0, kCfbEmitA, kCfbConsumeA, kCfbEmitB, kCfbStoreB, kCfbAssemble };
hipError_t launch_cfb(hipStream_t s, const SceneDev& sc, CfbArgs a, int phase, int round,
                      int* ok = nullptr, double* len = nullptr, int* npts = nullptr,
                      int* err = nullptr, int* items = nullptr, int* plist = nullptr);
hipError_t launch_cfb_steer(hipStream_t s, const SceneDev& sc, const CfbArgs& a, int max_tasks,
                            bool own_yaw, long long* wg_points = nullptr);
// a chunk of a round's steer: begin (the chunk's task count from the round's) or, after its walk,
// the None flags of its records into none[0, chunk->W)
hipError_t launch_cfb_chunk(hipStream_t s, const DevState* all, DevState* chunk, int base,
                            int cap, bool begin, const PrepRec* rec, unsigned char* none);
// the rounds' literal-path tasks re-run by steer_collide_literal (a scratch slot per wave)
hipError_t launch_cfb_literal(hipStream_t s, const SceneDev& sc, const CfbArgs& a, int max_tasks,
                              int* list, int* count, double* lit_scratch);
// cf_line_kernel's per-workgroup buffers: pts (3 x pts_cap doubles: x, y, hypots / words), etab
// (2 x (path_cap + kCfLevels + 1) ints) and path (path_cap ints) per workgroup.  spill != null
// (tier 1): a line deeper than path_cap or longer than pts_cap is appended to spill (the items
// layout, spill[0] its count, zeroed before the launch) instead of failing, and tier 2 — the full
// capacities (kCfMaxDepth, kCfPtsCap) on a few workgroups — runs the spill list
struct CfLineBufs {
    double* pts = nullptr;
    int pts_cap = 0;
    int* etab = nullptr;
    int* path = nullptr;
    int path_cap = kCfMaxDepth;
    int* spill = nullptr;
    int spill_cap = 0;
};
struct CfLines {
    int grid1 = 0;  // 0: no line kernel
    CfLineBufs t1;
    int grid2 = 0;  // tier 2 (when t1.spill)
    CfLineBufs t2;
};
hipError_t launch_check_finish(hipStream_t st, const SceneDev& sc, const SceneDev* scg,
                               const TreeDev& tr,
                               const int* nodes, int k, double gx, double gy, double gyaw,
                               double gyaw_opt, int level0, int mode, int want_line, int* ok,
                               double* len, int* npts, int* chain, double* lit_scratch,
                               int* lit_locks, const CfLines& lines, int* err, int grid,
                               long long* tally, const CfBatch& cb, int* gpath, int* items,
                               const int* blist = nullptr);
constexpr int kCfWaves = 4;                     // check_finish: waves (nodes in flight) per workgroup
constexpr int kCfItem = 4 + kCfLevels;          // a line item: b, s, verified, 0, pos[kCfLevels]

// pp_batch_plan: the (query, node) items of the accepted nodes (off: [Q + 1] exclusive scan of
// n_q - 1), and per query the first minimum length over its items' check_finish results
hipError_t launch_mq_plan_items(hipStream_t s, int Q, const int* off, int* qidx, int* nodes);
hipError_t launch_mq_plan_reduce(hipStream_t s, int Q, const int* off, const int* ok,
                                 const double* len, const int* npts, int* best_node,
                                 double* best_len, int* best_npts, int* n_fin);

// Multi-query batch: `steps` lockstep extend iterations of every query (config 3).
struct MqArgs {
    MqDev mq{};
    SceneDev sc{};
    DevState* st = nullptr;  // W = Q, ncomp = 0 (the steer kernels' task count)
    SteerTask* tasks = nullptr;
    PrepRec* rec = nullptr;
    int* status = nullptr;
    double* yaw = nullptr;
    double* lit_scratch = nullptr;  // kLiteralWaves buffers
    int* lit_locks = nullptr;       // their slot locks (0 free)
    int* err = nullptr;
    hipEvent_t* ev = nullptr;  // optional: 5 per step: before mq_sample_nn, then after it, steer_prep,
                               // steer_walk and mq_insert
    long long* wg_points = nullptr;  // profiling: walked points per walk workgroup (or null)
    const SceneDev* scp = nullptr;   // the scene in device memory: point_blocked (or null: none)
};
hipError_t launch_mq_steps(hipStream_t s, const MqArgs& a, int steps);
hipError_t launch_mq_init(hipStream_t s, const MqDev& mq, const double* starts);
// the per-query iteration targets of a pp_batch_extend(n_steps) call
hipError_t launch_mq_target(hipStream_t s, const MqDev& mq, int64_t n_steps, int64_t* target);

// RRT* query batch (config 5): `steps` lockstep RRT* iterations of every query.  Task arrays of
// round A hold Q entries, rounds B and C Q * kStarKMax; rec is shared by the rounds.
struct StarArgs {
    StarDev sd{};
    SceneDev sc{};
    SteerTask *tA = nullptr, *tB = nullptr, *tC = nullptr;
    StarTaskExt *eB = nullptr, *eC = nullptr;  // rounds B / C: cull limits, rewire child poses
    int *sA = nullptr, *sB = nullptr, *sC = nullptr;        // verdicts
    double *yA = nullptr, *yB = nullptr, *yC = nullptr;     // child yaw of each task
    double *cA = nullptr, *cB = nullptr, *cC = nullptr;     // Dubins cost of each task
    PrepRec* rec = nullptr;
    double* lit_scratch = nullptr;  // kLiteralWaves buffers
    int* err = nullptr;
    hipEvent_t* ev = nullptr;  // optional: 8 per step, around star_sample and each round's walk
    long long* wg_points = nullptr;  // profiling: walked points per walk workgroup (or null)
};
hipError_t launch_star_steps(hipStream_t s, const StarArgs& a, int steps);
hipError_t launch_star_init(hipStream_t s, const StarArgs& a, const double* starts);

// dubins_path_planning_from_origin for n (dx, dy, eyaw, c, step_size) configurations
hipError_t launch_dubins_origin(hipStream_t st, const double* conf, int n, int cap, double* px,
                                double* py, double* pyaw, int* n_out, int* word_out,
                                double* cost_out, int* status_out);
// the six Dubins words of n (alpha, beta, d) triples
hipError_t launch_dubins_words(hipStream_t st, const double* abd, int n, double* tpq, int* ok);

hipError_t launch_dubins_batch(hipStream_t st, const double* conf, int n, int cap, double* px,
                               double* py, double* pyaw, int* n_out, int* word_out,
                               double* cost_out, int* status_out);

}  // namespace ppamd
