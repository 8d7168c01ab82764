// pp_types.h — POD types shared by the host planner and the HIP kernels.
#pragma once

#include <stdint.h>

#include <hip/hip_runtime.h>  // uint4

namespace ppamd {

// dubins_literal return codes
enum : int { kSteerNone = 0, kSteerSome = 1, kSteerOverflow = -1 };

// Per-candidate verdict of the fused steer + collide kernel.
enum : int {
    kReject = 0,   // verify_node == false (out of bounds or an obstacle is hit)
    kAccept = 1,   // verify_node == true
    kLiteral = 2,  // fast path cannot reproduce the trim quirk exactly: rerun the literal path
    kError = 3,    // n_point overflow (the reference would panic) or scratch too small
};

constexpr int kCandCap = 16;         // in-window nearer-sample entries kept per sample
constexpr int kMaxChunks = 64;       // node chunks of the NN screen (partials per sample)
constexpr int kLiteralCap = 16384;   // points per literal-path scratch buffer
constexpr int kLiteralWaves = 256;   // literal scratch buffers (explicit-task kernel)
constexpr int kResolveThreads = 512;  // resolve_tail_kernel (8 waves, 256 VGPRs: the repair path)
constexpr int kMaxWindow = 4096;     // K limit: the resolve keeps the window's state in LDS
constexpr int kMinDynWindow = 128;   // the adaptive window's floor (DevState.kdyn)
constexpr int kSteerPrepBytes = 152; // sizeof(SteerPrep) (checked in pp_kernels.hip)
constexpr int kPrepLanes = 8;        // lanes per task in steer_prep's phase A
constexpr int kPrepThreads = 256;    // steer_prep workgroup: 32 tasks (8 per wave)
constexpr int kWalkThreads = 512;    // steer_walk workgroup: 8 tasks at a time (3 workgroups per CU)
constexpr int kWalkTallySlots = 4096;  // profiling: walk point tallies per workgroup (x2: arcs)
constexpr int kCfMaxDepth = 8192;    // check_finish: ancestor path per wave, in a global buffer of
                                     // grid * kCfWaves * kCfMaxDepth ints (32 MiB per 256
                                     // workgroups, allocated on the first check_finish)
constexpr int kCfLevels = 16;        // RECURSION_LIMIT, rrt.rs:14
constexpr int kCfMaxEdges = kCfLevels + 1 + kCfMaxDepth;
#ifndef PP_CF_MINW
#define PP_CF_MINW 2
#endif
constexpr int kCfMinW = PP_CF_MINW;  // check_finish: waves per SIMD (its register budget)
constexpr int kCfGrid = 256 * kCfMinW;  // check_finish workgroups: kCfMinW per CU

// Scene in device memory (Space, rrt.rs:70-78, with Q10 analytic discs).
struct SceneDev {
    double minx, maxx, miny, maxy;  // shrunken bounds rectangle (rrt.rs:82-106)
    double turn_radius;             // Robot.max_steer (rrt.rs:37-39, used at 424)
    double step_size;               // normalised Dubins step (rrt.rs:424 → dubins.rs:369)
    int m;                          // discs
    const double* cx;
    const double* cy;
    const double* r2;     // (r + width/2)^2
    const double* rcull;  // (r + width/2) * (1 + 1e-9) + 1e-9: conservative bbox cull radius
    // uniform grid over the discs: cell (gx, gy) = floor((v - g0) * ginv), clamped; a disc is
    // listed in every cell its cull box [c - rcull, c + rcull] touches (CSR: off, items)
    double gx0, gy0, ginv;
    double gcell;  // 1 / ginv (the cell size; s_classify's slabs)
    int gnx, gny;
    const int* goff;    // [gnx * gny + 1]
    const int* gitems;  // disc indices
    // LDS image of (goff, gitems, cx, cy, r2) — or of the occupancy bits — staged by the steer
    // kernels when it fits
    int lds_bytes;  // 0: read the scene from global memory
    const uint4* img;  // the LDS image, contiguous in global memory (lds_bytes / 16 words)
    int lds_goff, lds_items, lds_cx, lds_cy, lds_r2;  // byte offsets inside the image
    // the discs in f32 for the per-lane cull: (cx, cy, rcull rounded up, r + width/2)
    const float4* d4;
    int lds_d4;
    // occupancy grid (BASELINE config 4): when bits != nullptr the discs are ignored and every
    // polyline point probes its cell: (i, j) = (floor((x - bx0) * binv), floor((y - by0) * binv)),
    // bit i % 32 of word j * bwords + i / 32; a point outside the grid counts as occupied
    const uint32_t* bits;
    int bw, bh, bwords;
    double bx0, by0, binv;
    // polygon mode (pp_space_new_polygons, build-defined Q10p): when ne > 0 the grid items are
    // obstacle polygon edges (ex0, ey0)-(ex1, ey1) instead of discs (d4 = their f32 cull discs:
    // midpoint, half length + h rounded up); a segment hits an edge when they cross or an
    // endpoint of one lies within h of the other (h2 = (width/2)^2).  epoly: polygon id per edge
    // (a polygon's edges are consecutive) for the point-inside test.  nbv > 0: the bounds are the
    // polygon ring (bvx, bvy) eroded by h, on top of the rectangle test (its shrunken bbox).
    int ne;
    const double* ex0;
    const double* ey0;
    const double* ex1;
    const double* ey1;
    const int* epoly;
    double h2;
    int nbv;
    const double* bvx;
    const double* bvy;
    float cull_slack;  // f32 cull slack for the scene's coordinate magnitude
    // disc scenes: the cells of an ibn x ibn grid over the sampling box that lie wholly inside an
    // inflated disc (scene::inside_bitmap), the one-load point_blocked pre-test; null: none
    const uint32_t* ibits;
    int ibn, ibwords;
    double ibx0, iby0, ibinv;
    int root_blocked;  // planner (polygon mode): the root itself fails verify, so every
                       // line_to_origin does (check_finish: optimize accepts no candidate)
};

// Tree in device memory: f32 SoA for the NN screen, f64 SoA for everything exact.
struct TreeDev {
    float* x32;
    float* y32;
    double* x;
    double* y;
    double* yaw;
    int* parent;
};

// Device-resident planner state: the window kernels read it and the resolve kernel advances it,
// so windows are enqueued back to back without a host round trip.  Windows are pipelined: the
// window kernel of window w scans w's samples while its workgroup 0 resolves and commits window
// w - 1, so the scan-side fields are kept per window parity (p = w & 1).
struct DevState {
    int64_t it;      // next iteration (RNG counter base) = committed iterations
    int n;           // tree nodes (committed)
    int W;           // samples in the current window (0: nothing left to do / void window)
    int error;       // sticky kError seen (the reference would panic)
    int flag_count;  // NN samples flagged for the exact rescan (this window)
    int ncomp;       // candidate entries appended by nn_finalize's pair search (this window)
    int npend;       // samples queued for the resolve's round passes (this window)
    int weff;        // the window stops before this sample (a candidate list overflowed)
    int n_scan;      // tree nodes the next window's scan covers (nodes past it: nn_finalize)
    int64_t it_spec; // first iteration of the next window to scan
    int64_t wsp[2];  // per parity: first iteration of the window the scan generated
    int Wp[2];       // per parity: its sample count
    int nsp[2];      // per parity: tree nodes its scan covered
    int Wsp[2];      // per parity: samples the screen covers (the window's samples not in an
                     // obstacle: sorted positions [0, Wsp); samples_role)
    int chp[2];      // per parity: the screen's node chunks for those samples
    int64_t void_seq;  // window sequence number voided by a truncated predecessor (-1: none)
    int resolve_bail;  // the window kernel's resolve needed a repair: resolve_tail_kernel redoes it
    int kdyn;          // adaptive window: samples drawn per window (<= K; the commit adapts it)
    // statistics (pp_stats)
    int64_t iterations, accepted, windows, truncations, repair_rounds, repairs, literal_repairs,
        nn_flagged, node_evals;
    int64_t blocked;  // samples in an obstacle (point_blocked): rejected without steer or pair list
    // the query batch's active-task list (round 5): steer_prep / steer_walk run over i < W with the
    // compacted task i (its record at i) and store its yaw at slot alist[i], its verdict in list
    // order (MqDev::lstat); null: task i is slot i (the window pipeline, RRT*, the steer rounds)
    const int* alist;
    // list mode: the walk's verdict of task i sits at (i % lgrid) * lper + i / lgrid, so each
    // walk workgroup (it takes i = b, b + lgrid, ...) stores one contiguous run and a line of the
    // array is written back from one XCD's L2; the walk sets both for the insert
    int lgrid, lper;
};

// An explicit steer task: child (x, y) steered toward its parent — tree node `pnode` when
// pnode >= 0, else the explicit pose (px, py, pyaw).
struct SteerTask {
    double x, y, px, py, pyaw;
    int pnode;
    int literal;  // 1 = take the literal (single-lane) path
};

// RRT* extension of a SteerTask (a parallel array, so the extend batches keep 48-B tasks)
struct StarTaskExt {
    double cyaw;           // own_yaw: the child keeps this heading (rewire: an existing node's
                           // pose) instead of compute_yaw toward the parent (rrt.rs:267-271)
    double cbase, climit;  // cull: steer_prep settles the task as rejected, without a walk,
                           // unless cbase + its Dubins cost < climit (it cannot matter)
    int own_yaw;
    int cull;
    int node;  // rewire: the child's tree node
    int pad;
};

// A window sample i < j that is strictly nearer to sample j than j's snapshot NN, with the
// speculative verdict for (j, parent i) computed by the steer kernel.
struct CandEntry {
    int j, i;
    double d2;
    double yaw;
    int status;
    int pad;
};

// Per-task steer record of the window pipeline, written by steer_prep (8 lanes per task) and read
// by steer_walk (one wave per task) with scalar loads.  No grid points are stored: steer_walk
// generates the `pd` values of generate_local_course (dubins.rs:239-255) lane-parallel from the
// generator's initial state kept here (kPrepFallback; cnt[] is always 0, kept for the layout).
struct PrepRec {
    double x, y, px, py, yaw, pyaw;  // child (point 0), parent (the junction) and their headings
    double c, cw, sw;                // curvature, cos/sin(-yaw) of the world transform
    double ox[3], oy[3];             // segment origins in the local frame
    double ca[3], sa[3];             // segment trig: S cos/sin(o.yaw), L/R cos/sin(-o.yaw)
    double L[3];                     // segment lengths (the serial walk of kPrepFallback)
    double fb_pd, fb_dd;             // kPrepFallback: the generator's initial state (pd, d)
    long long n_point;               // dubins.rs:369
    int m[3], cnt[3];                // segment modes; cnt: unused (0)
    int state, fb_seg;               // kPrepNone / kPrepFallback or a verdict; the generator's
                                     // initial segment (0)
    int trim1;                       // the endpoint's local x is 0.0: the trim also pops the last
                                     // grid point (dubins.rs:281-288; the walk checks its x)
};
enum : int { kPrepWalk = -1, kPrepNone = 4, kPrepFallback = 5 };

// Multi-query batch (BASELINE config 3): Q independent trees, tree q in rows [q * cap, q * cap +
// n[q]) of the SoA arrays, all advanced one extend iteration per lockstep step.
struct MqDev {
    int Q;             // queries
    int cap;           // node rows per query (max_iter + 1: at most one insert per iteration)
    int64_t max_iter;  // RRT.max_iter of every query
    double* x;
    double* y;
    double* yaw;
    int* parent;
    int* n;                 // [Q] tree nodes
    int64_t* it;            // [Q] next iteration
    int64_t* evals;         // [Q] node-distance evaluations of the NN so far
    const uint64_t* seed;   // [Q] sampling stream
    const uint8_t* blocked; // [Q] polygon mode: the root fails verify, so every line_to_origin
                            // does and nothing is ever inserted (rrt.rs:414-426); may be null
    // speculative windows per query: every step evaluates the next K iterations of each query
    // against its tree at the step start (task q * K + k = iteration it[q] + k); the insert
    // replays them in order and stops at the first iteration whose nearest node would be one of
    // the window's own accepted samples (the next step resumes there), so the result equals
    // the one-iteration-per-step run for every K
    int K;
    const int64_t* target;  // [Q] iteration this pp_batch_extend call stops at
    double* nnd2;           // [Q * K] exact d2 of each task's snapshot nearest node
    // the verdict cache of the lockstep steps: it_prev[q] = the iteration of slot 0 of the tasks
    // now in the task region (the previous step's), so a window that starts T iterations later
    // finds iteration it + k in old slot k + T; null: no cache (RRT* rows)
    int64_t* it_prev = nullptr;
    int* status = nullptr;  // the previous step's verdicts (the task region's)
    // active-task compaction (round 5): mq_sample_nn settles the blocked and cached slots itself
    // (status, and tyaw = the cached task's yaw) and lists the slots that need a steer in
    // alist[0, st->W); the insert resets st->W.  null: every slot goes through the steer
    int* alist = nullptr;
    SteerTask* ctask = nullptr;  // the listed tasks, compacted (ctask[i] = tasks[alist[i]])
    // the listed tasks' verdicts in list order (the walk's stores stay contiguous); a listed
    // slot's status holds -2 - i until mq_insert resolves it from lstat[i]
    int* lstat = nullptr;
    DevState* st = nullptr;
    double* tyaw = nullptr;
};
// RRT* batch (BASELINE config 5; build-defined, oracle/pp_oracle.c orc_star_extend, DESIGN.md
// §3.7): Q independent RRT* trees in the MqDev rows (K = 1), one iteration per query and step in
// three steer rounds — A: the nearest edge (the gate), B: the other choose-parent candidates
// (X_near), C: the rewire edges X_near → new — each an explicit-task steer_prep / steer_walk pass
// whose task count the previous kernel sets on the device.
constexpr int kStarKMax = 63;  // neighbours per insert: with the nearest, <= 64 candidates (lanes)
struct StarDev {
    MqDev mq;            // trees, iteration counters, seeds, blocked roots, targets (K = 1)
    double* cost;        // [Q * cap] node cost, cost(root) = 0, cost = cost(parent) + elen
    double* elen;        // [Q * cap] Dubins cost of the node's edge to its parent
    int* mark;           // [Q * cap] subtree propagation: level stamp of the node
    int* stamp;          // [Q] next free level stamp
    const int* ksched;   // [cap + 1] |X_near| of an insert into an n-node tree (orc_star_k)
    double eta;          // Steer distance (0: the new node sits at the sample, Q5)
    double* px;          // [Q] the new point of the current iteration (after Steer)
    double* py;
    int* pn;             // [Q] its nearest node; -1: the query is idle this step
    int* near;           // [Q * kStarKMax] X_near in (d2, index) order
    int* nnear;          // [Q] |X_near|; -1: no insert this step (gate rejected, idle)
    int* bslot;          // [Q] first round-B task of the query
    uint64_t* bmask;     // [Q] X_near positions with a round-B task (not the nearest, not pruned)
    double curv;         // 1 / turn radius: the chord lower bound of a Dubins cost
    int* lit_locks;      // [kLiteralWaves] literal scratch slot locks (0 free)
    int* cslot;          // [Q] first round-C task; -1 none
    uint64_t* cmask;     // [Q] X_near positions with a round-C task
    double* cb;          // [Q] cost of the inserted node
    int64_t* rewires;    // [Q] rewires so far
    DevState* stA;       // W = Q (constant)
    DevState* stB;       // W = round-B task count (reset by star_sample, counted by star_knn)
    DevState* stC;       // W = round-C task count (counted by star_insert)
};

constexpr int kMqMaxK = 64;  // window limit per query (config 3's strong-scaling parallelism)
constexpr int kMqAutoK = 32; // the automatic window (halved while Q * K > 262144 tasks)

// Resolve scratch (global, one window; indexed by pending slot / list position).
struct ResolveScratch {
    int* order;     // [K * kCandCap] entry indices of list positions past the LDS-staged ones
    int* rep;       // [K] repair verdict (-1: none), | 16 when it came from the literal path
    double* repyaw; // [K]
};

// pp_rrt_extend_samples' per-iteration record (caller-drawn samples): the commit of a window
// writes, for every committed iteration it, the nearest node Node::new took as parent (rrt.rs:
// 169-175, 378-391), the new node's yaw and verify_node's verdict at [it - base]; each pointer
// may be null (all null: no record)
struct SampleRec {
    int64_t base;
    int* par;
    double* yaw;
    unsigned char* ok;
};

// window status word after the resolve (snap_status of a pending sample is overwritten with it):
// bit 0 = accepted, bit 2 = its parent is the window sample fin_par[j] (else its snapshot NN)
constexpr int kWinParent = 4;

}  // namespace ppamd
