/*
 * pathplanning_amd.h — C ABI of the MI355X-native RRT extend hot path.
 *
 * Drop-in boundary for tsturzl/rs-pathplanning's `rrt` / `dubins` public API (src/lib.rs:5-6):
 * a Rust host binds these symbols through a thin `extern "C"` block and keeps
 * its own types; everything here is plain pointers, sizes and status codes.
 *
 * Conventions
 *   - Every int-returning call returns PP_OK (0) or a negative PP_ERR_* code; no exception or
 *     panic crosses the boundary.  pp_last_error() gives the calling thread's last message.
 *   - The caller owns every host buffer; a context owns its device memory and HIP stream.
 *   - A context is not thread-safe: use one context per host thread (and per GPU).
 *   - Where the reference returns Option::None the ABI reports it in an output field
 *     (word = -1, idx = -1, ok = 0), not as an error.
 *   - The product path is HIP only: every compute call fails with PP_ERR_NO_DEVICE when no
 *     gfx950 device is present.  There is no CPU fallback.
 */
#ifndef PATHPLANNING_AMD_H
#define PATHPLANNING_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: pp_stats lost the diagnostic stamps and gained the batch / check_finish counters;
 *    pp_rrt_get_stats takes the caller's sizeof(pp_stats); pp_batch_plan added
 * 3: pp_batch_set_schedule, the persistent batch kernel; pp_stats appended its counters
 * 4: the persistent batch kernel and pp_batch_set_schedule removed (slower than the lockstep
 *    schedule on every workload measured: DESIGN.md §3.4); its pp_stats counters are reserved
 *    (always 0, the layout kept); pp_batch_set_finish_schedule replaces the library's former
 *    environment knobs
 * 5: pp_rrt_extend_samples and pp_rrt_tree_import (the host owns the RNG and the tree); nothing
 *    else changed */
#define PP_ABI_VERSION 5

#define PP_OK 0
#define PP_ERR_INVALID_ARGUMENT (-1)
#define PP_ERR_HIP (-2)
#define PP_ERR_NO_DEVICE (-3)
#define PP_ERR_CAPACITY (-4)
#define PP_ERR_STATE (-5)          /* no scene / no planner configured yet */
#define PP_ERR_STEER_OVERFLOW (-6) /* generate_local_course would index past n_point (panic) */
#define PP_ERR_REFERENCE_PANIC (-7) /* finalize: an edge with no feasible Dubins word (panic) */

typedef struct pp_ctx pp_ctx;

/* DubinsConfig, src/dubins.rs:315-324 (field order and meaning kept) */
typedef struct pp_dubins_config {
    double sx, sy, syaw;
    double ex, ey, eyaw;
    double turn_radius;
    double step_size;
} pp_dubins_config;

/* Counters of the batched extend driver (since pp_rrt_new / pp_batch_new / pp_star_new or the
 * last pp_rrt_reset_stats).  pp_rrt_get_stats copies min(out_size, sizeof(pp_stats)) bytes: the
 * size argument guards ABI 2+ callers only (ABI 1's entry point had no out_size and a different
 * layout; a v1 binary must be rebuilt).  From ABI 2 on, fields are only ever appended, so an ABI 2
 * caller of a later library gets the prefix it knows and never an overrun.
 * The *_ms fields are HIP-event spans on the kernel's own stream: with the query batches' two or
 * three sub-batch streams a span also covers time the other streams' kernels held the GPU, so
 * their sums are stream-span times, not isolated kernel durations (those come from a rocprofv3
 * kernel trace: profiles/r*_kernel_durations.json). */
typedef struct pp_stats {
    int64_t iterations;       /* extend iterations consumed (plan_one calls, minus check_finish) */
    int64_t accepted;         /* nodes inserted */
    int64_t windows;          /* speculative windows launched */
    int64_t truncations;      /* windows cut short by an in-window candidate-list overflow */
    int64_t repair_rounds;    /* extra steer launches for parents that changed inside a window */
    int64_t repairs;          /* candidates re-steered in those rounds */
    int64_t literal_repairs;  /* candidates re-run on the literal single-lane path */
    int64_t nn_flagged;       /* samples whose f32 NN screen needed the exact f64 rescan */
    int64_t node_evals;       /* sample-node distance evaluations of the NN screen: screened
                                 samples (not in an obstacle) x the tree nodes the screen scanned */
    /* HIP events around every kernel of a window / batch step (profiling on), summed over the
     * launches; the batches keep their timed schedule (sub-batch streams) while profiled */
    double nn_scan_ms;        /* window_kernel (the NN screen + the previous window's resolve), or
                                 the batch NN (mq_sample_nn / star_sample) */
    int64_t nn_scan_launches;
    double steer_ms;          /* steer_walk */
    int64_t steer_launches;
    double finalize_ms;       /* nn_finalize (one tree: one launch per nn_scan launch) */
    double prep_ms;           /* steer_prep (one launch per steer launch) */
    double insert_ms;         /* mq_insert (query batch: one launch per nn_scan launch) */
    int64_t walk_points;      /* polyline points the steer walk generated and verified (profiling on) */
    int64_t walk_arc_points;  /* ... of them on L / R segments (one sincos each) */
    int64_t batch_steps;      /* query batches: lockstep steps launched (each up to the window per query) */
    int64_t batch_passes;     /* query batches: host passes (the first plus the top-ups of stopped windows) */
    double finish_ms;         /* device time of check_finish_kernel (HIP events; profiling on) */
    int64_t finish_launches;
    int64_t finish_nodes;     /* nodes check_finish ran on (profiling on) */
    int64_t finish_edges;     /* Dubins edges steered + verified by check_finish (profiling on) */
    int64_t finish_points;    /* polyline points those edges walked (profiling on) */
    int64_t finish_arc_points;  /* ... of them on L / R segments */
    /* ABI 3's persistent query-batch counters, removed in ABI 4: always 0 (layout kept) */
    int64_t reserved_abi3[8];
    int64_t samples_evaluated;  /* extend samples evaluated (one tree: the iterations) */
    int64_t samples_blocked;    /* ... of them whose point lies in an obstacle: rejected whatever
                                   the parent, without steer_prep / steer_walk or a pair list */
    int64_t walk_tasks;         /* steer_walk tasks walked (profiling on; ABI 5, appended) */
} pp_stats;

int pp_abi_version(void);
const char* pp_last_error(void);
/* number of visible HIP devices (0 when none); never fails on a CPU-only host */
int pp_device_count(int* n);

int pp_create(int device, pp_ctx** out);
int pp_destroy(pp_ctx* ctx);
int pp_synchronize(pp_ctx* ctx);

/* ------------------------------------------------------------- seeded sampling (host) */
/* SplitMix64 output `ctr` of stream `seed`: the build's replacement for rand::thread_rng
 * (src/rrt.rs:140).  Draw 2*it is x, 2*it+1 is y of iteration `it`. */
uint64_t pp_rng_u64(uint64_t seed, uint64_t ctr);
/* rand 0.7 gen_range(low, high) for f64 on that stream (src/rrt.rs:142-143) */
double pp_gen_range(uint64_t seed, uint64_t ctr, double low, double high);

/* --------------------------------------------------------------- dubins (src/dubins.rs) */
double pp_mod2pi(double theta);   /* dubins.rs:18-20 */
double pp_pi_2_pi(double angle);  /* dubins.rs:22-24 */
/* dubins_path_planning (dubins.rs:401-428) for n configurations on the GPU.  Output slot i of
 * px/py/pyaw is [i*cap, i*cap+cap).  word[i] is the ALL_PLANNERS index (0 LSL, 1 RSR, 2 LSR,
 * 3 RSL, 4 RLR, 5 LRL) or -1 for None; n_points[i] the kept point count; cost[i] the normalised
 * cost.  A configuration whose n_point exceeds cap gets word -2 and the call returns
 * PP_ERR_CAPACITY after filling the others. */
int pp_dubins_path_planning_batch(pp_ctx* ctx, const pp_dubins_config* confs, int n, int cap,
                                  double* px, double* py, double* pyaw, int32_t* n_points,
                                  int32_t* word, double* cost);

/* dubins_path_planning_from_origin (dubins.rs:326-399) for n configurations on the GPU, each the
 * 5 doubles (dx, dy, eyaw, c, step_size) of the Rust arguments (c = curvature, 1 / turn radius):
 * the LOCAL points after generate_local_course's trim (dubins.rs:281-288) and the yaw as generated
 * (not wrapped by pi_2_pi).  Outputs and errors as pp_dubins_path_planning_batch. */
int pp_dubins_path_planning_from_origin_batch(pp_ctx* ctx, const double* conf5, int n, int cap,
                                              double* px, double* py, double* pyaw,
                                              int32_t* n_points, int32_t* word, double* cost);
/* lsl, rsr, lsr, rsl, rlr, lrl (dubins.rs:27-153) of n (alpha, beta, d) triples on the GPU:
 * tpq[18 i + 3 w + {0, 1, 2}] = (t, p, q) of word w in ALL_PLANNERS order (dubins.rs:291),
 * ok[6 i + w] = 0 where the word is None (then its t, p, q are 0). */
int pp_dubins_words_batch(pp_ctx* ctx, const double* abd, int n, double* tpq, int32_t* ok);

/* ------------------------------------------------------------------ scene (src/rrt.rs) */
/* create_circle(center, radius) (rrt.rs:43-60): the crate's polygon, n = ceil(2 pi r) chords and
 * the n + 1 vertices i = 0..=n at angle 2 pi / n * i, x then y interleaved in xy (2 (n + 1)
 * doubles, same evaluation order as the Rust expression; host arithmetic, like pp_mod2pi).
 * *n = the vertex count; PP_ERR_CAPACITY when cap (vertices) is too small. */
int pp_create_circle(double cx, double cy, double radius, double* xy, int cap, int* n);
/* Space::new(bounds, Robot::new(width, height, max_steer), obstacles) (rrt.rs:25,81-122) with
 * the bounds an axis-aligned rectangle (x0, y0)-(x1, y1) and the obstacles create_circle discs
 * (rrt.rs:43-60) given as centres and radii.  Bounds shrink and discs grow by width/2. */
int pp_space_new(pp_ctx* ctx, double x0, double y0, double x1, double y1, double robot_width,
                 double robot_height, double max_steer, const double* cx, const double* cy,
                 const double* r, int m);
/* BASELINE config 4: replace the obstacles of the current Space by a bit-packed occupancy grid
 * of w x h cells of size `cell` whose corner is (x0, y0): cell (i, j) is bit i % 32 of word
 * j * ceil(w / 32) + i / 32.  Verify then requires every point of the line inside the bounds and
 * in a free cell, with cell = (floor((x - x0) / cell), floor((y - y0) / cell)) and points outside
 * the grid counting as occupied; segments are not rasterised.  (The reference has no grid mode;
 * this is the build-defined semantics of SURVEY.md §8d config 4.)  A later pp_space_new clears
 * it; a planner must be created after it (pp_rrt_new / pp_batch_new). */
int pp_space_set_grid(pp_ctx* ctx, const uint32_t* bits, int w, int h, double x0, double y0,
                      double cell);
/* Space::new(bounds, Robot::new(width, height, max_steer), obstacles) (rrt.rs:25,81-122) with
 * polygon bounds and polygon obstacles, as examples/rrt/src/main.rs:30-45 builds them from its
 * JSON scene.  bounds_xy: nb vertices (x, y interleaved) of the bounds ring; obstacle o is the
 * ring obs_xy[2*obs_off[o] .. 2*obs_off[o+1]); a closing repeat of the first vertex is dropped.
 * Build-defined: geo-offset's buffers are the exact Minkowski buffers — an
 * obstacle grows by the closed disc of radius width/2 (a segment hits it when it crosses an edge
 * or comes within width/2 of one), the bounds shrink to the points at distance >= width/2 from
 * the ring inside it (tested on the line's points, like geo's Contains<LineString>).
 * rand_point samples the bounds' bbox shrunk by width/2.  Replaces the previous scene. */
int pp_space_new_polygons(pp_ctx* ctx, const double* bounds_xy, int nb, const double* obs_xy,
                          const int32_t* obs_off, int n_obs, double robot_width,
                          double robot_height, double max_steer);
/* Space::verify (rrt.rs:124-137) of k polylines on the GPU: line i is the points
 * [off[i], off[i+1]) of x / y; ok[i] = 1 when the line is inside the bounds and meets no
 * obstacle (a one-point line is tested as a point). */
int pp_space_verify_batch(pp_ctx* ctx, const double* x, const double* y, const int64_t* off,
                          int k, uint8_t* ok);
/* the shrunken bounds bbox (minx, maxx, miny, maxy) sampled by Space::rand_point (rrt.rs:84-106) */
int pp_space_get_bounds(pp_ctx* ctx, double out_minx_maxx_miny_maxy[4]);

/* ----------------------------------------------------------------- planner (src/rrt.rs) */
/* RRT::new(start, start_yaw, goal, goal_yaw, max_iter, step_size, space) (rrt.rs:335-355) plus
 * the sampling seed and an initial node capacity (grown on demand). */
int pp_rrt_new(pp_ctx* ctx, double sx, double sy, double syaw, double gx, double gy, double gyaw,
               int64_t max_iter, double step_size, uint64_t seed, int64_t capacity);
/* candidates per speculative window (K in [1, 4096]; default 4096).  Results do not depend on K. */
int pp_rrt_set_window(pp_ctx* ctx, int k);
/* n_iter iterations of plan_one's extend (rrt.rs:583-589: rand_point, get_nearest_node,
 * Node::new, verify_node, insert) with the sequential semantics of one rayon thread. */
int pp_rrt_extend(pp_ctx* ctx, int64_t n_iter, int64_t* n_accepted);
/* plan_one's extend (rrt.rs:583-589) over k CALLER-DRAWN samples: iteration it + i takes
 * (sx[i], sy[i]) as its Space::rand_point (rrt.rs:139-146, 406-412) instead of the seeded stream,
 * so a host that owns its RNG drives the same speculative GPU windows (SURVEY.md §8(b)'s
 * pp_extend_batch).  Sequential semantics: sample i sees the tree after samples < i; accepted
 * samples are inserted in order (rrt.rs:586-589).  Per sample (each output may be NULL):
 * nearest[i] = get_nearest_node (rrt.rs:378-391) of the tree as it stood, i.e. the parent
 * Node::new took; yaw[i] = that node's compute_yaw (rrt.rs:169-175, 267-271); ok[i] = 1 when
 * verify_node (rrt.rs:414-426) accepted and the node was inserted (it then has index
 * n_before + the number of ok samples before i).  *n_accepted (may be NULL) = the inserts.
 * Samples must be finite; the iteration counter advances by k.  With samples drawn as
 * pp_gen_range(seed, 2 it, ..), pp_gen_range(seed, 2 it + 1, ..) the tree equals pp_rrt_extend's. */
int pp_rrt_extend_samples(pp_ctx* ctx, const double* sx, const double* sy, int64_t k,
                          int32_t* nearest, double* yaw, uint8_t* ok, int64_t* n_accepted);
/* replace the planner's tree by n host-owned nodes (root first, as pp_rrt_tree_export returns
 * them: Node x, y, yaw (rrt.rs:161-166) and parent, -1 for node 0, otherwise an earlier node:
 * the crate's insertion order, rrt.rs:586-589).  The scene, goal, step size, seed, iteration
 * counter and statistics stay; later extends continue from this tree.  Export -> import -> extend
 * equals extend on the original. */
int pp_rrt_tree_import(pp_ctx* ctx, const double* x, const double* y, const double* yaw,
                       const int32_t* parent, int64_t n);
/* one plan_one extend (rrt.rs:583-589); *accepted = 1 when the node was inserted */
int pp_rrt_plan_one(pp_ctx* ctx, int32_t* accepted);
int pp_rrt_tree_size(pp_ctx* ctx, int64_t* n);
int pp_rrt_iteration(pp_ctx* ctx, int64_t* it);
/* copy the tree out (root first): coordinates, yaw (Node.yaw, rrt.rs:161-166), parent (-1 root) */
int pp_rrt_tree_export(pp_ctx* ctx, double* x, double* y, double* yaw, int32_t* parent,
                       int64_t cap, int64_t* n);
/* line_to_origin(node, Robot.max_steer, step_size) (rrt.rs:291-321) of tree node `node`: the
 * concatenated polyline node -> ... -> root in the sequential order (each edge's Dubins points
 * child -> parent, steered on the GPU; [(x, y)] of the child where the steer is None; the root
 * contributes [(root x, root y)]).  *n = its points; PP_ERR_CAPACITY when cap is too small (call
 * with cap 0 for the size). */
int pp_rrt_line_to_origin(pp_ctx* ctx, int32_t node, double* x, double* y, int64_t cap,
                          int64_t* n);
/* RRT::get_nearest_node (rrt.rs:378-391) for k points: exact nearest by dx*dx+dy*dy, lowest
 * index on ties; d2 may be NULL */
int pp_rrt_get_nearest_node_batch(pp_ctx* ctx, const double* qx, const double* qy, int k,
                                  int32_t* idx, double* d2);
/* RRT::verify_node(Node::new(point, tree[parent])) (rrt.rs:169-175, 414-426) for k candidates:
 * ok[i] = 1 when the line to the root verifies; yaw[i] = the new node's yaw (may be NULL) */
int pp_rrt_verify_node_batch(pp_ctx* ctx, const double* x, const double* y,
                             const int32_t* parent, int k, uint8_t* ok, double* yaw);

/* --------------------------------------------------- goal connection (src/rrt.rs:428-619) */
/* RRT::check_finish (rrt.rs:428-438) for k tree nodes: optimize_from_goal's shortcut search
 * (rrt.rs:463-501, RECURSION_LIMIT 16), finalize's line (rrt.rs:503-540) and its verify.
 * ok[i] = 1 when the line verifies (Some); length[i] = its euclidean_length, n_points[i] its
 * points (both may be NULL; computed for verified lines only).  chain (may be NULL) receives k
 * rows of PP_CF_CHAIN ints: [levels, edges, optimize's chosen ancestor per level...]. */
#define PP_CF_CHAIN 18
int pp_rrt_check_finish_batch(pp_ctx* ctx, const int32_t* nodes, int k, uint8_t* ok,
                              double* length, int32_t* n_points, int32_t* chain);
/* check_finish for one node with the line itself (root side first, as finalize returns it);
 * *n = 0 when *ok = 0.  PP_ERR_CAPACITY when cap is too small. */
int pp_rrt_check_finish(pp_ctx* ctx, int32_t node, uint8_t* ok, double* x, double* y,
                        int64_t cap, int64_t* n, double* length);
/* RRT::optimize(node, i) (rrt.rs:463-487) for tree node `node`: *n_chain = 0 when it returns None
 * (also for i >= RECURSION_LIMIT = 16), else the depth of the returned chain: chain[l] (at most
 * 16 - i entries) is the tree node the l-th copy connects to, i.e. the returned Node sits at
 * node's coordinates with parent a copy of chain[0] at its coordinates, ..., ending at the tree
 * node chain[n - 1]; each copy's yaw is Node::new's compute_yaw toward its parent. */
int pp_rrt_optimize(pp_ctx* ctx, int32_t node, int i, int32_t* chain, int* n_chain);
/* RRT::finalize(goal) (rrt.rs:489-540) for the caller-built goal node Node::new_goal((gx, gy),
 * parent, gyaw) with `parent` a tree node: optimize_from_goal (the planner's goal yaw when
 * optimize succeeds, rrt.rs:494-498), then every edge's Dubins points, reversed.  The line is
 * returned whether or not it verifies; *verified (may be NULL) = Space::verify of it (what
 * check_finish adds).  *n = its points (cap 0 or x/y NULL: the size only); a None steer on the
 * chain returns PP_ERR_REFERENCE_PANIC (rrt.rs:529). */
int pp_rrt_finalize(pp_ctx* ctx, double gx, double gy, double gyaw, int32_t parent, double* x,
                    double* y, int64_t cap, int64_t* n, uint8_t* verified);
/* RRT::plan (rrt.rs:599-619), sequential spec: n_iter plan_one iterations (extend + check_finish
 * on every accepted node); *best_node = the node whose finish has the minimum euclidean_length
 * (first on ties, -1 when none verified); the line via pp_rrt_check_finish(best_node). */
int pp_rrt_plan(pp_ctx* ctx, int64_t n_iter, int32_t* best_node, double* best_length,
                int64_t* n_finishes);

/* ------------------------------------------------ independent query batch (BASELINE config 3) */
/* q independent planners on the context's scene — RRT::new (rrt.rs:335-355) per query with
 * start starts[3i..3i+2] (x, y, yaw), goal goals[3i..] (may be NULL), sampling stream seeds[i],
 * the shared max_iter and step_size.  Replaces any previous batch of the context. */
int pp_batch_new(pp_ctx* ctx, int q, const double* starts, const double* goals,
                 const uint64_t* seeds, int64_t max_iter, double step_size);
/* speculative iterations per query and step (a power of two <= 64; 0 = automatic: 32, halved
 * while a step would hold more than 262144 tasks, i.e. q * k > 262144).  Results do not depend on
 * it: every query's tree equals its one-at-a-time sequential run.  Applies to the current batch
 * and the next ones. */
int pp_batch_set_window(pp_ctx* ctx, int k);
/* How pp_batch_plan runs check_finish (results are identical; for A/B measurement and tests):
 * rounds = 1 (default) in steer rounds, phase A taking span0 candidate edges per
 * node in its first round and span in the later ones (0 = the default, else 1..16); rounds = 0:
 * check_finish_kernel alone, one wave per (query, node).  Applies to the context's later plans. */
int pp_batch_set_finish_schedule(pp_ctx* ctx, int rounds, int span0, int span);
/* n_steps lockstep steps: every query runs one plan_one extend iteration (rrt.rs:583-589) per
 * step until it reaches max_iter.  Totals over the batch are returned (may be NULL).  On the
 * GPU a step evaluates up to the batch window's iterations per query at once. */
int pp_batch_extend(pp_ctx* ctx, int64_t n_steps, int64_t* n_iterations, int64_t* n_accepted);
/* per-query tree sizes (q int32), consumed iterations and NN node-distance evaluations (q int64
 * each); any may be NULL.  With pp_set_profiling on, pp_batch_extend times its NN kernel with
 * HIP events into pp_stats.nn_scan_ms / nn_scan_launches. */
int pp_batch_state(pp_ctx* ctx, int32_t* n_nodes, int64_t* iterations, int64_t* node_evals);
/* RRT::plan (rrt.rs:599-619) of every query of the batch, on its tree as extended so far:
 * check_finish (rrt.rs:428-438: optimize_from_goal, finalize, verify) of every node the query
 * inserted (1 .. n_q - 1 in insertion order, rrt.rs:591) with the query's goal from
 * pp_batch_new, then the first minimum euclidean_length (rrt.rs:607-617).  Per query (q entries
 * each, any may be NULL): best_node (-1: no finish, the reference's None), length (inf when none),
 * n_points of the finalized line, n_finishes (verified check_finish lines); n_checked = the
 * (query, node) pairs checked. */
int pp_batch_plan(pp_ctx* ctx, int32_t* best_node, double* length, int32_t* n_points,
                  int32_t* n_finishes, int64_t* n_checked);
/* one query's tree (root first), like pp_rrt_tree_export */
int pp_batch_tree_export(pp_ctx* ctx, int query, double* x, double* y, double* yaw,
                         int32_t* parent, int64_t cap, int64_t* n);

/* ------------------------------------------------- RRT* query batch (BASELINE config 5) */
/* Build-defined: the reference has no RRT* (SURVEY.md §8d config 5, §8f row 4).  q independent
 * k-nearest RRT* planners (Karaman & Frazzoli) in the crate's conventions (DESIGN.md §3.7,
 * oracle/pp_oracle.c orc_star_extend): rand_point and the exact nearest node as in the extend
 * (rrt.rs:139-146, 378-391); with eta > 0 a sample farther than eta from its nearest node moves
 * onto the chord at distance eta (eta = 0: the node sits at the sample, like Node::new); the edge
 * to the nearest node (verify_node, rrt.rs:414-426) gates the insert; the parent is the first
 * strict minimum of cost(p) + Dubins cost (dubins.rs:351-361) over the nearest node and the k
 * nearest nodes of the new point; then every one of those k nodes whose edge to the new node is
 * feasible and makes it strictly cheaper is rewired (its pose kept), costs of its subtree
 * recomputed.  k = 0: ceil(2e ln n) (at most 63 and n); 1..63: fixed.  Replaces any previous RRT*
 * batch of the context. */
int pp_star_new(pp_ctx* ctx, int q, const double* starts, const uint64_t* seeds,
                int64_t max_iter, double step_size, int k, double eta);
/* n_steps lockstep steps: every query runs one RRT* iteration per step until max_iter.  Batch
 * totals (each may be NULL): iterations, inserted nodes, rewires. */
int pp_star_extend(pp_ctx* ctx, int64_t n_steps, int64_t* n_iterations, int64_t* n_accepted,
                   int64_t* n_rewires);
/* per-query tree sizes (q int32), iterations, NN node-distance evaluations and rewires (q int64
 * each); any may be NULL */
int pp_star_state(pp_ctx* ctx, int32_t* n_nodes, int64_t* iterations, int64_t* node_evals,
                  int64_t* rewires);
/* one query's tree (root first): coordinates, yaw, parent (-1 root) and node cost (root 0) */
int pp_star_tree_export(pp_ctx* ctx, int query, double* x, double* y, double* yaw,
                        int32_t* parent, double* cost, int64_t cap, int64_t* n);

int pp_rrt_get_stats(pp_ctx* ctx, pp_stats* out, uint64_t out_size);
int pp_rrt_reset_stats(pp_ctx* ctx);
/* record HIP events around the hot kernels (adds a little host overhead per window) */
int pp_set_profiling(pp_ctx* ctx, int enabled);

#ifdef __cplusplus
}
#endif

#endif /* PATHPLANNING_AMD_H */
