/*
 * pp_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of tsturzl/rs-pathplanning's RRT extend hot path (Dubins steer + nearest
 * neighbour + collision verify), used as the parity checker for the HIP product path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / the timed CPU baseline — never as the thing shipped or measured.
 *
 * Parity status: the reference is Rust and cannot be built here (no cargo/rustc, crates.io
 * deps not vendored) and it ships no golden vectors or tests.  This file is
 * therefore "parity unpinned" against the crate itself; it is pinned against (a) an independent
 * pure-Python restatement (oracle/dubins_py.py) through the committed fixtures in tests/golden/,
 * and (b) the reference-supplied known inputs of examples/dubins/src/main.rs:131-164 and
 * benches/all.rs:8-42,102-111.
 *
 * Compile with -ffp-contract=off and no fast-math: Rust never contracts a*b+c into an FMA, and
 * every expression below keeps the reference's left-to-right evaluation order.  sin/cos/atan2/
 * acos/hypot come from the platform libm, exactly as Rust's std f64 methods do on Linux.
 *
 * Build-defined deviations:
 *   Q7  seeded counter RNG (SplitMix64) in place of rand::thread_rng, same draw order (x then y)
 *       and the same [1,2)-mantissa float construction as rand 0.7's UniformFloat::sample_single;
 *   Q8  sequential spec (one rayon thread) in place of the 4-thread pool;
 *   Q9  exact brute-force NN on dx*dx+dy*dy, lowest index wins ties (rstar's pruning is inexact);
 *   Q10 obstacles are analytic discs of radius r + robot.width/2 and the bounds an axis-aligned
 *       rectangle shrunk by robot.width/2; polyline-vs-disc uses exact segment distance;
 *   Q10p polygon scenes (examples/rrt/src/main.rs:30-45): the geo-offset buffers are the exact
 *       Minkowski buffers (obstacle polygon + closed disc of radius width/2; bounds polygon eroded
 *       by it), tested on the line's segments and points (see orc_verify_line).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_PI 3.14159265358979323846 /* == std::f64::consts::PI */
#define ORC_TWO_PI (2.0 * ORC_PI)

/* ---------------------------------------------------------------- dubins.rs restatement */

/* dubins.rs:14-16 */
static double fmodr(double x, double y) { return x - y * floor(x / y); }
/* dubins.rs:18-20 */
double orc_mod2pi(double theta) { return fmodr(theta, ORC_TWO_PI); }
/* dubins.rs:22-24 — Rust `%` on f64 is C fmod (truncated); negative inputs are not wrapped. */
double orc_pi_2_pi(double angle) { return fmod(angle + ORC_PI, ORC_TWO_PI) - ORC_PI; }

enum { M_L = 0, M_S = 1, M_R = 2 };
/* word order of ALL_PLANNERS, dubins.rs:291 */
enum { W_LSL = 0, W_RSR = 1, W_LSR = 2, W_RSL = 3, W_RLR = 4, W_LRL = 5 };
static const int WORD_MODES[6][3] = {
    {M_L, M_S, M_L}, {M_R, M_S, M_R}, {M_L, M_S, M_R},
    {M_R, M_S, M_L}, {M_R, M_L, M_R}, {M_L, M_R, M_L}};

typedef struct { int ok; double t, p, q; } orc_word;

/* dubins.rs:27-48 */
static orc_word lsl(double alpha, double beta, double d) {
    orc_word w = {0, 0, 0, 0};
    double sa = sin(alpha), sb = sin(beta), ca = cos(alpha), cb = cos(beta);
    double c_ab = cos(alpha - beta);
    double tmp0 = d + sa - sb;
    double p_squared = 2.0 + (d * d) - (2.0 * c_ab) + (2.0 * d * (sa - sb));
    if (p_squared < 0.0) return w;
    double tmp1 = atan2(cb - ca, tmp0);
    w.t = orc_mod2pi(-alpha + tmp1);
    w.p = sqrt(p_squared);
    w.q = orc_mod2pi(beta - tmp1);
    w.ok = 1;
    return w;
}
/* dubins.rs:51-71 */
static orc_word rsr(double alpha, double beta, double d) {
    orc_word w = {0, 0, 0, 0};
    double sa = sin(alpha), sb = sin(beta), ca = cos(alpha), cb = cos(beta);
    double c_ab = cos(alpha - beta);
    double tmp0 = d - sa + sb;
    double p_squared = 2.0 + (d * d) - (2.0 * c_ab) + (2.0 * d * (sb - sa));
    if (p_squared < 0.0) return w;
    double tmp1 = atan2(ca - cb, tmp0);
    w.t = orc_mod2pi(alpha - tmp1);
    w.p = sqrt(p_squared);
    w.q = orc_mod2pi(-beta + tmp1);
    w.ok = 1;
    return w;
}
/* dubins.rs:74-92 */
static orc_word lsr(double alpha, double beta, double d) {
    orc_word w = {0, 0, 0, 0};
    double sa = sin(alpha), sb = sin(beta), ca = cos(alpha), cb = cos(beta);
    double c_ab = cos(alpha - beta);
    double p_squared = -2.0 + (d * d) + (2.0 * c_ab) + (2.0 * d * (sa + sb));
    if (p_squared < 0.0) return w;
    double p = sqrt(p_squared);
    double tmp = atan2(-ca - cb, d + sa + sb) - atan2(-2.0, p);
    w.t = orc_mod2pi(-alpha + tmp);
    w.p = p;
    w.q = orc_mod2pi(-orc_mod2pi(beta) + tmp);
    w.ok = 1;
    return w;
}
/* dubins.rs:95-113 */
static orc_word rsl(double alpha, double beta, double d) {
    orc_word w = {0, 0, 0, 0};
    double sa = sin(alpha), sb = sin(beta), ca = cos(alpha), cb = cos(beta);
    double c_ab = cos(alpha - beta);
    double p_squared = -2.0 + (d * d) + (2.0 * c_ab) - (2.0 * d * (sa + sb));
    if (p_squared < 0.0) return w;
    double p = sqrt(p_squared);
    double tmp = atan2(ca + cb, d - sa - sb) - atan2(2.0, p);
    w.t = orc_mod2pi(alpha - tmp);
    w.p = p;
    w.q = orc_mod2pi(beta - tmp);
    w.ok = 1;
    return w;
}
/* dubins.rs:116-133 */
static orc_word rlr(double alpha, double beta, double d) {
    orc_word w = {0, 0, 0, 0};
    double sa = sin(alpha), sb = sin(beta), ca = cos(alpha), cb = cos(beta);
    double c_ab = cos(alpha - beta);
    double tmp_rlr = (6.0 - d * d + 2.0 * c_ab + 2.0 * d * (sa - sb)) / 8.0;
    if (fabs(tmp_rlr) > 1.0) return w;
    double p = orc_mod2pi(2.0 * ORC_PI - acos(tmp_rlr));
    double t = orc_mod2pi(alpha - atan2(ca - cb, d - sa + sb) + orc_mod2pi(p / 2.0));
    double q = orc_mod2pi(alpha - beta - t + orc_mod2pi(p));
    w.t = t; w.p = p; w.q = q; w.ok = 1;
    return w;
}
/* dubins.rs:136-153 */
static orc_word lrl(double alpha, double beta, double d) {
    orc_word w = {0, 0, 0, 0};
    double sa = sin(alpha), sb = sin(beta), ca = cos(alpha), cb = cos(beta);
    double c_ab = cos(alpha - beta);
    double tmp_lrl = (6.0 - d * d + 2.0 * c_ab + 2.0 * d * (-sa + sb)) / 8.0;
    if (fabs(tmp_lrl) > 1.0) return w;
    double p = orc_mod2pi(2.0 * ORC_PI - acos(tmp_lrl));
    double t = orc_mod2pi(-alpha - atan2(ca - cb, d + sa - sb) + p / 2.0);
    double q = orc_mod2pi(orc_mod2pi(beta) - alpha - t + orc_mod2pi(p));
    w.t = t; w.p = p; w.q = q; w.ok = 1;
    return w;
}

typedef orc_word (*planner_fn)(double, double, double);
static const planner_fn ALL_PLANNERS[6] = {lsl, rsr, lsr, rsl, rlr, lrl}; /* dubins.rs:291 */

/* dubins.rs:155-198 (directions are not part of the returned path and are omitted) */
static void interpolate(int ind, double length, int mode, double max_curvature, double origin_x,
                        double origin_y, double origin_yaw, double* path_x, double* path_y,
                        double* path_yaw) {
    if (mode == M_S) {
        path_x[ind] = origin_x + length / max_curvature * cos(origin_yaw);
        path_y[ind] = origin_y + length / max_curvature * sin(origin_yaw);
        path_yaw[ind] = origin_yaw;
    } else {
        double ldx = sin(length) / max_curvature;
        double ldy = 0.0;
        if (mode == M_L)
            ldy = (1.0 - cos(length)) / max_curvature;
        else
            ldy = (1.0 - cos(length)) / -max_curvature;
        double gdx = cos(-origin_yaw) * ldx + sin(-origin_yaw) * ldy;
        double gdy = -sin(-origin_yaw) * ldx + cos(-origin_yaw) * ldy;
        path_x[ind] = origin_x + gdx;
        path_y[ind] = origin_y + gdy;
    }
    if (mode == M_L)
        path_yaw[ind] = origin_yaw + length;
    else if (mode == M_R)
        path_yaw[ind] = origin_yaw - length;
}

/* dubins.rs:200-289.  Returns the kept length after the trailing-zero trim, or -1 when an index
 * would run past n_point (Rust panics there; unreachable for finite inputs). */
static int generate_local_course(const double lengths[3], const int mode[3], double max_curvature,
                                 double step_size, double* path_x, double* path_y, double* path_yaw,
                                 int n_point) {
    int ind = 1;
    double ll = 0.0;
    for (int i = 0; i < 3; ++i) {
        int m = mode[i];
        double l = lengths[i];
        double d = (l > 0.0) ? step_size : -step_size;
        double origin_x = path_x[ind], origin_y = path_y[ind], origin_yaw = path_yaw[ind];
        ind -= 1;
        double pd;
        if (i >= 1 && (lengths[i - 1] * lengths[i]) > 0.0)
            pd = -d - ll;
        else
            pd = d - ll;
        while (fabs(pd) <= fabs(l)) {
            ind += 1;
            if (ind >= n_point) return -1;
            interpolate(ind, pd, m, max_curvature, origin_x, origin_y, origin_yaw, path_x, path_y,
                        path_yaw);
            pd += d;
        }
        ll = l - pd - d;
        ind += 1;
        if (ind >= n_point) return -1;
        interpolate(ind, l, m, max_curvature, origin_x, origin_y, origin_yaw, path_x, path_y,
                    path_yaw);
    }
    int len = n_point;
    if (len <= 1) return 0; /* dubins.rs:274-279 (then 281 would panic on the empty vec) */
    /* dubins.rs:281-288: read the last element, then pop while the value read was 0.0 —
     * this pops every trailing zero AND the first non-zero element behind them. */
    double last = path_x[len - 1];
    while (len >= 1 && last == 0.0) {
        last = path_x[len - 1];
        len -= 1;
    }
    return len;
}

/* dubins.rs:326-399.  Writes LOCAL-frame points.  Returns 1 and fills outputs on Some, 0 on None,
 * -1 on capacity overflow (cap < n_point) or the unreachable index panic. */
static int from_origin(double dx, double dy, double eyaw, double c, double step_size, double* px,
                       double* py, double* pyaw, int cap, int* n_out, int* word_out,
                       double* cost_out, double* lengths_out) {
    double hyp = hypot(dx, dy);
    double d = hyp * c;
    double theta = orc_mod2pi(atan2(dy, dx));
    double alpha = orc_mod2pi(-theta);
    double beta = orc_mod2pi(eyaw - theta);

    double bcost = INFINITY;
    int bword = -1;
    double bt = 0, bp = 0, bq = 0;
    for (int i = 0; i < 6; ++i) {
        orc_word w = ALL_PLANNERS[i](alpha, beta, d);
        if (w.ok) {
            double cost = fabs(w.t) + fabs(w.p) + fabs(w.q);
            if (bcost > cost) { /* strict: first minimum wins (dubins.rs:354) */
                bt = w.t; bp = w.p; bq = w.q; bword = i; bcost = cost;
            }
        }
    }
    if (bword < 0) return 0;
    double lengths[3] = {bt, bp, bq};
    double total_length = 0.0; /* Iterator::sum folds from 0.0 */
    for (int i = 0; i < 3; ++i) total_length += lengths[i];
    double q = trunc(total_length / step_size);
    if (!(q >= 0.0) || q > 1e9) return -1;
    int n_point = (int)q + 3 + 4;
    if (n_point > cap) return -1;
    for (int i = 0; i < n_point; ++i) px[i] = py[i] = pyaw[i] = 0.0;
    int n = generate_local_course(lengths, WORD_MODES[bword], c, step_size, px, py, pyaw, n_point);
    if (n < 0) return -1;
    *n_out = n;
    *word_out = bword;
    *cost_out = bcost;
    if (lengths_out) { lengths_out[0] = bt; lengths_out[1] = bp; lengths_out[2] = bq; }
    return 1;
}

/* Upper bound on n_point for a given configuration is not known before the word is chosen; this
 * helper returns the n_point that dubins_path_planning would allocate (0 on None). */
int orc_dubins_n_point(const double conf[8]) {
    double sx = conf[0], sy = conf[1], syaw = conf[2], ex0 = conf[3], ey0 = conf[4], eyaw = conf[5];
    double R = conf[6], step = conf[7];
    double ex = ex0 - sx, ey = ey0 - sy, c = 1.0 / R;
    double lex = cos(syaw) * ex + sin(syaw) * ey;
    double ley = -(sin(syaw)) * ex + cos(syaw) * ey;
    double leyaw = eyaw - syaw;
    double hyp = hypot(lex, ley), d = hyp * c;
    double theta = orc_mod2pi(atan2(ley, lex));
    double alpha = orc_mod2pi(-theta), beta = orc_mod2pi(leyaw - theta);
    double bcost = INFINITY, tot = 0;
    int bword = -1;
    for (int i = 0; i < 6; ++i) {
        orc_word w = ALL_PLANNERS[i](alpha, beta, d);
        if (w.ok) {
            double cost = fabs(w.t) + fabs(w.p) + fabs(w.q);
            if (bcost > cost) { bcost = cost; bword = i; tot = ((0.0 + w.t) + w.p) + w.q; }
        }
    }
    if (bword < 0) return 0;
    return (int)trunc(tot / step) + 7;
}

/* dubins.rs:401-428.  conf = {sx, sy, syaw, ex, ey, eyaw, turn_radius, step_size}
 * (DubinsConfig, dubins.rs:315-324).  Returns 1 (Some), 0 (None) or -1 (cap too small). */
int orc_dubins(const double conf[8], double* px, double* py, double* pyaw, int cap, int* n,
               int* word, double* cost) {
    double sx = conf[0], sy = conf[1], syaw = conf[2], ex0 = conf[3], ey0 = conf[4], eyaw = conf[5];
    double turn_radius = conf[6], step_size = conf[7];
    double ex = ex0 - sx;
    double ey = ey0 - sy;
    double c = 1.0 / turn_radius;
    double lex = cos(syaw) * ex + sin(syaw) * ey;
    double ley = -(sin(syaw)) * ex + cos(syaw) * ey;
    double leyaw = eyaw - syaw;
    int r = from_origin(lex, ley, leyaw, c, step_size, px, py, pyaw, cap, n, word, cost, NULL);
    if (r != 1) return r;
    double cs = cos(-syaw), sn = sin(-syaw);
    for (int i = 0; i < *n; ++i) {
        double x = px[i], y = py[i];
        px[i] = cs * x + sn * y + sx;
        py[i] = -sn * x + cs * y + sy;
        pyaw[i] = orc_pi_2_pi(pyaw[i] + syaw);
    }
    return 1;
}

/* ------------------------------------------------------------------ seeded sampling (Q7) */

/* SplitMix64 output number `ctr` of the stream seeded with `seed`. */
uint64_t orc_rng_u64(uint64_t seed, uint64_t ctr) {
    uint64_t z = seed + (ctr + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* rand 0.7 UniformFloat<f64>::sample_single structure: 52 random mantissa bits under exponent 0
 * give [1,2); minus 1; times scale; plus low.  The (measure-zero) res >= high case narrows the
 * scale by one ulp and retries with the same bits instead of drawing again. */
double orc_gen_range(uint64_t seed, uint64_t ctr, double low, double high) {
    uint64_t bits = (orc_rng_u64(seed, ctr) >> 12) | 0x3FF0000000000000ULL;
    double value1_2;
    memcpy(&value1_2, &bits, sizeof value1_2);
    double value0_1 = value1_2 - 1.0;
    double scale = high - low;
    for (;;) {
        double res = value0_1 * scale + low;
        if (res < high) return res;
        scale = nextafter(scale, 0.0);
    }
}

/* ------------------------------------------------------------------------ scene (Q10) */

typedef struct {
    double minx, maxx, miny, maxy; /* bbox of the shrunken bounds (rrt.rs:82-106) */
    int m;                         /* obstacle discs */
    const double* cx;
    const double* cy;
    const double* r2; /* (r + width/2)^2 */
    double turn_radius;  /* Robot.max_steer (rrt.rs:37-39 → 424) */
    double step_size;
    /* config 4 occupancy grid (build-defined): when bits != NULL the discs are
     * ignored and every point of a line must lie in a free cell */
    const uint32_t* bits;
    int bw, bh, bwords;
    double bx0, by0, binv;
    /* polygon mode (pp_space_new_polygons; build-defined Q10p, see orc_verify_line): the bounds
     * polygon ring (nbv vertices, no closing repeat; 0 = the rectangle above only) and the
     * obstacle polygons as ne edges (ex0, ey0)-(ex1, ey1), the edges of one polygon consecutive
     * with their polygon id in epoly; h2 = (width/2)^2.  ne > 0 replaces the discs. */
    int nbv;
    const double* bvx;
    const double* bvy;
    int ne;
    const double* ex0;
    const double* ey0;
    const double* ex1;
    const double* ey1;
    const int* epoly;
    double h2;
} orc_scene;

typedef struct {
    double* x;
    double* y;
    double* yaw;
    int32_t* parent;
    int cap;
    int n;
} orc_tree;

/* squared distance from (cx, cy) to the closed segment a-b: exact closest point on the segment */
static double seg_point_d2(double ax, double ay, double bx, double by, double cx, double cy) {
    double vx = bx - ax, vy = by - ay;
    double wx = cx - ax, wy = cy - ay;
    double l2 = vx * vx + vy * vy;
    double t = 0.0;
    if (l2 > 0.0) {
        t = (wx * vx + wy * vy) / l2;
        if (t < 0.0) t = 0.0;
        else if (t > 1.0) t = 1.0;
    }
    double ex = wx - t * vx, ey = wy - t * vy;
    return ex * ex + ey * ey;
}

/* polyline segment vs closed disc */
static int seg_hits_disc(double ax, double ay, double bx, double by, double cx, double cy,
                         double r2) {
    return seg_point_d2(ax, ay, bx, by, cx, cy) <= r2;
}

/* ---- polygon mode (Q10p): geo's Contains / Intersects on geo-offset buffers (rrt.rs:62-68,
 * 82, 108-111, 124-137) restated as the exact Minkowski buffers of the polygons: an obstacle
 * grows by the closed disc of radius h = width/2, the bounds shrink to the points whose disc of
 * radius h stays inside.  geo-offset's arc approximation is not reproduced (parity unpinned,
 * SURVEY.md §8c). */

/* crossing-number step: the edge (xi, yi)-(xj, yj) crosses the ray from (px, py) toward +x
 * (half-open in y, the classic even-odd rule) */
static int ray_crosses(double px, double py, double xi, double yi, double xj, double yj) {
    return ((yi > py) != (yj > py)) && (px < (xj - xi) * (py - yi) / (yj - yi) + xi);
}

/* the point lies in the shrunken bounds polygon: inside the ring (even-odd) and at distance >= h
 * from every bounds edge */
static int in_poly_bounds(const orc_scene* sc, double x, double y) {
    int inside = 0;
    for (int i = 0; i < sc->nbv; ++i) {
        const int j = i + 1 == sc->nbv ? 0 : i + 1;
        const double xi = sc->bvx[i], yi = sc->bvy[i], xj = sc->bvx[j], yj = sc->bvy[j];
        if (ray_crosses(x, y, xi, yi, xj, yj)) inside ^= 1;
        if (seg_point_d2(xi, yi, xj, yj, x, y) < sc->h2) return 0;
    }
    return inside;
}

/* polyline segment a-b vs the buffer of one obstacle edge e0-e1: the segments cross properly,
 * or an endpoint of one lies within h of the other (touching counts: <= h^2) */
static int seg_hits_edge(double ax, double ay, double bx, double by, double e0x, double e0y,
                         double e1x, double e1y, double h2) {
    const double d1 = (e1x - e0x) * (ay - e0y) - (e1y - e0y) * (ax - e0x);
    const double d2 = (e1x - e0x) * (by - e0y) - (e1y - e0y) * (bx - e0x);
    const double d3 = (bx - ax) * (e0y - ay) - (by - ay) * (e0x - ax);
    const double d4 = (bx - ax) * (e1y - ay) - (by - ay) * (e1x - ax);
    if (((d1 > 0.0 && d2 < 0.0) || (d1 < 0.0 && d2 > 0.0)) &&
        ((d3 > 0.0 && d4 < 0.0) || (d3 < 0.0 && d4 > 0.0)))
        return 1;
    return seg_point_d2(e0x, e0y, e1x, e1y, ax, ay) <= h2 ||
           seg_point_d2(e0x, e0y, e1x, e1y, bx, by) <= h2 ||
           seg_point_d2(ax, ay, bx, by, e0x, e0y) <= h2 ||
           seg_point_d2(ax, ay, bx, by, e1x, e1y) <= h2;
}

/* the point lies inside some obstacle polygon (even-odd over each polygon's edges) */
static int in_obstacle(const orc_scene* sc, double x, double y) {
    int inside = 0;
    for (int k = 0; k < sc->ne; ++k) {
        if (k > 0 && sc->epoly[k] != sc->epoly[k - 1]) {
            if (inside) return 1;
            inside = 0;
        }
        if (ray_crosses(x, y, sc->ex0[k], sc->ey0[k], sc->ex1[k], sc->ey1[k])) inside ^= 1;
    }
    return inside;
}

static int in_bounds(const orc_scene* sc, double x, double y) {
    if (!(x >= sc->minx && x <= sc->maxx && y >= sc->miny && y <= sc->maxy)) return 0;
    return sc->nbv == 0 || in_poly_bounds(sc, x, y);
}

/* config 4 probe: cell (floor((x - x0) * inv), floor((y - y0) * inv)); outside = occupied */
static int grid_occupied(const orc_scene* sc, double x, double y) {
    double fx = floor((x - sc->bx0) * sc->binv), fy = floor((y - sc->by0) * sc->binv);
    if (!(fx >= 0.0) || !(fy >= 0.0) || fx >= (double)sc->bw || fy >= (double)sc->bh) return 1;
    int i = (int)fx, j = (int)fy;
    return (int)((sc->bits[(size_t)j * sc->bwords + (i >> 5)] >> (i & 31)) & 1u);
}

/* Space::verify, rrt.rs:124-137: bounds.contains(line) && no obstacle intersects the line.
 * A one-point line is tested as a point (degenerate segment).  With an occupancy grid: every
 * point in bounds and in a free cell.  Polygon mode (Q10p): every point in the bounds rectangle
 * and in the eroded bounds polygon (geo's Contains<LineString> tests the points against the
 * exterior), no segment within h of an obstacle edge or crossing it, and point 0 outside every
 * obstacle polygon (with no segment meeting an edge buffer the whole line is on one side). */
int orc_verify_line(const orc_scene* sc, const double* x, const double* y, int n) {
    if (n <= 0) return 1;
    for (int i = 0; i < n; ++i)
        if (!in_bounds(sc, x[i], y[i])) return 0;
    if (sc->bits) {
        for (int i = 0; i < n; ++i)
            if (grid_occupied(sc, x[i], y[i])) return 0;
        return 1;
    }
    if (sc->ne > 0) { /* polygon obstacles: every segment vs every edge buffer, then one point
                       * inside test (no segment meets a buffer: the line is on one side) */
        /* exact cull (speed only): an edge whose h-widened bbox misses the line's bbox is beyond
         * h of every segment (the widening is rounded up) */
        double lx0 = x[0], lx1 = x[0], ly0 = y[0], ly1 = y[0];
        for (int i = 1; i < n; ++i) {
            lx0 = fmin(lx0, x[i]); lx1 = fmax(lx1, x[i]);
            ly0 = fmin(ly0, y[i]); ly1 = fmax(ly1, y[i]);
        }
        const double hm = sqrt(sc->h2) * (1.0 + 1e-9) + 1e-9;
        for (int k = 0; k < sc->ne; ++k) {
            const double e0x = sc->ex0[k], e0y = sc->ey0[k], e1x = sc->ex1[k], e1y = sc->ey1[k];
            if (fmax(e0x, e1x) + hm < lx0 || fmin(e0x, e1x) - hm > lx1 ||
                fmax(e0y, e1y) + hm < ly0 || fmin(e0y, e1y) - hm > ly1)
                continue;
            if (n == 1 && seg_hits_edge(x[0], y[0], x[0], y[0], e0x, e0y, e1x, e1y, sc->h2))
                return 0;
            for (int i = 0; i + 1 < n; ++i)
                if (seg_hits_edge(x[i], y[i], x[i + 1], y[i + 1], e0x, e0y, e1x, e1y, sc->h2))
                    return 0;
        }
        return !in_obstacle(sc, x[0], y[0]);
    }
    if (n == 1) {
        for (int k = 0; k < sc->m; ++k)
            if (seg_hits_disc(x[0], y[0], x[0], y[0], sc->cx[k], sc->cy[k], sc->r2[k])) return 0;
        return 1;
    }
    /* exact cull (speed only): a disc whose centre lies farther than its radius (rounded up)
     * from the line's bbox is farther from every segment */
    double lx0 = x[0], lx1 = x[0], ly0 = y[0], ly1 = y[0];
    for (int i = 1; i < n; ++i) {
        lx0 = fmin(lx0, x[i]); lx1 = fmax(lx1, x[i]);
        ly0 = fmin(ly0, y[i]); ly1 = fmax(ly1, y[i]);
    }
    for (int k = 0; k < sc->m; ++k) {
        const double cx = sc->cx[k], cy = sc->cy[k];
        const double dx = fmax(fmax(lx0 - cx, cx - lx1), 0.0);
        const double dy = fmax(fmax(ly0 - cy, cy - ly1), 0.0);
        if (dx * dx + dy * dy > sc->r2[k] * (1.0 + 1e-9) + 1e-9) continue;
        for (int i = 0; i + 1 < n; ++i)
            if (seg_hits_disc(x[i], y[i], x[i + 1], y[i + 1], cx, cy, sc->r2[k]))
                return 0;
    }
    return 1;
}

/* exact brute-force NN (Q9): argmin dx*dx+dy*dy, lowest index wins ties */
int orc_nearest(const double* X, const double* Y, int n, double qx, double qy, double* d2_out) {
    int best = -1;
    double bd = INFINITY;
    for (int i = 0; i < n; ++i) {
        double dx = qx - X[i], dy = qy - Y[i];
        double d2 = dx * dx + dy * dy;
        if (d2 < bd) { bd = d2; best = i; }
    }
    if (d2_out) *d2_out = bd;
    return best;
}

/* compute_yaw, rrt.rs:267-271 */
static double compute_yaw(double fx, double fy, double tx, double ty) {
    return atan2(ty - fy, tx - fx);
}

/* growable point buffer for line building */
typedef struct { double* x; double* y; int n, cap; } pbuf;
static int pbuf_push(pbuf* b, double x, double y) {
    if (b->n == b->cap) {
        int nc = b->cap ? 2 * b->cap : 1024;
        double* nx = (double*)realloc(b->x, sizeof(double) * nc);
        double* ny = (double*)realloc(b->y, sizeof(double) * nc);
        if (!nx || !ny) { free(nx); free(ny); return -1; }
        b->x = nx; b->y = ny; b->cap = nc;
    }
    b->x[b->n] = x; b->y[b->n] = y; b->n++;
    return 0;
}

/* scratch for one Dubins segment */
typedef struct { double* px; double* py; double* pyaw; int cap; } dscratch;
static int dscratch_fit(dscratch* s, int need) {
    if (need <= s->cap) return 0;
    int nc = need + 1024;
    double* a = (double*)realloc(s->px, sizeof(double) * nc);
    double* b = (double*)realloc(s->py, sizeof(double) * nc);
    double* c = (double*)realloc(s->pyaw, sizeof(double) * nc);
    if (!a || !b || !c) return -1;
    s->px = a; s->py = b; s->pyaw = c; s->cap = nc;
    return 0;
}

/* one edge of line_to_origin (rrt.rs:295-315): the Dubins polyline child→parent, or [(sx,sy)]
 * when the steer fails.  Appends to `b`. */
static int push_edge(pbuf* b, dscratch* s, double sx, double sy, double syaw, double ex, double ey,
                     double eyaw, double R, double step) {
    double conf[8] = {sx, sy, syaw, ex, ey, eyaw, R, step};
    int need = orc_dubins_n_point(conf);
    if (need > 0 && dscratch_fit(s, need) != 0) return -1;
    int n = 0, word = -1;
    double cost = 0;
    int r = (need > 0) ? orc_dubins(conf, s->px, s->py, s->pyaw, s->cap, &n, &word, &cost) : 0;
    if (r < 0) return -1;
    if (r == 0) return pbuf_push(b, sx, sy);
    for (int i = 0; i < n; ++i)
        if (pbuf_push(b, s->px[i], s->py[i])) return -1;
    return 0;
}

/* RRT::verify_node(Node::new(sample, tree[p])) — rrt.rs:169-175, 414-426.
 * full_reverify=1 builds the whole line_to_origin (rrt.rs:291-321) like the reference; 0 verifies
 * edge(new→p) ++ [p] only (the ancestors' part was verified at their insert). */
static int verify_candidate(const orc_scene* sc, const orc_tree* tr, double x, double y, double yaw,
                            int p, int full_reverify, pbuf* b, dscratch* s) {
    b->n = 0;
    double R = sc->turn_radius, step = sc->step_size;
    if (push_edge(b, s, x, y, yaw, tr->x[p], tr->y[p], tr->yaw[p], R, step)) return -1;
    int cur = p;
    if (!full_reverify) {
        if (pbuf_push(b, tr->x[cur], tr->y[cur])) return -1;
    } else {
        for (;;) {
            int pp = tr->parent[cur];
            if (pp < 0) {
                if (pbuf_push(b, tr->x[cur], tr->y[cur])) return -1;
                break;
            }
            if (push_edge(b, s, tr->x[cur], tr->y[cur], tr->yaw[cur], tr->x[pp], tr->y[pp],
                          tr->yaw[pp], R, step))
                return -1;
            cur = pp;
        }
    }
    return orc_verify_line(sc, b->x, b->y, b->n);
}

/* Sequential spec of RRT::plan_one's extend (rrt.rs:583-589) for iterations [it0, it0+n_iter):
 * rand_point (x then y) → exact NN → Node::new → verify_node → insert.  check_finish is a
 * separate row.  Per-iteration logs: nearest index and accepted flag.
 * Returns the number of accepted nodes, or -1 (allocation / capacity failure). */
/* One iteration of plan_one's extend on the sample (x, y): exact NN → Node::new → verify_node →
 * insert (rrt.rs:583-589).  Returns 1 inserted, 0 rejected, -1 allocation / capacity failure;
 * *nn / *yaw_out: the nearest node and the new node's yaw (compute_yaw toward it). */
static int extend_one(const orc_scene* sc, orc_tree* tr, double x, double y, int full_reverify,
                      pbuf* b, dscratch* s, int* nn, double* yaw_out) {
    int p = orc_nearest(tr->x, tr->y, tr->n, x, y, NULL);
    *nn = p;
    *yaw_out = 0.0;
    if (p < 0) return 0;
    double yaw = compute_yaw(x, y, tr->x[p], tr->y[p]);
    *yaw_out = yaw;
    int ok = verify_candidate(sc, tr, x, y, yaw, p, full_reverify, b, s);
    if (ok <= 0) return ok;
    if (tr->n >= tr->cap) return -1;
    tr->x[tr->n] = x; tr->y[tr->n] = y; tr->yaw[tr->n] = yaw; tr->parent[tr->n] = p;
    tr->n++;
    return 1;
}

int64_t orc_rrt_extend(const orc_scene* sc, orc_tree* tr, uint64_t seed, int64_t it0,
                       int64_t n_iter, int full_reverify, int32_t* log_nn, int8_t* log_acc) {
    pbuf b = {0};
    dscratch s = {0};
    int64_t acc = 0;
    for (int64_t k = 0; k < n_iter; ++k) {
        uint64_t it = (uint64_t)(it0 + k);
        /* Space::rand_point, rrt.rs:139-146 (Q7: x = draw 2 it, y = draw 2 it + 1) */
        double x = orc_gen_range(seed, 2 * it, sc->minx, sc->maxx);
        double y = orc_gen_range(seed, 2 * it + 1, sc->miny, sc->maxy);
        int p;
        double yaw;
        int ok = extend_one(sc, tr, x, y, full_reverify, &b, &s, &p, &yaw);
        if (log_nn) log_nn[k] = p;
        if (ok < 0) { acc = -1; break; }
        acc += ok;
        if (log_acc) log_acc[k] = (int8_t)ok;
    }
    free(b.x); free(b.y);
    free(s.px); free(s.py); free(s.pyaw);
    return acc;
}

/* The same extend over caller-drawn samples (the host owns the RNG: pp_rrt_extend_samples):
 * iteration k takes (sx[k], sy[k]) as its rand_point.  Logs per sample: nearest node, yaw (the
 * node Node::new would build), inserted flag.  Returns the inserts, or -1. */
int64_t orc_rrt_extend_samples(const orc_scene* sc, orc_tree* tr, const double* sx,
                               const double* sy, int64_t n, int full_reverify, int32_t* log_nn,
                               double* log_yaw, int8_t* log_acc) {
    pbuf b = {0};
    dscratch s = {0};
    int64_t acc = 0;
    for (int64_t k = 0; k < n; ++k) {
        int p;
        double yaw;
        int ok = extend_one(sc, tr, sx[k], sy[k], full_reverify, &b, &s, &p, &yaw);
        if (ok < 0) { acc = -1; break; }
        acc += ok;
        if (log_nn) log_nn[k] = p;
        if (log_yaw) log_yaw[k] = yaw;
        if (log_acc) log_acc[k] = (int8_t)ok;
    }
    free(b.x); free(b.y);
    free(s.px); free(s.py); free(s.pyaw);
    return acc;
}

/* verify a single candidate against the tree (for per-candidate parity checks) */
int orc_verify_candidate(const orc_scene* sc, const orc_tree* tr, double x, double y, int p,
                         int full_reverify, double* yaw_out) {
    pbuf b = {0};
    dscratch s = {0};
    double yaw = compute_yaw(x, y, tr->x[p], tr->y[p]);
    if (yaw_out) *yaw_out = yaw;
    int ok = verify_candidate(sc, tr, x, y, yaw, p, full_reverify, &b, &s);
    free(b.x); free(b.y);
    free(s.px); free(s.py); free(s.pyaw);
    return ok;
}

/* ---------------------------------------- check_finish / optimize / finalize / plan (§8f) */
/* Node pool: ids [0, tr->n) are tree nodes, ids >= tr->n are the nodes optimize and
 * check_finish create (Node::new / Node::new_goal, rrt.rs:169-187), never inserted in the tree. */
typedef struct { double x, y, yaw; int parent; } orc_pnode;
typedef struct {
    const orc_scene* sc;
    const orc_tree* tr;
    int full_reverify;
    orc_pnode* v;
    int n, cap;
    pbuf b;
    dscratch s;
    int* chain;     /* optimize's chosen `to` per level (diagnostics) */
    int n_chain;
} orc_cf;

static double P_x(const orc_cf* C, int i) { return i < C->tr->n ? C->tr->x[i] : C->v[i - C->tr->n].x; }
static double P_y(const orc_cf* C, int i) { return i < C->tr->n ? C->tr->y[i] : C->v[i - C->tr->n].y; }
static double P_yaw(const orc_cf* C, int i) { return i < C->tr->n ? C->tr->yaw[i] : C->v[i - C->tr->n].yaw; }
static int P_par(const orc_cf* C, int i) { return i < C->tr->n ? C->tr->parent[i] : C->v[i - C->tr->n].parent; }

static int pool_new(orc_cf* C, double x, double y, double yaw, int parent) {
    if (C->n == C->cap) {
        int nc = C->cap ? 2 * C->cap : 64;
        orc_pnode* nv = (orc_pnode*)realloc(C->v, sizeof(orc_pnode) * nc);
        if (!nv) return -1;
        C->v = nv;
        C->cap = nc;
    }
    C->v[C->n] = (orc_pnode){x, y, yaw, parent};
    return C->tr->n + C->n++;
}

enum { ORC_NONE = -1, ORC_FAIL = -2, ORC_PANIC = -3 };

/* RRT::optimize, rrt.rs:463-487.  `node` is always a tree node here (optimize_from_goal passes the
 * goal's parent; the recursion passes ancestors from NodeIter).  The candidate line is
 * line_to_origin(Node::new(node, to)) (rrt.rs:476-477) — verified in full or as edge ++ [to]
 * (`to` is a tree node whose own line passed verify at its insert). */
static int optimize(orc_cf* C, int node, int i) {
    if (i >= 16) return ORC_NONE; /* RECURSION_LIMIT, rrt.rs:14 */
    int len = 0;
    for (int c = node; c >= 0; c = C->tr->parent[c]) len++;
    int* nodes = (int*)malloc(sizeof(int) * (size_t)len);
    if (!nodes) return ORC_FAIL;
    len = 0;
    for (int c = node; c >= 0; c = C->tr->parent[c]) nodes[len++] = c;
    int res = ORC_NONE;
    const double nx = C->tr->x[node], ny = C->tr->y[node];
    for (int k = len - 1; k >= 0; --k) { /* nodes_vec.into_iter().rev(): root first */
        const int to = nodes[k];
        const double yaw = compute_yaw(nx, ny, C->tr->x[to], C->tr->y[to]);
        int ok = verify_candidate(C->sc, C->tr, nx, ny, yaw, to, C->full_reverify, &C->b, &C->s);
        if (ok < 0) { res = ORC_FAIL; break; }
        if (!ok) continue;
        if (C->chain) C->chain[i] = to;
        if (C->n_chain < i + 1) C->n_chain = i + 1;
        int r = optimize(C, to, i + 1);
        if (r == ORC_FAIL) { res = ORC_FAIL; break; }
        if (r >= 0) /* Node::new(node, to') — yaw toward to' (at to's coordinates) */
            res = pool_new(C, nx, ny, compute_yaw(nx, ny, P_x(C, r), P_y(C, r)), r);
        else
            res = pool_new(C, nx, ny, yaw, to);
        if (res < 0) res = ORC_FAIL;
        break;
    }
    free(nodes);
    return res;
}

/* RRT::finalize, rrt.rs:503-540: NodeIter from the (optimised) goal, each node with a parent
 * contributes its Dubins points node→parent (None panics, rrt.rs:529), the root nothing; the
 * concatenation is reversed.  Writes into C->b. */
static int finalize_line(orc_cf* C, int goal) {
    pbuf tmp = {0};
    const double R = C->sc->turn_radius, step = C->sc->step_size;
    int rc = 0;
    for (int cur = goal; cur >= 0; cur = P_par(C, cur)) {
        const int par = P_par(C, cur);
        if (par < 0) break;
        double conf[8] = {P_x(C, cur), P_y(C, cur), P_yaw(C, cur), P_x(C, par), P_y(C, par),
                          P_yaw(C, par), R, step};
        int need = orc_dubins_n_point(conf);
        if (need <= 0) { rc = ORC_PANIC; break; }
        if (dscratch_fit(&C->s, need)) { rc = ORC_FAIL; break; }
        int n = 0, word = -1;
        double cost = 0;
        int r = orc_dubins(conf, C->s.px, C->s.py, C->s.pyaw, C->s.cap, &n, &word, &cost);
        if (r < 0) { rc = ORC_FAIL; break; }
        if (r == 0) { rc = ORC_PANIC; break; }
        for (int i = 0; i < n; ++i)
            if (pbuf_push(&tmp, C->s.px[i], C->s.py[i])) { rc = ORC_FAIL; break; }
        if (rc) break;
    }
    C->b.n = 0;
    if (!rc)
        for (int i = tmp.n - 1; i >= 0; --i) /* l.reverse(), rrt.rs:538 */
            if (pbuf_push(&C->b, tmp.x[i], tmp.y[i])) { rc = ORC_FAIL; break; }
    free(tmp.x);
    free(tmp.y);
    return rc;
}

/* geo 0.12 EuclideanLength for LineString: sum over consecutive points of hypot(dx, dy), in
 * line order (third-party arithmetic: parity unpinned). */
double orc_line_length(const double* x, const double* y, int n) {
    double s = 0.0;
    for (int i = 0; i + 1 < n; ++i) s += hypot(x[i + 1] - x[i], y[i + 1] - y[i]);
    return s;
}

/* RRT::check_finish, rrt.rs:428-438, for tree node `node`.  Returns 1 (Some: the line in
 * out_x/out_y, *n_out points, *len_out its euclidean_length), 0 (None), -1 (allocation or
 * capacity failure), -3 (finalize would panic).  chain_out (optional, 16 entries) receives
 * optimize's chosen `to` for each successful level, *n_chain their count. */
int orc_check_finish(const orc_scene* sc, const orc_tree* tr, int node, double gx, double gy,
                     double gyaw, int full_reverify, double* out_x, double* out_y, int cap,
                     int* n_out, double* len_out, int* chain_out, int* n_chain) {
    orc_cf C = {0};
    C.sc = sc;
    C.tr = tr;
    C.full_reverify = full_reverify;
    C.chain = chain_out;
    int rc;
    /* optimize_from_goal, rrt.rs:489-501 */
    int goal;
    int opt = optimize(&C, node, 0);
    if (opt == ORC_FAIL) { rc = -1; goto done; }
    goal = pool_new(&C, gx, gy, gyaw, opt >= 0 ? opt : node);
    if (goal < 0) { rc = -1; goto done; }
    rc = finalize_line(&C, goal);
    if (rc == ORC_FAIL) { rc = -1; goto done; }
    if (rc == ORC_PANIC) { rc = -3; goto done; }
    rc = orc_verify_line(sc, C.b.x, C.b.y, C.b.n) ? 1 : 0;
    if (n_out) *n_out = C.b.n;
    if (len_out) *len_out = orc_line_length(C.b.x, C.b.y, C.b.n);
    if (out_x && out_y) {
        if (C.b.n > cap) { rc = -1; goto done; }
        memcpy(out_x, C.b.x, sizeof(double) * (size_t)C.b.n);
        memcpy(out_y, C.b.y, sizeof(double) * (size_t)C.b.n);
    }
done:
    if (n_chain) *n_chain = C.n_chain;
    free(C.v);
    free(C.b.x); free(C.b.y);
    free(C.s.px); free(C.s.py); free(C.s.pyaw);
    return rc;
}

/* RRT::plan, rrt.rs:599-619, sequential spec: iterations [it0, it0+n_iter) of
 * plan_one (extend + check_finish on every accepted node); the answer is the first finish with
 * the minimum euclidean_length.  *best_node = -1 when no finish verified.  Returns accepted
 * nodes, or -1 / -3 like orc_check_finish. */
int64_t orc_plan(const orc_scene* sc, orc_tree* tr, uint64_t seed, int64_t it0, int64_t n_iter,
                 double gx, double gy, double gyaw, int full_reverify, int* best_node,
                 double* best_len, int32_t* finish_ok) {
    int64_t acc = 0;
    *best_node = -1;
    *best_len = INFINITY;
    for (int64_t k = 0; k < n_iter; ++k) {
        int n0 = tr->n;
        int64_t a = orc_rrt_extend(sc, tr, seed, it0 + k, 1, full_reverify, NULL, NULL);
        if (a < 0) return -1;
        if (finish_ok) finish_ok[k] = -1;
        if (a == 0) continue;
        acc += a;
        double len = 0;
        int r = orc_check_finish(sc, tr, n0, gx, gy, gyaw, full_reverify, NULL, NULL, 0, NULL, &len,
                                 NULL, NULL);
        if (r < 0) return r;
        if (finish_ok) finish_ok[k] = r;
        if (r == 1 && len < *best_len) { /* min_by keeps the first of equal minima */
            *best_len = len;
            *best_node = n0;
        }
    }
    return acc;
}

/* ------------------------------------------- multi-core CPU baseline (bench.py cpu_baseline) */
/* Independent sequential planners on T host threads (pthreads): the CPU analogue of the GPU
 * bench's parallelism.  Every job is one orc_rrt_extend run on its own tree, so results equal the
 * single-thread runs job by job; only the throughput is measured. */
typedef struct {
    const orc_scene* sc;
    const orc_tree* base;      /* replicas: the tree every job continues (copied) */
    const double* starts;      /* queries: 3 per job (x, y, yaw) */
    const uint64_t* seeds;     /* per job */
    int64_t it0, n_iter;
    int full_reverify;
    int n_jobs;
    int next;                  /* job counter (mutex) */
    pthread_mutex_t mu;
    int64_t accepted;
    int failed;
} orc_pool;

static void* pool_worker(void* arg) {
    orc_pool* P = (orc_pool*)arg;
    for (;;) {
        pthread_mutex_lock(&P->mu);
        const int j = P->next < P->n_jobs ? P->next++ : -1;
        pthread_mutex_unlock(&P->mu);
        if (j < 0) break;
        const int n0 = P->base ? P->base->n : 1;
        const int cap = n0 + (int)P->n_iter + 1;
        orc_tree t;
        t.x = (double*)malloc(sizeof(double) * (size_t)cap);
        t.y = (double*)malloc(sizeof(double) * (size_t)cap);
        t.yaw = (double*)malloc(sizeof(double) * (size_t)cap);
        t.parent = (int32_t*)malloc(sizeof(int32_t) * (size_t)cap);
        t.cap = cap;
        int64_t a = -1;
        if (t.x && t.y && t.yaw && t.parent) {
            if (P->base) {
                memcpy(t.x, P->base->x, sizeof(double) * (size_t)n0);
                memcpy(t.y, P->base->y, sizeof(double) * (size_t)n0);
                memcpy(t.yaw, P->base->yaw, sizeof(double) * (size_t)n0);
                memcpy(t.parent, P->base->parent, sizeof(int32_t) * (size_t)n0);
            } else {
                t.x[0] = P->starts[3 * j];
                t.y[0] = P->starts[3 * j + 1];
                t.yaw[0] = P->starts[3 * j + 2];
                t.parent[0] = -1;
            }
            t.n = n0;
            a = orc_rrt_extend(P->sc, &t, P->seeds[j], P->it0, P->n_iter, P->full_reverify, NULL,
                               NULL);
        }
        free(t.x); free(t.y); free(t.yaw); free(t.parent);
        pthread_mutex_lock(&P->mu);
        if (a < 0) P->failed = 1;
        else P->accepted += a;
        pthread_mutex_unlock(&P->mu);
    }
    return NULL;
}

static int64_t run_pool(orc_pool* P, int threads) {
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    if (!th) return -1;
    pthread_mutex_init(&P->mu, NULL);
    int started = 0;
    for (int i = 0; i < threads; ++i)
        if (pthread_create(&th[i], NULL, pool_worker, P) == 0) started++;
    if (started == 0) pool_worker(P);
    for (int i = 0; i < started; ++i) pthread_join(th[i], NULL);
    pthread_mutex_destroy(&P->mu);
    free(th);
    return P->failed ? -1 : P->accepted;
}

/* n_rep replicas of `base`, replica r continuing iterations [it0, it0+n_iter) with seeds[r] */
int64_t orc_extend_replicas(const orc_scene* sc, const orc_tree* base, const uint64_t* seeds,
                            int n_rep, int64_t it0, int64_t n_iter, int full_reverify, int threads) {
    orc_pool P;
    memset(&P, 0, sizeof P);
    P.sc = sc; P.base = base; P.seeds = seeds; P.it0 = it0; P.n_iter = n_iter;
    P.full_reverify = full_reverify; P.n_jobs = n_rep;
    return run_pool(&P, threads);
}

/* n_q independent queries (RRT::new at starts[3q..], seeds[q]), max_iter iterations each */
int64_t orc_queries(const orc_scene* sc, const double* starts, const uint64_t* seeds, int n_q,
                    int64_t max_iter, int full_reverify, int threads) {
    orc_pool P;
    memset(&P, 0, sizeof P);
    P.sc = sc; P.starts = starts; P.seeds = seeds; P.n_iter = max_iter;
    P.full_reverify = full_reverify; P.n_jobs = n_q;
    return run_pool(&P, threads);
}

/* ------------------------------------------------ RRT* (BASELINE config 5, build-defined) */
/* The reference has no RRT* (SURVEY.md §8d config 5, §8f row 4): this is the build's own spec,
 * k-nearest RRT* (Karaman & Frazzoli 2011, Alg. 6) in the crate's conventions, parity
 * "unpinned" against any reference and pinned against oracle/rrtstar_py.py instead.
 *   - sample and exact NN exactly as the extend (rrt.rs:139-146, 378-391); with eta > 0 a
 *     sample farther than eta from its nearest node x_nearest moves to x_nearest + (sample -
 *     x_nearest) * (eta / |sample - x_nearest|) (Steer; eta = 0 keeps the crate's node-at-the-
 *     sample, Q5); the edge new → x_nearest (Node::new, verify_node: rrt.rs:169-175, 414-426)
 *     gates the insert;
 *   - an edge is feasible when its Dubins steer is Some and verify(edge ++ [parent]) holds (the
 *     incremental verify of SURVEY.md §3.2; a None steer is infeasible here);
 *   - edge cost = the crate's Dubins cost (dubins.rs:351-361, |t|+|p|+|q| of the chosen word);
 *     node cost = cost(parent) + edge cost, accumulated root first in f64;
 *   - choose parent: X_near = the k nearest nodes of the new point by (d2, index); candidates
 *     x_nearest first, then X_near in order (x_nearest skipped); the first strict minimum of
 *     cost(p) + edge cost over the feasible edges new → p (yaw = compute_yaw toward p);
 *   - rewire: for m in X_near order, m != parent: the edge m → new keeps m's pose (x, y, yaw);
 *     when feasible and cost(new) + edge cost < cost(m) (current), m's parent becomes new and
 *     the costs of m's subtree are recomputed top down;
 *   - k = min(k_fixed, 63, n) when k_fixed > 0, else min(63, n, max(1, ceil(2e ln n))), with n the
 *     tree size before the insert (orc_star_k). */
int orc_star_k(int k_fixed, int n) {
    int k;
    if (k_fixed > 0) {
        k = k_fixed;
    } else {
        double v = n > 1 ? ceil(2.0 * 2.718281828459045 * log((double)n)) : 1.0;
        k = v < 1.0 ? 1 : (v > 63.0 ? 63 : (int)v);
    }
    if (k > 63) k = 63;
    return k < n ? k : n;
}

/* edge child (x, y, yaw) → parent pose: 1 feasible (Some and verify(edge ++ [parent])), 0 not,
 * -1 error (allocation / the reference's n_point panic); *cost = the Dubins cost */
static int star_edge(const orc_scene* sc, double x, double y, double yaw, double px, double py,
                     double pyaw, pbuf* b, dscratch* s, double* cost) {
    double conf[8] = {x, y, yaw, px, py, pyaw, sc->turn_radius, sc->step_size};
    *cost = INFINITY;
    int need = orc_dubins_n_point(conf);
    if (need <= 0) return 0; /* None */
    if (dscratch_fit(s, need) != 0) return -1;
    int n = 0, word = -1;
    int r = orc_dubins(conf, s->px, s->py, s->pyaw, s->cap, &n, &word, cost);
    if (r < 0) return -1;
    if (r == 0) { *cost = INFINITY; return 0; }
    b->n = 0;
    for (int i = 0; i < n; ++i)
        if (pbuf_push(b, s->px[i], s->py[i])) return -1;
    if (pbuf_push(b, px, py)) return -1;
    return orc_verify_line(sc, b->x, b->y, b->n);
}

/* the k nearest nodes by (d2, index), ascending */
static int star_knn(const orc_tree* tr, double qx, double qy, int k, int32_t* out, double* d2s) {
    int m = 0;
    for (int i = 0; i < tr->n; ++i) {
        double dx = qx - tr->x[i], dy = qy - tr->y[i];
        double d2 = dx * dx + dy * dy;
        if (m == k && !(d2 < d2s[m - 1])) continue; /* (d2, i) > the k-th: i is the larger index */
        int j = m < k ? m++ : m - 1;
        while (j > 0 && d2 < d2s[j - 1]) { d2s[j] = d2s[j - 1]; out[j] = out[j - 1]; --j; }
        d2s[j] = d2;
        out[j] = i;
    }
    return m;
}

/* recompute cost[] over the subtree of m (level by level: each level's parents are final) */
static int star_propagate(orc_tree* tr, double* cost, const double* elen, int m, uint8_t* fr,
                          uint8_t* nx) {
    memset(fr, 0, (size_t)tr->n);
    fr[m] = 1;
    for (;;) {
        int any = 0;
        memset(nx, 0, (size_t)tr->n);
        for (int i = 0; i < tr->n; ++i) {
            int p = tr->parent[i];
            if (p >= 0 && fr[p]) { cost[i] = cost[p] + elen[i]; nx[i] = 1; any = 1; }
        }
        if (!any) break;
        uint8_t* t = fr; fr = nx; nx = t;
    }
    return 0;
}

/* iterations [it0, it0 + n_iter) of RRT* on tree tr (with cost[], elen[] alongside; root cost
 * 0).  Logs (optional): nearest index and accepted flag per iteration.  *rewires_out += rewires.
 * Returns the accepted count, or -1 (allocation / capacity / steer overflow). */
int64_t orc_star_extend(const orc_scene* sc, orc_tree* tr, double* cost, double* elen,
                        uint64_t seed, int64_t it0, int64_t n_iter, int k_fixed, double eta,
                        int64_t* rewires_out, int32_t* log_nn, int8_t* log_acc) {
    pbuf b = {0};
    dscratch s = {0};
    int64_t acc = 0, rew = 0;
    int32_t near[63];
    double nd2[63];
    uint8_t* fr = (uint8_t*)malloc((size_t)tr->cap + 1);
    uint8_t* nx = (uint8_t*)malloc((size_t)tr->cap + 1);
    if (!fr || !nx) acc = -1;
    for (int64_t kk = 0; kk < n_iter && acc >= 0; ++kk) {
        uint64_t it = (uint64_t)(it0 + kk);
        double x = orc_gen_range(seed, 2 * it, sc->minx, sc->maxx);
        double y = orc_gen_range(seed, 2 * it + 1, sc->miny, sc->maxy);
        double d2;
        int p = orc_nearest(tr->x, tr->y, tr->n, x, y, &d2);
        if (log_nn) log_nn[kk] = p;
        if (log_acc) log_acc[kk] = 0;
        if (eta > 0.0 && d2 > eta * eta) { /* Steer(x_nearest, x_rand): eta along the chord */
            double f = eta / sqrt(d2);
            x = tr->x[p] + (x - tr->x[p]) * f;
            y = tr->y[p] + (y - tr->y[p]) * f;
        }
        double yb = compute_yaw(x, y, tr->x[p], tr->y[p]), eb;
        int ok = star_edge(sc, x, y, yb, tr->x[p], tr->y[p], tr->yaw[p], &b, &s, &eb);
        if (ok < 0) { acc = -1; break; }
        if (!ok) continue;
        int k = orc_star_k(k_fixed, tr->n);
        int kn = star_knn(tr, x, y, k, near, nd2);
        int best = p;
        double cb = cost[p] + eb;
        for (int j = 0; j < kn; ++j) {
            int q = near[j];
            if (q == p) continue; /* the nearest is the first candidate */
            double yq = compute_yaw(x, y, tr->x[q], tr->y[q]), eq;
            int o = star_edge(sc, x, y, yq, tr->x[q], tr->y[q], tr->yaw[q], &b, &s, &eq);
            if (o < 0) { acc = -1; break; }
            if (o) {
                double c = cost[q] + eq;
                if (c < cb) { cb = c; best = q; yb = yq; eb = eq; }
            }
        }
        if (acc < 0) break;
        if (tr->n >= tr->cap) { acc = -1; break; }
        int nw = tr->n;
        tr->x[nw] = x; tr->y[nw] = y; tr->yaw[nw] = yb; tr->parent[nw] = best;
        cost[nw] = cb; elen[nw] = eb;
        tr->n++;
        acc++;
        if (log_acc) log_acc[kk] = 1;
        for (int j = 0; j < kn; ++j) {
            int m = near[j];
            if (m == best || !(cb < cost[m])) continue; /* cb + e >= cb: no rewire possible */
            double em;
            int o = star_edge(sc, tr->x[m], tr->y[m], tr->yaw[m], x, y, yb, &b, &s, &em);
            if (o < 0) { acc = -1; break; }
            if (!o) continue;
            double cn = cb + em;
            if (cn < cost[m]) {
                tr->parent[m] = nw; elen[m] = em; cost[m] = cn;
                star_propagate(tr, cost, elen, m, fr, nx);
                rew++;
            }
        }
    }
    free(fr); free(nx);
    free(b.x); free(b.y);
    free(s.px); free(s.py); free(s.pyaw);
    if (rewires_out) *rewires_out += rew;
    return acc;
}

/* n_q independent RRT* queries on T threads (the config-5 CPU baseline) */
typedef struct {
    const orc_scene* sc;
    const double* starts;
    const uint64_t* seeds;
    int64_t n_iter;
    int k_fixed, n_jobs, next, failed;
    double eta;
    int64_t accepted, rewires;
    pthread_mutex_t mu;
} orc_star_pool;

static void* star_worker(void* arg) {
    orc_star_pool* P = (orc_star_pool*)arg;
    for (;;) {
        pthread_mutex_lock(&P->mu);
        const int j = P->next < P->n_jobs ? P->next++ : -1;
        pthread_mutex_unlock(&P->mu);
        if (j < 0) break;
        const int cap = (int)P->n_iter + 1;
        orc_tree t;
        t.x = (double*)malloc(sizeof(double) * (size_t)cap);
        t.y = (double*)malloc(sizeof(double) * (size_t)cap);
        t.yaw = (double*)malloc(sizeof(double) * (size_t)cap);
        t.parent = (int32_t*)malloc(sizeof(int32_t) * (size_t)cap);
        double* cost = (double*)malloc(sizeof(double) * (size_t)cap);
        double* elen = (double*)malloc(sizeof(double) * (size_t)cap);
        t.cap = cap;
        int64_t a = -1, rw = 0;
        if (t.x && t.y && t.yaw && t.parent && cost && elen) {
            t.x[0] = P->starts[3 * j]; t.y[0] = P->starts[3 * j + 1]; t.yaw[0] = P->starts[3 * j + 2];
            t.parent[0] = -1; cost[0] = 0.0; elen[0] = 0.0;
            t.n = 1;
            a = orc_star_extend(P->sc, &t, cost, elen, P->seeds[j], 0, P->n_iter, P->k_fixed, P->eta, &rw,
                                NULL, NULL);
        }
        free(t.x); free(t.y); free(t.yaw); free(t.parent); free(cost); free(elen);
        pthread_mutex_lock(&P->mu);
        if (a < 0) P->failed = 1;
        else { P->accepted += a; P->rewires += rw; }
        pthread_mutex_unlock(&P->mu);
    }
    return NULL;
}

int64_t orc_star_queries(const orc_scene* sc, const double* starts, const uint64_t* seeds, int n_q,
                         int64_t max_iter, int k_fixed, double eta, int threads,
                         int64_t* rewires_out) {
    orc_star_pool P;
    memset(&P, 0, sizeof P);
    P.sc = sc; P.starts = starts; P.seeds = seeds; P.n_iter = max_iter; P.k_fixed = k_fixed;
    P.eta = eta;
    P.n_jobs = n_q;
    if (threads < 1) threads = 1;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    if (!th) return -1;
    pthread_mutex_init(&P.mu, NULL);
    int started = 0;
    for (int i = 0; i < threads; ++i)
        if (pthread_create(&th[i], NULL, star_worker, &P) == 0) started++;
    if (started == 0) star_worker(&P);
    for (int i = 0; i < started; ++i) pthread_join(th[i], NULL);
    pthread_mutex_destroy(&P.mu);
    free(th);
    if (rewires_out) *rewires_out = P.rewires;
    return P.failed ? -1 : P.accepted;
}
