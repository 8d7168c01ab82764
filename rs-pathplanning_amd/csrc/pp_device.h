// pp_device.h — device-side building blocks of the RRT extend hot path (gfx950, f64 steer).
//
// Restates the arithmetic of tsturzl/rs-pathplanning src/dubins.rs (mod2pi, the six Dubins
// words, interpolate, generate_local_course) and of src/rrt.rs (compute_yaw, Space::verify) for
// device code.  Every expression keeps the reference's left-to-right evaluation order and the
// library is compiled with -ffp-contract=off, so results differ from the Rust crate only by the
// ulp-level differences between ocml's and glibc's sin/cos/atan2/acos/hypot.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pp_types.h"

namespace ppamd {

constexpr double kPi = 3.14159265358979323846;  // std::f64::consts::PI
constexpr double kTwoPi = 2.0 * kPi;

// dubins.rs:14-20
// theta / 2pi as the correctly rounded FMA quotient (q = RN(theta r), r = RN(1 / 2pi), then
// RN(q + fma(-q, 2pi, theta) r): Markstein's theorem, bit-identical to the IEEE division;
// tests/test_div_identity.py checks it for 2pi), 3 FP64 ops instead of the division sequence
constexpr double kInvTwoPi = 1.0 / kTwoPi;
// x / c given rc = RN(1 / c): the same correctly rounded quotient
__host__ __device__ inline double div_by(double x, double c, double rc) {
    const double q = x * rc;
    return fma(fma(-q, c, x), rc, q);
}
__host__ __device__ inline double mod2pi(double theta) {
    const double q = theta * kInvTwoPi;
    const double quo = fma(fma(-q, kTwoPi, theta), kInvTwoPi, q);
    return theta - kTwoPi * floor(quo);
}
// dubins.rs:22-24 (Rust `%` == fmod: truncated, negative angles are not wrapped)
__host__ __device__ inline double pi_2_pi(double angle) {
    return fmod(angle + kPi, kTwoPi) - kPi;
}

// Mode {L, S, R} (dubins.rs:4-9) and the ALL_PLANNERS order (dubins.rs:291).
enum : int { kModeL = 0, kModeS = 1, kModeR = 2 };
__host__ __device__ inline int word_mode(int word, int seg) {
    // LSL, RSR, LSR, RSL, RLR, LRL
    const int first = (word == 0 || word == 2 || word == 5) ? kModeL : kModeR;
    const int mid = (word < 4) ? kModeS : (word == 4 ? kModeL : kModeR);
    const int last = (word == 0 || word == 3 || word == 5) ? kModeL : kModeR;
    return seg == 0 ? first : (seg == 1 ? mid : last);
}

struct Word {
    int ok;
    double t, p, q;
};

// sin and cos of x, |x| < 2^30, bit for bit the values ROCm's __ocml_sincos_f64 returns (its
// trigredsmall Cody-Waite reduction by pi/2 in three parts and its sincosred2 polynomials, the
// same operations in the same order; -ffp-contract=off keeps every plain product a product).
// The walk's arc points call it with |pd| < 2 pi + step (every L/R segment length is a mod2pi
// value), so the caller routes any other argument to the literal path.  Why not ocml itself:
// the compiler hoists ocml's 17 f64 constants out of the walk's chunk loop into VGPRs, and at the
// 6-waves-per-SIMD budget two of them spilled (20 B per lane).  Here they are read
// through `tab`, a pointer the caller makes opaque inside the loop (scalar loads from the
// constant cache, re-issued per chunk) — nothing is loop-invariant to hoist.
// tab: kSinCosTab, in this order: 2/pi, -pi/2 (hi), -pi/2 (mid), pi/2 (mid), -pi/2 (lo), then the
// cos polynomial c6..c1 and the sin polynomial s5..s2 and s1.
__device__ inline void sincos_small(double x, const double* __restrict__ tab, double* sp,
                                    double* cp) {
    const double ax = fabs(x);
    // __ocmlpriv_trigredsmall_f64
    const double q = __builtin_rint(ax * tab[0]);
    const double a = __builtin_fma(q, tab[1], ax);
    const double b = __builtin_fma(q, tab[2], a);
    const double p = q * tab[3];
    const double pe = __builtin_fma(q, tab[3], -p);
    const double t9 = a - p;
    const double t10 = a - t9;
    const double t11 = t10 - p;
    const double t12 = t9 - b;
    const double t13 = t12 + t11;
    const double t14 = t13 - pe;
    const double t15 = __builtin_fma(q, tab[4], t14);
    const double hi = b + t15;
    const double t17 = hi - b;
    const double lo = t15 - t17;
    const int i = (int)q & 3;
    // __ocmlpriv_sincosred2_f64(hi, lo)
    const double x2 = hi * hi;
    const double hx2 = x2 * 0.5;
    const double c1 = 1.0 - hx2;
    const double t6 = 1.0 - c1;
    const double t7 = t6 - hx2;
    const double x4 = x2 * x2;
    double pc = __builtin_fma(x2, tab[5], tab[6]);
    pc = __builtin_fma(x2, pc, tab[7]);
    pc = __builtin_fma(x2, pc, tab[8]);
    pc = __builtin_fma(x2, pc, tab[9]);
    pc = __builtin_fma(x2, pc, tab[10]);
    const double t15b = __builtin_fma(hi, -lo, t7);
    const double t16 = __builtin_fma(x4, pc, t15b);
    const double cv = c1 + t16;
    double ps = __builtin_fma(x2, tab[11], tab[12]);
    ps = __builtin_fma(x2, ps, tab[13]);
    ps = __builtin_fma(x2, ps, tab[14]);
    ps = __builtin_fma(x2, ps, tab[15]);
    const double t23 = hi * -x2;
    const double t24 = lo * 0.5;
    const double t25 = __builtin_fma(t23, ps, t24);
    const double t26 = __builtin_fma(x2, t25, -lo);
    const double t27 = __builtin_fma(t23, tab[16], t26);
    const double sv = hi - t27;
    // __ocml_sincos_f64: quadrant and signs (|x| finite here)
    const unsigned flip = i > 1 ? 0x80000000u : 0u;
    const bool even = (i & 1) == 0;
    const double sm = even ? sv : cv;
    const double cm = even ? cv : -sv;
    const unsigned long long xs = (unsigned long long)__double_as_longlong(x) & 0x8000000000000000ull;
    const unsigned long long fl = (unsigned long long)flip << 32;
    *sp = __longlong_as_double((long long)((unsigned long long)__double_as_longlong(sm) ^ xs ^ fl));
    *cp = __longlong_as_double((long long)((unsigned long long)__double_as_longlong(cm) ^ fl));
}

// The six closed forms share sin/cos(alpha), sin/cos(beta) and cos(alpha - beta); each is
// computed once here (the reference recomputes identical values per word).
struct Trig {
    double sa, sb, ca, cb, c_ab;
};
__device__ inline Trig make_trig(double alpha, double beta) {
    Trig g;
    g.sa = sin(alpha);
    g.sb = sin(beta);
    g.ca = cos(alpha);
    g.cb = cos(beta);
    g.c_ab = cos(alpha - beta);
    return g;
}

// dubins.rs:27-48
__device__ inline Word word_lsl(double alpha, double beta, double d, const Trig& g) {
    Word w{0, 0.0, 0.0, 0.0};
    double tmp0 = d + g.sa - g.sb;
    double p_squared = 2.0 + (d * d) - (2.0 * g.c_ab) + (2.0 * d * (g.sa - g.sb));
    if (p_squared < 0.0) return w;
    double tmp1 = atan2(g.cb - g.ca, tmp0);
    w.t = mod2pi(-alpha + tmp1);
    w.p = sqrt(p_squared);
    w.q = mod2pi(beta - tmp1);
    w.ok = 1;
    return w;
}
// dubins.rs:51-71
__device__ inline Word word_rsr(double alpha, double beta, double d, const Trig& g) {
    Word w{0, 0.0, 0.0, 0.0};
    double tmp0 = d - g.sa + g.sb;
    double p_squared = 2.0 + (d * d) - (2.0 * g.c_ab) + (2.0 * d * (g.sb - g.sa));
    if (p_squared < 0.0) return w;
    double tmp1 = atan2(g.ca - g.cb, tmp0);
    w.t = mod2pi(alpha - tmp1);
    w.p = sqrt(p_squared);
    w.q = mod2pi(-beta + tmp1);
    w.ok = 1;
    return w;
}
// dubins.rs:74-92
__device__ inline Word word_lsr(double alpha, double beta, double d, const Trig& g) {
    Word w{0, 0.0, 0.0, 0.0};
    double p_squared = -2.0 + (d * d) + (2.0 * g.c_ab) + (2.0 * d * (g.sa + g.sb));
    if (p_squared < 0.0) return w;
    double p = sqrt(p_squared);
    double tmp = atan2(-g.ca - g.cb, d + g.sa + g.sb) - atan2(-2.0, p);
    w.t = mod2pi(-alpha + tmp);
    w.p = p;
    w.q = mod2pi(-mod2pi(beta) + tmp);
    w.ok = 1;
    return w;
}
// dubins.rs:95-113
__device__ inline Word word_rsl(double alpha, double beta, double d, const Trig& g) {
    Word w{0, 0.0, 0.0, 0.0};
    double p_squared = -2.0 + (d * d) + (2.0 * g.c_ab) - (2.0 * d * (g.sa + g.sb));
    if (p_squared < 0.0) return w;
    double p = sqrt(p_squared);
    double tmp = atan2(g.ca + g.cb, d - g.sa - g.sb) - atan2(2.0, p);
    w.t = mod2pi(alpha - tmp);
    w.p = p;
    w.q = mod2pi(beta - tmp);
    w.ok = 1;
    return w;
}
// dubins.rs:116-133
__device__ inline Word word_rlr(double alpha, double beta, double d, const Trig& g) {
    Word w{0, 0.0, 0.0, 0.0};
    double tmp_rlr = (6.0 - d * d + 2.0 * g.c_ab + 2.0 * d * (g.sa - g.sb)) / 8.0;
    if (fabs(tmp_rlr) > 1.0) return w;
    double p = mod2pi(2.0 * kPi - acos(tmp_rlr));
    double t = mod2pi(alpha - atan2(g.ca - g.cb, d - g.sa + g.sb) + mod2pi(p / 2.0));
    double q = mod2pi(alpha - beta - t + mod2pi(p));
    w.t = t;
    w.p = p;
    w.q = q;
    w.ok = 1;
    return w;
}
// dubins.rs:136-153
__device__ inline Word word_lrl(double alpha, double beta, double d, const Trig& g) {
    Word w{0, 0.0, 0.0, 0.0};
    double tmp_lrl = (6.0 - d * d + 2.0 * g.c_ab + 2.0 * d * (-g.sa + g.sb)) / 8.0;
    if (fabs(tmp_lrl) > 1.0) return w;
    double p = mod2pi(2.0 * kPi - acos(tmp_lrl));
    double t = mod2pi(-alpha - atan2(g.ca - g.cb, d + g.sa - g.sb) + p / 2.0);
    double q = mod2pi(mod2pi(beta) - alpha - t + mod2pi(p));
    w.t = t;
    w.p = p;
    w.q = q;
    w.ok = 1;
    return w;
}

// Result of the word selection of dubins_path_planning_from_origin (dubins.rs:333-363).
struct Steer {
    int word;  // -1 = None (no feasible word)
    double t, p, q, cost;
};

// dubins.rs:333-363: evaluate LSL, RSR, LSR, RSL, RLR, LRL in order and keep the first strict
// minimum of |t|+|p|+|q|.  All lanes compute the same (wave-uniform) values.
// (select_word_fi / interp_local_fi: always inlined, for a literal path that must take its
// caller's register budget; the plain names are ordinary inline functions)
__device__ __forceinline__ Steer select_word_fi(double lex, double ley, double leyaw, double c) {
    const double hyp = hypot(lex, ley);
    const double d = hyp * c;
    const double theta = mod2pi(atan2(ley, lex));
    const double alpha = mod2pi(-theta);
    const double beta = mod2pi(leyaw - theta);
    const Trig g = make_trig(alpha, beta);
    Steer s{-1, 0.0, 0.0, 0.0, 0.0};
    double bcost = __builtin_inf();
    Word w[6];
    w[0] = word_lsl(alpha, beta, d, g);
    w[1] = word_rsr(alpha, beta, d, g);
    w[2] = word_lsr(alpha, beta, d, g);
    w[3] = word_rsl(alpha, beta, d, g);
    w[4] = word_rlr(alpha, beta, d, g);
    w[5] = word_lrl(alpha, beta, d, g);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        if (w[i].ok) {
            double cost = fabs(w[i].t) + fabs(w[i].p) + fabs(w[i].q);
            if (bcost > cost) {
                s.word = i;
                s.t = w[i].t;
                s.p = w[i].p;
                s.q = w[i].q;
                bcost = cost;
            }
        }
    }
    s.cost = bcost;
    return s;
}
__device__ inline Steer select_word(double lex, double ley, double leyaw, double c) {
    return select_word_fi(lex, ley, leyaw, c);
}

struct Pose {
    double x, y, yaw;
};

// dubins.rs:155-198 (x, y, yaw of one sample; directions are not part of the output)
__device__ __forceinline__ Pose interp_local_fi(int mode, double length, double max_curvature,
                                                Pose o) {
    Pose r;
    if (mode == kModeS) {
        r.x = o.x + length / max_curvature * cos(o.yaw);
        r.y = o.y + length / max_curvature * sin(o.yaw);
        r.yaw = o.yaw;
    } else {
        double ldx = sin(length) / max_curvature;
        double ldy;
        if (mode == kModeL)
            ldy = (1.0 - cos(length)) / max_curvature;
        else
            ldy = (1.0 - cos(length)) / -max_curvature;
        double gdx = cos(-o.yaw) * ldx + sin(-o.yaw) * ldy;
        double gdy = -sin(-o.yaw) * ldx + cos(-o.yaw) * ldy;
        r.x = o.x + gdx;
        r.y = o.y + gdy;
        r.yaw = o.yaw;
    }
    if (mode == kModeL)
        r.yaw = o.yaw + length;
    else if (mode == kModeR)
        r.yaw = o.yaw - length;
    return r;
}
__device__ inline Pose interp_local(int mode, double length, double max_curvature, Pose o) {
    return interp_local_fi(mode, length, max_curvature, o);
}

// Literal single-thread restatement of dubins_path_planning_from_origin (dubins.rs:326-399): the
// LOCAL points after generate_local_course's trim, yaw as generated (not wrapped).  Returns
// kSteerSome / kSteerNone / kSteerOverflow (cap < n_point or the Rust index panic).
template <bool kFI = false>
__device__ inline int dubins_local(double lex, double ley, double leyaw, double c, double step_size,
                                   double* px, double* py, double* pyaw, int cap, int* n_out,
                                   int* word_out, double* cost_out) {
    const Steer s = kFI ? select_word_fi(lex, ley, leyaw, c) : select_word(lex, ley, leyaw, c);
    if (s.word < 0) return kSteerNone;
    const double lengths[3] = {s.t, s.p, s.q};
    double total = 0.0;
    total += s.t;
    total += s.p;
    total += s.q;
    const double nq = trunc(total / step_size);
    if (!(nq >= 0.0) || nq > 1.0e8) return kSteerOverflow;
    const int n_point = (int)nq + 3 + 4;
    if (n_point > cap) return kSteerOverflow;
    for (int i = 0; i < n_point; ++i) px[i] = py[i] = pyaw[i] = 0.0;
    // generate_local_course, dubins.rs:200-272
    int ind = 1;
    double ll = 0.0;
    for (int i = 0; i < 3; ++i) {
        const int m = word_mode(s.word, i);
        const double l = lengths[i];
        const double d = (l > 0.0) ? step_size : -step_size;
        const Pose o{px[ind], py[ind], pyaw[ind]};
        ind -= 1;
        double pd = (i >= 1 && (lengths[i - 1] * lengths[i]) > 0.0) ? (-d - ll) : (d - ll);
        while (fabs(pd) <= fabs(l)) {
            ind += 1;
            if (ind >= n_point) return kSteerOverflow;
            Pose r = kFI ? interp_local_fi(m, pd, c, o) : interp_local(m, pd, c, o);
            px[ind] = r.x;
            py[ind] = r.y;
            pyaw[ind] = r.yaw;
            pd += d;
        }
        ll = l - pd - d;
        ind += 1;
        if (ind >= n_point) return kSteerOverflow;
        Pose r = kFI ? interp_local_fi(m, l, c, o) : interp_local(m, l, c, o);
        px[ind] = r.x;
        py[ind] = r.y;
        pyaw[ind] = r.yaw;
    }
    // trailing-zero trim, dubins.rs:281-288 (pops every trailing 0.0 plus one more element)
    int len = n_point;
    double last = px[len - 1];
    while (len >= 1 && last == 0.0) {
        last = px[len - 1];
        len -= 1;
    }
    *n_out = len;
    *word_out = s.word;
    *cost_out = s.cost;
    return kSteerSome;
}

// Literal single-thread restatement of dubins_path_planning (dubins.rs:401-428) writing WORLD
// points: the slow path for the measure-zero trim cases, and the pp_dubins_batch API.
// Returns kSteerSome / kSteerNone / kSteerOverflow (cap < n_point or the Rust index panic).
// kYaw = false: the world yaws are not wrapped back (pyaw keeps the local ones): check_finish's
// lines need the points only, and pi_2_pi's fmod per point cost more than the points
template <bool kFI = false, bool kYaw = true>
__device__ inline int dubins_literal(double sx, double sy, double syaw, double ex0, double ey0,
                                     double eyaw, double turn_radius, double step_size, double* px,
                                     double* py, double* pyaw, int cap, int* n_out, int* word_out,
                                     double* cost_out) {
    const double ex = ex0 - sx, ey = ey0 - sy;
    const double c = 1.0 / turn_radius;
    const double lex = cos(syaw) * ex + sin(syaw) * ey;
    const double ley = -(sin(syaw)) * ex + cos(syaw) * ey;
    const double leyaw = eyaw - syaw;
    int len = 0;
    const int r = dubins_local<kFI>(lex, ley, leyaw, c, step_size, px, py, pyaw, cap, &len, word_out,
                               cost_out);
    if (r != kSteerSome) return r;
    // back to the world frame, dubins.rs:412-422
    const double cs = cos(-syaw), sn = sin(-syaw);
    for (int i = 0; i < len; ++i) {
        const double x = px[i], y = py[i];
        px[i] = cs * x + sn * y + sx;
        py[i] = -sn * x + cs * y + sy;
        if (kYaw) pyaw[i] = pi_2_pi(pyaw[i] + syaw);
    }
    *n_out = len;
    return kSteerSome;
}

// Squared distance from (cx, cy) to the closed segment a-b: exact closest point of the segment.
__host__ __device__ inline double seg_point_d2(double ax, double ay, double bx, double by,
                                               double cx, double cy) {
    const double vx = bx - ax, vy = by - ay;
    const double wx = cx - ax, wy = cy - ay;
    const double l2 = vx * vx + vy * vy;
    double t = 0.0;
    if (l2 > 0.0) {
        t = (wx * vx + wy * vy) / l2;
        if (t < 0.0)
            t = 0.0;
        else if (t > 1.0)
            t = 1.0;
    }
    const double ex = wx - t * vx, ey = wy - t * vy;
    return ex * ex + ey * ey;
}

// Polyline segment vs closed disc.
__device__ inline bool seg_hits_disc(double ax, double ay, double bx, double by, double cx,
                                     double cy, double r2) {
    return seg_point_d2(ax, ay, bx, by, cx, cy) <= r2;
}

// ---- polygon mode (Q10p): geo's Contains / Intersects on the geo-offset buffers (rrt.rs:62-68,
// 82, 108-111, 124-137) as exact Minkowski buffers — an obstacle polygon grows by the closed disc
// of radius h = width/2, the bounds polygon shrinks to the points whose disc stays inside.  The
// same arithmetic as the oracle (oracle/pp_oracle.c), so verdicts agree bit for bit.

// crossing-number step: edge (xi, yi)-(xj, yj) crosses the ray from (px, py) toward +x
__host__ __device__ inline bool ray_crosses(double px, double py, double xi, double yi, double xj,
                                            double yj) {
    return ((yi > py) != (yj > py)) && (px < (xj - xi) * (py - yi) / (yj - yi) + xi);
}

// the point lies in the bounds polygon eroded by h: inside the ring (even-odd) and at distance
// >= h from every bounds edge
__host__ __device__ inline bool in_poly_bounds(int nbv, const double* bvx, const double* bvy,
                                               double h2, double x, double y) {
    bool inside = false;
    for (int i = 0; i < nbv; ++i) {
        const int j = i + 1 == nbv ? 0 : i + 1;
        const double xi = bvx[i], yi = bvy[i], xj = bvx[j], yj = bvy[j];
        if (ray_crosses(x, y, xi, yi, xj, yj)) inside = !inside;
        if (seg_point_d2(xi, yi, xj, yj, x, y) < h2) return false;
    }
    return inside;
}

// polyline segment a-b vs the buffer of the obstacle edge e0-e1: a proper crossing, or an
// endpoint of one segment within h of the other (touching counts)
__host__ __device__ inline bool seg_hits_edge(double ax, double ay, double bx, double by,
                                              double e0x, double e0y, double e1x, double e1y,
                                              double h2) {
    const double d1 = (e1x - e0x) * (ay - e0y) - (e1y - e0y) * (ax - e0x);
    const double d2 = (e1x - e0x) * (by - e0y) - (e1y - e0y) * (bx - e0x);
    const double d3 = (bx - ax) * (e0y - ay) - (by - ay) * (e0x - ax);
    const double d4 = (bx - ax) * (e1y - ay) - (by - ay) * (e1x - ax);
    if (((d1 > 0.0 && d2 < 0.0) || (d1 < 0.0 && d2 > 0.0)) &&
        ((d3 > 0.0 && d4 < 0.0) || (d3 < 0.0 && d4 > 0.0)))
        return true;
    return seg_point_d2(e0x, e0y, e1x, e1y, ax, ay) <= h2 ||
           seg_point_d2(e0x, e0y, e1x, e1y, bx, by) <= h2 ||
           seg_point_d2(ax, ay, bx, by, e0x, e0y) <= h2 ||
           seg_point_d2(ax, ay, bx, by, e1x, e1y) <= h2;
}

// the point lies inside some obstacle polygon (even-odd over each polygon's consecutive edges)
__host__ __device__ inline bool in_obstacle(int ne, const double* ex0, const double* ey0,
                                            const double* ex1, const double* ey1,
                                            const int* epoly, double x, double y) {
    bool inside = false;
    for (int k = 0; k < ne; ++k) {
        if (k > 0 && epoly[k] != epoly[k - 1]) {
            if (inside) return true;
            inside = false;
        }
        if (ray_crosses(x, y, ex0[k], ey0[k], ex1[k], ey1[k])) inside = !inside;
    }
    return inside;
}

// a point in bounds: the (shrunken) rectangle, and the eroded bounds polygon when there is one
__host__ __device__ inline bool point_in_bounds(const SceneDev& sc, double x, double y) {
    if (!(x >= sc.minx && x <= sc.maxx && y >= sc.miny && y <= sc.maxy)) return false;
    return sc.nbv == 0 || in_poly_bounds(sc.nbv, sc.bvx, sc.bvy, sc.h2, x, y);
}

// --------------------------------------------------------- seeded sampling
// SplitMix64 output `ctr` of the stream `seed` (replaces rand::thread_rng, rrt.rs:140).
__host__ __device__ inline uint64_t rng_u64(uint64_t seed, uint64_t ctr) {
    uint64_t z = seed + (ctr + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
// rand 0.7 UniformFloat<f64>::sample_single: [1,2) from 52 random bits, minus 1, * scale + low
// (rrt.rs:142-143).  res >= high (measure zero) narrows scale by one ulp with the same bits.
__host__ __device__ inline double gen_range(uint64_t seed, uint64_t ctr, double low, double high) {
    const uint64_t bits = (rng_u64(seed, ctr) >> 12) | 0x3FF0000000000000ULL;
    const double value0_1 = __builtin_bit_cast(double, bits) - 1.0;
    double scale = high - low;
    for (;;) {
        const double res = value0_1 * scale + low;
        if (res < high) return res;
        scale = nextafter(scale, 0.0);
    }
}

// occupancy probe of config 4 (SceneDev::bits): true when the point's cell is occupied or the
// point lies outside the grid
__device__ inline bool grid_occupied(const uint32_t* B, int bw, int bh, int bwords, double bx0,
                                     double by0, double binv, double x, double y) {
    const double fx = floor((x - bx0) * binv), fy = floor((y - by0) * binv);
    if (!(fx >= 0.0) || !(fy >= 0.0) || fx >= (double)bw || fy >= (double)bh) return true;
    const int i = (int)fx, j = (int)fy;
    return (B[j * bwords + (i >> 5)] >> (i & 31)) & 1u;
}

// ------------------------------------------------------------------------- wave helpers
__device__ inline double wave_min(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}
// lane k's value (k wave-uniform) broadcast through SGPRs
__device__ inline double readlane_f64(double v, int k) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), k);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), k);
    return __hiloint2double(hi, lo);
}
__device__ inline double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}

// f32 wave reductions on DPP (no LDS round trips): quad swaps, half-row and row mirrors, then the
// gfx9 row broadcasts 15 and 31 into the upper rows; lane 63 holds the result.  All 64 lanes must
// be active.
template <int kCtrl, int kRowMask = 0xF>
__device__ inline float dpp_f32(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v),
                                                                 __builtin_bit_cast(int, v), kCtrl,
                                                                 kRowMask, 0xF, false));
}
__device__ inline float readlane_f32(float v, int k) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), k));
}
__device__ inline float wave_min_f32(float v) {
    v = __builtin_fminf(v, dpp_f32<0xB1>(v));       // quad_perm [1,0,3,2]
    v = __builtin_fminf(v, dpp_f32<0x4E>(v));       // quad_perm [2,3,0,1]
    v = __builtin_fminf(v, dpp_f32<0x141>(v));      // row_half_mirror
    v = __builtin_fminf(v, dpp_f32<0x140>(v));      // row_mirror
    v = __builtin_fminf(v, dpp_f32<0x142, 0xA>(v)); // row_bcast:15 into rows 1, 3
    v = __builtin_fminf(v, dpp_f32<0x143, 0xC>(v)); // row_bcast:31 into rows 2, 3
    return readlane_f32(v, 63);
}
__device__ inline float wave_max_f32(float v) {
    v = __builtin_fmaxf(v, dpp_f32<0xB1>(v));
    v = __builtin_fmaxf(v, dpp_f32<0x4E>(v));
    v = __builtin_fmaxf(v, dpp_f32<0x141>(v));
    v = __builtin_fmaxf(v, dpp_f32<0x140>(v));
    v = __builtin_fmaxf(v, dpp_f32<0x142, 0xA>(v));
    v = __builtin_fmaxf(v, dpp_f32<0x143, 0xC>(v));
    return readlane_f32(v, 63);
}
// __shfl_up(v, 1) on DPP (wave_shr:1): lane l gets lane l - 1's value, lane 0 keeps its own
__device__ inline double shfl_up1_f64(double v) {
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(v), __double2loint(v), 0x138, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(v), __double2hiint(v), 0x138, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
// lane k of every 8-lane group broadcast to the group's lanes (steer_prep's per-task lane
// groups), on DPP: the quad broadcast of lane k % 4, then the half-row mirror for the other quad.
// All 64 lanes must be active.
template <int k>
__device__ inline int grp8_bcast_i32(int v) {
    static_assert(k >= 0 && k < 8, "lane of an 8-lane group");
    constexpr int q = k & 3;
    const int v1 = __builtin_amdgcn_update_dpp(v, v, q | (q << 2) | (q << 4) | (q << 6), 0xF, 0xF, false);
    const int v2 = __builtin_amdgcn_update_dpp(v1, v1, 0x141, 0xF, 0xF, false);  // row_half_mirror
    const bool low = (threadIdx.x & 4) == 0;
    return (k < 4) == low ? v1 : v2;
}
template <int k>
__device__ inline double grp8_bcast_f64(double v) {
    return __hiloint2double(grp8_bcast_i32<k>(__double2hiint(v)), grp8_bcast_i32<k>(__double2loint(v)));
}
// Butterfly steps without LDS round trips (all 64 lanes active): dpp_pair<kCtrl> gives every lane
// its partner's 32-bit value under a DPP pattern that pairs disjoint lane sets (quad_perm [1,0,3,2]
// and [2,3,0,1], row_half_mirror, row_mirror); swap16 / swap32 (gfx950 v_permlane16/32_swap) give
// every lane the pair {v[l], v[l ^ 16]} / {v[l], v[l ^ 32]} (scripts/micro/permlane_check.hip).
template <int kCtrl>
__device__ inline int dpp_pair(int v) {
    return __builtin_amdgcn_update_dpp(v, v, kCtrl, 0xF, 0xF, false);
}
struct LanePair {
    int a, b;
};
__device__ inline LanePair swap16(int v) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return {(int)r[0], (int)r[1]};
}
__device__ inline LanePair swap32(int v) {
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return {(int)r[0], (int)r[1]};
}
// argmin over (d, i) in (d, index) order (ties: lowest index), whole wave; every lane ends with it
__device__ inline void argmin_step(double& d, int& i, double od, int oi) {
    if (od < d || (od == d && oi < i)) {
        d = od;
        i = oi;
    }
}
template <int kCtrl>
__device__ inline void argmin_dpp(double& d, int& i) {
    const double od = __hiloint2double(dpp_pair<kCtrl>(__double2hiint(d)), dpp_pair<kCtrl>(__double2loint(d)));
    argmin_step(d, i, od, dpp_pair<kCtrl>(i));
}
template <bool k32>
__device__ inline void argmin_swap(double& d, int& i) {
    const LanePair h = k32 ? swap32(__double2hiint(d)) : swap16(__double2hiint(d));
    const LanePair l = k32 ? swap32(__double2loint(d)) : swap16(__double2loint(d));
    const LanePair x = k32 ? swap32(i) : swap16(i);
    d = __hiloint2double(h.a, l.a);
    i = x.a;
    argmin_step(d, i, __hiloint2double(h.b, l.b), x.b);
}
__device__ inline void wave_argmin(double& d, int& i) {
    argmin_dpp<0xB1>(d, i);
    argmin_dpp<0x4E>(d, i);
    argmin_dpp<0x141>(d, i);
    argmin_dpp<0x140>(d, i);
    argmin_swap<false>(d, i);
    argmin_swap<true>(d, i);
}
// inclusive prefix sum over the wave's 64 lanes on DPP (all lanes active): within each row the
// three row shifts then the bank-masked shifts by 4 and 8, then the row broadcasts 15 and 31
template <int kCtrl, int kRowMask, int kBankMask>
__device__ inline int dpp_zero(int v) {  // lanes without a source (or masked off) read 0
    return __builtin_amdgcn_update_dpp(0, v, kCtrl, kRowMask, kBankMask, true);
}
__device__ inline int wave_incl_scan(int v) {
    int x = v + dpp_zero<0x111, 0xF, 0xF>(v);  // row_shr:1
    x += dpp_zero<0x112, 0xF, 0xF>(v);         // row_shr:2
    x += dpp_zero<0x113, 0xF, 0xF>(v);         // row_shr:3
    x += dpp_zero<0x114, 0xF, 0xE>(x);         // row_shr:4, banks 1-3
    x += dpp_zero<0x118, 0xF, 0xC>(x);         // row_shr:8, banks 2-3
    x += dpp_zero<0x142, 0xA, 0xF>(x);         // row_bcast:15 into rows 1, 3
    x += dpp_zero<0x143, 0xC, 0xF>(x);         // row_bcast:31 into rows 2, 3
    return x;
}
// f32 bounds of an f64 value: lo <= v <= hi (the conversion rounds to nearest; a rounded-past
// value moves out by far more than its rounding error)
__device__ inline float f32_below(double v) {
    const float f = (float)v;
    return (double)f > v ? f - (__builtin_fabsf(f) * 1.0e-6f + 1.0e-30f) : f;
}
__device__ inline float f32_above(double v) {
    const float f = (float)v;
    return (double)f < v ? f + (__builtin_fabsf(f) * 1.0e-6f + 1.0e-30f) : f;
}

}  // namespace ppamd
