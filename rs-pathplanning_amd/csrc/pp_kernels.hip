// pp_kernels.hip — hand-written CDNA4 (gfx950) kernels of the RRT extend hot path.
//
//   nn_scan          K samples x N tree nodes, f32 SoA screen (s_load-broadcast nodes, 4 queries
//                    per lane, exact top-2 per lane, LDS merge of the 4 waves)       rrt.rs:378-391
//   nn_finalize      merge the node-chunk partials, flag near-ties, exact f64 d^2 of the winner
//   nn_rescan        exact f64 brute force for the flagged (near-tie) samples only
//   window_pairs     per sample: the earlier samples of the same window that are strictly nearer
//                    than its snapshot NN (the candidates of the sequential-consistency resolve)
//   steer_slots      one wave per (sample, parent) slot: compute_yaw + Dubins steer + sampled-arc
//                    collision check, fused, f64                rrt.rs:169-175,414-426, dubins.rs
//   steer_tasks      the same for an explicit task list (repairs; literal single-lane path)
//   dubins_batch     one lane per DubinsConfig: dubins_path_planning, literal (API surface)
//
// No MFMA anywhere: there is no dense contraction on this path.
#include <hip/hip_runtime.h>

#include "pp_device.h"
#include "pp_kernels.h"

namespace ppamd {

// ------------------------------------------------------------------------------ collision

// One 64-point chunk of a polyline, one point per lane: bounds for the lanes flagged
// `check_bounds`, then the segment (lane-1 → lane) of every lane flagged `seg_valid` against the
// discs that overlap the chunk's bounding box (Space::verify, rrt.rs:124-137, Q10).
// Must be called by all 64 lanes.  Returns true when the chunk rejects the line.
__device__ bool chunk_rejects(const SceneDev& sc, bool has, bool check_bounds, bool seg_valid,
                              double qx, double qy) {
    const bool oob =
        check_bounds && !(qx >= sc.minx && qx <= sc.maxx && qy >= sc.miny && qy <= sc.maxy);
    if (__any(oob)) return true;
    const double ax = __shfl_up(qx, 1);
    const double ay = __shfl_up(qy, 1);
    const double inf = __builtin_inf();
    const double bx0 = wave_min(has ? qx : inf);
    const double bx1 = wave_max(has ? qx : -inf);
    const double by0 = wave_min(has ? qy : inf);
    const double by1 = wave_max(has ? qy : -inf);
    const int lane = threadIdx.x & 63;
    for (int base = 0; base < sc.m; base += 64) {
        const int k = base + lane;
        bool ov = false;
        if (k < sc.m) {
            const double cx = sc.cx[k], cy = sc.cy[k], rc = sc.rcull[k];
            ov = (cx + rc >= bx0) && (cx - rc <= bx1) && (cy + rc >= by0) && (cy - rc <= by1);
        }
        unsigned long long mask = __ballot(ov);
        while (mask) {
            const int b = __ffsll((unsigned long long)mask) - 1;
            mask &= mask - 1;
            const int kk = base + b;
            const double cx = sc.cx[kk], cy = sc.cy[kk], r2 = sc.r2[kk];
            const bool hit = seg_valid && seg_hits_disc(ax, ay, qx, qy, cx, cy, r2);
            if (__any(hit)) return true;
        }
    }
    return false;
}

// Fast path of verify_node for the edge child (x, y, yaw) → parent (px, py, pyaw):
// the Dubins polyline of line_to_origin (rrt.rs:295-315) plus the junction to the parent, whose
// own line was verified when it was inserted.  The word choice and the segment
// origins are wave-uniform; the pd accumulation of generate_local_course (dubins.rs:239-255) is
// replayed uniformly and each lane captures one grid point, so every point carries exactly the
// reference's `pd += d` value; interpolation and the collision test then run lane-parallel.
__device__ int steer_collide_fast(const SceneDev& sc, double x, double y, double yaw, double px,
                                  double py, double pyaw) {
    const int lane = threadIdx.x & 63;
    const double step = sc.step_size;
    // dubins_path_planning, dubins.rs:401-408 (s = child, e = parent)
    const double ex = px - x, ey = py - y;
    const double c = 1.0 / sc.turn_radius;
    const double lex = cos(yaw) * ex + sin(yaw) * ey;
    const double ley = -(sin(yaw)) * ex + cos(yaw) * ey;
    const double leyaw = pyaw - yaw;
    const Steer s = select_word(lex, ley, leyaw, c);
    if (s.word < 0) {
        // steer failed: line_to_origin contributes [(sx, sy)] (rrt.rs:313)
        const bool has = lane < 2;
        const double qx = lane == 0 ? x : px, qy = lane == 0 ? y : py;
        return chunk_rejects(sc, has, lane == 0, lane == 1, qx, qy) ? kReject : kAccept;
    }
    const double L0 = s.t, L1 = s.p, L2 = s.q;
    const int m0 = word_mode(s.word, 0), m1 = word_mode(s.word, 1), m2 = word_mode(s.word, 2);
    double total = 0.0;
    total += L0;
    total += L1;
    total += L2;
    const double nq = trunc(total / step);
    if (!(nq >= 0.0) || nq > 1.0e8) return kError;
    const long n_point = (long)nq + 3 + 4;
    // segment origins = previous segment's endpoint (dubins.rs:230, 258-271)
    const Pose O0{0.0, 0.0, 0.0};
    const Pose O1 = interp_local(m0, L0, c, O0);
    const Pose O2 = interp_local(m1, L1, c, O1);
    const Pose E = interp_local(m2, L2, c, O2);
    // The trim (dubins.rs:281-288) drops exactly the final endpoint unless its local x is 0.0
    // (then it keeps popping) or the array has no trailing zero: both go to the literal path.
    if (E.x == 0.0) return kLiteral;
    const double cw = cos(-yaw), sw = sin(-yaw);

    int seg = 0;
    double dd = (L0 > 0.0) ? step : -step;
    double pd = dd - 0.0;
    long grid = 0;
    double carry_x = x, carry_y = y;  // point 0 of the edge is the child itself
    bool first = true;
    for (;;) {
        int my_seg = 0;
        double my_pd = 0.0;
        int cnt = 0;
        while (cnt < 63 && seg < 3) {
            const double Ls = seg == 0 ? L0 : (seg == 1 ? L1 : L2);
            if (fabs(pd) <= fabs(Ls)) {
                if (lane == cnt + 1) {
                    my_seg = seg;
                    my_pd = pd;
                }
                ++cnt;
                pd += dd;
            } else {
                const double ll = Ls - pd - dd;
                ++seg;
                if (seg < 3) {
                    const double Ln = seg == 1 ? L1 : L2;
                    dd = (Ln > 0.0) ? step : -step;
                    pd = ((Ls * Ln) > 0.0) ? (-dd - ll) : (dd - ll);
                }
            }
        }
        grid += cnt;
        const bool junction_here = (seg >= 3) && cnt < 63;
        double qx = carry_x, qy = carry_y;
        bool has = (lane == 0), isgrid = false;
        if (lane >= 1 && lane <= cnt) {
            const Pose o = my_seg == 0 ? O0 : (my_seg == 1 ? O1 : O2);
            const int mm = my_seg == 0 ? m0 : (my_seg == 1 ? m1 : m2);
            const Pose r = interp_local(mm, my_pd, c, o);
            qx = cw * r.x + sw * r.y + x;   // dubins.rs:415
            qy = -sw * r.x + cw * r.y + y;  // dubins.rs:420
            has = true;
            isgrid = true;
        } else if (junction_here && lane == cnt + 1) {
            qx = px;
            qy = py;
            has = true;
        }
        const bool check_bounds = isgrid || (first && lane == 0);
        if (chunk_rejects(sc, has, check_bounds, has && lane >= 1, qx, qy)) return kReject;
        if (junction_here) break;
        carry_x = __shfl(qx, cnt);
        carry_y = __shfl(qy, cnt);
        first = false;
    }
    if (1 + grid > n_point - 2) return kLiteral;
    return kAccept;
}

// Literal path (measure-zero trim cases): lane 0 runs dubins_literal into its scratch buffer and
// verifies the polyline alone.  Slow, exact, essentially never taken.
__device__ int steer_collide_literal(const SceneDev& sc, double x, double y, double yaw, double px,
                                     double py, double pyaw, double* bx, double* by, double* byaw) {
    const int lane = threadIdx.x & 63;
    int st = kReject;
    if (lane == 0) {
        int n = 0, word = -1;
        double cost = 0.0;
        const int r = dubins_literal(x, y, yaw, px, py, pyaw, sc.turn_radius, sc.step_size, bx,
                                     by, byaw, kLiteralCap - 1, &n, &word, &cost);
        if (r == kSteerOverflow) {
            st = kError;
        } else {
            if (r == kSteerNone) {
                bx[0] = x;
                by[0] = y;
                n = 1;
            }
            bool ok = true;
            for (int i = 0; i < n && ok; ++i)
                ok = bx[i] >= sc.minx && bx[i] <= sc.maxx && by[i] >= sc.miny && by[i] <= sc.maxy;
            bx[n] = px;
            by[n] = py;
            const int np = n + 1;
            double x0 = bx[0], x1 = bx[0], y0 = by[0], y1 = by[0];
            for (int i = 1; i < np; ++i) {
                x0 = fmin(x0, bx[i]);
                x1 = fmax(x1, bx[i]);
                y0 = fmin(y0, by[i]);
                y1 = fmax(y1, by[i]);
            }
            for (int k = 0; k < sc.m && ok; ++k) {
                const double cx = sc.cx[k], cy = sc.cy[k], rc = sc.rcull[k];
                if (!((cx + rc >= x0) && (cx - rc <= x1) && (cy + rc >= y0) && (cy - rc <= y1)))
                    continue;
                for (int i = 0; i + 1 < np && ok; ++i)
                    if (seg_hits_disc(bx[i], by[i], bx[i + 1], by[i + 1], cx, cy, sc.r2[k]))
                        ok = false;
            }
            st = ok ? kAccept : kReject;
        }
    }
    return __shfl(st, 0);
}

// ------------------------------------------------------------------------- steer kernels

// Tasks [0, W): sample j → its snapshot NN (tree node nn_idx[j]).  Tasks [W, W + *ncomp):
// candidate entry e: sample E.j → window sample E.i, with E.i's yaw taken under ITS snapshot
// parent (the speculation the host resolve validates).
__global__ __launch_bounds__(256) void steer_window_kernel(
    SceneDev sc, TreeDev tr, const double* __restrict__ wsx, const double* __restrict__ wsy,
    const int* __restrict__ nn_idx, const CandEntry* __restrict__ cand,
    const int* __restrict__ ncomp, int W, int* __restrict__ snap_status,
    double* __restrict__ snap_yaw, int* __restrict__ spec_status, double* __restrict__ spec_yaw) {
    const int lane = threadIdx.x & 63;
    const int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int nw = (int)((gridDim.x * blockDim.x) >> 6);
    const int total = W + *ncomp;
    for (int t = gw; t < total; t += nw) {
        int j;
        double px, py, pyaw;
        if (t < W) {
            j = t;
            const int p = nn_idx[j];
            px = tr.x[p];
            py = tr.y[p];
            pyaw = tr.yaw[p];
        } else {
            const CandEntry ce = cand[t - W];
            j = ce.j;
            const int ni = nn_idx[ce.i];
            px = wsx[ce.i];
            py = wsy[ce.i];
            pyaw = atan2(tr.y[ni] - py, tr.x[ni] - px);
        }
        const double x = wsx[j], y = wsy[j];
        const double yaw = atan2(py - y, px - x);  // compute_yaw, rrt.rs:267-271
        const int st = steer_collide_fast(sc, x, y, yaw, px, py, pyaw);
        if (lane == 0) {
            if (t < W) {
                snap_status[t] = st;
                snap_yaw[t] = yaw;
            } else {
                spec_status[t - W] = st;
                spec_yaw[t - W] = yaw;
            }
        }
    }
}

// Explicit tasks (repairs, the verify_node API); waves <= kLiteralWaves so each wave owns one
// literal scratch buffer.
__global__ __launch_bounds__(256) void steer_tasks_kernel(SceneDev sc, TreeDev tr,
                                                          const SteerTask* __restrict__ tasks,
                                                          int n, int* __restrict__ out_status,
                                                          double* __restrict__ out_yaw,
                                                          double* __restrict__ scratch) {
    const int lane = threadIdx.x & 63;
    const int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int nw = (int)((gridDim.x * blockDim.x) >> 6);
    double* bx = scratch ? scratch + (size_t)gw * 3 * kLiteralCap : nullptr;
    for (int t = gw; t < n; t += nw) {
        const SteerTask tk = tasks[t];
        double px = tk.px, py = tk.py, pyaw = tk.pyaw;
        if (tk.pnode >= 0) {
            px = tr.x[tk.pnode];
            py = tr.y[tk.pnode];
            pyaw = tr.yaw[tk.pnode];
        }
        const double yaw = atan2(py - tk.y, px - tk.x);
        int st;
        if (tk.literal && bx)
            st = steer_collide_literal(sc, tk.x, tk.y, yaw, px, py, pyaw, bx, bx + kLiteralCap,
                                       bx + 2 * kLiteralCap);
        else if (tk.literal)
            st = kError;
        else
            st = steer_collide_fast(sc, tk.x, tk.y, yaw, px, py, pyaw);
        if (lane == 0) {
            out_status[t] = st;
            out_yaw[t] = yaw;
        }
    }
}

// Space::rand_point for iterations [it0, it0 + W): x = draw 2*it, y = draw 2*it + 1
// (rrt.rs:139-146 on the seeded stream).
__global__ __launch_bounds__(256) void sample_kernel(uint64_t seed, int64_t it0, int W, double minx,
                                                     double maxx, double miny, double maxy,
                                                     double* __restrict__ wsx,
                                                     double* __restrict__ wsy) {
    const int j = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (j >= W) return;
    const uint64_t it = (uint64_t)(it0 + j);
    wsx[j] = gen_range(seed, 2 * it, minx, maxx);
    wsy[j] = gen_range(seed, 2 * it + 1, miny, maxy);
}

// insert (rrt.rs:586-589) of the resolved, accepted window samples, in sequential order
__global__ __launch_bounds__(256) void append_kernel(const CommitEntry* __restrict__ ents, int n_new,
                                                     int n0, const double* __restrict__ wsx,
                                                     const double* __restrict__ wsy,
                                                     const int* __restrict__ nn_idx,
                                                     float* __restrict__ x32,
                                                     float* __restrict__ y32, double* __restrict__ X,
                                                     double* __restrict__ Y,
                                                     double* __restrict__ YAW,
                                                     int* __restrict__ PAR) {
    const int r = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (r >= n_new) return;
    const CommitEntry e = ents[r];
    const int node = n0 + r;
    const double x = wsx[e.j], y = wsy[e.j];
    X[node] = x;
    Y[node] = y;
    x32[node] = (float)x;
    y32[node] = (float)y;
    YAW[node] = e.yaw;
    PAR[node] = e.parent >= 0 ? e.parent : nn_idx[e.j];
}

// --------------------------------------------------------------------------------- dubins

__global__ __launch_bounds__(64) void dubins_batch_kernel(const double* __restrict__ conf, int n,
                                                          int cap, double* __restrict__ px,
                                                          double* __restrict__ py,
                                                          double* __restrict__ pyaw,
                                                          int* __restrict__ n_out,
                                                          int* __restrict__ word_out,
                                                          double* __restrict__ cost_out,
                                                          int* __restrict__ status_out) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const double* c = conf + (size_t)i * 8;
    int np = 0, word = -1;
    double cost = 0.0;
    const int r = dubins_literal(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7],
                                 px + (size_t)i * cap, py + (size_t)i * cap,
                                 pyaw + (size_t)i * cap, cap, &np, &word, &cost);
    n_out[i] = np;
    word_out[i] = word;
    cost_out[i] = cost;
    status_out[i] = r;
}

// ------------------------------------------------------------------------- nearest neighbour

constexpr int kQPL = 4;                // samples per lane
constexpr int kQPB = 64 * kQPL;        // samples per workgroup (all 4 waves share them)

struct Top2 {
    float b, s;
    int i;
};
__device__ inline Top2 merge_top2(Top2 a, Top2 c) {
    Top2 r;
    float other;
    if (c.b < a.b || (c.b == a.b && c.i >= 0 && (a.i < 0 || c.i < a.i))) {
        r.b = c.b;
        r.i = c.i;
        other = a.b;
    } else {
        r.b = a.b;
        r.i = a.i;
        other = c.b;
    }
    r.s = fminf(fminf(a.s, c.s), other);
    return r;
}

// grid (ceil(nq / 256), n_chunks), 256 threads.  Each wave scans a quarter of the chunk; tree
// coordinates are wave-uniform loads (scalar cache, broadcast as SGPR operands) and every lane
// holds 4 samples, so one node feeds 4 distance evaluations per lane.
__global__ __launch_bounds__(256) void nn_scan_kernel(const float* __restrict__ nx,
                                                      const float* __restrict__ ny, int n_nodes,
                                                      const double* __restrict__ qx,
                                                      const double* __restrict__ qy, int nq,
                                                      int chunk_len, int stride,
                                                      float* __restrict__ pbest,
                                                      float* __restrict__ psecond,
                                                      int* __restrict__ pidx) {
    __shared__ float s_b[4][kQPB];
    __shared__ float s_s[4][kQPB];
    __shared__ int s_i[4][kQPB];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int qbase = blockIdx.x * kQPB;
    float qxr[kQPL], qyr[kQPL], best[kQPL], second[kQPL];
    int bi[kQPL];
#pragma unroll
    for (int r = 0; r < kQPL; ++r) {
        const int q = qbase + r * 64 + lane;
        qxr[r] = q < nq ? (float)qx[q] : 0.0f;
        qyr[r] = q < nq ? (float)qy[q] : 0.0f;
        best[r] = __builtin_inff();
        second[r] = __builtin_inff();
        bi[r] = -1;
    }
    const int c0 = blockIdx.y * chunk_len;
    const int c1 = min(c0 + chunk_len, n_nodes);
    const int per = (((c1 - c0) + 3) / 4 + 7) & ~7;
    // wave-uniform range: readfirstlane lets the compiler use scalar loads for the nodes
    const int w0 = __builtin_amdgcn_readfirstlane(min(c0 + wave * per, c1));
    const int w1 = __builtin_amdgcn_readfirstlane(min(w0 + per, c1));
    int k = w0;
    for (; k + 8 <= w1; k += 8) {
        float px[8], py[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            px[u] = nx[k + u];
            py[u] = ny[k + u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
#pragma unroll
            for (int r = 0; r < kQPL; ++r) {
                const float dx = qxr[r] - px[u];
                const float dy = qyr[r] - py[u];
                const float d = __builtin_fmaf(dy, dy, dx * dx);
                second[r] = __builtin_amdgcn_fmed3f(best[r], d, second[r]);
                if (d < best[r]) {
                    best[r] = d;
                    bi[r] = k + u;
                }
            }
        }
    }
    for (; k < w1; ++k) {
        const float px = nx[k], py = ny[k];
#pragma unroll
        for (int r = 0; r < kQPL; ++r) {
            const float dx = qxr[r] - px;
            const float dy = qyr[r] - py;
            const float d = __builtin_fmaf(dy, dy, dx * dx);
            second[r] = __builtin_amdgcn_fmed3f(best[r], d, second[r]);
            if (d < best[r]) {
                best[r] = d;
                bi[r] = k;
            }
        }
    }
#pragma unroll
    for (int r = 0; r < kQPL; ++r) {
        s_b[wave][r * 64 + lane] = best[r];
        s_s[wave][r * 64 + lane] = second[r];
        s_i[wave][r * 64 + lane] = bi[r];
    }
    __syncthreads();
    // wave w merges sample group r = w across the 4 waves (ascending node ranges)
    const int slot = wave * 64 + lane;
    Top2 t{s_b[0][slot], s_s[0][slot], s_i[0][slot]};
#pragma unroll
    for (int w = 1; w < 4; ++w) t = merge_top2(t, Top2{s_b[w][slot], s_s[w][slot], s_i[w][slot]});
    const int q = qbase + slot;
    if (q < nq) {
        const size_t o = (size_t)blockIdx.y * stride + q;
        pbest[o] = t.b;
        psecond[o] = t.s;
        pidx[o] = t.i;
    }
}

// one thread per sample: merge chunk partials, decide whether the f32 winner is certainly the
// exact f64 winner (margin test against the f32 rounding bound), else queue an exact rescan.
__global__ __launch_bounds__(256) void nn_finalize_kernel(
    const float* __restrict__ pbest, const float* __restrict__ psecond,
    const int* __restrict__ pidx, int n_chunks, int stride, int nq, const double* __restrict__ qx,
    const double* __restrict__ qy, const double* __restrict__ X, const double* __restrict__ Y,
    double eps_coord, int* __restrict__ out_idx, double* __restrict__ out_d2,
    int* __restrict__ flag_list, int* __restrict__ flag_count) {
    const int q = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (q >= nq) return;
    Top2 t{pbest[q], psecond[q], pidx[q]};
    for (int c = 1; c < n_chunks; ++c) {
        const size_t o = (size_t)c * stride + q;
        t = merge_top2(t, Top2{pbest[o], psecond[o], pidx[o]});
    }
    bool flag = t.i < 0 || !(t.b < __builtin_inff());
    if (!flag && t.s < __builtin_inff()) {
        const double D1 = sqrt((double)t.b), D2 = sqrt((double)t.s);
        const double tau = 8.0 * eps_coord + 1.0e-6 * D2;
        flag = !(D2 - D1 > tau);
    }
    if (flag) {
        const int e = atomicAdd(flag_count, 1);
        flag_list[e] = q;
        out_idx[q] = -1;
    } else {
        const double dx = qx[q] - X[t.i], dy = qy[q] - Y[t.i];
        out_idx[q] = t.i;
        out_d2[q] = dx * dx + dy * dy;
    }
}

// exact f64 brute force (lowest index wins ties) for the flagged samples; grid-stride over the
// flagged list, one workgroup per sample.
__global__ __launch_bounds__(256) void nn_rescan_kernel(const int* __restrict__ flag_list,
                                                        const int* __restrict__ flag_count,
                                                        const double* __restrict__ qx,
                                                        const double* __restrict__ qy,
                                                        const double* __restrict__ X,
                                                        const double* __restrict__ Y, int n,
                                                        int* __restrict__ out_idx,
                                                        double* __restrict__ out_d2) {
    __shared__ double s_d[256];
    __shared__ int s_i[256];
    const int cnt = *flag_count;
    for (int e = blockIdx.x; e < cnt; e += gridDim.x) {
        const int q = flag_list[e];
        const double x = qx[q], y = qy[q];
        double best = __builtin_inf();
        int bi = 0x7fffffff;
        for (int k = threadIdx.x; k < n; k += 256) {
            const double dx = x - X[k], dy = y - Y[k];
            const double d2 = dx * dx + dy * dy;
            if (d2 < best) {
                best = d2;
                bi = k;
            }
        }
        s_d[threadIdx.x] = best;
        s_i[threadIdx.x] = bi;
        __syncthreads();
        for (int h = 128; h > 0; h >>= 1) {
            if ((int)threadIdx.x < h) {
                const double od = s_d[threadIdx.x + h];
                const int oi = s_i[threadIdx.x + h];
                if (od < s_d[threadIdx.x] || (od == s_d[threadIdx.x] && oi < s_i[threadIdx.x])) {
                    s_d[threadIdx.x] = od;
                    s_i[threadIdx.x] = oi;
                }
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            out_idx[q] = s_i[0];
            out_d2[q] = s_d[0];
        }
        __syncthreads();
    }
}

// one wave per sample j: the earlier window samples i < j with d2(j, i) < D2_j (its snapshot
// NN's squared distance).  cand_cnt[j] is the exact count; the first kCandCap of them (ascending
// i) are appended to the compact list `cand` (slots reserved with one atomic per sample).
__global__ __launch_bounds__(256) void window_pairs_kernel(const double* __restrict__ wsx,
                                                           const double* __restrict__ wsy,
                                                           const double* __restrict__ nn_d2, int W,
                                                           int* __restrict__ cand_cnt,
                                                           CandEntry* __restrict__ cand,
                                                           int* __restrict__ ncomp) {
    const int lane = threadIdx.x & 63;
    const int j = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    if (j >= W) return;
    const double x = wsx[j], y = wsy[j], D2 = nn_d2[j];
    int cnt = 0;
    for (int base = 0; base < j; base += 64) {
        const int i = base + lane;
        bool hit = false;
        if (i < j) {
            const double dx = x - wsx[i], dy = y - wsy[i];
            hit = dx * dx + dy * dy < D2;
        }
        cnt += __popcll(__ballot(hit));
    }
    if (cnt == 0) {
        if (lane == 0) cand_cnt[j] = 0;
        return;
    }
    const int keep = cnt < kCandCap ? cnt : kCandCap;
    int slot0 = 0;
    if (lane == 0) slot0 = atomicAdd(ncomp, keep);
    slot0 = __shfl(slot0, 0);
    int w = 0;
    for (int base = 0; base < j && w < keep; base += 64) {
        const int i = base + lane;
        bool hit = false;
        double d2 = 0.0;
        if (i < j) {
            const double dx = x - wsx[i], dy = y - wsy[i];
            d2 = dx * dx + dy * dy;
            hit = d2 < D2;
        }
        const unsigned long long mask = __ballot(hit);
        if (hit) {
            const int pos = w + __popcll(mask & ((1ull << lane) - 1ull));
            if (pos < keep) cand[slot0 + pos] = CandEntry{j, i, d2};
        }
        w += __popcll(mask);
    }
    if (lane == 0) cand_cnt[j] = cnt;
}

// --------------------------------------------------------------------------- launch wrappers

hipError_t launch_nn(hipStream_t st, const TreeDev& tr, const double* qx, const double* qy,
                     int nq, int stride, float* pbest, float* psecond, int* pidx, double eps_coord,
                     int* out_idx, double* out_d2, int* flag_list, int* flag_count,
                     hipEvent_t ev_scan0, hipEvent_t ev_scan1) {
    if (nq <= 0) return hipSuccess;
    const int n = tr.n;
    int chunk_len = (n + kMaxChunks - 1) / kMaxChunks;
    if (chunk_len < 512) chunk_len = 512;
    chunk_len = (chunk_len + 31) & ~31;
    const int n_chunks = (n + chunk_len - 1) / chunk_len;
    hipError_t e = hipMemsetAsync(flag_count, 0, sizeof(int), st);
    if (e != hipSuccess) return e;
    dim3 g1((nq + kQPB - 1) / kQPB, n_chunks);
    if (ev_scan0) (void)hipEventRecord(ev_scan0, st);
    nn_scan_kernel<<<g1, 256, 0, st>>>(tr.x32, tr.y32, n, qx, qy, nq, chunk_len, stride, pbest,
                                       psecond, pidx);
    if (ev_scan1) (void)hipEventRecord(ev_scan1, st);
    nn_finalize_kernel<<<(nq + 255) / 256, 256, 0, st>>>(pbest, psecond, pidx, n_chunks, stride,
                                                         nq, qx, qy, tr.x, tr.y, eps_coord,
                                                         out_idx, out_d2, flag_list, flag_count);
    const int g3 = nq < 256 ? nq : 256;
    nn_rescan_kernel<<<g3, 256, 0, st>>>(flag_list, flag_count, qx, qy, tr.x, tr.y, n, out_idx,
                                         out_d2);
    return hipGetLastError();
}

hipError_t launch_pairs(hipStream_t st, const double* wsx, const double* wsy, const double* nn_d2,
                        int W, int* cand_cnt, CandEntry* cand, int* ncomp) {
    if (W <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(ncomp, 0, sizeof(int), st);
    if (e != hipSuccess) return e;
    window_pairs_kernel<<<(W + 3) / 4, 256, 0, st>>>(wsx, wsy, nn_d2, W, cand_cnt, cand, ncomp);
    return hipGetLastError();
}

hipError_t launch_steer_window(hipStream_t st, const SceneDev& sc, const TreeDev& tr,
                               const double* wsx, const double* wsy, const int* nn_idx,
                               const CandEntry* cand, const int* ncomp, int W, int* snap_status,
                               double* snap_yaw, int* spec_status, double* spec_yaw) {
    if (W <= 0) return hipSuccess;
    // one wave per snapshot task; the (few) candidate tasks are picked up by the grid-stride loop
    int waves = W;
    if (waves > 16384) waves = 16384;
    steer_window_kernel<<<(waves + 3) / 4, 256, 0, st>>>(sc, tr, wsx, wsy, nn_idx, cand, ncomp, W,
                                                         snap_status, snap_yaw, spec_status,
                                                         spec_yaw);
    return hipGetLastError();
}

hipError_t launch_steer_tasks(hipStream_t st, const SceneDev& sc, const TreeDev& tr,
                              const SteerTask* tasks, int n, int* out_status, double* out_yaw,
                              double* scratch) {
    if (n <= 0) return hipSuccess;
    int waves = n;
    if (scratch && waves > kLiteralWaves) waves = kLiteralWaves;
    if (waves > 16384) waves = 16384;
    steer_tasks_kernel<<<(waves + 3) / 4, 256, 0, st>>>(sc, tr, tasks, n, out_status, out_yaw,
                                                        scratch);
    return hipGetLastError();
}

hipError_t launch_sample(hipStream_t st, uint64_t seed, int64_t it0, int W, double minx,
                         double maxx, double miny, double maxy, double* wsx, double* wsy) {
    if (W <= 0) return hipSuccess;
    sample_kernel<<<(W + 255) / 256, 256, 0, st>>>(seed, it0, W, minx, maxx, miny, maxy, wsx, wsy);
    return hipGetLastError();
}

hipError_t launch_append(hipStream_t st, const CommitEntry* ents, int n_new, int n0,
                         const double* wsx, const double* wsy, const int* nn_idx, float* x32,
                         float* y32, double* X, double* Y, double* YAW, int* PAR) {
    if (n_new <= 0) return hipSuccess;
    append_kernel<<<(n_new + 255) / 256, 256, 0, st>>>(ents, n_new, n0, wsx, wsy, nn_idx, x32, y32,
                                                       X, Y, YAW, PAR);
    return hipGetLastError();
}

hipError_t launch_dubins_batch(hipStream_t st, const double* conf, int n, int cap, double* px,
                               double* py, double* pyaw, int* n_out, int* word_out,
                               double* cost_out, int* status_out) {
    if (n <= 0) return hipSuccess;
    dubins_batch_kernel<<<(n + 63) / 64, 64, 0, st>>>(conf, n, cap, px, py, pyaw, n_out, word_out,
                                                      cost_out, status_out);
    return hipGetLastError();
}

}  // namespace ppamd
