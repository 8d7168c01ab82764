// pp_kernels.hip — hand-written CDNA4 (gfx950) kernels of the RRT extend hot path.
//
// Window pipeline (one speculative window of K iterations, device-resident state):
//   window_samples Space::rand_point for the window's iterations (seeded stream), Morton-sorted
//                  (the first window of a batch; later ones come from nn_finalize) rrt.rs:139-146
//   window_kernel  workgroups 1..: the NN screen, K samples x N tree nodes, f32 SoA, expanded form
//                  about each sample block's centre, scalar-broadcast nodes, 4 samples per lane,
//                  exact per-chunk top-2, XCD-aware mapping                          rrt.rs:378-391
//                  workgroup 0: resolve + commit of the previous window (sequential-consistency
//                  replay, repairs inline, in-order insert)                          rrt.rs:414-426
//   nn_finalize    merge the chunk partials and the appended nodes, exact f64 d2 of the winner,
//                  near-ties decided exactly (wave, or workgroup brute force), window pairs
//                  (earlier samples nearer than the snapshot NN), next window's samples
//   steer_prep     8 lanes per (sample, parent): compute_yaw + Dubins word + grid-point distances
//   steer_walk     one wave per task: sampled-arc polyline, bounds + disc collision, f64
//                                                               rrt.rs:169-175,414-426, dubins.rs
// API kernels: steer_tasks (verify_node batch), nn_fix (nearest batch), dubins_batch.
//
// No MFMA anywhere: there is no dense contraction on this path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

#include "pp_device.h"
#include "pp_kernels.h"

namespace ppamd {

typedef __attribute__((address_space(3))) void lds_void;  // LDS-DMA operands
typedef __attribute__((address_space(1))) void glb_void;

// ------------------------------------------------------------------------------ collision

// One 64-point chunk of a polyline, one point per lane: bounds for the lanes flagged
// `check_bounds`, then the segment (lane-1 → lane) of every lane flagged `seg_valid` against the
// discs listed in the grid cells the chunk's bounding box touches (Space::verify,
// rrt.rs:124-137, Q10).  A disc whose cull box meets the chunk's box shares a cell with it (the
// cell index is monotone in the coordinate), so the cull is exact.  Must be called by all 64
// lanes.  Returns true when the chunk rejects the line.
// (the clamp in the integer domain: v_cvt_i32_f64 saturates — NaN gives 0 — so no f64 bound has
// to stay live in the walk's registers; the same cell as clamping the double)
__device__ inline int grid_cell(double v, double v0, double inv, int n) {
    const double f = floor((v - v0) * inv);
    int i;
    asm("v_cvt_i32_f64 %0, %1" : "=v"(i) : "v"(f));
    return min(max(i, 0), n - 1);
}

// Dynamic LDS of the steer kernels: the scene image (SceneDev::lds_*) when kLds.
extern __shared__ __attribute__((aligned(16))) char pp_smem[];

// Copy the scene's LDS image (disc grid + discs, or the occupancy bits) into this workgroup's LDS
// (all threads call it): 16-byte words, 8 loads in flight per thread before their stores.
__device__ inline void stage_scene(const SceneDev& sc) {
    constexpr int U = 8;
    const int n16 = sc.lds_bytes >> 4;
    uint4* dst = reinterpret_cast<uint4*>(pp_smem);
    const int nt = blockDim.x;
    for (int base = threadIdx.x; base < n16; base += nt * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {  // unconditional (clamped) loads: all U stay in flight
            const int k = min(base + u * nt, n16 - 1);
            v[u] = sc.img[k];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = base + u * nt;
            if (k < n16) dst[k] = v[u];
        }
    }
    __syncthreads();
}

// The scene modes a walk can be compiled for: kSceneAny tests the SceneDev fields at run time;
// the others drop the code (and the kernel-argument registers) of the modes they exclude.
enum : int { kSceneAny = 0, kSceneDisc = 1, kSceneGrid = 2, kScenePoly = 3 };
__host__ __device__ inline int scene_kind(const SceneDev& sc) {
    if (sc.bits) return kSceneGrid;
    if (sc.ne > 0 || sc.nbv > 0) return kScenePoly;
    return kSceneDisc;
}

// box: the lane's point bounds the chunk's item search (default: every lane with a point; the
// walk leaves out lane 0 when its segment 0 -> 1 is an analytically cleared S chord, which is not
// tested, so the box need not cover it)
template <bool kLds, int kScene = kSceneAny>
__device__ __forceinline__ bool chunk_rejects(const SceneDev& sc, bool has, bool check_bounds,
                                              bool seg_valid, double qx, double qy,
                                              bool box = true) {
    bool oob =
        check_bounds && !(qx >= sc.minx && qx <= sc.maxx && qy >= sc.miny && qy <= sc.maxy);
    if (__any(oob)) return true;
    if ((kScene == kSceneAny || kScene == kScenePoly) && sc.nbv > 0) {
        // polygon bounds (Q10p): the eroded ring, per lane over every bounds edge
        oob = check_bounds && !in_poly_bounds(sc.nbv, sc.bvx, sc.bvy, sc.h2, qx, qy);
        if (__any(oob)) return true;
    }
    if (kScene == kSceneGrid || (kScene == kSceneAny && sc.bits)) {
        // config 4: every point of the line probes its cell (1 bit), no segments
        const uint32_t* B = kLds ? reinterpret_cast<const uint32_t*>(pp_smem) : sc.bits;
        const bool hit = check_bounds && grid_occupied(B, sc.bw, sc.bh, sc.bwords, sc.bx0, sc.by0,
                                                       sc.binv, qx, qy);
        return __any(hit);
    }
    if (kScene == kSceneDisc ? sc.m == 0
                             : (kScene == kScenePoly ? sc.ne == 0 : (sc.m == 0 && sc.ne == 0)))
        return false;
    // grid items are polygon edges (Q10p), else discs
    const bool poly = kScene == kScenePoly || (kScene == kSceneAny && sc.ne > 0);
    // the chunk's bounding box in f32, rounded outward (DPP reductions): a box that contains the
    // points selects a superset of the cells and items, and the exact test below decides
    const double ax = shfl_up1_f64(qx);
    const double ay = shfl_up1_f64(qy);
    const float inff = __builtin_inff();
    const bool inb = has && box;
    const float bx0 = wave_min_f32(inb ? f32_below(qx) : inff);
    const float bx1 = wave_max_f32(inb ? f32_above(qx) : -inff);
    const float by0 = wave_min_f32(inb ? f32_below(qy) : inff);
    const float by1 = wave_max_f32(inb ? f32_above(qy) : -inff);
    const int cx0 = __builtin_amdgcn_readfirstlane(grid_cell(bx0, sc.gx0, sc.ginv, sc.gnx));
    const int cx1 = __builtin_amdgcn_readfirstlane(grid_cell(bx1, sc.gx0, sc.ginv, sc.gnx));
    const int cy0 = __builtin_amdgcn_readfirstlane(grid_cell(by0, sc.gy0, sc.ginv, sc.gny));
    const int cy1 = __builtin_amdgcn_readfirstlane(grid_cell(by1, sc.gy0, sc.ginv, sc.gny));
    const int* goff = kLds ? reinterpret_cast<const int*>(pp_smem + sc.lds_goff) : sc.goff;
    const int* items = kLds ? reinterpret_cast<const int*>(pp_smem + sc.lds_items) : sc.gitems;
    const double* dcx = sc.cx;  // exact test: f64 discs from global memory (L2)
    const double* dcy = sc.cy;
    const double* dr2 = sc.r2;
    // the cull discs are in the LDS image too unless the scene only fit without them (lds_d4 < 0)
    const float4* d4 = (kLds && sc.lds_d4 >= 0)
                           ? reinterpret_cast<const float4*>(pp_smem + sc.lds_d4)
                           : sc.d4;
    // per-lane f32 cull: a segment a-b can only touch a disc / an edge buffer (exact test below)
    // if |a - c| <= rcull + |b - a| (c: the disc centre / the edge midpoint, rcull: the radius /
    // half length + h); cull_slack covers the f32 rounding of the scene's coordinates
    const float axf = (float)ax, ayf = (float)ay;
    const float vxf = (float)(qx - ax), vyf = (float)(qy - ay);
    const float l2f = vxf * vxf + vyf * vyf;
    const float Lf = __builtin_sqrtf(l2f) * 1.000001f + sc.cull_slack;
    // the closest-point parameter below uses 1 / |b - a|^2 (one reciprocal per lane and chunk, not
    // a division per item): t is only approximate anyway — any t in [0, 1] gives a point of the
    // segment, so "surely within" stays exact, and the error of "surely clear" is second order in
    // the error of t (t minimises the distance), far inside the band
    const float il2f = l2f > 0.0f ? __builtin_amdgcn_rcpf(l2f) : 0.0f;
    // the chunk's bbox in f32, widened by the rounding slack: an item whose cull disc misses it
    // cannot meet any of the chunk's segments
    const int lane = __lane_id();
    const float bxl = (float)bx0 - sc.cull_slack, bxh = (float)bx1 + sc.cull_slack;
    const float byl = (float)by0 - sc.cull_slack, byh = (float)by1 + sc.cull_slack;
    // up to 64 items in parallel, one per lane (kk: its index in the item list, valid: a lane with
    // an item): the cull disc against the chunk's bbox, then the survivors against every lane's
    // segment, one at a time
    auto items_reject = [&](bool valid, int kk) -> bool {
        int dl = 0;
        float4 Dl = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        bool ov = false;
        if (valid) {
            dl = items[kk];
            Dl = d4[dl];
            ov = Dl.x + Dl.z >= bxl && Dl.x - Dl.z <= bxh && Dl.y + Dl.z >= byl && Dl.y - Dl.z <= byh;
        }
        for (uint64_t m = __ballot(ov); m; m &= m - 1) {
            const int src = (int)__builtin_ctzll(m);
            const int d = __builtin_amdgcn_readlane(dl, src);
            float4 D;
            D.x = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, Dl.x), src));
            D.y = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, Dl.y), src));
            D.z = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, Dl.z), src));
            D.w = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, Dl.w), src));
            const float dxf = D.x - axf, dyf = D.y - ayf, thr = D.z + Lf;
            bool near = seg_valid && dxf * dxf + dyf * dyf <= thr * thr;
            if (!__any(near)) continue;
            if (!poly) {
                // f32 closest point of the segment to the disc centre, decisive outside a band of
                // +-eps around the radius (eps bounds the f32 rounding of the coordinates, the
                // radius and this arithmetic): only the band needs the exact f64 test and its
                // global loads
                const float t =
                    __builtin_fminf(__builtin_fmaxf((dxf * vxf + dyf * vyf) * il2f, 0.0f), 1.0f);
                const float ex = dxf - t * vxf, ey = dyf - t * vyf;
                const float e2 = ex * ex + ey * ey;
                const float eps = sc.cull_slack + 1.0e-4f * (1.0f + thr);
                const float lo = __builtin_fmaxf(D.w - eps, 0.0f), hi = D.w + eps;
                if (__any(near && e2 < lo * lo)) return true;  // surely within the disc
                near = near && e2 <= hi * hi;                  // else surely clear
                if (!__any(near)) continue;
            }
            const bool hit =
                near && (poly ? seg_hits_edge(ax, ay, qx, qy, sc.ex0[d], sc.ey0[d], sc.ex1[d],
                                              sc.ey1[d], sc.h2)
                              : seg_hits_disc(ax, ay, qx, qy, dcx[d], dcy[d], dr2[d]));
            if (__any(hit)) return true;
        }
        return false;
    };
    const int ncx = cx1 - cx0 + 1, ncy = cy1 - cy0 + 1;
    if (ncx <= 0 || ncy <= 0) return false;
    if (ncx * ncy <= 64) {
        // every cell of the box at once: lane c reads cell c's item range (one LDS round trip
        // instead of one per cell), then the cells' item lists are dealt out to the lanes as one
        // list (a cell's items follow the previous cell's), 64 at a time — the result is an OR
        // over (item, segment) pairs, so the order does not matter
        const int ncell = ncx * ncy;
        int k0v = 0, cntv = 0;
        if (lane < ncell) {
            const int ry = lane / ncx;
            const int cell = (cy0 + ry) * sc.gnx + cx0 + (lane - ry * ncx);
            k0v = goff[cell];
            cntv = goff[cell + 1] - k0v;
        }
        for (int mb = 0;; mb += 64) {
            const int m = mb + lane;
            int kk = -1, run = 0;
            for (int c = 0; c < ncell; ++c) {
                const int b = __builtin_amdgcn_readlane(k0v, c), n = __builtin_amdgcn_readlane(cntv, c);
                if (m >= run && m < run + n) kk = b + (m - run);
                run += n;
            }
            if (items_reject(kk >= 0, kk)) return true;
            if (mb + 64 >= run) break;
        }
        return false;
    }
    for (int gy = cy0; gy <= cy1; ++gy) {
        for (int gx = cx0; gx <= cx1; ++gx) {
            const int cell = gy * sc.gnx + gx;
            const int k0 = goff[cell], k1 = goff[cell + 1];
            for (int kb = k0; kb < k1; kb += 64)
                if (items_reject(kb + lane < k1, kb + lane)) return true;
        }
    }
    return false;
}

// ------------------------------------------------ straight segments, analytically (round 4)
//
// The S segment of LSL / LSR / RSL / RSR (segment 1) puts its grid points at A + (pd / c) u: A
// its origin, u its world direction, pd the generator's values (interpolate's S branch and the
// world transform, dubins.rs:168-171, 412-422), up to a few ulps of the coordinates (< 1e-12
// relative).  Against the discs of a Q10 scene, with dl = 1e-9 (1 + |A| + |B|) far above that
// rounding:
//   kSClear    every disc centre lies farther than r + dl from the ideal segment AB, and A, B lie
//              dl inside the bounds: every S point and every polyline segment between two S
//              points then lies farther than r from every centre and inside the bounds, so the
//              walk keeps only the first and the last S point (the chord between them clears
//              too) — the verdict is the one of the full polyline;
//   kSHit      some disc's (r - dl) chord on AB, clipped to the stretch the S points surely
//              cover (from 3d past A: the first pd is at most 3d, dubins.rs:239-241; to d
//              before B), is longer than the points' spacing: an S point lies strictly inside
//              the disc, and verify rejects (rrt.rs:124-137) whatever the other segments;
//   kSUnknown  otherwise: the walk tests every point.
// The discs come from the item grid's cells within dl of AB, row by row: lane r takes row
// cy0 + r, clips AB to the row's band (widened by dl; the edge rows extend to infinity, as the
// grid clamps), and the cells of that stretch (widened by dl) are one contiguous item range of
// the row-major CSR.  A disc within r + dl of AB has its cull box (>= r) within dl of AB, so in
// one of those cells.  Called by all 64 lanes; returns a wave-uniform class.
enum : int { kSUnknown = 0, kSClear = 1, kSHit = 2 };
constexpr int kSMinPts = 64;  // S segments shorter than this many points are walked as they are
template <bool kLds>
__device__ int s_classify(const SceneDev& sc, double ax, double ay, double bx, double by,
                          double t_lo, double t_hi, double gap, double dl) {
    const int lane = __lane_id();
    const double ux0 = bx - ax, uy0 = by - ay;
    const double len = sqrt(ux0 * ux0 + uy0 * uy0);
    if (!(len > 0.0)) return kSUnknown;
    const double ux = ux0 / len, uy = uy0 / len;
    int res = (fmin(ax, bx) >= sc.minx + dl && fmax(ax, bx) <= sc.maxx - dl &&
               fmin(ay, by) >= sc.miny + dl && fmax(ay, by) <= sc.maxy - dl)
                  ? kSClear
                  : kSUnknown;
    const int cy0 = __builtin_amdgcn_readfirstlane(grid_cell(fmin(ay, by) - dl, sc.gy0, sc.ginv, sc.gny));
    const int cy1 = __builtin_amdgcn_readfirstlane(grid_cell(fmax(ay, by) + dl, sc.gy0, sc.ginv, sc.gny));
    const int ny = cy1 - cy0 + 1;
    if (ny > 64) return kSUnknown;
    const int* goff = kLds ? reinterpret_cast<const int*>(pp_smem + sc.lds_goff) : sc.goff;
    const int* items = kLds ? reinterpret_cast<const int*>(pp_smem + sc.lds_items) : sc.gitems;
    int k0v = 0, cntv = 0;
    if (lane < ny) {
        const int gy = cy0 + lane;
        const double cell = sc.gcell;
        const double ylo = gy == 0 ? -__builtin_inf() : sc.gy0 + gy * cell - dl;
        const double yhi = gy == sc.gny - 1 ? __builtin_inf() : sc.gy0 + (gy + 1) * cell + dl;
        double t0 = 0.0, t1 = 1.0;
        if (uy0 != 0.0) {
            double ta = (ylo - ay) / uy0, tb = (yhi - ay) / uy0;
            if (ta > tb) {
                const double tt = ta;
                ta = tb;
                tb = tt;
            }
            t0 = fmax(t0, ta);
            t1 = fmin(t1, tb);
        } else if (!(ay >= ylo && ay <= yhi)) {
            t1 = -1.0;
        }
        if (t0 <= t1) {
            const double xa = ax + t0 * ux0, xb = ax + t1 * ux0;
            const int ca = grid_cell(fmin(xa, xb) - dl, sc.gx0, sc.ginv, sc.gnx);
            const int cb = grid_cell(fmax(xa, xb) + dl, sc.gx0, sc.ginv, sc.gnx);
            k0v = goff[gy * sc.gnx + ca];
            cntv = goff[gy * sc.gnx + cb + 1] - k0v;
        }
    }
    // the rows' item ranges dealt to the lanes as one list, 64 at a time (a disc listed in
    // several cells is tested several times).  Each disc is tested in f32 from its cull record
    // (LDS when the image holds it: no f64 loads, no f64 square roots), with margins that make
    // both answers conservative.  e = 2 cull_slack bounds the f32 error of a distance or of a
    // projection t here (cull_slack covers the rounding of the scene's coordinates, both ends
    // of a difference, both axes), and of D.w = fl(r + width / 2):
    //  - near: the f32 distance to AB within D.w + dl + 2e — every disc truly within r + dl;
    //  - hit: the f32 chord of radius ri = D.w - dl - 2e (<= the exact r - dl - e), shortened by
    //    e at each end, lies inside the exact (r - dl) chord, so its overlap with [t_lo, t_hi]
    //    of at least gap + 2e is an exact one of at least gap: an S point lies in the disc.
    // A disc the f32 test cannot decide either way only costs the walk its points (kSUnknown).
    const float4* d4 = (kLds && sc.lds_d4 >= 0)
                           ? reinterpret_cast<const float4*>(pp_smem + sc.lds_d4)
                           : sc.d4;
    const float e = 2.0f * sc.cull_slack;
    const float axf = (float)ax, ayf = (float)ay, uxf = (float)ux, uyf = (float)uy;
    const float lenf = (float)len, dlf = (float)dl;
    const float t_lof = (float)t_lo, t_hif = (float)t_hi, gapf = (float)gap + 2.0f * e;
    for (int mb = 0;; mb += 64) {
        const int m = mb + lane;
        int kk = -1, run = 0;
        for (int r = 0; r < ny; ++r) {
            const int b = __builtin_amdgcn_readlane(k0v, r), n = __builtin_amdgcn_readlane(cntv, r);
            if (m >= run && m < run + n) kk = b + (m - run);
            run += n;
        }
        bool near = false, hit = false;
        if (kk >= 0) {
            const float4 D = d4[items[kk]];
            const float wx = D.x - axf, wy = D.y - ayf;
            const float t = wx * uxf + wy * uyf;
            const float tc = __builtin_fminf(__builtin_fmaxf(t, 0.0f), lenf);
            const float ex = wx - tc * uxf, ey = wy - tc * uyf;
            const float ro = D.w + dlf + 2.0f * e;
            near = ex * ex + ey * ey <= ro * ro;
            const float px = wx - t * uxf, py = wy - t * uyf;
            const float p2 = px * px + py * py, ri = D.w - dlf - 2.0f * e;
            if (ri > 0.0f && p2 < ri * ri) {
                const float h = __builtin_sqrtf(ri * ri - p2) - e;
                hit = __builtin_fminf(t + h, t_hif) - __builtin_fmaxf(t - h, t_lof) >= gapf;
            }
        }
        if (__any(hit)) return kSHit;
        if (__any(near)) res = kSUnknown;
        if (mb + 64 >= run) break;
    }
    return res;
}

// Squared distance of the closed segments a-b and e0-e1: 0 when they cross properly, else the
// nearest endpoint-to-segment distance (the seg_hits_edge predicate as a distance).
__device__ __forceinline__ double seg_seg_d2(double ax, double ay, double bx, double by,
                                             double e0x, double e0y, double e1x, double e1y) {
    const double d1 = (e1x - e0x) * (ay - e0y) - (e1y - e0y) * (ax - e0x);
    const double d2 = (e1x - e0x) * (by - e0y) - (e1y - e0y) * (bx - e0x);
    const double d3 = (bx - ax) * (e0y - ay) - (by - ay) * (e0x - ax);
    const double d4 = (bx - ax) * (e1y - ay) - (by - ay) * (e1x - ax);
    if (((d1 > 0.0 && d2 < 0.0) || (d1 < 0.0 && d2 > 0.0)) &&
        ((d3 > 0.0 && d4 < 0.0) || (d3 < 0.0 && d4 > 0.0)))
        return 0.0;
    return fmin(fmin(seg_point_d2(e0x, e0y, e1x, e1y, ax, ay), seg_point_d2(e0x, e0y, e1x, e1y, bx, by)),
                fmin(seg_point_d2(ax, ay, bx, by, e0x, e0y), seg_point_d2(ax, ay, bx, by, e1x, e1y)));
}

// s_classify for polygon scenes (Q10p, round 5).  The S points lie within dl of AB and the
// polyline through them stays within dl of AB (the dl-neighbourhood of a segment is convex), and
// covers AB's stretch [t_lo, t_hi] continuously (its points advance monotonically along u).  So:
//   kSClear    A, B dl inside the rectangle; every bounds-ring edge farther than h + dl from AB
//              and A inside the ring (then every S point is inside and farther than h from the
//              ring: in_poly_bounds holds); every obstacle edge farther than h + dl from AB (no
//              polyline segment between S points comes within h: seg_hits_edge is false);
//   kSHit      some obstacle edge comes within h - 3 dl of the stretch [t_lo, t_hi]: the polyline
//              segment spanning the nearest point passes within h - 2 dl, so seg_hits_edge holds
//              for it and verify rejects (rrt.rs:124-137) whatever the other segments;
//   kSUnknown  otherwise.  (The bounds ring tests points only, so it never gives a sure hit.)
// The edges come from the item grid exactly as s_classify's discs: an edge within h + dl of AB
// has a point of its cull box (its h-neighbourhood) within dl of AB.  Wave-uniform result.
template <bool kLds>
__device__ int s_classify_poly(const SceneDev& sc, double ax, double ay, double bx, double by,
                               double t_lo, double t_hi, double dl) {
    const int lane = __lane_id();
    const double ux0 = bx - ax, uy0 = by - ay;
    const double len = sqrt(ux0 * ux0 + uy0 * uy0);
    if (!(len > 0.0)) return kSUnknown;
    const double ux = ux0 / len, uy = uy0 / len;
    int res = (fmin(ax, bx) >= sc.minx + dl && fmax(ax, bx) <= sc.maxx - dl &&
               fmin(ay, by) >= sc.miny + dl && fmax(ay, by) <= sc.maxy - dl)
                  ? kSClear
                  : kSUnknown;
    const double h = sqrt(sc.h2);
    const double ro = h + dl, ri = h - 3.0 * dl;
    if (res == kSClear && sc.nbv > 0) {
        // the ring, lane-parallel: clearance from every edge and A's crossing parity
        bool near = false;
        int par = 0;
        for (int i0 = 0; i0 < sc.nbv; i0 += 64) {
            const int i = i0 + lane;
            bool cr = false;
            if (i < sc.nbv) {
                const int j = i + 1 == sc.nbv ? 0 : i + 1;
                const double xi = sc.bvx[i], yi = sc.bvy[i], xj = sc.bvx[j], yj = sc.bvy[j];
                near = near || seg_seg_d2(ax, ay, bx, by, xi, yi, xj, yj) <= ro * ro;
                cr = ray_crosses(ax, ay, xi, yi, xj, yj);
            }
            par ^= __popcll(__ballot(cr)) & 1;
        }
        if (__any(near) || !par) res = kSUnknown;
    }
    if (sc.ne == 0) return res;
    const bool stretch = t_hi > t_lo && ri > 0.0;
    const double sax = ax + t_lo * ux, say = ay + t_lo * uy;
    const double sbx = ax + t_hi * ux, sby = ay + t_hi * uy;
    const int cy0 = __builtin_amdgcn_readfirstlane(grid_cell(fmin(ay, by) - dl, sc.gy0, sc.ginv, sc.gny));
    const int cy1 = __builtin_amdgcn_readfirstlane(grid_cell(fmax(ay, by) + dl, sc.gy0, sc.ginv, sc.gny));
    const int ny = cy1 - cy0 + 1;
    if (ny > 64) return kSUnknown;
    const int* goff = kLds ? reinterpret_cast<const int*>(pp_smem + sc.lds_goff) : sc.goff;
    const int* items = kLds ? reinterpret_cast<const int*>(pp_smem + sc.lds_items) : sc.gitems;
    int k0v = 0, cntv = 0;
    if (lane < ny) {
        const int gy = cy0 + lane;
        const double cell = sc.gcell;
        const double ylo = gy == 0 ? -__builtin_inf() : sc.gy0 + gy * cell - dl;
        const double yhi = gy == sc.gny - 1 ? __builtin_inf() : sc.gy0 + (gy + 1) * cell + dl;
        double t0 = 0.0, t1 = 1.0;
        if (uy0 != 0.0) {
            double ta = (ylo - ay) / uy0, tb = (yhi - ay) / uy0;
            if (ta > tb) {
                const double tt = ta;
                ta = tb;
                tb = tt;
            }
            t0 = fmax(t0, ta);
            t1 = fmin(t1, tb);
        } else if (!(ay >= ylo && ay <= yhi)) {
            t1 = -1.0;
        }
        if (t0 <= t1) {
            const double xa = ax + t0 * ux0, xb = ax + t1 * ux0;
            const int ca = grid_cell(fmin(xa, xb) - dl, sc.gx0, sc.ginv, sc.gnx);
            const int cb = grid_cell(fmax(xa, xb) + dl, sc.gx0, sc.ginv, sc.gnx);
            k0v = goff[gy * sc.gnx + ca];
            cntv = goff[gy * sc.gnx + cb + 1] - k0v;
        }
    }
    for (int mb = 0;; mb += 64) {
        const int m = mb + lane;
        int kk = -1, run = 0;
        for (int r = 0; r < ny; ++r) {
            const int b = __builtin_amdgcn_readlane(k0v, r), n = __builtin_amdgcn_readlane(cntv, r);
            if (m >= run && m < run + n) kk = b + (m - run);
            run += n;
        }
        bool near = false, hit = false;
        if (kk >= 0) {
            const int e = items[kk];
            const double e0x = sc.ex0[e], e0y = sc.ey0[e], e1x = sc.ex1[e], e1y = sc.ey1[e];
            near = seg_seg_d2(ax, ay, bx, by, e0x, e0y, e1x, e1y) <= ro * ro;
            hit = near && stretch && seg_seg_d2(sax, say, sbx, sby, e0x, e0y, e1x, e1y) < ri * ri;
        }
        if (__any(hit)) return kSHit;
        if (__any(near)) res = kSUnknown;
        if (mb + 64 >= run) break;
    }
    return res;
}

// Count-only run of the `pd += d` generator over one segment from its first value w (the same
// passes as walk_rec's generator, every lane a value: the closed form inside a binade, else the
// serial chain through the wave's LDS slots gs): n values with |pd| <= |Ls|, the last of them
// and the first one past (the segment's end, dubins.rs:243-256).  Wave-uniform results.
__device__ inline void seg_count(double w, double dd, double Ls, double* __restrict__ gs,
                                 long long& n, double& last, double& exitv) {
    const int lane = __lane_id();
    const double aL = fabs(Ls);
    n = 0;
    last = w;
    for (;;) {
        int u = 63;
        double v = w;
        const double w1 = w + dd, w2 = w1 + dd;
        bool cf = (w1 - w) == (w2 - w1);
        if (cf) {
            const double vc = __builtin_fma((double)lane, w1 - w, w);
            const uint64_t fm = __ballot(!(fabs(vc) <= aL));
            const int fl = fm ? (int)__builtin_ctzll(fm) : 63;
            cf = __ballot(lane <= fl && (__double2hiint(vc) >> 20) != (__double2hiint(w) >> 20)) == 0;
            v = vc;
        }
        if (!cf) {
            double s = w;
            if (lane == 0) gs[0] = s;
            u = 0;
            bool ended = !(fabs(s) <= aL);
            while (!ended && u < 63) {
                double t4[4];
#pragma unroll
                for (int z = 0; z < 4; ++z) {
                    s += dd;
                    t4[z] = s;
                }
                if (lane == 0) {
#pragma unroll
                    for (int z = 0; z < 4; ++z) gs[u + 1 + z] = t4[z];
                }
                u += 4;
                ended = !(fabs(s) <= aL);
            }
            u = min(u, 63);
            __builtin_amdgcn_wave_barrier();
            v = lane <= u ? gs[lane] : w;
            __builtin_amdgcn_wave_barrier();
        }
        const uint64_t bad = __ballot(lane > u || !(fabs(v) <= aL));
        const int m = bad ? (int)__builtin_ctzll(bad) : 64;
        n += m;
        if (m > 0) last = readlane_f64(v, m - 1);
        if (m <= 63) {
            exitv = readlane_f64(v, m);
            return;
        }
        w = readlane_f64(v, 63) + dd;
    }
}

// Point 0 of a candidate's line — the sample itself — inside an obstacle: the line is rejected
// whatever its parent and its Dubins path (verify, rrt.rs:124-137: the first segment starts inside
// the disc / on an occupied cell), so the candidate needs neither steer_prep nor steer_walk and its
// verdict cannot depend on which node is its parent.  Discs: one bit of the inside bitmap (the
// point's cell lies wholly inside a disc), else the disc grid's cell of the point (every disc is
// listed in each cell its cull box touches); clearly inside only — d2 below r2 by a relative 1e-9,
// far beyond the rounding of the walk's exact segment test, which therefore finds the same hit;
// the grid mode probes the very bit the walk probes.  Polygon scenes: no pre-test.
template <bool kLds, int kScene>
__device__ __forceinline__ bool point_blocked(const SceneDev& sc, double x, double y) {
    if (kScene == kSceneGrid || (kScene == kSceneAny && sc.bits)) {
        const uint32_t* B = kLds ? reinterpret_cast<const uint32_t*>(pp_smem) : sc.bits;
        return grid_occupied(B, sc.bw, sc.bh, sc.bwords, sc.bx0, sc.by0, sc.binv, x, y);
    }
    if (kScene == kScenePoly || (kScene == kSceneAny && (sc.ne > 0 || sc.nbv > 0)) || sc.m == 0)
        return false;
    if (sc.ibits) {  // one load: the cell lies wholly inside a disc (scene::inside_bitmap)
        const double fx = floor((x - sc.ibx0) * sc.ibinv), fy = floor((y - sc.iby0) * sc.ibinv);
        if (!(fx >= 0.0) || !(fy >= 0.0) || fx >= (double)sc.ibn || fy >= (double)sc.ibn)
            return false;
        const int i = (int)fx, j = (int)fy;
        return (sc.ibits[(size_t)j * sc.ibwords + (i >> 5)] >> (i & 31)) & 1u;
    }
    const int* goff = kLds ? reinterpret_cast<const int*>(pp_smem + sc.lds_goff) : sc.goff;
    const int* items = kLds ? reinterpret_cast<const int*>(pp_smem + sc.lds_items) : sc.gitems;
    const int cell = grid_cell(y, sc.gy0, sc.ginv, sc.gny) * sc.gnx + grid_cell(x, sc.gx0, sc.ginv, sc.gnx);
    const int k1 = goff[cell + 1];
    for (int k = goff[cell]; k < k1; ++k) {
        const int d = items[k];
        const double dx = x - sc.cx[d], dy = y - sc.cy[d];
        if (dx * dx + dy * dy < sc.r2[d] * (1.0 - 1.0e-9)) return true;
    }
    return false;
}

// Fast path of verify_node for the edge child (x, y, yaw) → parent (px, py, pyaw): the Dubins
// polyline of line_to_origin (rrt.rs:295-315) plus the junction to the parent, whose own line
// was verified when it was inserted.  Split in two:
//   steer_prep  per lane (one task per lane): word choice, lengths, segment origins, the trim
//               checks — all the per-task scalar math;
//   steer_walk  per wave (one task per wave): the `pd += d` walk of generate_local_course
//               (dubins.rs:239-255) replayed uniformly, each lane capturing one grid point so
//               every point carries exactly the reference's accumulated value; interpolation
//               and the collision test then run lane-parallel, 63 points per chunk.
struct SteerPrep {
    double x, y, px, py;      // child (point 0 of the edge) and parent (the junction)
    double c, cw, sw;         // curvature, cos/sin(-yaw) of the world transform
    double L0, L1, L2;        // segment lengths
    double o1x, o1y, o1yaw;   // origin of segment 1 (endpoint of segment 0)
    double o2x, o2y, o2yaw;   // origin of segment 2
    long long n_point;        // dubins.rs:369
    int m0, m1, m2;           // segment modes
    int state;                // -1: walk; kReject/kAccept: decided; kLiteral; kError; 4: None
};
static_assert(sizeof(SteerPrep) == kSteerPrepBytes, "SteerPrep layout");

__device__ __forceinline__ SteerPrep steer_prep(const SceneDev& sc, double x, double y,
                                                double yaw, double px, double py, double pyaw) {
    SteerPrep r;
    r.x = x;
    r.y = y;
    r.px = px;
    r.py = py;
    const double step = sc.step_size;
    // dubins_path_planning, dubins.rs:401-408 (s = child, e = parent)
    const double ex = px - x, ey = py - y;
    const double c = 1.0 / sc.turn_radius;
    const double lex = cos(yaw) * ex + sin(yaw) * ey;
    const double ley = -(sin(yaw)) * ex + cos(yaw) * ey;
    const double leyaw = pyaw - yaw;
    const Steer s = select_word(lex, ley, leyaw, c);
    r.c = c;
    r.cw = cos(-yaw);
    r.sw = sin(-yaw);
    if (s.word < 0) {  // steer failed: line_to_origin contributes [(sx, sy)] (rrt.rs:313)
        r.state = kPrepNone;
        return r;
    }
    r.L0 = s.t;
    r.L1 = s.p;
    r.L2 = s.q;
    r.m0 = word_mode(s.word, 0);
    r.m1 = word_mode(s.word, 1);
    r.m2 = word_mode(s.word, 2);
    double total = 0.0;
    total += s.t;
    total += s.p;
    total += s.q;
    const double nq = trunc(total / step);
    if (!(nq >= 0.0) || nq > 1.0e8) {
        r.state = kError;
        return r;
    }
    r.n_point = (long long)nq + 3 + 4;
    // segment origins = previous segment's endpoint (dubins.rs:230, 258-271)
    const Pose O0{0.0, 0.0, 0.0};
    const Pose O1 = interp_local(r.m0, r.L0, c, O0);
    const Pose O2 = interp_local(r.m1, r.L1, c, O1);
    const Pose E = interp_local(r.m2, r.L2, c, O2);
    r.o1x = O1.x;
    r.o1y = O1.y;
    r.o1yaw = O1.yaw;
    r.o2x = O2.x;
    r.o2y = O2.y;
    r.o2yaw = O2.yaw;
    // The trim (dubins.rs:281-288) drops exactly the final endpoint unless its local x is 0.0
    // (then it keeps popping) or the array has no trailing zero: both go to the literal path.
    r.state = E.x == 0.0 ? kLiteral : kPrepWalk;
    return r;
}

// The record's fields travel as scalars (a struct passed by reference ends up on the private
// stack once the per-lane segment select turns into an indexed load).
struct WalkIn {
    double x, y, px, py, c, cw, sw, L0, L1, L2, o1x, o1y, o1yaw, o2x, o2y, o2yaw;
    long long n_point;
    int m0, m1, m2, state;
};
__device__ __forceinline__ WalkIn walk_in(const SteerPrep* __restrict__ p) {
    WalkIn w;
    w.x = p->x;
    w.y = p->y;
    w.px = p->px;
    w.py = p->py;
    w.c = p->c;
    w.cw = p->cw;
    w.sw = p->sw;
    w.L0 = p->L0;
    w.L1 = p->L1;
    w.L2 = p->L2;
    w.o1x = p->o1x;
    w.o1y = p->o1y;
    w.o1yaw = p->o1yaw;
    w.o2x = p->o2x;
    w.o2y = p->o2y;
    w.o2yaw = p->o2yaw;
    w.n_point = p->n_point;
    w.m0 = p->m0;
    w.m1 = p->m1;
    w.m2 = p->m2;
    w.state = p->state;
    return w;
}
__device__ __forceinline__ WalkIn walk_in(const SteerPrep& p) { return walk_in(&p); }

// walked / walked_arc (optional, wave-uniform): += the polyline points generated and verified /
// those of them on L and R segments (the sincos points of the walk's FLOP count)
template <bool kLds>
__device__ __forceinline__ int steer_walk(const SceneDev& sc, const WalkIn r,
                                          bool junction = true, int* walked = nullptr,
                                          int* walked_arc = nullptr) {
    const int lane = __lane_id();
    if (r.state == kPrepNone) {  // polyline [(x, y), (px, py)]
        if (walked) *walked += 2;
        const bool has = lane < 2;
        const double qx = lane == 0 ? r.x : r.px, qy = lane == 0 ? r.y : r.py;
        return chunk_rejects<kLds>(sc, has, has, lane == 1, qx, qy) ? kReject : kAccept;
    }
    if (r.state != kPrepWalk) return r.state;
    const double step = sc.step_size;
    const double L0 = r.L0, L1 = r.L1, L2 = r.L2;
    const int m0 = r.m0, m1 = r.m1, m2 = r.m2;
    const double o1x = r.o1x, o1y = r.o1y, o1yaw = r.o1yaw;
    const double o2x = r.o2x, o2y = r.o2y, o2yaw = r.o2yaw;
    int seg = 0;
    double dd = (L0 > 0.0) ? step : -step;
    double pd = dd - 0.0;
    long long grid = 0;
    double carry_x = r.x, carry_y = r.y;  // point 0 of the edge is the child itself
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
        const bool end_here = (seg >= 3) && cnt < 63;
        const bool junction_here = end_here && junction;
        double qx = carry_x, qy = carry_y;
        bool has = (lane == 0), isgrid = false, isjunction = false, isarc = false;
        if (lane >= 1 && lane <= cnt) {
            Pose o;
            o.x = my_seg == 0 ? 0.0 : (my_seg == 1 ? o1x : o2x);
            o.y = my_seg == 0 ? 0.0 : (my_seg == 1 ? o1y : o2y);
            o.yaw = my_seg == 0 ? 0.0 : (my_seg == 1 ? o1yaw : o2yaw);
            const int mm = my_seg == 0 ? m0 : (my_seg == 1 ? m1 : m2);
            isarc = mm != kModeS;
            const Pose p = interp_local(mm, my_pd, r.c, o);
            qx = r.cw * p.x + r.sw * p.y + r.x;   // dubins.rs:415
            qy = -r.sw * p.x + r.cw * p.y + r.y;  // dubins.rs:420
            has = true;
            isgrid = true;
        } else if (junction_here && lane == cnt + 1) {
            qx = r.px;
            qy = r.py;
            has = true;
            isjunction = true;  // the parent: already checked unless it is the root
        }
        const bool check_bounds = isgrid || isjunction || (first && lane == 0);
        const bool rej = chunk_rejects<kLds>(sc, has, check_bounds, has && lane >= 1, qx, qy);
        if (walked) *walked += cnt + (first ? 1 : 0) + (junction_here ? 1 : 0);
        if (walked_arc) *walked_arc += __popcll(__ballot(isarc));
        if (rej) return kReject;
        if (end_here) break;
        carry_x = readlane_f64(qx, cnt);
        carry_y = readlane_f64(qy, cnt);
        first = false;
    }
    if (1 + grid > r.n_point - 2) return kLiteral;
    return kAccept;
}

// Both halves on one wave (uniform prep): the repair and verify_node paths.
// junction = false: the polyline ends at the edge's last point (finalize's edge into the root,
// rrt.rs:532, contributes no root point).
template <bool kLds>
__device__ int steer_collide_fast(const SceneDev& sc, double x, double y, double yaw, double px,
                                  double py, double pyaw, bool junction = true) {
    const SteerPrep r = steer_prep(sc, x, y, yaw, px, py, pyaw);
    return steer_walk<kLds>(sc, walk_in(r), junction);
}

// Literal path (the trim cases the fast walk cannot reproduce: an endpoint local x of 0.0, a
// buffer with no trailing zero): lane 0 runs dubins_literal into its scratch buffer, then the
// whole wave verifies the polyline with the walk's chunk test — chunks of 63 segments, lane 0 the
// previous chunk's last point (bounds-checked in the first chunk only), lanes 1..63 the next
// points — instead of one lane looping over every point and obstacle.  Rare in the extend, but
// check_finish meets it on optimize's self-connections (a node's copy into the node itself): the
// serial test held a scratch slot of the shared pool for a whole scene scan, and hundreds of waves
// queued for the slots.
template <bool kFI>
__device__ __forceinline__ int steer_collide_literal_body(const SceneDev& sc, double x, double y,
                                                          double yaw, double px, double py,
                                                          double pyaw, double* bx, double* by,
                                                          double* byaw, bool junction) {
    const int lane = __lane_id();
    int n = 0, r = 0;
    if (lane == 0) {
        int word = -1;
        double cost = 0.0;
        r = dubins_literal<kFI>(x, y, yaw, px, py, pyaw, sc.turn_radius, sc.step_size, bx, by, byaw,
                           kLiteralCap - 1, &n, &word, &cost);
        if (r != kSteerOverflow) {
            if (r == kSteerNone) {
                bx[0] = x;
                by[0] = y;
                n = 1;
            }
            bx[n] = px;
            by[n] = py;
        }
    }
    r = __shfl(r, 0);
    n = __shfl(n, 0);
    if (r == kSteerOverflow) return kError;
    __threadfence_block();  // lane 0's points before the wave reads them
    const int np = junction ? n + 1 : n;  // the junction point is bounds-checked too
    for (int base = 0; base == 0 || base + 1 < np; base += 63) {
        const int i = base + lane;
        const bool has = i < np;
        const double qx = has ? bx[i] : x, qy = has ? by[i] : y;
        if (chunk_rejects<false>(sc, has, has && (lane >= 1 || base == 0), has && lane >= 1, qx, qy))
            return kReject;
    }
    return kAccept;
}
__device__ int steer_collide_literal(const SceneDev& sc, double x, double y, double yaw, double px,
                                     double py, double pyaw, double* bx, double* by, double* byaw,
                                     bool junction = true) {
    return steer_collide_literal_body<false>(sc, x, y, yaw, px, py, pyaw, bx, by, byaw, junction);
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

// dubins_path_planning_from_origin (dubins.rs:326-399) for n configurations (dx, dy, eyaw, c,
// step_size): local points, yaw as generated
__global__ __launch_bounds__(64) void dubins_origin_kernel(const double* __restrict__ conf, int n,
                                                           int cap, double* __restrict__ px,
                                                           double* __restrict__ py,
                                                           double* __restrict__ pyaw,
                                                           int* __restrict__ n_out,
                                                           int* __restrict__ word_out,
                                                           double* __restrict__ cost_out,
                                                           int* __restrict__ status_out) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const double* c = conf + (size_t)i * 5;
    int np = 0, word = -1;
    double cost = 0.0;
    const int r = dubins_local(c[0], c[1], c[2], c[3], c[4], px + (size_t)i * cap,
                               py + (size_t)i * cap, pyaw + (size_t)i * cap, cap, &np, &word,
                               &cost);
    n_out[i] = np;
    word_out[i] = word;
    cost_out[i] = cost;
    status_out[i] = r;
}

// the six words lsl, rsr, lsr, rsl, rlr, lrl (dubins.rs:27-153) of n (alpha, beta, d) triples:
// tpq[18 i + 3 w ..] = (t, p, q) of word w, ok[6 i + w] = 0 where the word is None
__global__ __launch_bounds__(64) void dubins_words_kernel(const double* __restrict__ abd, int n,
                                                          double* __restrict__ tpq,
                                                          int* __restrict__ ok) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= n) return;
    const double alpha = abd[3 * i], beta = abd[3 * i + 1], d = abd[3 * i + 2];
    const Trig g = make_trig(alpha, beta);
    Word w[6];
    w[0] = word_lsl(alpha, beta, d, g);
    w[1] = word_rsr(alpha, beta, d, g);
    w[2] = word_lsr(alpha, beta, d, g);
    w[3] = word_rsl(alpha, beta, d, g);
    w[4] = word_rlr(alpha, beta, d, g);
    w[5] = word_lrl(alpha, beta, d, g);
    for (int k = 0; k < 6; ++k) {
        ok[6 * i + k] = w[k].ok ? 1 : 0;
        tpq[18 * i + 3 * k] = w[k].ok ? w[k].t : 0.0;
        tpq[18 * i + 3 * k + 1] = w[k].ok ? w[k].p : 0.0;
        tpq[18 * i + 3 * k + 2] = w[k].ok ? w[k].q : 0.0;
    }
}

// ------------------------------------------------------------------------- window pipeline
//
// One speculative window w = window_kernel (w's NN screen ‖ resolve + commit of w - 1) →
// nn_finalize (+ window pairs, + w + 1's samples) → steer_prep → steer_walk; window w's resolve and commit
// run inside window w + 1's window_kernel (or the batch's drain launch).  Everything reads the
// device-resident DevState, so the host enqueues windows back to back and synchronises once per
// batch.

constexpr int kQPL = 8;                     // samples per lane in the screen
constexpr int kQPB = 64 * kQPL;                  // samples per screen workgroup (its waves share them)
constexpr int kScanThreads = 512;                // window_kernel workgroup (8 waves, 256 VGPRs)
constexpr bool kWinRepair = true;                // repairs inside the window kernel (no spill)
constexpr int kScanWaves = kScanThreads / 64;
constexpr int kScanBlk = 16;             // nodes per block (one block minimum per sample)
constexpr int kStage = 7936;                     // chunk nodes staged in LDS per round
constexpr int kGrab = 64;                        // nodes a screen wave takes from the counter
constexpr int kExactNode = 1 << 30;              // screen partial key: a node index, not a block
// LDS of a screen workgroup: the wave merge (best, second, key per wave and sample; sample ids;
// the samples' f32 operands), then the staged chunk
constexpr int kScreenStageOff = (3 * kScanWaves + 3) * kQPB * 4;
constexpr int kScanGrid = 255;           // screen workgroups per window (one per CU, with
                                                 // the resolve workgroup: <= 256 CUs)

// node chunks of the screen for a window of K samples: the nqb sample blocks x chunks workgroups
// fill kScanGrid; every chunk is a whole number of kScanBlk blocks
__host__ __device__ inline int scan_chunks(int K) {
    const int nqb = (K + kQPB - 1) / kQPB;
    int c = kScanGrid / nqb;
    if (c > kMaxChunks) c = kMaxChunks;
    return c < 1 ? 1 : c;
}
__host__ __device__ inline int scan_chunk_len(int n, int chunks) {
    int cl = (n + chunks - 1) / chunks;
    if (cl < kScanWaves * kScanBlk) cl = kScanWaves * kScanBlk;
    return (cl + kScanBlk - 1) & ~(kScanBlk - 1);
}
__host__ __device__ inline int scan_chunks_used(int n, int chunks) {
    const int cl = scan_chunk_len(n, chunks);
    return (n + cl - 1) / cl;
}

__device__ inline void argmin_pair(double& d, int& i, double od, int oi) {
    if (od < d || (od == d && oi < i)) {
        d = od;
        i = oi;
    }
}

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

// sincos_small's constants (pp_device.h): __ocml_sincos_f64's, bit for bit
__constant__ double kSinCosTab[17] = {
    0x1.45f306dc9c883p-1,  -0x1.921fb54442d18p+0,  -0x1.1a62633145c00p-54,
    0x1.1a62633145c00p-54, -0x1.b839a252049c0p-104,
    -0x1.907db46cc5e42p-37, 0x1.1eeb69037ab78p-29, -0x1.27e4fa17f65f6p-22,
    0x1.a01a019f4ec90p-16,  -0x1.6c16c16c16967p-10, 0x1.5555555555555p-5,
    0x1.5e0b2f9a43bb8p-33,  -0x1.ae600b42fdfa7p-26, 0x1.71de3796cde01p-19,
    -0x1.a01a019e83e5cp-13, 0x1.1111111110bb3p-7,   -0x1.5555555555555p-3};

__device__ __forceinline__ float scan_d2(float qx, float qy, float nx, float ny) {
    const float dx = qx - nx, dy = qy - ny;
    return __builtin_fmaf(dy, dy, dx * dx);
}

// window_samples: Space::rand_point for the iterations [start, start + W) of a window
// (rrt.rs:139-146, seeded: Q7 — x = draw 2*it, y = draw 2*it + 1), W = min(K, target - start),
// and a counting sort of the samples by the Morton index of their cell in a 16 x 16 grid over the
// sampling box: perm[pos] = sample, so a screen block of 256 consecutive sorted samples is
// spatially compact (the expanded screen's precision).  Within a cell the order is arbitrary —
// the results never depend on it (only which samples meet the exact rescan).
struct SamplesArgs {
    int K;
    int64_t target;
    uint64_t seed;
    double minx, maxx, miny, maxy;
    double* wsx[2];
    double* wsy[2];
    float* wsx32[2];
    float* wsy32[2];
    int* perm[2];
    int* cofs[2];     // [257] first sorted position of each Morton cell (cell 256: W)
    float2* sxy[2];   // sorted position -> (x, y) f32 (the pair search's prefilter)
    double* ssx[2];   // sorted position -> x, y (f64): the screen's coalesced sample loads
    double* ssy[2];
    float2* ob[2];    // [K / kQPB] the screen block's centre o (f32) of each kQPB sorted samples
    double* sq[2];    // sample -> |q - o|^2 about its block's centre (f64, exact)
    int* ipos[2];     // sample -> sorted position (the screen's partials are stored by position)
    const SceneDev* scp = nullptr;       // the scene in device memory (point_blocked)
    unsigned char* blk[2] = {nullptr, nullptr};  // sample -> its point lies in an obstacle
    // caller-drawn samples (pp_rrt_extend_samples): iteration it's sample is (hsx, hsy)[it -
    // hs_base] instead of the seeded stream (null: the stream)
    const double* hsx = nullptr;
    const double* hsy = nullptr;
    int64_t hs_base = 0;
};

// Space::rand_point of iteration itj (rrt.rs:139-146): the seeded stream (Q7: x = draw 2 it,
// y = draw 2 it + 1), or the caller's own sample of that iteration
__device__ __forceinline__ void draw_sample(const SamplesArgs& g, uint64_t itj, double& x,
                                            double& y) {
    if (g.hsx) {
        const int64_t i = (int64_t)itj - g.hs_base;
        x = g.hsx[i];
        y = g.hsy[i];
    } else {
        x = gen_range(g.seed, 2 * itj, g.minx, g.maxx);
        y = gen_range(g.seed, 2 * itj + 1, g.miny, g.maxy);
    }
}

__device__ inline int morton16(int x, int y) {
    int m = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) m |= (((x >> b) & 1) << (2 * b)) | (((y >> b) & 1) << (2 * b + 1));
    return m;
}

// LDS of samples_role: the Morton histogram, each sample's cell, the sorted window's sample ids,
// the count of samples in an obstacle
constexpr int kSamplesLds = 256 * 4 + kMaxWindow + kMaxWindow * 4 + 16 + kMaxWindow;

// The screen's geometry for Ws screened samples (window mode): nqb blocks of kQPB samples x
// chunks node chunks on at most kScanGrid workgroups, nqb x chunks a multiple of 8 when it can be
// (the XCD-aware mapping), chunks <= kMaxChunks (the partials' capacity).
__host__ __device__ inline int screen_chunks(int Ws) {
    const int nqb = (Ws + kQPB - 1) / kQPB;
    if (nqb <= 0) return 1;
    int c = kScanGrid / nqb;
    if (c > kMaxChunks) c = kMaxChunks;
    for (int d = c; d >= 1 && d * 4 >= c * 3; --d)
        if (((nqb * d) & 7) == 0) return d;
    return c < 1 ? 1 : c;
}

__device__ void samples_role(DevState* st, const SamplesArgs& g, int np, int64_t start,
                             char* smem) {
    int* s_hist = reinterpret_cast<int*>(smem);                  // [256]
    unsigned char* s_cell = reinterpret_cast<unsigned char*>(s_hist + 256);  // [K]
    int* s_j = reinterpret_cast<int*>(smem + 256 * 4 + kMaxWindow);  // [K] sorted position -> sample
    int* s_nb = s_j + kMaxWindow;  // samples in an obstacle (sorted after the screened ones)
    unsigned char* s_bk = reinterpret_cast<unsigned char*>(s_nb + 4);  // [K] sample in an obstacle
    const int tid = threadIdx.x, NT = blockDim.x;
    const int64_t rem = g.target - start;
    // the adaptive window (kdyn, set by the commits; results never depend on the window size)
    const int Kw = st->kdyn > 0 ? min(g.K, st->kdyn) : g.K;
    const int W = (rem <= 0 || st->error) ? 0 : (rem < Kw ? (int)rem : Kw);
    if (tid == 0) {
        st->Wp[np] = W;
        st->wsp[np] = start;
    }
    for (int i = tid; i < 256; i += NT) s_hist[i] = 0;
    if (tid == 0) *s_nb = 0;
    __syncthreads();
    const double fx = 16.0 / (g.maxx - g.minx), fy = 16.0 / (g.maxy - g.miny);
    // (kU samples per thread per pass: their pre-test loads are in flight together)
    constexpr int kU = 4;
    const bool pre = g.blk[np] != nullptr;
    // the pre-test's scene fields, loaded once (through the pointer they would be reloaded after
    // every store below, which the compiler cannot prove disjoint)
    SceneDev scl{};
    if (pre) {
        scl.bits = g.scp->bits;
        scl.bw = g.scp->bw;
        scl.bh = g.scp->bh;
        scl.bwords = g.scp->bwords;
        scl.bx0 = g.scp->bx0;
        scl.by0 = g.scp->by0;
        scl.binv = g.scp->binv;
        scl.ne = g.scp->ne;
        scl.nbv = g.scp->nbv;
        scl.m = g.scp->m;
        scl.ibits = g.scp->ibits;
        scl.ibn = g.scp->ibn;
        scl.ibwords = g.scp->ibwords;
        scl.ibx0 = g.scp->ibx0;
        scl.iby0 = g.scp->iby0;
        scl.ibinv = g.scp->ibinv;
        scl.goff = g.scp->goff;
        scl.gitems = g.scp->gitems;
        scl.cx = g.scp->cx;
        scl.cy = g.scp->cy;
        scl.r2 = g.scp->r2;
        scl.gx0 = g.scp->gx0;
        scl.gy0 = g.scp->gy0;
        scl.ginv = g.scp->ginv;
        scl.gnx = g.scp->gnx;
        scl.gny = g.scp->gny;
    }
    for (int j0 = tid; j0 < W; j0 += NT * kU) {
        double xs[kU], ys[kU];
        bool bks[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int j = j0 + u * NT;
            xs[u] = ys[u] = 0.0;
            if (j < W) {
                draw_sample(g, (uint64_t)(start + j), xs[u], ys[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < kU; ++u)
            bks[u] = pre && j0 + u * NT < W && point_blocked<false, kSceneAny>(scl, xs[u], ys[u]);
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const int j = j0 + u * NT;
            const bool valid = j < W;
            // a sample in an obstacle needs no nearest node and is nobody's candidate parent: it
            // is sorted after the screened samples, out of the screen and the pair grid (counted
            // per wave: one LDS atomic instead of one per sample on a single address)
            const uint64_t mb = __ballot(valid && bks[u]);
            if ((__lane_id()) == 0 && mb) atomicAdd(s_nb, (int)__popcll(mb));
            if (!valid) continue;
            const double x = xs[u], y = ys[u];
            g.wsx[np][j] = x;
            g.wsy[np][j] = y;
            g.wsx32[np][j] = (float)x;
            g.wsy32[np][j] = (float)y;
            if (pre) g.blk[np][j] = bks[u] ? 1 : 0;
            s_bk[j] = bks[u] ? 1 : 0;
            const int cx = min(max((int)((x - g.minx) * fx), 0), 15);  // == sample_cell
            const int cy = min(max((int)((y - g.miny) * fy), 0), 15);
            const int cell = morton16(cx, cy);
            s_cell[j] = (unsigned char)cell;
            if (!bks[u]) atomicAdd(&s_hist[cell], 1);
        }
    }
    __syncthreads();
    const int Ws = W - *s_nb;  // screened samples: sorted positions [0, Ws)
    if (tid == 0) {
        st->Wsp[np] = Ws;
        st->chp[np] = screen_chunks(Ws);
    }
    if (tid < 64) {  // exclusive prefix of the 256 cell counts, 4 per lane
        int v[4], sum = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            v[u] = s_hist[4 * tid + u];
            sum += v[u];
        }
        const int x = wave_incl_scan(sum);
        int base = x - sum;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            s_hist[4 * tid + u] = base;
            base += v[u];
        }
    }
    __syncthreads();
    for (int i = tid; i < 256; i += NT) g.cofs[np][i] = s_hist[i];
    if (tid == 0) {
        g.cofs[np][256] = Ws;
        *s_nb = Ws;  // (now the next free position of the blocked bucket)
    }
    __syncthreads();  // the cell starts are read before the scatter advances them
    for (int j0 = tid - (tid & 63); j0 < W; j0 += NT) {  // whole waves (the ballot below)
        const int j = j0 + (tid & 63);
        const bool bk = j < W && s_bk[j];
        // the blocked bucket: a wave's blocked samples take consecutive positions (one atomic)
        const uint64_t mb = __ballot(bk);
        int base = 0;
        if ((tid & 63) == 0 && mb) base = atomicAdd(s_nb, (int)__popcll(mb));
        base = __builtin_amdgcn_readfirstlane(base);
        if (j >= W) continue;
        s_j[bk ? base + (int)__popcll(mb & ((1ull << (tid & 63)) - 1)) : atomicAdd(&s_hist[s_cell[j]], 1)] = j;
    }
    __syncthreads();
    // the screen's blocks of kQPB sorted samples, one wave each: the sorted window (coalesced; the
    // coordinates drawn again from the stream, bit-identical), the centre o of the block's
    // bounding box (f32) and every sample's |q - o|^2 in f64 — (q - o) rounded to f32 per axis,
    // the screen's own operands, squared exactly (nn_finalize adds it back to the screen values)
    const int lane = tid & 63, wv = tid >> 6;
    for (int pos = Ws + tid; pos < W; pos += NT) {  // the blocked bucket: perm / ipos only
        const int j = s_j[pos];
        g.perm[np][pos] = j;
        g.ipos[np][j] = pos;
    }
    // every thread takes sorted positions tid, tid + NT, ... (a wave: 64 consecutive positions,
    // inside one block): the coordinates again from the stream, the position's stores, and the
    // wave's f32 bounding box into LDS slot pos / 64 (s_hist is free by now); then one thread per
    // block merges its waves' boxes into the centre o, and every position stores |q - o|^2.  (r03
    // gave each block to one wave, 8 samples per lane, and 16 waves shared 4-8 blocks: the
    // sampling workgroup was nn_finalize's long pole, ~30 of its 27-30 us)
    // s_bb: [kMaxWindow / 64][4] wave boxes (x0, x1, y0, y1), then [kMaxWindow / kQPB][2] block
    // centres — over s_hist and the head of s_cell, both dead after the scatter
    float* s_bb = reinterpret_cast<float*>(s_hist);
    (void)wv;
    __syncthreads();  // (s_hist's last readers: the scatter above)
    constexpr int kMaxK = 4;  // positions per thread: both callers run 1024 threads
    static_assert(kMaxWindow <= 1024 * kMaxK, "samples_role: positions per thread");
    static_assert((4 * (kMaxWindow / 64) + 2 * (kMaxWindow / kQPB)) * 4 <= 256 * 4 + kMaxWindow,
                  "samples_role: the box slots fit s_hist and s_cell");
    double xs[kMaxK], ys[kMaxK];
#pragma unroll
    for (int k = 0; k < kMaxK; ++k) {
        const int pos = tid + k * NT;
        xs[k] = ys[k] = 0.0;
        const bool in = pos < Ws;
        if (in) {
            const int j = s_j[pos];
            draw_sample(g, (uint64_t)(start + j), xs[k], ys[k]);
            g.perm[np][pos] = j;
            g.ipos[np][j] = pos;
            g.sxy[np][pos] = make_float2((float)xs[k], (float)ys[k]);
            g.ssx[np][pos] = xs[k];
            g.ssy[np][pos] = ys[k];
        }
        const int wbase = pos - lane;  // the wave's first position (uniform)
        if (wbase < Ws) {
            const float inff = __builtin_inff();
            const float bx0 = wave_min_f32(in ? f32_below(xs[k]) : inff);
            const float bx1 = wave_max_f32(in ? f32_above(xs[k]) : -inff);
            const float by0 = wave_min_f32(in ? f32_below(ys[k]) : inff);
            const float by1 = wave_max_f32(in ? f32_above(ys[k]) : -inff);
            if (lane == 0) {
                float* b = s_bb + 4 * (wbase >> 6);
                b[0] = bx0;
                b[1] = bx1;
                b[2] = by0;
                b[3] = by1;
            }
        }
        if (NT * (k + 1) >= kMaxWindow) break;
    }
    __syncthreads();
    const int nqb = (Ws + kQPB - 1) / kQPB;
    if (tid < nqb) {  // block tid's centre: the middle of its samples' box (f32)
        float x0 = __builtin_inff(), x1 = -__builtin_inff(), y0 = __builtin_inff(), y1 = -__builtin_inff();
        for (int w = tid * (kQPB / 64); w < (tid + 1) * (kQPB / 64) && w * 64 < Ws; ++w) {
            const float* b = s_bb + 4 * w;
            x0 = fminf(x0, b[0]);
            x1 = fmaxf(x1, b[1]);
            y0 = fminf(y0, b[2]);
            y1 = fmaxf(y1, b[3]);
        }
        const float2 o = make_float2((float)(0.5 * ((double)x0 + (double)x1)),
                                     (float)(0.5 * ((double)y0 + (double)y1)));
        g.ob[np][tid] = o;
        s_bb[4 * (kMaxWindow / 64) + 2 * tid] = o.x;  // (after the wave slots)
        s_bb[4 * (kMaxWindow / 64) + 2 * tid + 1] = o.y;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kMaxK; ++k) {
        const int pos = tid + k * NT;
        if (pos < Ws) {
            const int qb = pos / kQPB;
            const float oxf = s_bb[4 * (kMaxWindow / 64) + 2 * qb];
            const float oyf = s_bb[4 * (kMaxWindow / 64) + 2 * qb + 1];
            const float qpx = (float)(xs[k] - (double)oxf), qpy = (float)(ys[k] - (double)oyf);
            g.sq[np][s_j[pos]] = (double)qpx * (double)qpx + (double)qpy * (double)qpy;
        }
        if (NT * (k + 1) >= kMaxWindow) break;
    }
}

// the Morton cell coordinate of v along one axis (samples_role's binning, clamped)
__device__ inline int sample_cell(double v, double v0, double f) {
    return min(max((int)((v - v0) * f), 0), 15);
}

// Arguments of the window kernel.  Sample buffers are double-buffered by window parity: the
// screen of window w writes wsx/wsy[p], the resolve of w - 1 reads [1 - p].
struct WinKArgs {
    DevState* st;
    SceneDev sc;
    TreeDev tr;
    int K;              // samples per window
    int Kcap;           // buffer capacity per window (stride of the partials)
    int nqb, chunks;    // screen geometry (scan_chunks)
    int p;              // parity of the screened window
    int gen;            // 1: window mode (sorted samples, expanded screen); 0: given wsx/wsy[p]
    int resolve;        // 1: workgroup 0 resolves + commits the previous window
    int scan;           // 0: the drain launch (resolve only)
    int64_t seq;        // sequence number of the screened window
    int64_t target;     // iteration the enqueued windows stop at
    uint64_t seed;
    double* wsx[2];
    double* wsy[2];
    float* wsx32[2];    // f32 copies (the pair search's prefilter)
    float* wsy32[2];
    int* perm[2];       // window mode: sorted position -> sample (window_samples)
    double* sq[2];      // window mode: |q - o|^2 of every sample (the screen's block origin)
    float* pbest;
    float* psecond;
    int* pidx;
    // resolve + commit of the previous window (parity 1 - p)
    const int* nn_idx;
    int* cand_cnt;
    const CandEntry* cand;
    const int* pend;
    int* snap_status;
    double* snap_yaw;
    int* fin_par;
    ResolveScratch rs;
    double* lit_scratch;
    // window mode: workgroup 0 draws the next window's samples (parity 1 - p) after its commit
    int gen_next;
    SamplesArgs g;
    SampleRec hrec;     // pp_rrt_extend_samples: the commit's per-iteration record
};

// RRT::get_nearest_node screen (rrt.rs:378-391): f32 SoA nodes x the window's samples.  The
// screen workgroup b (mapped XCD-aware, so the sample blocks that stream one node chunk share an
// XCD's L2) takes sample block qb and node chunk c.  Its waves split the chunk; every lane holds 4
// samples; node coordinates are wave-uniform scalar loads (the next block in flight) used directly
// as SGPR operands.  Per block of kScanBlk nodes each sample keeps only the block minimum (v_min3),
// merges it into (best, second) with med3 and records the block that first attained the best; the
// winning block is re-evaluated afterwards with the same arithmetic (bit-identical) for the lowest
// index and the in-block second best.  Result: the exact per-chunk top-2 of the screen values.
//
// kExp (window mode): the samples come spatially sorted (window_samples: perm), so a block of 256
// is compact and the screen runs in the expanded form about the block's centre o:
//     e(n) = |n - o|^2 - 2 (q - o).(n - o)  =  |q - n|^2 - |q - o|^2
// two FMAs per (node, sample) after a per-node prologue (n - o, |n - o|^2: four ops per wave,
// shared by the lane's 4 samples) — 3.5 VALU per evaluation instead of 4.5.  nn_finalize adds
// |q - o|^2 back (sq) and widens the near-tie margin by the expanded form's rounding bound.
// !kExp (nearest API): the given samples, direct form (sub, sub, mul, fma).
// The screen's winner re-evaluation of a block no longer in LDS (trees past one staging round):
// the block's 16 nodes from global memory with the screen's own prep and arithmetic, the lowest
// u with value == best and the minimum of the others.  Out of line: inlined, the compiler merges
// it with the LDS path into flat loads.
template <bool kExp, int kNodes = kScanBlk>
__device__ __attribute__((noinline)) void screen_block_global(const float* __restrict__ bx,
                                                              const float* __restrict__ by, float qx,
                                                              float qy, float oxf, float oyf,
                                                              float best, int& ui, float& other) {
    for (int u = 0; u < kNodes; ++u) {
        float px = bx[u], py = by[u], pw = 0.0f;
        if (kExp) {
            px = px - oxf;
            py = py - oyf;
            pw = __builtin_fmaf(py, py, px * px);
        }
        const float d = kExp ? __builtin_fmaf(qx, px, __builtin_fmaf(qy, py, pw))
                             : scan_d2(qx, qy, px, py);
        if (ui < 0 && d == best)
            ui = u;
        else
            other = __builtin_fminf(other, d);
    }
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <bool kExp>
__device__ __attribute__((always_inline)) inline void scan_role(const WinKArgs& a, int b,
                                                               char* smem) {
    DevState* st = a.st;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // window mode: the samples not in an obstacle (sorted first) on the geometry samples_role
    // chose for them; the nearest API: the given samples on the launch's geometry
    const int W = kExp ? st->Wsp[a.p] : st->Wp[a.p];
    const int ns = st->n_scan;
    if (b == 0 && tid == 0) st->nsp[a.p] = ns;
    const int chunks = kExp ? st->chp[a.p] : a.chunks;
    const int nqb = kExp ? (W + kQPB - 1) / kQPB : a.nqb;
    const int G = nqb * chunks;
    if (b >= G) return;
    const int t = (G & 7) == 0 ? (b & 7) * (G >> 3) + (b >> 3) : b;
    const int qb = t % nqb, c = t / nqb;
    const int qbase = qb * kQPB;
    if (qbase >= W) return;
    const int cl = scan_chunk_len(ns, chunks);
    const int c0 = c * cl;
    if (c0 >= ns) return;
    const int L = min(c0 + cl, ns) - c0;  // the chunk's nodes
    const float* nx = a.tr.x32;
    const float* ny = a.tr.y32;
    // The chunk goes through the workgroup's LDS (x | y | |n-o|^2, kStage nodes a round; one
    // round up to ~250k tree nodes at K = 4096): LDS-DMA (global_load_lds_dwordx4, lane l brings
    // nodes 4l..4l+3 of a 256-node quarter, no registers) issued before the samples are read, so
    // the two latencies overlap; each thread then preps its own float4s in place — (n - o,
    // |n - o|^2) in the expanded form, each node once instead of once per lane.  The waves take
    // kGrab-node pieces from an LDS counter (no wave idles at the merge barrier while another
    // still screens); a wave's pieces come in increasing order, so its first block to reach the
    // best is its lowest.  The block loop reads its 16 nodes as broadcast ds_read_b128.
    float* stg = reinterpret_cast<float*>(smem + kScreenStageOff);
    int* s_next = reinterpret_cast<int*>(stg + 3 * kStage);
    auto issue_round = [&](int r0) {
        const int len = min(kStage, L - r0);
        for (int q4 = wave; q4 * 256 < len; q4 += kScanWaves) {
            if (q4 * 256 + 4 * lane < len) {  // (a partial float4 reads up to 3 padding floats)
                const size_t gi = (size_t)(c0 + r0 + q4 * 256 + 4 * lane);
                __builtin_amdgcn_global_load_lds((glb_void*)(nx + gi), (lds_void*)(stg + q4 * 256), 16, 0, 0);
                __builtin_amdgcn_global_load_lds((glb_void*)(ny + gi), (lds_void*)(stg + kStage + q4 * 256), 16, 0, 0);
            }
        }
    };
    issue_round(0);
    float qxr[kQPL], qyr[kQPL], best[kQPL], second[kQPL];
    int sid[kQPL], blk[kQPL], bi[kQPL];
    float oxf = 0.0f, oyf = 0.0f;
    if (kExp) {
        // window mode: samples_role left the window sorted (f64, coalesced), each screen block's
        // centre o and every sample's |q - o|^2 (for nn_finalize)
        const float2 o = a.g.ob[a.p][qb];
        oxf = o.x;
        oyf = o.y;
#pragma unroll
        for (int r = 0; r < kQPL; ++r) {
            const int pos = qbase + r * 64 + lane;
            const bool in = pos < W;
            sid[r] = in ? a.perm[a.p][pos] : -1;
            const double xs = in ? a.g.ssx[a.p][pos] : (double)oxf;
            const double ys = in ? a.g.ssy[a.p][pos] : (double)oyf;
            const float qpx = (float)(xs - (double)oxf), qpy = (float)(ys - (double)oyf);
            qxr[r] = -2.0f * qpx;  // exact scaling
            qyr[r] = -2.0f * qpy;
        }
    } else {
        const double* qxs = a.wsx[a.p];
        const double* qys = a.wsy[a.p];
#pragma unroll
        for (int r = 0; r < kQPL; ++r) {
            const int pos = qbase + r * 64 + lane;
            sid[r] = pos < W ? pos : -1;
            qxr[r] = sid[r] >= 0 ? (float)qxs[pos] : 0.0f;
            qyr[r] = sid[r] >= 0 ? (float)qys[pos] : 0.0f;
        }
    }
#pragma unroll
    for (int r = 0; r < kQPL; ++r) {
        best[r] = __builtin_inff();
        second[r] = __builtin_inff();
        blk[r] = -1;
        bi[r] = -1;
    }
    {  // wave 0 parks the samples' operands for the winner re-evaluation (read after barriers)
        float* s_qx = reinterpret_cast<float*>(smem) + (3 * kScanWaves + 1) * kQPB;
        if (wave == 0) {
#pragma unroll
            for (int r = 0; r < kQPL; ++r) {
                s_qx[r * 64 + lane] = qxr[r];
                s_qx[kQPB + r * 64 + lane] = qyr[r];
            }
        }
    }
    // screen value of (sample r, node (nx, ny)); expanded: the node's (x - ox, y - oy, |.|^2)
    auto val = [&](int r, float px, float py, float pw) {
        if (kExp) return __builtin_fmaf(qxr[r], px, __builtin_fmaf(qyr[r], py, pw));
        return scan_d2(qxr[r], qyr[r], px, py);
    };
    auto prep = [&](float& px, float& py, float& pw) {
        if (kExp) {
            px = px - oxf;
            py = py - oyf;
            pw = __builtin_fmaf(py, py, px * px);
        } else {
            pw = 0.0f;
        }
    };
    int r0 = 0;
    for (;;) {
        const int len = min(kStage, L - r0);
        if (tid == 0) *s_next = 0;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA has landed
        __syncthreads();                                   // ... and every other wave's
        for (int i = 4 * tid; i < len; i += 4 * kScanThreads) {  // prep in place
            float4 x4 = *reinterpret_cast<const float4*>(stg + i);
            float4 y4 = *reinterpret_cast<const float4*>(stg + kStage + i);
            float4 w4;
            prep(x4.x, y4.x, w4.x);
            prep(x4.y, y4.y, w4.y);
            prep(x4.z, y4.z, w4.z);
            prep(x4.w, y4.w, w4.w);
            *reinterpret_cast<float4*>(stg + i) = x4;
            *reinterpret_cast<float4*>(stg + kStage + i) = y4;
            *reinterpret_cast<float4*>(stg + 2 * kStage + i) = w4;
        }
        __syncthreads();
        for (;;) {
            int g0 = 0;
            if (lane == 0) g0 = atomicAdd(s_next, kGrab);
            g0 = __builtin_amdgcn_readfirstlane(__shfl(g0, 0));
            if (g0 >= len) break;
            const int g1 = min(g0 + kGrab, len);
            const int gb = g0 + ((g1 - g0) & ~(kScanBlk - 1));  // whole blocks (a tail: the last)
            for (int u0 = g0; u0 < gb; u0 += kScanBlk) {
                float px[kScanBlk], py[kScanBlk], pw[kScanBlk];
#pragma unroll
                for (int v = 0; v < kScanBlk / 4; ++v) {
                    const float4 ax = *reinterpret_cast<const float4*>(stg + u0 + 4 * v);
                    const float4 ay = *reinterpret_cast<const float4*>(stg + kStage + u0 + 4 * v);
                    const float4 aw = *reinterpret_cast<const float4*>(stg + 2 * kStage + u0 + 4 * v);
                    px[4 * v] = ax.x, px[4 * v + 1] = ax.y, px[4 * v + 2] = ax.z, px[4 * v + 3] = ax.w;
                    py[4 * v] = ay.x, py[4 * v + 1] = ay.y, py[4 * v + 2] = ay.z, py[4 * v + 3] = ay.w;
                    pw[4 * v] = aw.x, pw[4 * v + 1] = aw.y, pw[4 * v + 2] = aw.z, pw[4 * v + 3] = aw.w;
                }
                float bm[kQPL];
                if (kExp) {
                    // two nodes per packed FMA (v_pk_fma_f32: each half the exactly rounded
                    // fmaf of the scalar form, so the winner re-evaluation below stays
                    // bit-identical), the pair's minimum folded in by one v_min3
#pragma unroll
                    for (int u = 0; u < kScanBlk; u += 2) {
                        const f32x2 PX = {px[u], px[u + 1]}, PY = {py[u], py[u + 1]};
                        const f32x2 PW = {pw[u], pw[u + 1]};
#pragma unroll
                        for (int r = 0; r < kQPL; ++r) {
                            const f32x2 QX = {qxr[r], qxr[r]}, QY = {qyr[r], qyr[r]};
                            const f32x2 d = __builtin_elementwise_fma(
                                QX, PX, __builtin_elementwise_fma(QY, PY, PW));
                            const float m = __builtin_fminf(d.x, d.y);
                            bm[r] = u == 0 ? m : __builtin_fminf(bm[r], m);
                        }
                    }
                } else {
#pragma unroll
                    for (int u = 0; u < kScanBlk; ++u) {
#pragma unroll
                        for (int r = 0; r < kQPL; ++r) {
                            const float d = val(r, px[u], py[u], pw[u]);
                            bm[r] = u == 0 ? d : __builtin_fminf(bm[r], d);
                        }
                    }
                }
                const int k = c0 + r0 + u0;
#pragma unroll
                for (int r = 0; r < kQPL; ++r) {
                    second[r] = __builtin_amdgcn_fmed3f(best[r], bm[r], second[r]);
                    if (bm[r] < best[r]) {
                        best[r] = bm[r];
                        blk[r] = k;
                    }
                }
            }
            for (int u = gb; u < g1; ++u) {  // the chunk's tail (< kScanBlk nodes): exact top-2
                const float px = stg[u], py = stg[kStage + u], pw = stg[2 * kStage + u];
#pragma unroll
                for (int r = 0; r < kQPL; ++r) {
                    const float d = val(r, px, py, pw);
                    second[r] = __builtin_amdgcn_fmed3f(best[r], d, second[r]);
                    if (d < best[r]) {
                        best[r] = d;
                        bi[r] = c0 + r0 + u;
                        blk[r] = -1;  // the best is a tail node, not a block's
                    }
                }
            }
        }
        if (r0 + len >= L) break;
        r0 += len;
        __syncthreads();  // every wave is done with this round before the next overwrites it
        issue_round(r0);
    }
    // The waves' partials per sample go to LDS — (best, second, key): key = the best block's start,
    // or kExactNode | index when the best is a tail node (tail nodes follow every block of the
    // chunk, so keys order ties by node index either way), 0x7fffffff when the wave saw no node —
    // and one thread per sample merges them; only then is the winning block re-evaluated (one
    // block per sample, not one per wave): the same arithmetic again, bit-identical, for the lowest
    // index of the best value and the best of the block's other nodes (the block minima carried one
    // each).  From LDS when the block is in the last round (always up to ~250k nodes).
    float* s_b = reinterpret_cast<float*>(smem);              // [kScanWaves][kQPB]
    float* s_s = s_b + kScanWaves * kQPB;
    int* s_i = reinterpret_cast<int*>(s_s + kScanWaves * kQPB);
    int* s_sid = s_i + kScanWaves * kQPB;                      // [kQPB]
#pragma unroll
    for (int r = 0; r < kQPL; ++r) {
        s_b[wave * kQPB + r * 64 + lane] = best[r];
        s_s[wave * kQPB + r * 64 + lane] = second[r];
        s_i[wave * kQPB + r * 64 + lane] =
            blk[r] >= 0 ? blk[r] : (bi[r] >= 0 ? (bi[r] | kExactNode) : 0x7fffffff);
        if (wave == 0) s_sid[r * 64 + lane] = sid[r];
    }
    __syncthreads();
    if (tid < kQPB) {  // one thread per sample (sorted position qbase + tid)
        float bb = s_b[tid], ss = s_s[tid];
        int key = s_i[tid];
#pragma unroll
        for (int w = 1; w < kScanWaves; ++w) {
            const float ob = s_b[w * kQPB + tid], os = s_s[w * kQPB + tid];
            const int ok = s_i[w * kQPB + tid];
            const bool take = ob < bb || (ob == bb && ok < key);  // (branch-free)
            ss = fminf(fminf(ss, os), take ? bb : ob);
            bb = take ? ob : bb;
            key = take ? ok : key;
        }
        const int q = s_sid[tid];
        int idx = key == 0x7fffffff ? -1 : (key & ~kExactNode);
        if (q >= 0 && key != 0x7fffffff && !(key & kExactNode)) {
            // the sample's screen operands, as wave 0 held them
            const float* s_qx = reinterpret_cast<const float*>(smem) + (3 * kScanWaves + 1) * kQPB;
            const float qx = s_qx[tid], qy = s_qx[kQPB + tid];
            const int rel = key - c0 - r0;
            int ui = -1;
            float other = __builtin_inff();
            if (rel >= 0) {  // (LDS only: a shared pointer select would make these flat loads)
                float vx[kScanBlk], vy[kScanBlk], vw[kScanBlk];
#pragma unroll
                for (int v = 0; v < kScanBlk / 4; ++v) {
                    const float4 a4 = *reinterpret_cast<const float4*>(stg + rel + 4 * v);
                    const float4 b4 = *reinterpret_cast<const float4*>(stg + kStage + rel + 4 * v);
                    const float4 w4 = *reinterpret_cast<const float4*>(stg + 2 * kStage + rel + 4 * v);
                    vx[4 * v] = a4.x, vx[4 * v + 1] = a4.y, vx[4 * v + 2] = a4.z, vx[4 * v + 3] = a4.w;
                    vy[4 * v] = b4.x, vy[4 * v + 1] = b4.y, vy[4 * v + 2] = b4.z, vy[4 * v + 3] = b4.w;
                    vw[4 * v] = w4.x, vw[4 * v + 1] = w4.y, vw[4 * v + 2] = w4.z, vw[4 * v + 3] = w4.w;
                }
#pragma unroll
                for (int u = 0; u < kScanBlk; ++u) {
                    const float d = kExp ? __builtin_fmaf(qx, vx[u], __builtin_fmaf(qy, vy[u], vw[u]))
                                         : scan_d2(qx, qy, vx[u], vy[u]);
                    if (ui < 0 && d == bb)
                        ui = u;
                    else
                        other = __builtin_fminf(other, d);
                }
            } else {
                screen_block_global<kExp>(nx + key, ny + key, qx, qy, oxf, oyf, bb, ui, other);
            }
            idx = key + ui;
            ss = __builtin_fminf(ss, other);
        }
        if (q >= 0) {  // by sorted position: coalesced (nn_finalize maps samples through ipos)
            const size_t o = (size_t)c * a.Kcap + qbase + tid;
            a.pbest[o] = bb;
            a.psecond[o] = ss;
            a.pidx[o] = idx;
        }
    }
}


// The first window of a batch: its samples (the later ones come from the previous window kernel
// workgroup 0, after the commit that decides where the next window starts).
__global__ __launch_bounds__(1024) void window_samples_kernel(DevState* st, SamplesArgs g, int np) {
    __shared__ __attribute__((aligned(16))) char smem[kSamplesLds];
    samples_role(st, g, np, st->it_spec, smem);
}


// nn_finalize: kFinSamples samples per workgroup, one wave per sample.
//  1. The wave merges the sample's screen partials (lane c: chunk c) and screens the nodes the
//     window's screen did not cover — the ones appended since (the previous window's commit) —
//     with the same f32 arithmetic (lanes stride them), then reduces the top-2 across the wave.
//     Margin test against the f32 rounding bound: certain → exact f64 d2 of the winner; else the
//     wave's exact f64 brute force over the screen chunks whose f32 minimum could hide the exact
//     nearest and over the appended nodes (rrt.rs:378-391; lowest index on exact ties, Q9).
//  2. Window pairs (window mode): for each of the workgroup's samples j (one wave each), the
//     earlier window samples i < j strictly nearer than j's snapshot NN — the candidates of the
//     sequential-consistency resolve.  The window's samples are binned in a 16 x 16 Morton grid
//     (samples_role: perm, cofs, sorted f32 copies), so the wave visits only the cells j's disc
//     of radius sqrt(D2) touches; an f32 distance within the rounding margin of the NN distance
//     goes to the exact f64 test (dx*dx + dy*dy < nn_d2, the oracle's arithmetic).  Hits stay in
//     LDS (at most kCandCap per sample, the count exact) and are appended with one global atomic
//     per workgroup.
// Workgroup 0 also publishes the window (W, or 0 when a truncated predecessor voided it) for the
// later kernels and advances the next window's screen position.
constexpr int kFinThreads = 1024;
constexpr int kFinWaves = kFinThreads / 64;
constexpr int kFinSamples = kFinWaves;  // one wave per sample
constexpr int kFinDelta = 4096;         // appended nodes staged in LDS (beyond: global loads)

// The window's samples binned by Morton cell (samples_role): the pair search's spatial index.
struct PairGrid {
    const int* perm;     // sorted position -> sample
    const int* cofs;     // [257] first sorted position of each cell
    const float2* sxy;   // sorted position -> (x, y) f32
    const double* ssx;   // sorted position -> x, y f64 (the samples' own coordinates, bit for bit)
    const double* ssy;
    double minx, miny, fx, fy;  // samples_role's binning: cell = (v - v0) * f, clamped to 0..15
    float slack;         // f32 prefilter margin for the coordinates' magnitude
};

// the wave's top-2 (every lane ends with it): butterfly steps that merge disjoint lane sets, on
// DPP and the gfx950 lane swaps (merge_top2 is not idempotent: a set merged with itself would
// report its best as its second)
template <int kCtrl>
__device__ inline Top2 top2_dpp(Top2 t) {
    return Top2{__builtin_bit_cast(float, dpp_pair<kCtrl>(__builtin_bit_cast(int, t.b))),
                __builtin_bit_cast(float, dpp_pair<kCtrl>(__builtin_bit_cast(int, t.s))),
                dpp_pair<kCtrl>(t.i)};
}
template <bool k32>
__device__ inline Top2 top2_swap(Top2 t) {
    const LanePair b = k32 ? swap32(__builtin_bit_cast(int, t.b)) : swap16(__builtin_bit_cast(int, t.b));
    const LanePair s = k32 ? swap32(__builtin_bit_cast(int, t.s)) : swap16(__builtin_bit_cast(int, t.s));
    const LanePair i = k32 ? swap32(t.i) : swap16(t.i);
    return merge_top2(Top2{__builtin_bit_cast(float, b.a), __builtin_bit_cast(float, s.a), i.a},
                      Top2{__builtin_bit_cast(float, b.b), __builtin_bit_cast(float, s.b), i.b});
}
__device__ inline Top2 wave_top2(Top2 t) {
    t = merge_top2(t, top2_dpp<0xB1>(t));   // quad_perm [1,0,3,2]
    t = merge_top2(t, top2_dpp<0x4E>(t));   // quad_perm [2,3,0,1]
    t = merge_top2(t, top2_dpp<0x141>(t));  // row_half_mirror
    t = merge_top2(t, top2_dpp<0x140>(t));  // row_mirror
    t = top2_swap<false>(t);
    return top2_swap<true>(t);
}

#ifdef PP_FIN_STAMPS  // diagnostic builds only: wall-clock phase stamps of nn_finalize per workgroup
__device__ unsigned long long g_fin_stamps[kFinStampSlots * kFinStampWGs];
#define FS(k)                                                                          \
    if (threadIdx.x == 0 && blockIdx.x < kFinStampWGs)                                 \
        g_fin_stamps[kFinStampSlots * blockIdx.x + (k)] = wall_clock64();
#define FSW(k)                                                                         \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < kFinStampWGs)                         \
        atomicMax(&g_fin_stamps[kFinStampSlots * blockIdx.x + (k)], wall_clock64());
hipError_t fin_stamps_copy(unsigned long long* out, size_t n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fin_stamps), n * sizeof(unsigned long long));
}
#else
#define FS(k)
#define FSW(k)
#endif

// 8 waves per SIMD (<= 64 VGPRs): two 1024-thread workgroups per CU, so the extra sampling
// workgroup (the grid's last) runs beside the others instead of waiting for a CU to drain.
__global__ __launch_bounds__(kFinThreads, 8) void nn_finalize_kernel(
    DevState* __restrict__ st, int p, int64_t seq, int chunks_api, const float* __restrict__ pbest,
    const float* __restrict__ psecond, const int* __restrict__ pidx, int stride,
    const double* __restrict__ qx, const double* __restrict__ qy, const float* __restrict__ x32,
    const float* __restrict__ y32, const double* __restrict__ X, const double* __restrict__ Y,
    const double* __restrict__ YAW, double eps_coord, int* __restrict__ out_idx,
    double* __restrict__ out_d2, double* __restrict__ out_pose, PairGrid pg,
    int* __restrict__ cand_cnt, CandEntry* __restrict__ cand,
    int* __restrict__ pend, const double* __restrict__ sq, const int* __restrict__ ipos,
    SamplesArgs gen, int gen_next, const unsigned char* __restrict__ blk) {
    __shared__ double s_nd2[kFinSamples];  // exact snapshot NN d2 of each sample
    __shared__ int s_pc[kFinSamples];      // pair search: nearer window samples found
    __shared__ int s_pi[kFinSamples][kCandCap];
    __shared__ double s_pd[kFinSamples][kCandCap];
    __shared__ int s_pbase, s_pnb;
    __shared__ uint32_t s_fmask;         // samples (waves) that need the exact brute force
    __shared__ double s_fd[kFinSamples];  // candidate-chunk bound on pbest of a near-tie
    __shared__ uint64_t s_cmask;
    __shared__ double s_rd[kFinWaves];
    __shared__ int s_ri[kFinWaves];
    __shared__ float2 s_dn[kFinDelta];   // nodes appended after the screen's snapshot (f32)
    FS(0)
    const bool voided = st->void_seq == seq || st->error;
    if (gen_next && blockIdx.x == gridDim.x - 1) {
        // the extra workgroup: Space::rand_point of the window after this one, into the parity
        // the committed previous window freed — it starts where this window ends, or, when the
        // commit voided this window (a truncation), where the committed one stopped (it_spec;
        // workgroup 0 advances it_spec only when this window is not voided).  Off the critical
        // path: steer_prep and steer_walk of this window run before the next screen.
        __shared__ __attribute__((aligned(16))) char s_gen[kSamplesLds];
        const int64_t start = voided ? st->it_spec : st->wsp[p] + st->Wp[p];
        samples_role(st, gen, 1 - p, start, s_gen);
        FS(9)
        return;
    }
    const int W = voided ? 0 : st->Wp[p];
    const int ns = st->nsp[p], n = st->n;
    const int chunks = cand ? st->chp[p] : chunks_api;  // window mode: samples_role's geometry
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        st->W = W;
        st->n_scan = n;
        if (!voided) st->it_spec = st->wsp[p] + W;
    }
    const int q0 = (int)blockIdx.x * kFinSamples;
    if (q0 >= W) return;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int q = q0 + wave;
    // a sample in an obstacle is rejected whatever its parent: no nearest node, no pair list, and
    // it is nobody's candidate parent (samples_role's point_blocked)
    const bool qblk = blk && q < W && blk[q];
    const bool in = q < W && !qblk;
    const int D = n - ns, Dl = min(D, kFinDelta);  // appended nodes (staged: the first kFinDelta)
    for (int k = tid; k < Dl; k += kFinThreads) s_dn[k] = make_float2(x32[ns + k], y32[ns + k]);
    if (tid < kFinSamples) s_pc[tid] = 0;
    if (tid == 0) s_fmask = 0;
    __syncthreads();
    FS(1)
    // ---- 1. the sample's nearest node
    if (in) {
        const int n_chunks = scan_chunks_used(ns, chunks);
        Top2 t{__builtin_inff(), __builtin_inff(), -1};
        const double qq = sq ? sq[q] : 0.0;  // window mode: screen values are d2 - |q - o|^2
        float cb = __builtin_inff(), cs = __builtin_inff();  // this lane's chunk: raw screen top-2
        int ci = -1;
        const int pq = ipos ? ipos[q] : q;  // the sample's sorted position (the partials' index)
        if (lane < n_chunks) {
            const size_t o = (size_t)lane * stride + pq;
            cb = pbest[o];
            cs = psecond[o];
            ci = pidx[o];
            t = Top2{(float)((double)cb + qq), (float)((double)cs + qq), ci};
        }
        FSW(2)
        const double xq = qx[q], yq = qy[q];
        const float fx = (float)xq, fy = (float)yq;
        for (int k = lane; k < D; k += 64) {  // appended nodes: exact top-2 per lane
            const float2 v = k < Dl ? s_dn[k] : make_float2(x32[ns + k], y32[ns + k]);
            const float d = scan_d2(fx, fy, v.x, v.y);
            const Top2 c{d, __builtin_inff(), ns + k};
            t = merge_top2(t, c);
        }
        t = wave_top2(t);
        bool flag = t.i < 0 || !(t.b < __builtin_inff());
        double cthr = __builtin_inf();  // near-tie: the chunks with pbest <= cthr are rescanned
        if (!flag) {
            const double D1 = sqrt((double)t.b);
            if (!sq) {  // direct screen: f32 rounding of the coordinates and the arithmetic
                const double tc = 16.0 * eps_coord + 4.0e-6 * (D1 + 1.0);
                cthr = (D1 + tc) * (D1 + tc);
                if (t.s < __builtin_inff()) {
                    const double D2 = sqrt((double)t.s);
                    flag = !(D2 - D1 > 8.0 * eps_coord + 1.0e-6 * D2);
                }
            } else {  // expanded screen: rounding of |n-o|^2 - 2(q-o).(n-o) about the block centre
                const double qn = sqrt(qq);
                const double D = (t.s < __builtin_inff() ? sqrt((double)t.s) : D1) + 1.0;
                // |dE| <= 5u (|n-o|^2 + 2|q-o||n-o|) for the f32 inputs and arithmetic
                // (u = 2^-24, |n-o| <= |q-o| + D for the winner and the runner-up), plus the f32
                // rounding of the node coordinates (|dn| <= eps_coord / 2 per axis)
                const double E = 4.0e-7 * ((qn + D) * (qn + D) + 2.0 * qn * (qn + D)) +
                                 8.0 * eps_coord * (D + 1.0);
                cthr = (double)t.b + 2.0 * E - qq;
                if (t.s < __builtin_inff()) flag = !((double)t.s - (double)t.b > 2.0 * E);
            }
        }
        FSW(3)
        if (!flag) {
            const int bi = t.i;
            const double dx = xq - X[bi], dy = yq - Y[bi];
            const double bd = dx * dx + dy * dy;
            FSW(4)
            if (lane == 0) {
                out_idx[q] = bi;
                out_d2[q] = bd;
                s_nd2[wave] = bd;
                if (out_pose) {
                    out_pose[3 * q] = X[bi];
                    out_pose[3 * q + 1] = Y[bi];
                    out_pose[3 * q + 2] = YAW[bi];
                }
            }
        } else {
            // a near-tie: the nodes that can still be the exact nearest are those whose screen
            // value is <= cthr.  When every candidate chunk holds one of them (its second > cthr),
            // they are the chunks' known winners: the wave decides exactly on those and the
            // appended nodes.  A chunk with two (or more) falls to the workgroup's brute force.
            // The appended nodes are screened again in the direct form against the exact
            // distance U of a known node: only those within its f32 rounding bound load f64.
            bool need = false;
            double bd = __builtin_inf();
            int bi = 0x7fffffff;
            if (t.i >= 0) {  // the screen's winner (a chunk's or an appended node)
                const double dx = xq - X[t.i], dy = yq - Y[t.i];
                bd = dx * dx + dy * dy;
                bi = t.i;
            }
            if (!((double)cb > cthr)) {
                if (!((double)cs > cthr) || ci < 0) {
                    need = true;
                } else {
                    const double dx = xq - X[ci], dy = yq - Y[ci];
                    argmin_pair(bd, bi, dx * dx + dy * dy, ci);
                }
            }
            wave_argmin(bd, bi);
            if (D > 0 && !__any(need)) {
                const double U = sqrt(bd), tu = 16.0 * eps_coord + 4.0e-6 * (U + 1.0);
                const double lim = (U + tu) * (U + tu);
                for (int k = lane; k < D; k += 64) {
                    const float2 v = k < Dl ? s_dn[k] : make_float2(x32[ns + k], y32[ns + k]);
                    if (!((double)scan_d2(fx, fy, v.x, v.y) > lim)) {
                        const double dx = xq - X[ns + k], dy = yq - Y[ns + k];
                        argmin_pair(bd, bi, dx * dx + dy * dy, ns + k);
                    }
                }
                wave_argmin(bd, bi);
            }
            if (lane == 0) atomicAdd(&st->flag_count, 1);  // statistics (nn_flagged)
            if (__any(need) || bi == 0x7fffffff) {
                if (lane == 0) {
                    atomicOr(&s_fmask, 1u << wave);
                    s_fd[wave] = cthr;
                }
            } else if (lane == 0) {
                out_idx[q] = bi;
                out_d2[q] = bd;
                s_nd2[wave] = bd;
                if (out_pose) {
                    out_pose[3 * q] = X[bi];
                    out_pose[3 * q + 1] = Y[bi];
                    out_pose[3 * q + 2] = YAW[bi];
                }
            }
        }
    }
    __syncthreads();
    FS(5)
    // near-ties: the workgroup's exact f64 brute force, over the screen chunks whose f32 minimum
    // could hide the exact nearest (f32 distance within the rounding bound of the f32 winner)
    // and over the appended nodes; lowest index on exact ties (rrt.rs:378-391, Q9)
    for (uint32_t fm = s_fmask; fm; fm &= fm - 1) {
        const int w = (int)__builtin_ctz(fm);
        const int qf = q0 + w;
        const double cthr = s_fd[w];
        const int n_chunks = scan_chunks_used(ns, chunks);
        if (wave == 0) {
            const int pf = ipos ? ipos[qf] : qf;
            const bool cc = lane < n_chunks && !((double)pbest[(size_t)lane * stride + pf] > cthr);
            const uint64_t cm = __ballot(cc);
            if (lane == 0) s_cmask = cm;
        }
        __syncthreads();
        const int cl = scan_chunk_len(ns, chunks);
        const double xq = qx[qf], yq = qy[qf];
        double bd = __builtin_inf();
        int bi = 0x7fffffff;
        for (uint64_t cm = s_cmask; cm; cm &= cm - 1) {
            const int c = (int)__builtin_ctzll(cm);
            const int c1 = min(c * cl + cl, ns);
            for (int k = c * cl + tid; k < c1; k += kFinThreads) {
                const double dx = xq - X[k], dy = yq - Y[k];
                argmin_pair(bd, bi, dx * dx + dy * dy, k);
            }
        }
        for (int k = ns + tid; k < n; k += kFinThreads) {
            const double dx = xq - X[k], dy = yq - Y[k];
            argmin_pair(bd, bi, dx * dx + dy * dy, k);
        }
        wave_argmin(bd, bi);
        if (lane == 0) {
            s_rd[wave] = bd;
            s_ri[wave] = bi;
        }
        __syncthreads();
        if (tid == 0) {
            double d = s_rd[0];
            int i = s_ri[0];
            for (int v = 1; v < kFinWaves; ++v) argmin_pair(d, i, s_rd[v], s_ri[v]);
            out_idx[qf] = i;
            out_d2[qf] = d;
            s_nd2[w] = d;
            if (out_pose) {
                out_pose[3 * qf] = X[i];
                out_pose[3 * qf + 1] = Y[i];
                out_pose[3 * qf + 2] = YAW[i];
            }
        }
        __syncthreads();
    }
    if (!cand) return;  // nearest-only launch (no window)
    FS(6)
    // ---- 2. window pairs
    {
        // wave w: sample j = q0 + w against the window samples i < j of the Morton cells its
        // disc of radius sqrt(D2) touches (the binning is monotone, so the cells are a superset)
        const int j = q0 + wave;
        if (j < W && !qblk) {
            const double xj = qx[j], yj = qy[j];
            const float xjf = (float)xj, yjf = (float)yj;
            const double D2 = s_nd2[wave];
            const float df = __builtin_sqrtf((float)D2) + pg.slack;
            const float thr = df * df;
            const double R = sqrt(D2) * (1.0 + 1e-9) + 1e-9;
            const int cx0 = sample_cell(xj - R, pg.minx, pg.fx), cx1 = sample_cell(xj + R, pg.minx, pg.fx);
            const int cy0 = sample_cell(yj - R, pg.miny, pg.fy), cy1 = sample_cell(yj + R, pg.miny, pg.fy);
            for (int cy = cy0; cy <= cy1; ++cy) {
                for (int cx = cx0; cx <= cx1; ++cx) {
                    const int m = morton16(cx, cy);
                    const int a1 = pg.cofs[m + 1];
                    // (the cells list only the screened samples, none in an obstacle; a
                    // candidate's index and f64 coordinates are read by sorted position, beside
                    // its f32 prefilter, not through perm)
                    for (int pos = pg.cofs[m] + lane; pos < a1; pos += 64) {
                        const float2 v = pg.sxy[pos];
                        const int ii = pg.perm[pos];
                        const double sx = pg.ssx[pos], sy = pg.ssy[pos];
                        if (!(scan_d2(xjf, yjf, v.x, v.y) <= thr)) continue;
                        if (ii >= j) continue;
                        const double dx = xj - sx, dy = yj - sy;
                        const double d2 = dx * dx + dy * dy;
                        if (d2 < D2) {  // strictly nearer than the snapshot NN (which wins ties)
                            const int at = atomicAdd(&s_pc[wave], 1);
                            if (at < kCandCap) {
                                s_pi[wave][at] = ii;
                                s_pd[wave][at] = d2;
                            }
                        }
                    }
                }
            }
        }
    }
    __syncthreads();
    FS(7)
    if (wave == 0) {
        const int j = q0 + lane;
        const bool jin = lane < kFinSamples && j < W;
        const int cnt = jin ? s_pc[lane] : 0;
        const int keep = min(cnt, kCandCap);
        if (jin) cand_cnt[j] = cnt;
        // one reservation per workgroup for the entries and for the queue of pending samples
        const int ex = wave_incl_scan(keep), pc = wave_incl_scan(cnt > 0 ? 1 : 0);
        const int eo = ex - keep, po = pc - (cnt > 0 ? 1 : 0);
        if (lane == 63) {
            s_pbase = ex > 0 ? atomicAdd(&st->ncomp, ex) : 0;
            s_pnb = pc > 0 ? atomicAdd(&st->npend, pc) : 0;
        }
        const uint64_t ov = __ballot(cnt > kCandCap);  // a list overflowed: the window stops there
        __builtin_amdgcn_wave_barrier();
        const int eb = s_pbase + eo, pb = s_pnb + po;
        for (int k = 0; k < keep; ++k)
            cand[eb + k] = CandEntry{j, s_pi[lane][k], s_pd[lane][k], 0.0, -1, 0};
        if (cnt > 0) pend[pb] = j;
        if (lane == 0 && ov) atomicMin(&st->weff, q0 + (int)__builtin_ctzll(ov));
        if (blk) {  // statistics (pp_stats.samples_blocked): one atomic per workgroup
            const uint64_t bm = __ballot(jin && blk[j]);
            if (lane == 0 && bm) atomicAdd((unsigned long long*)&st->blocked, (unsigned long long)__popcll(bm));
        }
        FS(8)
    }
}

// Task t of a window: t < W is (sample t → its snapshot NN); t >= W is candidate entry t - W
// (sample E.j → window sample E.i, with E.i's yaw under ITS snapshot parent: the speculation the
// resolve validates).
__device__ inline void window_task(int t, int W, const double* wsx, const double* wsy,
                                   const double* snap_pose, const CandEntry* cand, int* j_out,
                                   double* px, double* py, double* pyaw) {
    if (t < W) {  // parent = the snapshot NN, whose pose nn_finalize wrote
        *j_out = t;
        *px = snap_pose[3 * t];
        *py = snap_pose[3 * t + 1];
        *pyaw = snap_pose[3 * t + 2];
    } else {  // parent = window sample i, heading toward ITS snapshot NN (compute_yaw)
        const CandEntry ce = cand[t - W];
        *j_out = ce.j;
        *px = wsx[ce.i];
        *py = wsy[ce.i];
        *pyaw = atan2(snap_pose[3 * ce.i + 1] - *py, snap_pose[3 * ce.i] - *px);
    }
}

// One segment's endpoint from its origin (interpolate at the full length, dubins.rs:155-198)
// with the transcendental values supplied: ca/sa as in PrepRec, sl/cl = sin/cos(length).
struct Pt {
    double x, y;
};
// (x / c as div_by: the correctly rounded FMA quotient, bit-identical to the division)
__device__ inline Pt seg_end(int mode, double len, double c, double rc, double ox, double oy,
                             double ca, double sa, double sl, double cl) {
    Pt r;
    if (mode == kModeS) {
        const double lc = div_by(len, c, rc);
        r.x = ox + lc * ca;
        r.y = oy + lc * sa;
    } else {
        const double ldx = div_by(sl, c, rc);
        const double l1 = div_by(1.0 - cl, c, rc);  // (1 - cos) / -c = -((1 - cos) / c)
        const double ldy = mode == kModeL ? l1 : -l1;
        const double gdx = ca * ldx + sa * ldy;
        const double gdy = -sa * ldx + ca * ldy;
        r.x = ox + gdx;
        r.y = oy + gdy;
    }
    return r;
}

// The per-task body of steer_prep: the 8 lanes r of one task group (all 64 lanes of the wave
// call it: the word choice broadcasts within 8-lane groups).  act: an active task (else a
// kReject record); write: this group owns task t (lane r == 0 stores rec[t], *yaw_dst and
// cost_out[t]).
__device__ __forceinline__ void prep_task(const SceneDev& sc, int r, int g0, int t, bool write,
                                          bool act, double x, double y, double px, double py,
                                          double pyaw, int own, double cyaw, int cull, double cbase,
                                          double climit, PrepRec* __restrict__ rec,
                                          double* yaw_dst, double* __restrict__ cost_out,
                                          int force_state = -1) {
    const double step = sc.step_size;
    const double c = 1.0 / sc.turn_radius;
    const double cy_atan = atan2(py - y, px - x);
    const double yaw = own ? cyaw : cy_atan;
    // dubins_path_planning, dubins.rs:401-408 (s = child, e = parent)
    const double ex = px - x, ey = py - y;
    const double cyw = cos(yaw), syw = sin(yaw);
    const double lex = cyw * ex + syw * ey;
    const double ley = -(syw)*ex + cyw * ey;
    const double leyaw = pyaw - yaw;
    // dubins_path_planning_from_origin, dubins.rs:333-348
    const double hyp = hypot(lex, ley);
    const double d = hyp * c;
    const double theta = mod2pi(atan2(ley, lex));
    const double alpha = mod2pi(-theta);
    const double beta = mod2pi(leyaw - theta);
    // lanes 0/1: sin(alpha), sin(beta); lanes 0/1/2: cos(alpha), cos(beta), cos(alpha - beta)
    const double s_in = sin(r == 0 ? alpha : beta);
    const double c_in = cos(r == 0 ? alpha : (r == 1 ? beta : alpha - beta));
    const double sa = grp8_bcast_f64<0>(s_in), sb = grp8_bcast_f64<1>(s_in);
    const double ca = grp8_bcast_f64<0>(c_in), cb = grp8_bcast_f64<1>(c_in),
                 c_ab = grp8_bcast_f64<2>(c_in);
    // lane r < 6 evaluates word r of ALL_PLANNERS (dubins.rs:27-153, 291)
    const double dd2 = d * d;
    double ya = 0.0, xa = 1.0, psq = -1.0, tmpc = 2.0;
    if (r == 0) {
        psq = 2.0 + dd2 - (2.0 * c_ab) + (2.0 * d * (sa - sb));
        ya = cb - ca;
        xa = d + sa - sb;
    } else if (r == 1) {
        psq = 2.0 + dd2 - (2.0 * c_ab) + (2.0 * d * (sb - sa));
        ya = ca - cb;
        xa = d - sa + sb;
    } else if (r == 2) {
        psq = -2.0 + dd2 + (2.0 * c_ab) + (2.0 * d * (sa + sb));
        ya = -ca - cb;
        xa = d + sa + sb;
    } else if (r == 3) {
        psq = -2.0 + dd2 + (2.0 * c_ab) - (2.0 * d * (sa + sb));
        ya = ca + cb;
        xa = d - sa - sb;
    } else if (r == 4) {
        tmpc = (6.0 - dd2 + 2.0 * c_ab + 2.0 * d * (sa - sb)) / 8.0;
        ya = ca - cb;
        xa = d - sa + sb;
    } else if (r == 5) {
        tmpc = (6.0 - dd2 + 2.0 * c_ab + 2.0 * d * (-sa + sb)) / 8.0;
        ya = ca - cb;
        xa = d + sa - sb;
    }
    const bool wok = r < 4 ? !(psq < 0.0) : (r < 6 ? !(fabs(tmpc) > 1.0) : false);
    const double A1 = atan2(ya, xa);
    const double pp = sqrt(r < 4 && wok ? psq : 0.0);
    const double A2 = atan2(r == 2 ? -2.0 : 2.0, pp);
    const double Cc = acos(r >= 4 && wok ? tmpc : 0.0);
    double wt = 0.0, wp = 0.0, wq = 0.0;
    if (r == 0) {
        wt = mod2pi(-alpha + A1);
        wp = pp;
        wq = mod2pi(beta - A1);
    } else if (r == 1) {
        wt = mod2pi(alpha - A1);
        wp = pp;
        wq = mod2pi(-beta + A1);
    } else if (r == 2) {
        const double tm = A1 - A2;
        wt = mod2pi(-alpha + tm);
        wp = pp;
        wq = mod2pi(-mod2pi(beta) + tm);
    } else if (r == 3) {
        const double tm = A1 - A2;
        wt = mod2pi(alpha - tm);
        wp = pp;
        wq = mod2pi(beta - tm);
    } else if (r == 4) {
        wp = mod2pi(2.0 * kPi - Cc);
        wt = mod2pi(alpha - A1 + mod2pi(wp / 2.0));
        wq = mod2pi(alpha - beta - wt + mod2pi(wp));
    } else if (r == 5) {
        wp = mod2pi(2.0 * kPi - Cc);
        wt = mod2pi(-alpha - A1 + wp / 2.0);
        wq = mod2pi(mod2pi(beta) - alpha - wt + mod2pi(wp));
    }
    const double wcost = fabs(wt) + fabs(wp) + fabs(wq);
    // first strict minimum in ALL_PLANNERS order (dubins.rs:351-360: bcost starts at inf and a
    // word wins on `bcost > cost`, so a NaN or inf cost never wins and ties keep the earlier
    // word) = the (cost, word) argmin over the group's valid words: a DPP butterfly over the
    // 8-lane group (xor 1, xor 2, half-row mirror), no per-word broadcasts
    double bc = (r < 6 && wok && wcost < __builtin_inf()) ? wcost : __builtin_inf();
    int bw = bc < __builtin_inf() ? r : 0x7fffffff;
    argmin_dpp<0xB1>(bc, bw);
    argmin_dpp<0x4E>(bc, bw);
    argmin_dpp<0x141>(bc, bw);
    if (!(bc < __builtin_inf())) bw = -1;
    const int src = g0 + (bw < 0 ? 0 : bw);
    const double L0 = __shfl(wt, src), L1 = __shfl(wp, src), L2 = __shfl(wq, src);
    const int m0 = word_mode(bw, 0), m1 = word_mode(bw, 1), m2 = word_mode(bw, 2);
    int state = !act ? kReject : (bw < 0 ? kPrepNone : kPrepWalk);
    double tot = 0.0;
    tot += L0;
    tot += L1;
    tot += L2;
    const double nq = trunc(tot / step);
    if (state == kPrepWalk && (!(nq >= 0.0) || nq > 1.0e8)) state = kError;
    // segment origin headings (interpolate's yaw, dubins.rs:191-196)
    const double oy0 = 0.0;
    const double oy1 = m0 == kModeL ? oy0 + L0 : (m0 == kModeR ? oy0 - L0 : oy0);
    const double oy2 = m1 == kModeL ? oy1 + L1 : (m1 == kModeR ? oy1 - L1 : oy1);
    // lanes 0..2: segment trig, 3..5: sin/cos of the lengths, 6: the world transform
    double arg = 0.0;
    if (r < 3) {
        const int ms = r == 0 ? m0 : (r == 1 ? m1 : m2);
        const double oys = r == 0 ? oy0 : (r == 1 ? oy1 : oy2);
        arg = ms == kModeS ? oys : -oys;
    } else if (r < 6) {
        arg = r == 3 ? L0 : (r == 4 ? L1 : L2);
    } else if (r == 6) {
        arg = -yaw;
    }
    const double sv = sin(arg), cv = cos(arg);
    const double ca0 = grp8_bcast_f64<0>(cv), ca1 = grp8_bcast_f64<1>(cv), ca2 = grp8_bcast_f64<2>(cv);
    const double sa0 = grp8_bcast_f64<0>(sv), sa1 = grp8_bcast_f64<1>(sv), sa2 = grp8_bcast_f64<2>(sv);
    const double sl0 = grp8_bcast_f64<3>(sv), sl1 = grp8_bcast_f64<4>(sv), sl2 = grp8_bcast_f64<5>(sv);
    const double cl0 = grp8_bcast_f64<3>(cv), cl1 = grp8_bcast_f64<4>(cv), cl2 = grp8_bcast_f64<5>(cv);
    const double cw = grp8_bcast_f64<6>(cv), sw = grp8_bcast_f64<6>(sv);
    const double rc = 1.0 / c;
    const Pt O1 = seg_end(m0, L0, c, rc, 0.0, 0.0, ca0, sa0, sl0, cl0);
    const Pt O2 = seg_end(m1, L1, c, rc, O1.x, O1.y, ca1, sa1, sl1, cl1);
    const Pt E = seg_end(m2, L2, c, rc, O2.x, O2.y, ca2, sa2, sl2, cl2);
    // the trim (dubins.rs:281-288) drops exactly the endpoint unless its local x is 0.0; then it
    // drops the last grid point too, and goes on while the dropped x is 0.0: the walk drops that
    // point and hands the rest (its x 0.0 as well) to the literal path
    const int trim1 = (state == kPrepWalk && E.x == 0.0) ? 1 : 0;
    int cnt0 = 0, cnt1 = 0, cnt2 = 0, fb_seg = 0;
    double fb_pd = 0.0, fb_dd = 0.0;
    // no grid points are stored: steer_walk generates them all, lane-parallel and bit-exact,
    // from the walk's initial state (segment 0, pd = d - 0.0, dubins.rs:239-241), and runs
    // the trailing-zero check itself
    if (state == kPrepWalk) {
        state = kPrepFallback;
        fb_dd = (L0 > 0.0) ? step : -step;
        fb_pd = fb_dd - 0.0;
    }
    // RRT* cull: an edge whose cost cannot beat the limit is settled without its walk
    if (act && cull && !(cbase + bc < climit)) state = kReject;
    // the query batch's verdict cache (mq_sample_nn): the same child and parent as a task the
    // previous step walked — its verdict, no walk
    if (act && force_state >= 0) state = force_state;
    if (write && r == 0) {  // idle batch tasks get a kReject record (act == false)
        PrepRec o;
        o.x = x;
        o.y = y;
        o.px = px;
        o.py = py;
        o.yaw = yaw;
        o.pyaw = pyaw;
        o.c = c;
        o.cw = cw;
        o.sw = sw;
        o.ox[0] = 0.0;
        o.oy[0] = 0.0;
        o.ox[1] = O1.x;
        o.oy[1] = O1.y;
        o.ox[2] = O2.x;
        o.oy[2] = O2.y;
        o.ca[0] = ca0;
        o.ca[1] = ca1;
        o.ca[2] = ca2;
        o.sa[0] = sa0;
        o.sa[1] = sa1;
        o.sa[2] = sa2;
        o.L[0] = L0;
        o.L[1] = L1;
        o.L[2] = L2;
        o.n_point = (long long)nq + 3 + 4;
        o.fb_pd = fb_pd;
        o.fb_dd = fb_dd;
        o.fb_seg = fb_seg;
        o.m[0] = m0;
        o.m[1] = m1;
        o.m[2] = m2;
        o.cnt[0] = cnt0;
        o.cnt[1] = cnt1;
        o.cnt[2] = cnt2;
        o.state = state;
        o.trim1 = trim1;
        rec[t] = o;
        if (yaw_dst) *yaw_dst = yaw;
        // the Dubins cost (dubins.rs:351-361; inf on None): the RRT* edge cost
        if (cost_out) cost_out[t] = bc;
    }
}

// steer_prep: kPrepLanes lanes per task, 8 tasks per wave (persistent grid over the
// window's W + ncomp tasks): compute_yaw (rrt.rs:267-271),
// dubins_path_planning's frame change and word choice (dubins.rs:333-363, 401-408) and the
// segment origins.  Every transcendental sits at a call site all lanes reach with per-lane
// arguments (lane r evaluates word r; one sin and one cos call give all the segment trig), so a
// task's chain is ~9 calls deep instead of ~32.  The `pd += d` walk of generate_local_course
// (dubins.rs:200-272) is left to steer_walk (lane-parallel, exact).
__global__ __launch_bounds__(kPrepThreads) void steer_prep_kernel(
    const DevState* __restrict__ st, SceneDev sc, const double* __restrict__ wsx,
    const double* __restrict__ wsy, const double* __restrict__ snap_pose,
    CandEntry* __restrict__ cand, PrepRec* __restrict__ rec, double* __restrict__ snap_yaw, const SteerTask* __restrict__ tasks,
    double* __restrict__ cost_out = nullptr, const StarTaskExt* __restrict__ ext = nullptr,
    const unsigned char* __restrict__ blk_in = nullptr) {
    // tasks != nullptr: explicit (child, parent pose) tasks [0, W) (multi-query batch); a task
    // with pnode < 0 is idle; own_yaw: the child keeps its heading cyaw (RRT* rewire edges)
    const int W = st->W;
    const int total = W + st->ncomp;
    const int lane = __lane_id(), wave = threadIdx.x >> 6;
    const int r = lane & (kPrepLanes - 1), g0 = lane & ~(kPrepLanes - 1);
    constexpr int TPW = 64 / kPrepLanes;  // tasks per wave in phase A
    static_assert(kPrepLanes == 8, "the per-task broadcasts are grp8_bcast (8-lane groups)");
    constexpr int TPB = kPrepThreads / 64 * TPW;  // tasks per workgroup
    const int* __restrict__ al = st->alist;  // (the batch's active-task list)
    for (int blk = blockIdx.x; blk * TPB < total; blk += gridDim.x) {
        const int ti = blk * TPB + wave * TPW + lane / kPrepLanes;
        const bool valid = ti < total;
        // t: the slot (the yaw's); list mode reads the compacted task and writes the record at ti
        const int t = (al && valid) ? al[ti] : ti;
        const int ri = al ? ti : t;
        // (window mode: a sample in an obstacle needs no steer — a kReject record)
        bool act = valid && !(blk_in && t < W && blk_in[t]);
        int j = 0, own = 0, cull = 0;
        double x = 0.0, y = 0.0, px = 1.0, py = 0.0, pyaw = 0.0, cyaw = 0.0;
        double cbase = 0.0, climit = 0.0;
        int force = -1;
        if (act && tasks) {
            const SteerTask tk = tasks[ri];
            act = tk.pnode >= 0;
            if (tk.literal >= 2) force = tk.literal - 2;  // (a cached verdict, mq_sample_nn)
            x = tk.x;
            y = tk.y;
            px = act ? tk.px : 1.0;
            py = act ? tk.py : 0.0;
            pyaw = act ? tk.pyaw : 0.0;
            if (ext) {
                const StarTaskExt ex = ext[t];
                own = ex.own_yaw;
                cyaw = ex.cyaw;
                cull = ex.cull;
                cbase = ex.cbase;
                climit = ex.climit;
            }
        } else if (act) {
            window_task(t, W, wsx, wsy, snap_pose, cand, &j, &px, &py, &pyaw);
            x = wsx[j];
            y = wsy[j];
        }
        double* yaw_dst = nullptr;
        if (valid) yaw_dst = (t < W || tasks) ? snap_yaw + t : &cand[t - W].yaw;
        prep_task(sc, r, g0, ri, valid, act, x, y, px, py, pyaw, own, cyaw, cull, cbase, climit,
                  rec, yaw_dst, cost_out, force);
    }
}

// steer_walk for one PrepRec (called by all 64 lanes; the record is wave-uniform).  Chunks of 63
// grid points: lane k >= 1 interpolates grid point base + k - 1 (interpolate, dubins.rs:155-198,
// then the world transform dubins.rs:412-422), lane 0 carries the previous chunk's last point,
// and the junction to the parent follows the last grid point.  The grid points' pd values come
// from the lane-parallel `pd += d` generator below, started from the state steer_prep kept
// (segment 0, pd = d), each lane capturing its own point.  npts (wave-uniform) += the polyline points generated and verified
// (grid points plus the junction; the profiled walk roofline's unit).
//
// gs: the wave's kGenSlots LDS doubles — the generator's kGenPts value slots, then the task's
// segment table (kSegRow doubles per segment: origin x, y, trig ca, sa, mode), written once per task
// by lanes 0-2, from which each point's lane reads its own segment's row (two ds_read_b128)
// instead of selecting among the twelve wave-uniform values.
//
// The three divisions by the curvature c per point (dubins.rs:169-178: length / c, sin / c,
// (1 - cos) / +-c) are x / c = q + (x - q c) / c rounded once: q = RN(x rc), the residual
// fma(-q, c, x) is exact, and RN(q + residual rc) with rc = RN(1 / c) is the correctly rounded
// quotient (Markstein's theorem; no x here is subnormal), i.e. bit-identical to the division —
// tests/test_div_identity.py checks the identity for the scenes' curvatures.  3 VALU instead of 9.
// A wave-uniform value into SGPRs: walk_rec's record fields.  A record in LDS is read with
// ds_read into VGPRs (~60 of them for the ~30 fields the walk keeps live); readfirstlane moves
// each into SGPRs, as the scalar loads of a global record do (there it folds away).
__device__ __forceinline__ double ufl(double v) {
    return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                            __builtin_amdgcn_readfirstlane(__double2loint(v)));
}
__device__ __forceinline__ int ufl(int v) { return __builtin_amdgcn_readfirstlane(v); }
constexpr int kGenPts = 68;  // generator slots: 63 points + 4 overshoot + 1
constexpr int kSegRow = 6;   // segment-table row (16-byte aligned rows: ds_read_b128)
template <bool kLds, int kScene = kSceneAny, bool kS = false>
__device__ __forceinline__ int walk_rec(const SceneDev& sc, const PrepRec* __restrict__ p,
                                        double* __restrict__ gs, int& npts, int& napts,
                                        bool junction = true) {
    const int lane = __lane_id();
    const int state = ufl(p->state);
    const double x = ufl(p->x), y = ufl(p->y), px = ufl(p->px), py = ufl(p->py);
    if (state == kPrepNone) {  // steer failed: polyline [(x, y), (px, py)] (rrt.rs:313)
        const bool has = lane < 2;
        const double qx = lane == 0 ? x : px, qy = lane == 0 ? y : py;
        npts += 2;
        return chunk_rejects<kLds, kScene>(sc, has, has, lane == 1, qx, qy) ? kReject : kAccept;
    }
    // (steer_prep stores no grid points: every walkable record is kPrepFallback at point 0)
    if (state != kPrepFallback) return state == kPrepWalk ? kError : state;
    const double step = sc.step_size;
    const double c = ufl(p->c), cw = ufl(p->cw), sw = ufl(p->sw);
    const double ox1 = ufl(p->ox[1]), oy1 = ufl(p->oy[1]), ox2 = ufl(p->ox[2]), oy2 = ufl(p->oy[2]);
    const double ca0 = ufl(p->ca[0]), ca1 = ufl(p->ca[1]), ca2 = ufl(p->ca[2]);
    const double sa0 = ufl(p->sa[0]), sa1 = ufl(p->sa[1]), sa2 = ufl(p->sa[2]);
    const double L0 = ufl(p->L[0]), L1 = ufl(p->L[1]), L2 = ufl(p->L[2]);
    const int m0 = ufl(p->m[0]), m1 = ufl(p->m[1]), m2 = ufl(p->m[2]);
    const double rc = 1.0 / c;
    double* segt = gs + kGenPts;
    if (lane < 3) {
        double* row = segt + kSegRow * lane;
        row[0] = lane == 0 ? 0.0 : (lane == 1 ? ox1 : ox2);
        row[1] = lane == 0 ? 0.0 : (lane == 1 ? oy1 : oy2);
        row[2] = lane == 0 ? ca0 : (lane == 1 ? ca1 : ca2);
        row[3] = lane == 0 ? sa0 : (lane == 1 ? sa1 : sa2);
        row[4] = (double)(lane == 0 ? m0 : (lane == 1 ? m1 : m2));
    }
    __builtin_amdgcn_wave_barrier();
    // the generator's initial state (segment 0, pd = d - 0.0, dubins.rs:239-241), from steer_prep
    int gseg = ufl(p->fb_seg);
    double gdd = ufl(p->fb_dd);
    double gpd = ufl(p->fb_pd);
    long long grid = 0;  // grid points generated (and counted) so far
    double carry_x = x, carry_y = y;
    npts += 1;  // point 0, the child
    // a long S segment against the discs (s_classify) or the polygon edges and bounds ring
    // (s_classify_poly), analytically: a sure hit rejects at once,
    // a sure clearance keeps only its first and last point (s_state 1: counted, s_emit of them
    // placed in lanes so far)
    bool s_clear = false;
    int s_state = 0, s_emit = 0;
    long long s_n = 0;
    double s_first = 0.0, s_last = 0.0, s_exit = 0.0;
    const int trim1 = ufl(p->trim1);
    const bool discs = kS && !trim1 &&
                       (kScene == kSceneDisc ||
                        (kScene == kSceneAny && !sc.bits && sc.ne == 0 && sc.nbv == 0)) &&
                       sc.m > 0;
    const bool polys = kS && !trim1 &&
                       (kScene == kScenePoly ||
                        (kScene == kSceneAny && !sc.bits && (sc.ne > 0 || sc.nbv > 0)));
    if ((discs || polys) && m1 == kModeS && L1 >= kSMinPts * step) {
        const double ax = cw * ox1 + sw * oy1 + x, ay = -sw * ox1 + cw * oy1 + y;
        const double pcb = div_by(L1, c, rc);
        const double lxb = ox1 + pcb * ca1, lyb = oy1 + pcb * sa1;
        const double bx = cw * lxb + sw * lyb + x, by = -sw * lxb + cw * lyb + y;
        const double dl = 1.0e-9 * (1.0 + fabs(ax) + fabs(ay) + fabs(bx) + fabs(by));
        const double sp = step * rc;  // the S points' spacing along AB
        const double t_lo = 3.0 * sp * (1.0 + 1.0e-9) + dl;
        const double t_hi = (L1 - step) * rc * (1.0 - 1.0e-9) - dl;
        const int cls = polys ? s_classify_poly<kLds>(sc, ax, ay, bx, by, t_lo, t_hi, dl)
                              : s_classify<kLds>(sc, ax, ay, bx, by, t_lo, t_hi,
                                                 sp * (1.0 + 1.0e-9) + 2.0 * dl, dl);
        if (cls == kSHit) return kReject;
        s_clear = cls == kSClear;
    }
    for (int base = 0;; base += 63) {
        int cnt = 0, my_seg = 0;
        double my_pd = 0.0;
        bool done;
        bool chord = false;  // lane 1 holds the cleared S segment's last point, lane 0 its first
        {
            // lane-parallel `pd += d` (dubins.rs:239-255): lane l >= pos replays l - pos
            // additions from the uniform start value — the serial walk's exact rounding
            // sequence — and the first lane whose |pd| exceeds |L| ends the segment (its value
            // gives ll and the next segment's start, dubins.rs:256-259)
            int pos = 1;
            while (pos <= 63 && gseg < 3) {
                if (s_clear && gseg == 1) {
                    // the cleared S segment: its first and last points only (s_classify), the
                    // rest counted; then the segment's end as the generator would reach it
                    if (s_state == 0) {
                        seg_count(gpd, gdd, L1, gs, s_n, s_last, s_exit);
                        s_first = gpd;
                        s_state = 1;
                    }
                    // The chord between the two lies within rounding of AB, so it clears and is
                    // not tested: the chunk ends after the first point, and the next one starts
                    // with the chord (lanes 0 -> 1), its box without lane 0 — so the long chord
                    // neither widens a chunk's item search nor meets the exact tests
                    const int n_emit = s_n >= 2 ? 2 : (int)s_n;
                    while (s_emit < n_emit && pos <= 63) {
                        if (s_emit == 1 && pos > 1) break;
                        if (lane == pos) {
                            my_seg = 1;
                            my_pd = s_emit == 0 ? s_first : s_last;
                        }
                        if (s_emit == 1) chord = true;
                        ++s_emit;
                        ++pos;
                        ++cnt;
                    }
                    if (s_emit < n_emit) break;  // the chunk ends: the next one goes on
                    grid += s_n - n_emit;
                    npts += s_n - n_emit;
                    const double ll = L1 - s_exit - gdd;
                    gseg = 2;
                    gdd = (L2 > 0.0) ? step : -step;
                    gpd = ((L1 * L2) > 0.0) ? (-gdd - ll) : (gdd - ll);
                    continue;
                }
                const double Ls = gseg == 0 ? L0 : (gseg == 1 ? L1 : L2);
                // the serial chain w_u = gpd (+ gdd) x u is the same in every lane: one f64 add
                // per step, lane 0 parks the values in the wave's LDS slots (gs) and lane pos + u
                // picks w_u up afterwards.  Within a segment the passing values form a prefix
                // (|pd| can only shrink before it grows), so the chain stops, 4 steps at a time,
                // once its latest value fails; lanes past the last generated value count as failed
                const int kk = lane - pos;
                const double aL = fabs(Ls);
                const int umax = 63 - pos;
                int u = umax;
                double v = gpd;
                // Closed form first: while the values keep w0's sign and exponent (one ulp u),
                // fl(w + d) = w + RN_u(d), so when the first two steps agree (w1 - w0 == w2 - w1
                // = delta; a tie-to-even would alternate them) w_k = w0 + k delta exactly — one
                // fma per lane, representable, so exact.  Checked over every value up to the
                // first one past |L|; any other pass (a binade or sign crossing inside the
                // chunk) takes the serial chain.  tests/test_walk_generator.py restates both.
                const double w1 = gpd + gdd, w2 = w1 + gdd;
                bool cf = (w1 - gpd) == (w2 - w1);
                if (cf) {
                    const double vc = __builtin_fma((double)(kk > 0 ? kk : 0), w1 - gpd, gpd);
                    const uint64_t fm = __ballot(kk >= 0 && !(fabs(vc) <= aL));
                    const int fl = fm ? (int)__builtin_ctzll(fm) : 63;
                    cf = __ballot(kk >= 0 && lane <= fl &&
                                  (__double2hiint(vc) >> 20) != (__double2hiint(gpd) >> 20)) == 0;
                    if (kk >= 0) v = vc;
                }
                if (!cf) {
                    double w = gpd;
                    if (lane == 0) gs[0] = w;
                    u = 0;
                    bool ended = !(fabs(w) <= aL);
                    while (!ended && u < umax) {
                        double t4[4];
#pragma unroll
                        for (int z = 0; z < 4; ++z) {
                            w += gdd;
                            t4[z] = w;
                        }
                        if (lane == 0) {
#pragma unroll
                            for (int z = 0; z < 4; ++z) gs[u + 1 + z] = t4[z];
                        }
                        u += 4;
                        ended = !(fabs(w) <= aL);
                    }
                    u = min(u, umax);
                    __builtin_amdgcn_wave_barrier();
                    v = (kk >= 0 && kk <= u) ? gs[kk] : gpd;
                }
                const uint64_t bad = __ballot(lane >= pos && (kk > u || !(fabs(v) <= aL)));
                const int m = bad ? (int)__builtin_ctzll(bad) : 64;
                if (lane >= pos && lane < m) {
                    my_seg = gseg;
                    my_pd = v;
                }
                if (m <= 63) {
                    const double pend = readlane_f64(v, m);
                    const double ll = Ls - pend - gdd;
                    if (++gseg < 3) {
                        const double Ln = gseg == 1 ? L1 : L2;
                        gdd = (Ln > 0.0) ? step : -step;
                        gpd = ((Ls * Ln) > 0.0) ? (-gdd - ll) : (gdd - ll);
                    }
                    cnt += m - pos;
                    pos = m;
                } else {
                    gpd = readlane_f64(v, 63) + gdd;
                    cnt += 64 - pos;
                    pos = 64;
                }
            }
            grid += cnt;
            done = gseg >= 3;
            // trim1: the last segment's final grid point landed in lane 63 (its next value is
            // past |L|): end here, so the drop below pops it in this chunk instead of one already
            // tested (the segment's end, dubins.rs:256, needs no ll: nothing follows)
            if (trim1 && !done && gseg == 2 && pos > 63 && !(fabs(gpd) <= fabs(L2))) {
                gseg = 3;
                done = true;
            }
        }
        // trim1 (prep_task): the chunk where the last segment ends pops its last grid point with
        // the endpoint; one generated in the previous chunk was tested already: literal path
        const bool drop = trim1 && done;
        if (drop && cnt == 0) return kLiteral;
        const int cnt_gen = cnt;  // grid points generated in this chunk (lanes 1 .. cnt_gen)
        if (drop) cnt -= 1;       // ... and kept
        const bool junction_here = done && cnt < 63;
        const bool isgen = lane >= 1 && lane <= cnt_gen;
        const bool isgrid = lane >= 1 && lane <= cnt;
        const bool isj = junction && junction_here && lane == cnt + 1;
        double qx = carry_x, qy = carry_y;
        int mm = kModeS;
        bool pop_more = false;  // the popped point's local x is 0.0 too: the trim goes on
        bool bad_arg = false;   // an arc point's pd outside sincos_small's range
        if (isgen) {
            const double* row = segt + kSegRow * my_seg;
            const double2 o2 = *reinterpret_cast<const double2*>(row);
            const double2 t2 = *reinterpret_cast<const double2*>(row + 2);
            mm = (int)row[4];
            const double ox = o2.x, oy = o2.y, ca = t2.x, sa = t2.y;
            const double pd = my_pd;
            double lx, ly;
            if (mm == kModeS) {
                const double pc = div_by(pd, c, rc);
                lx = ox + pc * ca;
                ly = oy + pc * sa;
            } else {
                // one argument reduction for both (walk -2..3%): ocml's own sincos, restated with
                // its constants behind an opaque pointer (sincos_small: no hoisted, spilled
                // coefficients); |pd| >= 2^30 (never on an L / R segment) goes to the literal path
                const double* tab = kSinCosTab;
                asm volatile("" : "+s"(tab));
                bad_arg = !(fabs(pd) < 0x1p30);
                double sp, cp;
                sincos_small(pd, tab, &sp, &cp);
                const double ldx = div_by(sp, c, rc);
                const double ld1 = div_by(1.0 - cp, c, rc);  // (1 - cos) / -c = -((1 - cos) / c)
                const double ldy = mm == kModeL ? ld1 : -ld1;
                const double gdx = ca * ldx + sa * ldy;
                const double gdy = -sa * ldx + ca * ldy;
                lx = ox + gdx;
                ly = oy + gdy;
            }
            qx = cw * lx + sw * ly + x;   // dubins.rs:415
            qy = -sw * lx + cw * ly + y;  // dubins.rs:420
            pop_more = drop && lane == cnt_gen && lx == 0.0;
        }
        if (isj) {
            qx = px;
            qy = py;
        }
        if (__any(pop_more || bad_arg)) return kLiteral;
        const bool has = lane == 0 || isgrid || isj;
        const bool chk = isgrid || isj || (base == 0 && lane == 0);
        npts += cnt + (junction && junction_here ? 1 : 0);
        napts += __popcll(__ballot(isgrid && mm != kModeS));
        if (chunk_rejects<kLds, kScene>(sc, has, chk, has && lane >= 1 && !(chord && lane == 1),
                                        qx, qy, !(chord && lane == 0)))
            return kReject;
        if (junction_here) break;
        // (the last point: lane 63, or lane cnt of a chunk ended before the chord)
        carry_x = readlane_f64(qx, cnt);
        carry_y = readlane_f64(qy, cnt);
    }
    // no trailing zero left for the trim (dubins.rs:281-288): the literal path decides
    if (1 + grid > (long long)ufl((double)p->n_point) - 2) return kLiteral;
    return kAccept;
}

// One edge on one wave from the wave-uniform SteerPrep of steer_prep(): the PrepRec that
// steer_prep_kernel would have written for it (segment trig of the origin yaws, the generator's
// initial state, no stored grid points), walked by walk_rec — the lane-parallel exact `pd`
// generator instead of the serial one of steer_walk.  junction = false: the polyline ends at the
// edge's last point (finalize's edge into the root).  gs: this wave's kGenSlots LDS doubles.
template <bool kLds, bool kS = false>
__device__ __forceinline__ int walk_edge(const SceneDev& sc, const SteerPrep& r, double* gs,
                                         bool junction, int& npts, int& napts) {
    if (r.state != kPrepWalk && r.state != kPrepNone) return r.state;
    PrepRec p;
    p.x = r.x;
    p.y = r.y;
    p.px = r.px;
    p.py = r.py;
    p.c = r.c;
    p.cw = r.cw;
    p.sw = r.sw;
    p.ox[0] = 0.0;
    p.oy[0] = 0.0;
    p.ox[1] = r.o1x;
    p.oy[1] = r.o1y;
    p.ox[2] = r.o2x;
    p.oy[2] = r.o2y;
    // segment trig (dubins.rs:155-198): S cos/sin(origin yaw), L/R cos/sin(-origin yaw)
    const double a0 = 0.0;
    const double a1 = r.m1 == kModeS ? r.o1yaw : -r.o1yaw;
    const double a2 = r.m2 == kModeS ? r.o2yaw : -r.o2yaw;
    p.ca[0] = cos(a0);
    p.sa[0] = sin(a0);
    p.ca[1] = cos(a1);
    p.sa[1] = sin(a1);
    p.ca[2] = cos(a2);
    p.sa[2] = sin(a2);
    p.L[0] = r.L0;
    p.L[1] = r.L1;
    p.L[2] = r.L2;
    p.m[0] = r.m0;
    p.m[1] = r.m1;
    p.m[2] = r.m2;
    p.cnt[0] = p.cnt[1] = p.cnt[2] = 0;
    p.n_point = r.n_point;
    p.state = r.state == kPrepNone ? kPrepNone : kPrepFallback;
    p.fb_dd = (r.L0 > 0.0) ? sc.step_size : -sc.step_size;
    p.fb_pd = p.fb_dd - 0.0;  // dubins.rs:239-241
    p.fb_seg = 0;
    p.trim1 = 0;
    p.yaw = p.pyaw = 0.0;
    return walk_rec<kLds, kSceneAny, kS>(sc, &p, gs, npts, napts, junction);
}

// steer_walk, one task per wave (persistent grid, grid-stride over the W + ncomp tasks); kLds:
// the scene's disc grid is staged into this workgroup's LDS first.
constexpr int kGenSlots = kGenPts + 3 * kSegRow;  // per-wave LDS doubles of walk_rec

// Explicit tasks (the verify_node API); waves <= kLiteralWaves so each wave owns one literal
// scratch buffer.  The fast path is the product's walk (walk_rec through walk_edge, with the
// analytic S segments), so the API's verdicts test the same code the planners run.
__global__ __launch_bounds__(256) void steer_tasks_kernel(SceneDev sc, TreeDev tr,
                                                          const SteerTask* __restrict__ tasks,
                                                          int n, int* __restrict__ out_status,
                                                          double* __restrict__ out_yaw,
                                                          double* __restrict__ scratch) {
    const int lane = __lane_id();
    const int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int nw = (int)((gridDim.x * blockDim.x) >> 6);
    double* bx = scratch ? scratch + (size_t)gw * 3 * kLiteralCap : nullptr;
    __shared__ double s_gen[4][kGenSlots];
    double* gs = s_gen[__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6))];
    int np = 0, na = 0;
    for (int t = gw; t < n; t += nw) {
        const SteerTask tk = tasks[t];
        double px = tk.px, py = tk.py, pyaw = tk.pyaw;
        if (tk.pnode >= 0) {
            px = tr.x[tk.pnode];
            py = tr.y[tk.pnode];
            pyaw = tr.yaw[tk.pnode];
        }
        const double yaw = atan2(py - tk.y, px - tk.x);
        int s;
        if (tk.literal && bx)
            s = steer_collide_literal(sc, tk.x, tk.y, yaw, px, py, pyaw, bx, bx + kLiteralCap,
                                      bx + 2 * kLiteralCap);
        else if (tk.literal)
            s = kError;
        else
            s = walk_edge<false, true>(sc, steer_prep(sc, tk.x, tk.y, yaw, px, py, pyaw), gs, true,
                                       np, na);
        if (lane == 0) {
            out_status[t] = s;
            out_yaw[t] = yaw;
        }
    }
}

constexpr int kWalkMaxWG = 768;  // 3 resident workgroups per CU
__host__ __device__ inline int walk_lds_bytes(int scene_bytes) {
    return scene_bytes + kWalkThreads / 64 * kGenSlots * 8;
}
// Window mode (pend != nullptr): a snapshot task whose verdict is not final (literal path,
// error) and that has no nearer window sample is queued for the resolve (the others were queued
// by nn_finalize's pair search).  wg_points (profiling only, else null): workgroup b adds its
// walked polyline points to wg_points[b] (its own slot: no atomics on a shared address).
// kMinW: minimum waves per SIMD the compiler must allow (register budget).  The window pipeline
// walks ~1 task per wave (1: 94 VGPRs, 2 workgroups per CU); the query batches walk dozens of
// tasks per wave, latency-bound, and run better at 6 (80 VGPRs, 3 workgroups per CU: config 3
// 279 -> 309 M it/s; 8 spills too much).
constexpr int kWalkMinWWindow = 1;
constexpr int kWalkMinWBatch = 6;
// RRT* scenes (config 5) carry a ~58 KB LDS image, so LDS holds the walk at 2 workgroups per CU
// whatever the register budget: the uncapped budget wins there (16.46 vs 15.96 M it/s, r02 A/B).
constexpr int kWalkMinWStar = kWalkMinWWindow;
template <bool kLds, int kMinW, int kScene, bool kS>
__global__ __launch_bounds__(kWalkThreads, kMinW) void steer_walk_kernel(DevState* __restrict__ st,
                                                         SceneDev sc,
                                                         const PrepRec* __restrict__ rec,
                                                         CandEntry* __restrict__ cand,
                                                         int* __restrict__ snap_status,
                                                         const int* __restrict__ cand_cnt,
                                                         int* __restrict__ pend,
                                                         long long* __restrict__ wg_points) {
    const int lane = __lane_id();
    const int W = st->W;
    const int total = W + st->ncomp;
    if ((int)blockIdx.x >= total) return;
    // (the wave index as a wave-uniform value: threadIdx.x itself need not stay live)
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const bool t0 = threadIdx.x == 0;
    if (kLds) stage_scene(sc);
    double* gs = reinterpret_cast<double*>(pp_smem + (kLds ? sc.lds_bytes : 0)) +
                 wv * kGenSlots;  // this wave's generator slots
    int npts = 0, napts = 0, ntasks = 0;
    // Workgroup b walks the tasks b, b + G, b + 2G, ... (G = the grid); its waves take them one
    // at a time from an LDS counter, so a wave that drew short paths takes more of them (a
    // workgroup's share is a sum of dozens of tasks: far more even than a wave's handful under a
    // static stride), and consecutive tasks — one query's window, similar paths — land on
    // different workgroups.  No global atomics.  (Contiguous ranges per workgroup measured 10%
    // slower on config 5's walk.)
    __shared__ int s_next;
    const int G = (int)gridDim.x;
    if (t0) s_next = 0;
    const int* __restrict__ al = st->alist;  // (the batch's active-task list)
    const int lper = (total + G - 1) / G;
    if (al && blockIdx.x == 0 && t0) {
        st->lgrid = G;
        st->lper = lper;
    }
    __syncthreads();
    for (;;) {
        int k = 0;
        if (lane == 0) k = atomicAdd(&s_next, 1);
        const int ti = (int)blockIdx.x + G * __builtin_amdgcn_readlane(k, 0);
        if (ti >= total) break;
        // (list mode: the record is at ti; the slot t only addresses the verdict's store)
        const int t = al ? al[ti] : ti;
        const int s = walk_rec<kLds, kScene, kS>(sc, rec + ti, gs, npts, napts);
        ++ntasks;
        if (lane == 0) {
            if (al || t < W) {
                // (list mode: the workgroup's run of verdicts, DevState::lgrid / lper)
                snap_status[al ? (int)blockIdx.x * lper + (ti - (int)blockIdx.x) / G : t] = s;
                if (pend && s != kAccept && s != kReject && cand_cnt[t] == 0)
                    pend[atomicAdd(&st->npend, 1)] = t;
            } else {
                cand[t - W].status = s;
            }
        }
    }
    if (wg_points) {  // [b]: points, [kWalkTallySlots + b]: their arc points, [2 kWalkTallySlots + b]: tasks
        __shared__ int s_np[3][kWalkThreads / 64];
        if (lane == 0) {
            s_np[0][wv] = npts;
            s_np[1][wv] = napts;
            s_np[2][wv] = ntasks;
        }
        __syncthreads();
        if (wv == 0 && lane < 3) {
            long long sum = 0;
            for (int w = 0; w < kWalkThreads / 64; ++w) sum += s_np[lane][w];
            wg_points[blockIdx.x + lane * kWalkTallySlots] += sum;
        }
    }
}

// The walk's persistent grid: the workgroups that can be resident at once, so no workgroup starts
// late with a share of tasks — the device's CU count times the workgroups per CU the occupancy
// API gives for this instantiation and its dynamic LDS (the scene image decides; at most 4 of 8
// waves each), read once per (device, image size) instead of assuming 256 CUs and 160 KB.
// kMaxPerCU: the query batch's walk runs beside the other sub-batch stream's kernels and does best
// at 2 workgroups per CU although 3 fit (a 1024-query shard 171 -> 179-183 M it/s, the 8192-query
// batch unchanged).
// The walk instantiation for a scene: LDS image or not, and its mode (scene_kind), as a callable
// applied to the kernel (launch or occupancy query).
// (polygon scenes walk at most 5 waves per SIMD: their edge tests do not fit the 6-wave budget
// without scratch; with the analytic S segments at most 4: s_classify_poly spills ~80 B at 5)
template <int kMinW, bool kS = false, typename F>
inline hipError_t walk_kernel_for(const SceneDev& sc, F&& f) {
    const bool lds = sc.lds_bytes > 0;
    constexpr int kPolyCap = kS ? 4 : 5;
    constexpr int kMinWPoly = kMinW > kPolyCap ? kPolyCap : kMinW;
    switch (scene_kind(sc)) {
        case kSceneGrid:
            return lds ? f(steer_walk_kernel<true, kMinW, kSceneGrid, kS>)
                       : f(steer_walk_kernel<false, kMinW, kSceneGrid, kS>);
        case kScenePoly:
            return lds ? f(steer_walk_kernel<true, kMinWPoly, kScenePoly, kS>)
                       : f(steer_walk_kernel<false, kMinWPoly, kScenePoly, kS>);
        default:
            return lds ? f(steer_walk_kernel<true, kMinW, kSceneDisc, kS>)
                       : f(steer_walk_kernel<false, kMinW, kSceneDisc, kS>);
    }
}

// (kS: the instantiation that is launched — the S classes change a polygon walk's budget)
template <int kMinW = kWalkMinWWindow, int kMaxPerCU = 4, bool kS = false>
inline int walk_grid_cap(const SceneDev& sc) {
    static std::mutex mu;
    static std::map<std::tuple<int, int, int>, int> cache;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    std::lock_guard<std::mutex> lk(mu);
    const std::tuple<int, int, int> key{dev, sc.lds_bytes, scene_kind(sc)};
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int cus = 256, per_cu = 0;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0)
        cus = prop.multiProcessorCount;
    const hipError_t e = walk_kernel_for<kMinW, kS>(sc, [&](auto kern) {
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kWalkThreads,
                                                            walk_lds_bytes(sc.lds_bytes));
    });
    if (e != hipSuccess || per_cu < 1) per_cu = 1;
    per_cu = std::min(kMaxPerCU, per_cu);
    const int cap = cus * per_cu;
    cache[key] = cap;
    return cap;
}

// steer_walk_kernel over a task set on stream s (its instantiation for the scene)
template <int kMinW, bool kS = false>
inline void launch_walk(hipStream_t s, int blocks, DevState* st, const SceneDev& sc,
                        const PrepRec* rec, CandEntry* cand, int* status,
                        const int* cand_cnt, int* pend, long long* wg_points) {
    (void)walk_kernel_for<kMinW, kS>(sc, [&](auto kern) {
        kern<<<blocks, kWalkThreads, walk_lds_bytes(sc.lds_bytes), s>>>(
            st, sc, rec, cand, status, cand_cnt, pend, wg_points);
        return hipSuccess;
    });
}

// A resolve repair (one wave): the (child, parent pose) pair steered and collision-checked anew
// (only resolve_tail_kernel compiles it: inlined there it needs no scratch).
__device__ __forceinline__ int resolve_repair(const SceneDev& sc, double x, double y,
                                                        double yaw, double px, double py,
                                                        double pyaw, int lit, double* bx) {
    return lit ? steer_collide_literal(sc, x, y, yaw, px, py, pyaw, bx, bx + kLiteralCap,
                                       bx + 2 * kLiteralCap)
               : steer_collide_fast<false>(sc, x, y, yaw, px, py, pyaw);
}

// The sequential-consistency resolve of one window's PENDING samples, on one workgroup with its
// state in LDS.  A sample is pending when nn_finalize's pair search found an earlier window sample strictly
// nearer than its snapshot NN, or when its snapshot verdict is not final (literal path, error);
// every other sample is decided by its snapshot verdict and never touches the resolve.  The
// replay: sample j's parent is the first ACCEPTED entry of its candidate list in (d2, i) order,
// else its snapshot NN.  Output per pending j < weff: snap_status[j] = verdict | kWinParent
// (parent = window sample fin_par[j]), snap_yaw[j] = its final yaw.  commit_role then appends
// the window.
constexpr int kResolveEnt = 1024;  // candidate-list positions staged in LDS (the rest: rs.order)
struct ResolveLds {
    double yaw[kMaxWindow];          // slot: snapshot yaw, then a repair's, then the final one
    double ed[kResolveEnt];          // list position: d2 (the sort key), then the entry's yaw
    int j[kMaxWindow];               // slot -> sample
    int round[kMaxWindow];           // slot: decided flag (published last)
    int par[kMaxWindow];             // slot: -1 snapshot NN, else window sample index
    int off[kMaxWindow];             // slot: first list position
    int cnt[kMaxWindow];             // slot: list length (<= kCandCap); first the fill counter
    int ei[kResolveEnt];             // list position: candidate sample i
    int ee[kResolveEnt];             // list position: entry index into cand[]
    int ec[kResolveEnt];             // list position: i's slot, or -1 / -2 (rejected / accepted by
                                     // its snapshot verdict)
    short slot[kMaxWindow];          // sample -> pending slot, -1: decided by its snapshot
    signed char verdict[kMaxWindow]; // slot: snapshot status until decided, then 0/1
    signed char rep[kMaxWindow];     // slot: repair verdict (-1: none) | 16 if literal
    signed char es[kResolveEnt];     // list position: the entry's speculative status
    int total, err, bail;
    int stat[4];                     // repair passes, repairs, literal repairs, max passes of a wave
};

// kRepair = false (the window kernel): no repair code is compiled in (it would spill at the
// window kernel's 128-VGPR budget); a window that needs a repair returns false without
// publishing anything and resolve_tail_kernel redoes it with repairs.
template <bool kRepair, int NT>
__device__ __attribute__((always_inline)) inline bool resolve_role(
    DevState* __restrict__ st, const SceneDev& sc, const TreeDev& tr,
    const double* __restrict__ wsx, const double* __restrict__ wsy,
    const int* __restrict__ nn_idx, const int* __restrict__ cand_cnt,
    const CandEntry* __restrict__ cand, const int* __restrict__ pend,
    int* __restrict__ snap_status, double* __restrict__ snap_yaw, int* __restrict__ fin_par,
    ResolveScratch rs, double* __restrict__ lit_scratch, int W, char* smem) {
    constexpr int KW = kMaxWindow;
    constexpr int kEntLds = kResolveEnt;
    ResolveLds& L = *reinterpret_cast<ResolveLds*>(smem);
    auto& s_slot = L.slot;
    auto& s_j = L.j;
    auto& s_round = L.round;
    auto& s_par = L.par;
    auto& s_yaw = L.yaw;
    auto& s_off = L.off;
    auto& s_cnt = L.cnt;
    auto& s_verdict = L.verdict;
    auto& s_rep = L.rep;
    auto& s_ei = L.ei;
    auto& s_ee = L.ee;
    auto& s_ec = L.ec;
    auto& s_ed = L.ed;
    auto& s_es = L.es;
    auto& s_total = L.total;
    auto& s_err = L.err;
    auto& s_stat = L.stat;
    auto& s_bail = L.bail;
    const int Weff = min(W, st->weff);
    const int npend = min(st->npend, KW);
    const int ncomp = st->ncomp;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    if (tid < 4) s_stat[tid] = 0;
    if (tid == 0) {
        s_total = 0;
        s_err = 0;
        s_bail = 0;
    }
    for (int j = tid; j < W; j += NT) s_slot[j] = -1;
    __syncthreads();
    // 1. slots: every load of the pass is issued before any of them is used
    for (int q = tid; q < npend; q += NT) {
        const int j = pend[q];
        const int c = cand_cnt[j];
        const int ss = snap_status[j];
        const double sy = snap_yaw[j];
        s_slot[j] = (short)q;
        s_j[q] = j;
        s_round[q] = 0;
        const int k = min(c, kCandCap);
        s_off[q] = atomicAdd(&s_total, k);
        s_cnt[q] = 0;
        s_verdict[q] = (signed char)ss;
        s_yaw[q] = sy;
        s_rep[q] = -1;
    }
    __syncthreads();
    // 2. lists: each entry goes to its sample's segment (then sorted by (d2, i))
    for (int e = tid; e < ncomp; e += NT) {
        const CandEntry ce = cand[e];
        const int q = s_slot[ce.j];
        const int k = s_off[q] + atomicAdd(&s_cnt[q], 1);
        const int qi = s_slot[ce.i];
        const int code = qi >= 0 ? qi : (snap_status[ce.i] == kAccept ? -2 : -1);
        if (k < kEntLds) {
            s_ei[k] = ce.i;
            s_ee[k] = e;
            s_ec[k] = code;
            s_ed[k] = ce.d2;
        } else {
            rs.order[k] = e;
        }
    }
    __syncthreads();
    auto ent_e = [&](int k) { return k < kEntLds ? s_ee[k] : rs.order[k]; };
    auto ent_i = [&](int k) { return k < kEntLds ? s_ei[k] : cand[rs.order[k]].i; };
    auto ent_c = [&](int k) {
        if (k < kEntLds) return s_ec[k];
        const int i = cand[rs.order[k]].i;
        const int qi = s_slot[i];
        return qi >= 0 ? qi : (snap_status[i] == kAccept ? -2 : -1);
    };
    for (int q = tid; q < npend; q += NT) {  // insertion sort of each list by (d2, i)
        const int o = s_off[q], k = s_cnt[q];
        if (o + k > kEntLds) continue;  // lists past the LDS part: sorted below (global)
        for (int a2 = 1; a2 < k; ++a2) {
            const double d = s_ed[o + a2];
            const int ii = s_ei[o + a2], ee = s_ee[o + a2], cc = s_ec[o + a2];
            int b2 = a2 - 1;
            while (b2 >= 0 && (s_ed[o + b2] > d || (s_ed[o + b2] == d && s_ei[o + b2] > ii))) {
                s_ed[o + b2 + 1] = s_ed[o + b2];
                s_ei[o + b2 + 1] = s_ei[o + b2];
                s_ee[o + b2 + 1] = s_ee[o + b2];
                s_ec[o + b2 + 1] = s_ec[o + b2];
                --b2;
            }
            s_ed[o + b2 + 1] = d;
            s_ei[o + b2 + 1] = ii;
            s_ee[o + b2 + 1] = ee;
            s_ec[o + b2 + 1] = cc;
        }
    }
    for (int q = tid; q < npend; q += NT) {  // the rare lists that straddle or pass kEntLds
        const int o = s_off[q], k = s_cnt[q];
        if (o + k <= kEntLds) continue;
        // materialise the whole list in rs.order, then sort it there
        for (int a2 = 0; a2 < k; ++a2)
            if (o + a2 < kEntLds) rs.order[o + a2] = s_ee[o + a2];
        for (int a2 = 1; a2 < k; ++a2) {
            const int e = rs.order[o + a2];
            const double d = cand[e].d2;
            const int ii = cand[e].i;
            int b2 = a2 - 1;
            while (b2 >= 0) {
                const int eb = rs.order[o + b2];
                if (cand[eb].d2 < d || (cand[eb].d2 == d && cand[eb].i < ii)) break;
                rs.order[o + b2 + 1] = eb;
                --b2;
            }
            rs.order[o + b2 + 1] = e;
        }
        for (int a2 = 0; a2 < k && o + a2 < kEntLds; ++a2) {  // refresh the LDS part
            const int e = rs.order[o + a2];
            const int i = cand[e].i;
            const int qi = s_slot[i];
            s_ee[o + a2] = e;
            s_ei[o + a2] = i;
            s_ed[o + a2] = cand[e].d2;
            s_ec[o + a2] = qi >= 0 ? qi : (snap_status[i] == kAccept ? -2 : -1);
        }
    }
    __syncthreads();
    for (int k = tid; k < min(s_total, kEntLds); k += NT) {  // the entries' speculative verdicts
        const int e = s_ee[k];
        const int es = cand[e].status;
        const double ey = cand[e].yaw;
        s_es[k] = (signed char)es;
        s_ed[k] = ey;
    }
    __syncthreads();
    // 3. decisions, without workgroup barriers: every wave passes over its own slots until all of
    //    them are decided, reading the other slots' decisions from LDS as they appear.  A decision
    //    is final once published (its flag is stored last, with release order), and every
    //    dependency points to an earlier sample, so the earliest undecided slot can always be
    //    decided: the passes terminate.  A pair nobody speculated on is re-steered by the wave
    //    that owns the slot, between its passes.
    int64_t n_rounds_rep = 0, n_rep = 0, n_lit = 0, n_rounds = 0;
    for (int pass = 0; pass < (1 << 20); ++pass) {
        ++n_rounds;
        bool left = false;
        int rq = -1, rpar = -1, rlit = 0;  // this lane's repair request (one per pass)
        for (int q = tid; q < npend; q += NT) {
            if (__hip_atomic_load(&s_round[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
                continue;
            const int j = s_j[q];
            if (j >= Weff) continue;
            int parent = -1, pos = -1, pq = -1;
            bool blocked = false;
            const int k = s_cnt[q], o = s_off[q];
            int a2 = 0;
            for (; a2 < k; ++a2) {
                const int code = ent_c(o + a2);
                if (code >= 0) {
                    if (!__hip_atomic_load(&s_round[code], __ATOMIC_ACQUIRE,
                                           __HIP_MEMORY_SCOPE_WORKGROUP)) {
                        blocked = true;  // an earlier candidate is still undecided
                        break;
                    }
                    if (!s_verdict[code]) continue;
                } else if (code == -1) {
                    continue;
                }
                parent = ent_i(o + a2);
                pos = o + a2;
                pq = code;
                break;
            }
            if (blocked) {
                // the entries before the blocker are final rejections: the next pass starts at
                // the blocker (only this thread touches slot q's list bounds in the passes)
                s_off[q] = o + a2;
                s_cnt[q] = k - a2;
                left = true;
                continue;
            }
            int status = -1, lit_done = 0;
            double y = 0.0;
            const int rp = s_rep[q];
            if (rp >= 0) {
                status = rp & 15;
                lit_done = rp >> 4;
                y = s_yaw[q];
            } else if (parent < 0) {
                status = s_verdict[q];
                y = s_yaw[q];
            } else if (pq < 0 || s_par[pq] < 0) {  // parent kept its snapshot parent: speculated
                if (pos < kEntLds) {
                    status = s_es[pos];
                    y = s_ed[pos];
                } else {
                    const int e = ent_e(pos);
                    status = cand[e].status;
                    y = cand[e].yaw;
                }
            }
            if (status < 0 || (status == kLiteral && !lit_done)) {
                left = true;
                if (rq < 0) {
                    rq = q;
                    rpar = parent;
                    rlit = status == kLiteral;
                }
                continue;
            }
            if (status != kAccept && status != kReject) s_err = 1;  // kError
            s_verdict[q] = status == kAccept;
            s_par[q] = parent;
            s_yaw[q] = y;
            __hip_atomic_store(&s_round[q], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        // repairs requested by this wave's lanes, one wave-wide steer each
        uint64_t m = __ballot(rq >= 0);
        if constexpr (!kRepair) {
            if (m && lane == 0) s_bail = 1;
            if (__hip_atomic_load(&s_bail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
        } else {
            if (m) ++n_rounds_rep;
            while (m) {
                const int l = (int)__builtin_ctzll(m);
                m &= m - 1;
                const int q = __shfl(rq, l), p = __shfl(rpar, l), lit = __shfl(rlit, l);
                const int j = s_j[q];
                const double x = wsx[j], y = wsy[j];
                double px, py, pyaw;
                if (p < 0) {
                    const int nq = nn_idx[j];
                    px = tr.x[nq];
                    py = tr.y[nq];
                    pyaw = tr.yaw[nq];
                } else {
                    px = wsx[p];
                    py = wsy[p];
                    const int pq = s_slot[p];
                    pyaw = pq >= 0 ? s_yaw[pq] : snap_yaw[p];
                }
                const double yaw = atan2(py - y, px - x);
                double* bx = lit_scratch + (size_t)wave * 3 * kLiteralCap;
                const int sres = resolve_repair(sc, x, y, yaw, px, py, pyaw, lit, bx);
                if (lane == 0) {
                    s_rep[q] = (signed char)(sres | (lit << 4));
                    s_yaw[q] = yaw;
                }
                ++n_rep;
                n_lit += lit;
            }
        }
        if (!__any(left)) break;
    }
    if (lane == 0) {  // per-wave statistics (wave-uniform values)
        atomicAdd(&s_stat[0], (int)n_rounds_rep);
        atomicAdd(&s_stat[1], (int)n_rep);
        atomicAdd(&s_stat[2], (int)n_lit);
        atomicMax(&s_stat[3], (int)n_rounds);
    }
    __syncthreads();
    if (!kRepair && s_bail) return false;
    // 4. publish the pending verdicts for window_commit
    for (int q = tid; q < npend; q += NT) {
        const int j = s_j[q];
        if (j >= Weff) continue;
        const int p = s_par[q];
        snap_status[j] = (s_verdict[q] ? kAccept : kReject) | (p >= 0 ? kWinParent : 0);
        snap_yaw[j] = s_yaw[q];
        fin_par[j] = p;
    }
    if (tid == 0) {
        if (s_err) st->error = 1;
        st->repair_rounds += s_stat[0];
        st->repairs += s_stat[1];
        st->literal_repairs += s_stat[2];
    }
    return true;
}

// Append the window (rrt.rs:586-589): the accepted samples j < weff get consecutive node indices
// in iteration order (a prefix sum of the verdict words in LDS, so a window parent's node index is
// known), then DevState advances.  A truncated window (weff < W) restarts the next window at
// sample weff: the window screened concurrently (seq) is void.
template <int NT>
__device__ __attribute__((always_inline)) inline void commit_role(
    DevState* __restrict__ st, const TreeDev& tr, const double* __restrict__ wsx,
    const double* __restrict__ wsy, const int* __restrict__ nn_idx,
    const int* __restrict__ snap_status, const double* __restrict__ snap_yaw,
    const int* __restrict__ fin_par, int* __restrict__ cand_cnt, int W, int64_t void_next,
    int64_t screened, const SampleRec& hrec, char* smem) {
    constexpr int PER = kMaxWindow / NT;
    static_assert(PER % 4 == 0, "commit: whole int4 loads per thread");
    int* s_node = reinterpret_cast<int*>(smem);
    int* s_wave = s_node + kMaxWindow;
    const int Weff = min(W, st->weff);
    const int n0 = st->n;
    const int64_t it0 = st->it;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int j0 = tid * PER;
    int v[PER];
    if (j0 + PER <= Weff) {
#pragma unroll
        for (int u = 0; u < PER; u += 4) {
            const int4 w4 = *reinterpret_cast<const int4*>(snap_status + j0 + u);
            v[u] = w4.x;
            v[u + 1] = w4.y;
            v[u + 2] = w4.z;
            v[u + 3] = w4.w;
        }
    } else {
#pragma unroll
        for (int u = 0; u < PER; ++u) v[u] = j0 + u < Weff ? snap_status[j0 + u] : 0;
    }
    int local = 0;
#pragma unroll
    for (int u = 0; u < PER; ++u) local += v[u] & 1;
    const int x = wave_incl_scan(local);
    if (lane == 63) s_wave[wave] = x;
    __syncthreads();
    int base = 0, total = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
        base += w < wave ? s_wave[w] : 0;
        total += s_wave[w];
    }
    int node = n0 + base + x - local;
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        s_node[j0 + u] = node;
        node += v[u] & 1;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int j = j0 + u;
        if (j < Weff && (v[u] & 1)) {
            const int nd = s_node[j];
            const double xx = wsx[j], yy = wsy[j];
            tr.x[nd] = xx;
            tr.y[nd] = yy;
            tr.x32[nd] = (float)xx;
            tr.y32[nd] = (float)yy;
            tr.yaw[nd] = snap_yaw[j];
            tr.parent[nd] = (v[u] & kWinParent) ? s_node[fin_par[j]] : nn_idx[j];
        }
        if (j < W) cand_cnt[j] = 0;  // the next window's pair counts start at zero
    }
    if (hrec.par || hrec.yaw || hrec.ok) {  // pp_rrt_extend_samples: every committed iteration
#pragma unroll
        for (int u = 0; u < PER; ++u) {
            const int j = j0 + u;
            if (j >= Weff) continue;
            const int64_t r = it0 + j - hrec.base;
            if (hrec.ok) hrec.ok[r] = (unsigned char)(v[u] & 1);
            if (hrec.par) hrec.par[r] = (v[u] & kWinParent) ? s_node[fin_par[j]] : nn_idx[j];
            if (hrec.yaw) hrec.yaw[r] = snap_yaw[j];
        }
    }
    if (tid == 0) {
        st->n = n0 + total;
        st->it = it0 + Weff;
        st->iterations += Weff;
        st->accepted += total;
        st->windows += 1;
        st->truncations += Weff < W;
        st->nn_flagged += st->flag_count;
        // the screen's distance evaluations: the samples it covered (not in an obstacle) x the
        // tree nodes it scanned (nodes past n_scan are nn_finalize's, a few per window)
        st->node_evals += screened;
        if (Weff < W) {
            st->it_spec = it0 + Weff;
            if (void_next >= 0) st->void_seq = void_next;
        }
        // adaptive window (a young tree: the window's samples are mostly nearer to each other than
        // to the tree, lists overflow and windows are cut): a cut window shrinks the next draws to
        // the power of two at or above where it stopped, a full one doubles them (<= K, clamped by
        // the draws).  Only the speed depends on it: the results are those of one sample at a time.
        int kd = st->kdyn > 0 ? st->kdyn : kMaxWindow;
        if (Weff < W) {
            kd = kMinDynWindow;
            while (kd < Weff) kd <<= 1;
        } else if (W >= kd) {
            kd = min(2 * kd, kMaxWindow);
        }
        st->kdyn = kd;
    }
}

// The window kernel: workgroup 0 resolves and commits the previous window (or, in the drain
// launch, the batch's last one) while workgroups 1.. screen this window's samples.  One LDS image
// serves the role of each workgroup (ResolveLds / the commit prefix / the screen's wave merge).
constexpr int kWinLds = (int)sizeof(ResolveLds);
static_assert(kWinLds <= 160 * 1024, "window kernel LDS");
static_assert((int)((3 * kScanWaves + 1) * kQPB * 4) <= kWinLds, "screen merge fits the LDS image");
static_assert(kSamplesLds <= kWinLds, "samples_role fits the window kernel's LDS image");
static_assert(kScreenStageOff % 16 == 0 && kScreenStageOff + 3 * kStage * 4 + 16 <= kWinLds,
              "screen staging (x, y, |n-o|^2 of kStage nodes + the piece counter) fits");
static_assert(kStage % 256 == 0 && kGrab % kScanBlk == 0, "whole DMA quarters and blocks");


__global__ __launch_bounds__(kScanThreads) void window_kernel(WinKArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[kWinLds];
    if (blockIdx.x == 0) {
        DevState* st = a.st;
        if (a.resolve) {
            const int W = st->W;
            if (W > 0) {
                const int q = 1 - a.p;
                if (!resolve_role<kWinRepair, kScanThreads>(st, a.sc, a.tr, a.wsx[q], a.wsy[q], a.nn_idx,
                                                       a.cand_cnt, a.cand, a.pend, a.snap_status,
                                                       a.snap_yaw, a.fin_par, a.rs, a.lit_scratch,
                                                       W, smem)) {
                    if (threadIdx.x == 0) st->resolve_bail = 1;  // resolve_tail_kernel redoes it
                    return;
                }
                // (same workgroup: the barrier's workgroup-scope fence orders these stores)
                __syncthreads();
                commit_role<kScanThreads>(st, a.tr, a.wsx[q], a.wsy[q], a.nn_idx, a.snap_status,
                                          a.snap_yaw, a.fin_par, a.cand_cnt, W,
                                          a.scan ? a.seq : -1,
                                          (int64_t)st->Wsp[q] * st->nsp[q], a.hrec, smem);
            }
        }
        if (threadIdx.x == 0) {  // the screened window's counters start at zero
            st->flag_count = 0;
            st->ncomp = 0;
            st->npend = 0;
            // no cut yet: nn_finalize's workgroups lower it with atomicMin in any order (a plain
            // store there raced with the early finishers)
            st->weff = 0x7fffffff;
        }
        return;
    }
    if (a.scan) {
        if (a.gen)
            scan_role<true>(a, (int)blockIdx.x - 1, smem);
        else
            scan_role<false>(a, (int)blockIdx.x - 1, smem);
    }
}

// The resolve + commit of a window whose resolve in the window kernel needed a repair (a pair
// nobody speculated on, or the literal path): redone here with the repairs, at kResolveThreads
// (256 VGPRs each, no spill).  A no-op launch otherwise.
__global__ __launch_bounds__(kResolveThreads) void resolve_tail_kernel(WinKArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[kWinLds];
    DevState* st = a.st;
    if (!st->resolve_bail) return;
    const int q = 1 - a.p;
    const int W = st->W;
    resolve_role<true, kResolveThreads>(st, a.sc, a.tr, a.wsx[q], a.wsy[q], a.nn_idx, a.cand_cnt,
                                         a.cand, a.pend, a.snap_status, a.snap_yaw, a.fin_par,
                                         a.rs, a.lit_scratch, W, smem);
    // (same workgroup: the barrier's workgroup-scope fence orders these stores)
    __syncthreads();
    commit_role<kResolveThreads>(st, a.tr, a.wsx[q], a.wsy[q], a.nn_idx, a.snap_status,
                                 a.snap_yaw, a.fin_par, a.cand_cnt, W, a.scan ? a.seq : -1,
                                 (int64_t)st->Wsp[q] * st->nsp[q], a.hrec, smem);
    if (threadIdx.x == 0) {
        st->resolve_bail = 0;
        st->flag_count = 0;
        st->ncomp = 0;
        st->npend = 0;
        st->weff = 0x7fffffff;
    }
}

// ---------------------------------------------------------------- check_finish
//
// RRT::check_finish (rrt.rs:428-438) for a batch of tree nodes, ONE WAVE PER NODE (kCfWaves
// independent waves per workgroup, nodes from a launch-wide counter), the node's ancestor path
// root..node in the wave's region of a global path buffer (kCfMaxDepth ints per wave):
//   optimize (rrt.rs:463-487)   level i: candidates path[0..L] root first, steered + collided one
//                               at a time on the wave, the first accepted one wins (memoised per
//                               tree node in ftab); recursion = the next level on that ancestor;
//                               RECURSION_LIMIT 16.  Every candidate parent is a tree node, so
//                               verifying edge ++ [to] is verify(line_to_origin(new)) (§3.2).
//   finalize (rrt.rs:503-540)   the chain goal → optimised copies → tree path → root; every edge
//                               is verified with its junction chord, the edge into the root
//                               without one (the root contributes no point); a None steer is the
//                               reference's panic (rrt.rs:529).
//   length                      verified finishes: the edges' literal Dubins points, then
//                               euclidean_length of the reversed line summed in line order.
struct CfPose {
    double x, y, yaw;
};
constexpr int kCfThreads = 64 * kCfWaves;

__device__ inline bool same_pose(const CfPose& a, const CfPose& b) {
    return __double_as_longlong(a.x) == __double_as_longlong(b.x) &&
           __double_as_longlong(a.y) == __double_as_longlong(b.y) &&
           __double_as_longlong(a.yaw) == __double_as_longlong(b.yaw);
}

// verify one edge a → b (+ junction chord to b unless junction is false) on one wave; kCfPanic
// when the steer is None (finalize's panic; verify_node's callers never pass such an edge here).
enum : int { kCfPanic = 6 };
// A literal-path scratch buffer (3 x kLiteralCap doubles) from a pool of kLiteralWaves slots,
// so kernels of any width can run the measure-zero literal path: lane 0 takes a free slot with
// atomicCAS (0 free, 1 taken), spinning over the pool if every slot is held — a holder is a
// running wave that releases after its bounded literal walk.  Called by all lanes.
__device__ __forceinline__ int lit_acquire(int* locks, int hint) {
    int slot = 0;
    if ((__lane_id()) == 0)
        for (int i = 0;; ++i) {
            const int sl = (hint + i) % kLiteralWaves;
            if (atomicCAS(&locks[sl], 0, 1) == 0) {
                slot = sl;
                break;
            }
        }
    slot = __shfl(slot, 0);
    __threadfence();
    return slot;
}
__device__ __forceinline__ void lit_release(int* locks, int slot) {
    __threadfence();
    if ((__lane_id()) == 0) atomicExch(&locks[slot], 0);
}

// returns the verdict | (polyline points walked << 4) | (their arc points << 34)
// The edge's steer_prep runs on the wave's eight 8-lane groups (prep_task: the word choice across
// a group's lanes, ~9 transcendental calls deep instead of ~32 on one lane), every group on the
// same edge; group 0 writes the record to the wave's LDS slot lrec, which walk_rec then walks.
// ONE out-of-line body for both call sites, reading the scene through a device-memory pointer
// (round 4): a reference to the kernel-argument SceneDev would copy the struct to the stack, and
// inlined at two sites (round 3) the kernel sat at 256 VGPRs with 608 B/lane of scratch and 571
// SGPR spills (the literal call's save area) — 2 waves per SIMD.
// the edge's prep and walk as separate bodies: each gets its own register allocation under the
// kernel's budget (one inlined body held both chains' values at once)
__device__ __noinline__ void cf_prep(const SceneDev* __restrict__ scg, double ax, double ay,
                                     double ayaw, double bx, double by, double byaw,
                                     PrepRec* lrec) {
    const int lane = __lane_id();
    prep_task(*scg, lane & 7, lane & ~7, 0, lane < 8, true, ax, ay, bx, by, byaw, 1, ayaw, 0,
              0.0, 0.0, lrec, nullptr, nullptr);
}
// (the walked point tallies go to the wave's LDS slot `tally`: reference out-parameters would
// live in the caller's stack frame, i.e. scratch)
__device__ __forceinline__ int cf_walk(const SceneDev* __restrict__ scg, const PrepRec* lrec,
                                    double* gs, bool junction, int* tally) {
    int w = 0, wa = 0;
    const int st = walk_rec<false, kSceneAny, true>(*scg, lrec, gs, w, wa, junction);
    if (__lane_id() == 0) {
        tally[0] = w;
        tally[1] = wa;
    }
    return st;
}
__device__ __forceinline__ long long cf_edge_check(const SceneDev* __restrict__ scg, double ax,
                                                double ay, double ayaw, double bx, double by,
                                                double byaw, int flags, double* lit_scratch,
                                                int* lit_locks, double* gs, PrepRec* lrec) {
    const SceneDev& sc = *scg;
    const bool junction = flags & 1, allow_none = flags & 2;
    cf_prep(scg, ax, ay, ayaw, bx, by, byaw, lrec);
    __builtin_amdgcn_wave_barrier();
    if (!allow_none && ufl(lrec->state) == kPrepNone) return kCfPanic;
    // (lrec's fb_seg / cnt[0] are dead once the walk started: its tallies come back there)
    int* tally = &lrec->cnt[0];
    int st = cf_walk(scg, lrec, gs, junction, tally);
    __builtin_amdgcn_wave_barrier();
    const long long walked = ufl(tally[0]), walked_arc = ufl(tally[1]);
    if (st == kLiteral) {  // (measure-zero) a scratch buffer from the pool, for this edge only
        const int slot = lit_acquire(lit_locks, (int)blockIdx.x);
        double* sx = lit_scratch + (size_t)slot * 3 * kLiteralCap;
        st = steer_collide_literal(sc, ax, ay, ayaw, bx, by, byaw, sx, sx + kLiteralCap,
                                   sx + 2 * kLiteralCap, junction);
        lit_release(lit_locks, slot);
    }
    return (long long)st | (walked << 4) | (walked_arc << 34);
}

// compute_yaw out of line: check_finish_kernel's own body is bookkeeping, and an inlined ocml
// atan2 (its polynomial constants hoisted out of the item loop) held ~100 VGPRs live across the
// edge calls
__device__ __noinline__ double cf_atan2(double y, double x) { return atan2(y, x); }

// n_point of dubins_path_planning(a → b) (dubins.rs:369), 0 when the steer is None; the chosen
// word in st
__device__ inline int cf_npoint_steer(const SceneDev& sc, CfPose a, CfPose b, Steer& st) {
    const double ex = b.x - a.x, ey = b.y - a.y;
    const double c = 1.0 / sc.turn_radius;
    const double lex = cos(a.yaw) * ex + sin(a.yaw) * ey;
    const double ley = -(sin(a.yaw)) * ex + cos(a.yaw) * ey;
    st = select_word(lex, ley, b.yaw - a.yaw, c);
    if (st.word < 0) return 0;
    double tot = 0.0;
    tot += st.t;
    tot += st.p;
    tot += st.q;
    const double nq = trunc(tot / sc.step_size);
    if (!(nq >= 0.0) || nq > 1.0e8) return -1;
    return (int)nq + 7;
}
__device__ inline int cf_npoint(const SceneDev& sc, CfPose a, CfPose b) {
    Steer st;
    return cf_npoint_steer(sc, a, b, st);
}

__device__ __noinline__ int cf_npoint_ool(const SceneDev* __restrict__ scg, CfPose a, CfPose b) {
    return cf_npoint(*scg, a, b);
}

// mode kCfCheck: check_finish of nodes[b] (the goal node Node::new_goal(goal, node, gyaw));
// kCfOptimize: optimize(nodes[b], level0) alone (ok_out: Some, chain_out: the chosen ancestors);
// kCfFinalize: finalize of the goal node (gx, gy, gyaw) with parent nodes[b] — the line is built
// whether it verifies or not (ok_out: it does).  optimize_from_goal gives the goal gyaw_opt when
// optimize succeeds (rrt.rs:489-501: the planner's goal yaw), else the goal node keeps gyaw.
// cb.qidx != nullptr (a query batch, pp_batch_plan): work item b is node nodes[b] of query
// qidx[b], whose tree is rows [q * row_cap, ...) of the SoA arrays and whose goal (both yaws) is
// goals[3q..3q+2]; its polygon-mode root block flag is blocked[q].
//
// Two launches.  check_finish_kernel: ONE WAVE PER NODE — the waves of a workgroup are
// independent (no barrier): each takes nodes from a launch-wide counter and runs optimize and
// finalize's verification edge by edge, in the reference's own order, so no edge is steered
// speculatively (the r02 form checked four candidates at a time across the workgroup's waves and
// discarded the ones past the first accept; it also held the workgroup at a barrier per round).
// A node whose line is wanted (a verified finish, or kCfFinalize) becomes a line item; the
// points and the length of the line items are cf_line_kernel's, one workgroup per item.
__device__ inline void cf_node_setup(const TreeDev& tr_in, const CfBatch& cb, int b,
                                     double gx_in, double gy_in, double gyaw_in,
                                     double gyaw_opt_in, int root_blocked_in, TreeDev& tr,
                                     double& gx, double& gy, double& gyaw, double& gyaw_opt,
                                     int& root_blocked, int** ftab = nullptr,
                                     int** gtab = nullptr) {
    tr = tr_in;
    if (ftab) *ftab = cb.ftab;
    if (gtab) *gtab = cb.gtab;
    gx = gx_in;
    gy = gy_in;
    gyaw = gyaw_in;
    gyaw_opt = gyaw_opt_in;
    root_blocked = root_blocked_in;
    if (cb.qidx) {
        const int q = cb.qidx[b];
        const size_t o = (size_t)q * cb.row_cap;
        tr.x += o;
        tr.y += o;
        tr.yaw += o;
        tr.parent += o;
        gx = cb.goals[3 * q];
        gy = cb.goals[3 * q + 1];
        gyaw = gyaw_opt = cb.goals[3 * q + 2];
        root_blocked = cb.blocked ? cb.blocked[q] : 0;
        // the memo rows are compact: query q's n_q nodes at mo(q) = its items before + q
        const size_t m = cb.moff ? (size_t)cb.moff[q] + q : o;
        if (ftab && *ftab) *ftab += m;
        if (gtab && *gtab) *gtab += m;
    }
}

// A node's ancestor path root first into path[0, D) (NodeIter, rrt.rs:253-265, reversed), by the
// calling wave (lane 0 follows the parents, then the lanes reverse it); -1 past kCfMaxDepth.
__device__ inline int cf_path(const TreeDev& tr, int node, int* __restrict__ path,
                              int cap = kCfMaxDepth) {
    const int lane = __lane_id();
    int d = 0;
    if (lane == 0) {
        int c = node;
        while (c >= 0 && d < cap) {
            path[d++] = c;
            c = tr.parent[c];
        }
        if (c >= 0) d = -1;
    }
    d = __shfl(d, 0);
    __builtin_amdgcn_wave_barrier();
    if (d > 0)
        for (int i = lane; i < d / 2; i += 64) {
            const int t = path[i];
            path[i] = path[d - 1 - i];
            path[d - 1 - i] = t;
        }
    __builtin_amdgcn_wave_barrier();
    return d;
}


__global__ __launch_bounds__(kCfThreads, kCfMinW) void check_finish_kernel(
    const SceneDev* __restrict__ scg, TreeDev tr_in, const int* __restrict__ nodes, int k, double gx_in, double gy_in,
    double gyaw_in, double gyaw_opt_in, int level0, int mode, int want_line,
    int* __restrict__ ok_out, double* __restrict__ len_out,
    int* __restrict__ npts_out, int* __restrict__ chain_out, double* __restrict__ lit_scratch,
    int* __restrict__ lit_locks, int* __restrict__ err, long long* __restrict__ tally, CfBatch cb,
    int* __restrict__ gpath, int* __restrict__ items, const int* __restrict__ blist) {
    __shared__ __attribute__((aligned(16))) double s_gs[kCfWaves][kGenSlots];  // walk_rec's LDS, one set per wave
    __shared__ int s_pos[kCfWaves][kCfLevels];  // the optimize chain's path positions per wave
    __shared__ PrepRec s_rec[kCfWaves];          // the wave's edge record (cf_edge_check)
    const SceneDev& sc = *scg;
    const int lane = __lane_id();
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    int* path = gpath + ((size_t)blockIdx.x * kCfWaves + wave) * kCfMaxDepth;  // this wave's
    double* gs = s_gs[wave];
    int* pos = s_pos[wave];
    PrepRec* lrec = &s_rec[wave];
    long long t_nodes = 0, t_edges = 0, t_pts = 0, t_arc = 0;  // this wave's work (profiling)
    for (;;) {
        // nodes one at a time from a launch-wide counter (err[1], zeroed with err): a node's
        // cost varies with its depth and how far optimize climbs
        int b = 0;
        if (lane == 0) b = atomicAdd(&err[1], 1);
        b = __builtin_amdgcn_readfirstlane(__shfl(b, 0));
        if (b >= k) break;
        if (blist) b = __builtin_amdgcn_readfirstlane(blist[b]);  // (a sub-list of the items)
        ++t_nodes;
        TreeDev tr;
        double gx, gy, gyaw, gyaw_opt;
        int root_blocked;
        int *ftab = nullptr, *gtab = nullptr;
        cf_node_setup(tr_in, cb, b, gx_in, gy_in, gyaw_in, gyaw_opt_in, sc.root_blocked, tr, gx,
                      gy, gyaw, gyaw_opt, root_blocked, &ftab, &gtab);
        const int D = cf_path(tr, nodes[b], path);
        if (D < 0) {
            if (lane == 0) {
                ok_out[b] = 0;
                atomicOr(err, 1);
            }
            continue;
        }
        // optimize (rrt.rs:463-487), level by level: candidates path[0..L] root first, the first
        // accepted one wins (kError before it: the reference's panic); RECURSION_LIMIT levels
        // The first verifying candidate of a tree node c (root first over c's ancestors and c)
        // depends on c alone — its ancestors' poses — not on the item whose chain reaches it, and
        // every item of a plan climbs through its ancestors' own levels: ftab memoises it
        // (cb.ftab; the value is the candidate's depth, which is its position in every path through
        // c).  Concurrent waves computing the same entry store the same value.
        int bad = 0;
        int L = D - 1, s_lv = 0;
        int fnone = 0;  // the last accepted candidate edge's steer was None (finalize panics)
        for (int level = 0; level < kCfLevels - level0; ++level) {
            const int Lstart = L;
            const int c = path[L];
            const int fm = ftab ? __builtin_amdgcn_readfirstlane(ftab[c]) : 0;
            int found = -1;
            if (fm >= 2) {
                found = fm & 0x3fffffff;
                found -= 2;
                fnone = fm >> 30;
            } else if (fm == 0) {
                const double ax = tr.x[c], ay = tr.y[c];
                for (int m = 0; m <= L && !root_blocked; ++m) {
                    const int to = path[m];
                    const CfPose bt{tr.x[to], tr.y[to], tr.yaw[to]};
                    const CfPose a{ax, ay, cf_atan2(bt.y - ay, bt.x - ax)};
                    const long long rv = cf_edge_check(scg, a.x, a.y, a.yaw, bt.x, bt.y, bt.yaw,
                                                       3, lit_scratch, lit_locks, gs, lrec);
                    const int st = (int)(rv & 15);
                    ++t_edges;
                    t_pts += (rv >> 4) & 0x3fffffff;
                    t_arc += rv >> 34;
                    if (st == kReject) continue;
                    found = st == kAccept ? m : -2;
                    fnone = lrec->state == kPrepNone ? 1 : 0;
                    break;
                }
                if (ftab && lane == 0 && found != -2)
                    ftab[c] = found >= 0 ? (2 + found) | (fnone << 30) : 1;
            }
            if (found == -2) {
                bad = 4;
                break;
            }
            if (found < 0) break;
            if (lane == 0) pos[level] = found;
            __builtin_amdgcn_wave_barrier();
            L = found;
            s_lv = level + 1;
            if (Lstart == 0) {
                // a level at the root tried its one candidate, the root copy (yaw atan2(0, 0))
                // into the root itself, and accepted it: every further level is the very same
                // edge with the same verdict — the chain of root copies
                // runs to the recursion limit
                if (lane == 0)
                    for (int l2 = level + 1; l2 < kCfLevels - level0; ++l2) pos[l2] = 0;
                __builtin_amdgcn_wave_barrier();
                s_lv = kCfLevels - level0;
                break;
            }
        }
        if (mode == kCfOptimize) {
            if (lane == 0) {
                ok_out[b] = (bad == 0 && s_lv > 0) ? 1 : 0;
                len_out[b] = 0.0;
                npts_out[b] = 0;
                if (bad) atomicOr(err, bad);
                if (chain_out) {
                    chain_out[(size_t)b * (kCfLevels + 2)] = s_lv;
                    chain_out[(size_t)b * (kCfLevels + 2) + 1] = 0;
                    for (int i = 0; i < s_lv; ++i)
                        chain_out[(size_t)b * (kCfLevels + 2) + 2 + i] = path[pos[i]];
                }
            }
            continue;
        }
        // finalize (rrt.rs:503-540): the chain goal -> optimised copies -> tree path -> root,
        // every edge verified with its junction chord, the edge into the root without one
        const int s = s_lv;
        const double gyaw_e = s > 0 ? gyaw_opt : gyaw;  // optimize_from_goal (rrt.rs:489-501)
        const int ps = s > 0 ? pos[s - 1] : D - 1;
        const int E = 1 + s + ps;
        bool vok = bad == 0;
        // pose j of the chain (cf_pose's indexing, the chain positions in registers)
        auto pose = [&](int j) -> CfPose {
            if (j == 0) return CfPose{gx, gy, gyaw_e};
            if (j <= s) {
                const int i = j - 1;
                const int here = path[i == 0 ? D - 1 : pos[i - 1]];
                const int to = path[pos[i]];
                const double x = tr.x[here], y = tr.y[here];
                return CfPose{x, y, cf_atan2(tr.y[to] - y, tr.x[to] - x)};  // Node::new (compute_yaw)
            }
            const int node = path[ps - (j - s - 1)];
            return CfPose{tr.x[node], tr.y[node], tr.yaw[node]};
        };
        // Only the goal edge and the s copy edges are steered: edges s + 1 .. E - 1 are tree edges
        // (node -> parent, both with their stored poses) whose polyline with its junction chord
        // passed verify when the node was inserted (verify_node, rrt.rs:414-426: the incremental
        // form, §2), and the edge into the root is checked without its chord, a subset.  Both
        // Contains and Intersects decompose over the concatenation, so those edges cannot change
        // the verdict (tests: every check_finish verdict equals the oracle's full-line verify).
        // Edge s (the last copy into the tree node optimize's last level accepted) is that
        // level's candidate edge: it verified with its junction chord (without the chord, into
        // the root, a subset), so only its None steer matters (finalize's panic; fnone).  Copy
        // edge e in 1..s-1 runs from the copy at chain node v = path[pos[e - 2]] (the item's node
        // for e = 1) toward F(v) to the copy at F(v) toward F(F(v)): a function of v alone, so
        // gtab memoises its verdict like ftab.
        const int Ev = 1 + s;
        if (vok) {
            CfPose prev{0.0, 0.0, 0.0}, a = pose(0);
            int prev_st = kAccept;
            for (int e = 0; e < Ev; ++e) {
                const CfPose bp = pose(e + 1);
                // an edge identical to the previous one (consecutive root copies: both poses
                // equal bit for bit, both with the junction) has that edge's verdict
                const bool dup = e >= 1 && e < E - 1 && same_pose(prev, a) && same_pose(a, bp);
                const int gv = (e >= 1 && e < s) ? path[e == 1 ? D - 1 : pos[e - 2]] : -1;
                // the goal edge's verdict from the batch plan's steer round (cb.gotab), the copy
                // edges' from gtab
                const int gm = (e == 0 && cb.gotab)
                                   ? __builtin_amdgcn_readfirstlane(cb.gotab[b])
                                   : ((gtab && gv >= 0) ? __builtin_amdgcn_readfirstlane(gtab[gv]) : 0);
                int st = prev_st;
                if (e >= 1 && e == s) {
                    st = fnone ? kCfPanic : kAccept;
                } else if (gm > 0) {
                    st = gm - 1;
                } else if (!dup) {
                    const long long rv = cf_edge_check(scg, a.x, a.y, a.yaw, bp.x, bp.y, bp.yaw,
                                                       e < E - 1 ? 1 : 0, lit_scratch, lit_locks,
                                                       gs, lrec);
                    st = (int)(rv & 15);
                    ++t_edges;
                    t_pts += (rv >> 4) & 0x3fffffff;
                    t_arc += rv >> 34;
                    if (gtab && gv >= 0 && lane == 0) gtab[gv] = st + 1;
                }
                if (st != kAccept) {
                    if (st == kCfPanic) bad = 2;
                    else if (st == kError) bad = 4;
                    vok = false;
                    break;
                }
                prev = a;
                a = bp;
                prev_st = st;
            }
        }
        // polygon mode: the chain's line is connected and no segment met an edge buffer, so it
        // lies on one side of every obstacle boundary — the goal decides (Q10p)
        if (vok && sc.ne > 0 && in_obstacle(sc.ne, sc.ex0, sc.ey0, sc.ex1, sc.ey1, sc.epoly, gx, gy))
            vok = false;
        // a panic anywhere in finalize wins over a rejection (the reference builds the whole line
        // before it verifies): the other edges' steers, lane-parallel.  A verified chain also
        // scans its tree edges s + 1 .. E - 1, which were not steered above: insertion accepts a
        // None steer as the straight polyline (rrt.rs:313), finalize panics on it (rrt.rs:529).
        // (None needs a non-finite pose — LSL's and RSR's p² differ only in the sign of one
        // term, so one of them is >= 0 — e.g. a NaN start yaw; only finishes pay the scan.)
        if (bad == 0 && (!vok || E > Ev)) {
            bool none = false;
            for (int e = (vok ? Ev : 0) + lane; e < E; e += 64)
                if (cf_npoint_ool(scg, pose(e), pose(e + 1)) == 0) none = true;
            if (__any(none)) bad = 2;
        }
        if ((vok || mode == kCfFinalize) && bad == 0 && want_line) {
            // the line's points and length: a cf_line_kernel item
            if (lane == 0) {
                const int it = atomicAdd(&items[0], 1);
                int* o = items + 1 + (size_t)it * kCfItem;
                o[0] = b;
                o[1] = s;
                o[2] = vok ? 1 : 0;
                o[3] = 0;
                for (int i = 0; i < kCfLevels; ++i) o[4 + i] = i < s ? pos[i] : 0;
            }
        } else if (lane == 0) {
            ok_out[b] = (vok && bad == 0) ? 1 : 0;
            len_out[b] = 0.0;
            npts_out[b] = 0;
            if (bad) atomicOr(err, bad);
        }
        if (lane == 0 && chain_out) {
            chain_out[(size_t)b * (kCfLevels + 2)] = s;
            chain_out[(size_t)b * (kCfLevels + 2) + 1] = E;
            for (int i = 0; i < s; ++i)
                chain_out[(size_t)b * (kCfLevels + 2) + 2 + i] = path[pos[i]];
        }
    }
    if (tally && lane == 0) {  // profiling: nodes, edges, points
        unsigned long long* tl = reinterpret_cast<unsigned long long*>(tally);
        atomicAdd(&tl[0], (unsigned long long)t_nodes);
        atomicAdd(&tl[1], (unsigned long long)t_edges);
        atomicAdd(&tl[2], (unsigned long long)t_pts);
        atomicAdd(&tl[3], (unsigned long long)t_arc);
    }
}

// cf_line_kernel's workgroup: one wave per line item.  An item's path walk and its ordered length
// sum are serial, so a 4-wave workgroup left 3 waves waiting at its barriers; one wave per item
// puts 4x the items in flight at the same occupancy
constexpr int kCfLineThreads = 64;
static_assert(kCfLineThreads == 64, "cf_line_kernel: one wave per item (its edge table and sums are wave-wide)");
#ifdef PP_LINE_TIMING  // diagnostic builds only: phase stamps of cf_line_kernel's items
#define LT(k) const unsigned long long lt##k = wall_clock64();
#else
#define LT(k)
#endif

// dubins_literal<false, false> (dubins.rs:326-428) of one edge by one wave: the WORLD points of
// the trimmed course into px / py (cap >= n_point), *n_out = their count.  generate_local_course
// (dubins.rs:200-272) writes the origin at index 0, each segment's grid points from the slot of
// the previous segment's end on (that end is overwritten), and the last segment's end after its
// grid points; the rest of the n_point slots stay 0.0.  The grid values of a segment are the
// serial chain pd, pd + d, ... (every lane runs the uniform chain and keeps its own term, the
// same rounding sequence), 64 per pass; each lane interpolates its point (dubins.rs:155-198) and
// moves it to the world frame (dubins.rs:412-422).  The trim (dubins.rs:281-288) keeps the
// indices below the last one whose local x is nonzero (none: 0), or all n_point when the last
// slot is written and nonzero.  Returns kSteerSome / kSteerNone / kSteerOverflow like the
// literal restatement.
__device__ int line_edge_wave(double sx, double sy, double syaw, const double* __restrict__ word,
                              double turn_radius, double step_size, double* px, double* py,
                              int cap, int lane, int* n_out) {
    // the word (dubins.rs:333-363) as cf_npoint_steer chose it for this edge: {word, t, p, q}
    const double c = 1.0 / turn_radius;
    const double rc = 1.0 / c;
    Steer s;
    s.word = (int)word[0];
    s.t = word[1];
    s.p = word[2];
    s.q = word[3];
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
    // every sin / cos the edge needs in one lane-parallel round (the same calls on the same
    // arguments as interp_local and the world transform make, so the same values): lanes 0..2 the
    // segment origins' yaw trig (S: cos / sin of the yaw; L, R: of minus the yaw), 3..5 sin / cos
    // of the segment lengths (their end points), 6 the world transform's cos / sin(-syaw)
    const int m0 = word_mode(s.word, 0), m1 = word_mode(s.word, 1), m2 = word_mode(s.word, 2);
    const double oy0 = 0.0;  // interpolate's yaw chain, dubins.rs:191-196
    const double oy1 = m0 == kModeL ? oy0 + s.t : (m0 == kModeR ? oy0 - s.t : oy0);
    const double oy2 = m1 == kModeL ? oy1 + s.p : (m1 == kModeR ? oy1 - s.p : oy1);
    double arg = 0.0;
    if (lane < 3) {
        const int ms = lane == 0 ? m0 : (lane == 1 ? m1 : m2);
        const double oys = lane == 0 ? oy0 : (lane == 1 ? oy1 : oy2);
        arg = ms == kModeS ? oys : -oys;
    } else if (lane < 6) {
        arg = lane == 3 ? s.t : (lane == 4 ? s.p : s.q);
    } else if (lane == 6) {
        arg = -syaw;
    }
    const double sv = sin(arg), cv = cos(arg);
    const double cs = readlane_f64(cv, 6), sn = readlane_f64(sv, 6);
    if (lane == 0) {  // the origin, index 0
        px[0] = cs * 0.0 + sn * 0.0 + sx;
        py[0] = -sn * 0.0 + cs * 0.0 + sy;
    }
    int ind = 0;      // the last index written
    int lastnz = -1;  // the last index whose local x is nonzero
    double lastx = 0.0;
    Pose o{0.0, 0.0, 0.0};
    double ll = 0.0;
    for (int i = 0; i < 3; ++i) {
        const int m = word_mode(s.word, i);
        const double l = lengths[i];
        const double d = (l > 0.0) ? step_size : -step_size;
        // interp_local's trig of the segment's origin yaw (per point in the serial form, the same
        // values): S cos / sin(yaw), L / R cos / sin(-yaw)
        const double ca = readlane_f64(cv, i), sa = readlane_f64(sv, i);
        const double co = ca, so = sa, cmo = ca, smo = sa;
        const double al = fabs(l);
        double pd = (i >= 1 && (lengths[i - 1] * lengths[i]) > 0.0) ? (-d - ll) : (d - ll);
        int base = i == 0 ? 1 : ind;  // the slot of this segment's first grid point
        ind = base - 1;               // (dubins.rs:227: ind -= 1)
        for (;;) {
            double my = 0.0, w = pd;
            // walk_rec's closed form first: while the values keep pd's sign and exponent,
            // fl(w + d) = w + delta exactly (delta = w1 - pd, when the first two steps agree), so
            // lane k's value is one exact fma; checked over every value up to the first one past
            // |l| (the one the segment end needs).  Otherwise the serial chain.
            const double w1 = pd + d, w2 = w1 + d;
            bool cf = (w1 - pd) == (w2 - w1);
            if (cf) {
                const double vc = __builtin_fma((double)lane, w1 - pd, pd);
                const uint64_t fm = __ballot(!(fabs(vc) <= al));
                const int fl = fm ? (int)__builtin_ctzll(fm) : 63;
                cf = __ballot(lane <= fl && (__double2hiint(vc) >> 20) != (__double2hiint(pd) >> 20)) == 0;
                if (cf) {
                    my = vc;
                    w = readlane_f64(vc, 63) + d;
                }
            }
            if (!cf) {
                for (int u = 0; u < 64; ++u) {
                    if (lane == u) my = w;
                    w += d;
                }
            }
            const uint64_t bad = __ballot(!(fabs(my) <= al));
            const int cnt = bad ? (int)__builtin_ctzll(bad) : 64;
            if (cnt > 0 && base + cnt - 1 >= n_point) return kSteerOverflow;
            if (lane < cnt) {
                // (x / c as div_by: the correctly rounded quotient, bit-identical to the division)
                double lx, ly;
                if (m == kModeS) {
                    lx = o.x + div_by(my, c, rc) * co;
                    ly = o.y + div_by(my, c, rc) * so;
                } else {
                    const double ldx = div_by(sin(my), c, rc);
                    const double l1 = div_by(1.0 - cos(my), c, rc);
                    const double ldy = m == kModeL ? l1 : -l1;
                    lx = o.x + (cmo * ldx + smo * ldy);
                    ly = o.y + (-smo * ldx + cmo * ldy);
                }
                px[base + lane] = cs * lx + sn * ly + sx;
                py[base + lane] = -sn * lx + cs * ly + sy;
                const uint64_t nz = __ballot(lx != 0.0);
                if (nz) lastnz = base + 63 - (int)__builtin_clzll(nz);
                lastx = lx;
            }
            if (cnt > 0) {
                ind = base + cnt - 1;
                lastx = readlane_f64(lastx, cnt - 1);
            }
            if (cnt < 64) {
                ll = l - readlane_f64(my, cnt) - d;
                break;
            }
            base += 64;
            pd = w;
        }
        // the segment's end (dubins.rs:262-267) at the next slot; the next segment starts there
        ind += 1;
        if (ind >= n_point) return kSteerOverflow;
        // interp_local(m, l, c, o) with the round's values
        Pose r;
        if (m == kModeS) {
            r.x = o.x + l / c * co;
            r.y = o.y + l / c * so;
        } else {
            const double sl = readlane_f64(sv, 3 + i), cl = readlane_f64(cv, 3 + i);
            const double ldx = sl / c;
            const double ldy = m == kModeL ? (1.0 - cl) / c : (1.0 - cl) / -c;
            r.x = o.x + (cmo * ldx + smo * ldy);
            r.y = o.y + (-smo * ldx + cmo * ldy);
        }
        r.yaw = 0.0;  // (the next segment's trig comes from the round)
        if (i == 2) {
            if (lane == 0) {
                px[ind] = cs * r.x + sn * r.y + sx;
                py[ind] = -sn * r.x + cs * r.y + sy;
            }
            if (r.x != 0.0) lastnz = ind;
            lastx = r.x;
        }
        o = r;
    }
    // the trim: every trailing 0.0 (the unwritten slots) and one more element
    *n_out = (ind == n_point - 1 && lastx != 0.0) ? n_point : (lastnz > 0 ? lastnz : 0);
    return kSteerSome;
}

// The lines of check_finish_kernel's line items: workgroup w takes items w, w + grid, ... (item
// i < grid: the workgroup-i buffers, so a one-node call's line is in workgroup 0's); every
// edge's literal Dubins points (line_edge_wave, a wave per edge) into the workgroup's pts / etab,
// then l.reverse() and geo's euclidean_length in that order (rrt.rs:538: the hypots in parallel,
// their sum in line order).
// a line item past tier 1's capacities onto the spill list (all 64 lanes of the item's wave)
// (past the list's capacity: the point-capacity error)
__device__ inline void cf_spill(const CfLineBufs& lb, const int* __restrict__ o, int tid,
                                int* __restrict__ err) {
    int w = 0;
    if (tid == 0) w = atomicAdd(&lb.spill[0], 1);
    w = __shfl(w, 0);
    if (w >= lb.spill_cap) {
        if (tid == 0) atomicOr(err, 8);
    } else if (tid < kCfItem) {
        lb.spill[1 + (size_t)w * kCfItem + tid] = o[tid];
    }
}

__global__ __launch_bounds__(kCfLineThreads) void cf_line_kernel(
    SceneDev sc, TreeDev tr_in, const int* __restrict__ nodes, double gx_in, double gy_in,
    double gyaw_in, double gyaw_opt_in, int* __restrict__ ok_out, double* __restrict__ len_out,
    int* __restrict__ npts_out, CfLineBufs lb, int* __restrict__ err, CfBatch cb,
    const int* __restrict__ items) {
    __shared__ int s_off, s_bad;
    __shared__ int s_pos[kCfLevels];
    const int tid = threadIdx.x;
    // this workgroup's buffers: points (x, y, hypots / words), edge table, ancestor path
    const int pts_cap = lb.pts_cap;
    double* px = lb.pts + (size_t)blockIdx.x * 3 * pts_cap;
    double* py = px + pts_cap;
    double* pyw = py + pts_cap;
    int* et = lb.etab + (size_t)blockIdx.x * 2 * (lb.path_cap + kCfLevels + 1);
    int* path = lb.path + (size_t)blockIdx.x * lb.path_cap;
    const int n_items = items[0];
    for (int it = blockIdx.x; it < n_items; it += gridDim.x) {
        const int* o = items + 1 + (size_t)it * kCfItem;
        const int b = o[0], s = o[1], vok = o[2];
        LT(0)
        if (tid < kCfLevels) s_pos[tid] = o[4 + tid];
        const int* pos = s_pos;
        TreeDev tr;
        double gx, gy, gyaw, gyaw_opt;
        int root_blocked;
        cf_node_setup(tr_in, cb, b, gx_in, gy_in, gyaw_in, gyaw_opt_in, sc.root_blocked, tr, gx,
                      gy, gyaw, gyaw_opt, root_blocked);
        int D = 0;
        if (tid < 64) D = cf_path(tr, nodes[b], path, lb.path_cap);
        if (tid == 0) s_off = D;
        __syncthreads();
        D = s_off;
        // tier 1: a path deeper than this tier's capacity goes to tier 2 (the spill list); at the
        // full capacity it is check_finish_kernel's depth error
        if (D < 0) {
            if (lb.spill) {
                cf_spill(lb, o, tid, err);
            } else if (tid == 0) {
                ok_out[b] = 0;
                atomicOr(err, 1);
            }
            __syncthreads();
            continue;
        }
        LT(1)
        const double gyaw_e = s > 0 ? gyaw_opt : gyaw;
        const int ps = s > 0 ? pos[s - 1] : D - 1;
        const int E = 1 + s + ps;
        auto pose = [&](int j) -> CfPose {
            if (j == 0) return CfPose{gx, gy, gyaw_e};
            if (j <= s) {
                const int i = j - 1;
                const int here = path[i == 0 ? D - 1 : pos[i - 1]];
                const int to = path[pos[i]];
                const double x = tr.x[here], y = tr.y[here];
                return CfPose{x, y, atan2(tr.y[to] - y, tr.x[to] - x)};
            }
            const int node = path[ps - (j - s - 1)];
            return CfPose{tr.x[node], tr.y[node], tr.yaw[node]};
        };
        if (tid == 0) s_bad = 0;
        // every edge's word and point count, a lane per edge; the words wait in the hypot buffer
        // (4 doubles an edge, 4 kCfMaxEdges <= pts_cap) for the generation below
        for (int e = tid; e < E; e += kCfLineThreads) {
            Steer w;
            et[2 * e] = cf_npoint_steer(sc, pose(e), pose(e + 1), w);
            double* wd = pyw + 4 * (size_t)e;
            wd[0] = (double)w.word;
            wd[1] = w.t;
            wd[2] = w.p;
            wd[3] = w.q;
        }
        __syncthreads();
        if (tid == 0) {  // edge capacities -> offsets
            int off = 0;
            bool none = false, neg = false;
            for (int e = 0; e < E; ++e) {
                const int c = et[2 * e];
                none |= c == 0;
                neg |= c < 0;
                et[2 * e] = off;
                off += c > 0 ? c : 0;
            }
            // a None steer is finalize's panic (rrt.rs:529); an overflowing count or a line
            // past the point capacity is the capacity error — in tier 1, a line longer than the
            // tier's capacity goes to tier 2 (-3)
            s_off = none ? -2 : neg ? -1 : off <= pts_cap ? off : lb.spill ? -3 : -1;
        }
        __syncthreads();
        const int total = s_off;
        LT(2)
        if (total == -3) {  // spilled: tier 2 writes this item's outputs
            cf_spill(lb, o, tid, err);
            __syncthreads();
            continue;
        }
        if (total < 0) {
            if (tid == 0) s_bad = total == -2 ? 2 : 8;
        } else {
            const int lane = tid & 63;
            for (int e = tid >> 6; e < E; e += kCfLineThreads / 64) {
                const int off = et[2 * e];
                const int cap = (e + 1 < E ? et[2 * e + 2] : total) - off;
                const CfPose a = pose(e);
                int n = 0;
                const int r = line_edge_wave(a.x, a.y, a.yaw, pyw + 4 * (size_t)e, sc.turn_radius,
                                             sc.step_size, px + off, py + off, cap, lane, &n);
                if (lane == 0) {
                    et[2 * e + 1] = r == kSteerSome ? n : 0;
                    // a None steer is finalize's panic (rrt.rs:529); an n_point overflow is the
                    // steer-overflow error (round 5 reported both as the panic)
                    if (r == kSteerNone) atomicOr(&s_bad, 2);
                    else if (r != kSteerSome) atomicOr(&s_bad, 4);
                }
            }
        }
        __syncthreads();
        // l.reverse() (rrt.rs:538), then euclidean_length in that order: the line's points in
        // forward order f = 0 .. np - 1 (edge by edge), the reversed line's k-th segment is
        // (f + 1 -> f) for f = np - 2 down to 0.  Every segment's hypot in parallel (into the
        // yaw buffer, by forward index), then one lane adds them in the reversed order — the
        // same operands, the same order of the sum
        const int bad0 = s_bad;
        LT(3)
        int npts_all = 0;
        if (bad0 == 0 && E <= 64) {
            // (one wave, at most 64 edges: the edge table in registers — lane e holds edge e's
            // offset, count, compact base and the offset of the next edge with points — so the
            // loop over the edges waits on no table load)
            const int eoff = tid < E ? et[2 * tid] : 0, en = tid < E ? et[2 * tid + 1] : 0;
            const uint64_t ne = __ballot(en > 0);
            const uint64_t above = tid >= 63 ? 0ull : (ne & (~0ull << (tid + 1)));
            const int nxl = above ? (int)__builtin_ctzll(above) : 0;
            const int nxo = __shfl(eoff, nxl);
            const int nx = above ? nxo : -1;
            const int incl = wave_incl_scan(en);
            const int cbv = incl - en;
            npts_all = __builtin_amdgcn_readlane(incl, 63);
            for (int e = 0; e < E; ++e) {
                const int off = __builtin_amdgcn_readlane(eoff, e);
                const int n = __builtin_amdgcn_readlane(en, e);
                const int cb = __builtin_amdgcn_readlane(cbv, e);
                const int nxe = __builtin_amdgcn_readlane(nx, e);
                for (int i = tid; i < n; i += kCfLineThreads) {
                    const int noff = i + 1 < n ? off + i + 1 : nxe;
                    if (noff >= 0)
                        pyw[cb + i] = hypot(px[off + i] - px[noff], py[off + i] - py[noff]);
                }
            }
        } else if (bad0 == 0) {
            int cb = 0;
            for (int e = 0; e < E; ++e) {
                const int off = et[2 * e], n = et[2 * e + 1];
                for (int i = tid; i < n; i += kCfLineThreads) {
                    int noff = -1;
                    if (i + 1 < n) {
                        noff = off + i + 1;
                    } else {
                        for (int e2 = e + 1; e2 < E; ++e2)
                            if (et[2 * e2 + 1] > 0) {
                                noff = et[2 * e2];
                                break;
                            }
                    }
                    if (noff >= 0)
                        pyw[cb + i] = hypot(px[off + i] - px[noff], py[off + i] - py[noff]);
                }
                cb += n;
            }
            npts_all = cb;
        }
        __syncthreads();
        LT(4)
        if (tid < 64) {
            // the reversed sum, wave 0: 64 hypots a load (lane j holds pyw[hi - j], the next
            // chunk's load in flight), added in lane order by readlane — the serial order
            double len = 0.0;
            int npts = 0;
            const int bad = s_bad;
            if (bad == 0) {
                npts = npts_all;
                int hi = npts - 2;
                double v = hi - tid >= 0 ? pyw[hi - tid] : 0.0;
                for (; hi >= 0; hi -= 64) {
                    const double cur = v;
                    v = hi - 64 - tid >= 0 ? pyw[hi - 64 - tid] : 0.0;
                    if (hi >= 63) {  // a full chunk: constant lane indices
#pragma unroll
                        for (int j = 0; j < 64; ++j) len += readlane_f64(cur, j);
                    } else {
                        for (int j = 0; j <= hi; ++j) len += readlane_f64(cur, j);
                    }
                }
            }
            if (tid == 0) {
                ok_out[b] = (vok && bad == 0) ? 1 : 0;
                len_out[b] = bad == 0 ? len : 0.0;
                npts_out[b] = bad == 0 ? npts : 0;
                if (bad) atomicOr(err, bad);
            }
        }
        __syncthreads();  // the buffers and s_off serve the next item
#ifdef PP_LINE_TIMING
        {
            LT(5)
            if (tid == 0 && it % 97 == 0)
                printf("LT it %d D %d E %d path %llu cnt %llu gen %llu hyp %llu sum %llu\n", it, D, E,
                       lt1 - lt0, lt2 - lt1, lt3 - lt2, lt4 - lt3, lt5 - lt4);
        }
#endif
    }
}

hipError_t launch_check_finish(hipStream_t st, const SceneDev& sc, const SceneDev* scg,
                               const TreeDev& tr,
                               const int* nodes, int k, double gx, double gy, double gyaw,
                               double gyaw_opt, int level0, int mode, int want_line, int* ok,
                               double* len, int* npts, int* chain, double* lit_scratch,
                               int* lit_locks, const CfLines& lines, int* err, int grid,
                               long long* tally, const CfBatch& cb, int* gpath, int* items,
                               const int* blist) {
    if (k <= 0 && lines.grid1 <= 0) return hipSuccess;
    const int wgs = std::min(grid, (k + kCfWaves - 1) / kCfWaves);
    if (k > 0)
        check_finish_kernel<<<wgs, kCfThreads, 0, st>>>(scg, tr, nodes, k, gx, gy, gyaw, gyaw_opt,
                                                        level0, mode, want_line, ok, len, npts,
                                                        chain, lit_scratch, lit_locks, err, tally,
                                                        cb, gpath, items, blist);
    if (want_line && mode != kCfOptimize && lines.grid1 > 0) {
        cf_line_kernel<<<lines.grid1, kCfLineThreads, 0, st>>>(sc, tr, nodes, gx, gy, gyaw,
                                                               gyaw_opt, ok, len, npts, lines.t1,
                                                               err, cb, items);
        if (lines.t1.spill)  // the lines past tier 1's capacities, at the full ones
            cf_line_kernel<<<lines.grid2, kCfLineThreads, 0, st>>>(sc, tr, nodes, gx, gy, gyaw,
                                                                   gyaw_opt, ok, len, npts,
                                                                   lines.t2, err, cb,
                                                                   lines.t1.spill);
    }
    return hipGetLastError();
}

// ------------------------------------------------------------ RRT::plan of a query batch
//
// pp_batch_plan: check_finish (rrt.rs:428-438) of every accepted node of every query — nodes
// 1 .. n_q - 1 in insertion (= iteration) order, rrt.rs:591 — by check_finish_kernel over the
// flattened (query, node) items, then per query the first minimum euclidean_length
// (rrt.rs:607-617).  Items of query q are [off[q], off[q + 1]), node = 1 + (b - off[q]).
__global__ __launch_bounds__(256) void mq_plan_items_kernel(int Q, const int* __restrict__ off,
                                                            int* __restrict__ qidx,
                                                            int* __restrict__ nodes) {
    const int lane = __lane_id();
    const int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int nw = (int)((gridDim.x * blockDim.x) >> 6);
    for (int q = gw; q < Q; q += nw) {
        const int a = off[q], e = off[q + 1];
        for (int b = a + lane; b < e; b += 64) {
            qidx[b] = q;
            nodes[b] = 1 + (b - a);
        }
    }
}

__global__ __launch_bounds__(256) void mq_plan_reduce_kernel(
    int Q, const int* __restrict__ off, const int* __restrict__ ok, const double* __restrict__ len,
    const int* __restrict__ npts, int* __restrict__ best_node, double* __restrict__ best_len,
    int* __restrict__ best_npts, int* __restrict__ n_fin) {
    const int lane = __lane_id();
    const int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int nw = (int)((gridDim.x * blockDim.x) >> 6);
    for (int q = gw; q < Q; q += nw) {
        const int a = off[q], e = off[q + 1];
        double bd = __builtin_inf();
        int bi = 0x7fffffff, cnt = 0;
        for (int b = a + lane; b < e; b += 64) {
            if (!ok[b]) continue;
            ++cnt;
            argmin_pair(bd, bi, len[b], b);  // first minimum: the lowest item on ties
        }
        wave_argmin(bd, bi);
        for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
        if (lane == 0) {
            const bool any = bi != 0x7fffffff;
            best_node[q] = any ? 1 + (bi - a) : -1;
            best_len[q] = any ? bd : __builtin_inf();
            best_npts[q] = any ? npts[bi] : 0;
            n_fin[q] = cnt;
        }
    }
}

hipError_t launch_mq_plan_items(hipStream_t s, int Q, const int* off, int* qidx, int* nodes) {
    mq_plan_items_kernel<<<std::min((Q + 3) / 4, 4096), 256, 0, s>>>(Q, off, qidx, nodes);
    return hipGetLastError();
}

hipError_t launch_mq_plan_reduce(hipStream_t s, int Q, const int* off, const int* ok,
                                 const double* len, const int* npts, int* best_node,
                                 double* best_len, int* best_npts, int* n_fin) {
    mq_plan_reduce_kernel<<<std::min((Q + 3) / 4, 4096), 256, 0, s>>>(
        Q, off, ok, len, npts, best_node, best_len, best_npts, n_fin);
    return hipGetLastError();
}

// --------------------------------- check_finish of a query batch in steer rounds (round 4)
//
// check_finish_kernel runs every item's edges one after the other on one wave, at 2 waves per
// SIMD (its register budget): a latency chain.  For a batch plan, every edge whose verdict
// depends on one tree node or one item is steered up front instead, by the query batch's own
// steer_prep / steer_walk at their occupancy, and written to the memo tables the kernel already
// reads (CfBatch::ftab / gtab, and gotab: the goal edge of each item):
//   phase A  ftab of every node (optimize's level for node c: the first of c's ancestors, root
//            first, and c itself whose edge verifies, rrt.rs:463-487): rounds of kCfbSpan
//            candidates per open node, in order; a node settles at its first verdict that is
//            not a rejection (a literal-path or error verdict leaves ftab unknown);
//   phase B  each item's chain follows ftab; its goal edge (Node::new_goal, rrt.rs:430-436,
//            the goal keeping its own yaw) and its copy edges (one per chain node v, claimed by
//            the first item that reaches v) are steered in one round: gotab / gtab;
//   assemble one lane per item: the chain, the verdicts in finalize's order, the panic scan from
//            the None flags (a None steer is a panic status in the memo; the tree edges' flags
//            are tnone_up), the outputs or a line item.  An item with any unknown verdict goes
//            to a list that check_finish_kernel runs as before (with every memo entry there).
// Results are those of check_finish_kernel: the same edges, the same verdicts, the same order
// of precedence (a panic anywhere wins over a rejection; verify decides the rest).

// phase A node list: b < nitems is item b (qidx[b], nodes[b]); b - nitems < Q is query's root
// query q's first memo row: the memo tables are compact, q's n_q nodes after the nodes of the
// queries before it (their items plus their roots)
__device__ inline size_t cfb_memo_row(const CfbArgs& a, int q) {
    return (size_t)a.moff[q] + q;
}

__device__ inline void cfb_node(const CfbArgs& a, int b, int& q, int& c) {
    if (b < a.nitems) {
        q = a.qidx[b];
        c = a.nodes[b];
    } else {
        q = b - a.nitems;
        c = 0;
    }
}

// depth of every phase-A node, its own tree edge's None flag (the steer from its pose to its
// parent's, rrt.rs:313 / 529), and the open state; maxdepth for the host
__global__ __launch_bounds__(256) void cfb_depth_kernel(CfbArgs a, SceneDev sc) {
    // (the depth histogram per workgroup in LDS, then one atomic per nonzero bin: the host bounds
    // each steer round's task count by it)
    __shared__ int s_h[kCfbDepthBins];
    if (threadIdx.x < kCfbDepthBins) s_h[threadIdx.x] = 0;
    __syncthreads();
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = b < a.nitems + a.Q;
    if (in) {
        int q0, c0;
        cfb_node(a, b, q0, c0);
        const size_t o0 = (size_t)q0 * a.row_cap;
        int d0 = 0;
        for (int k = c0; a.tr.parent[o0 + k] >= 0; k = a.tr.parent[o0 + k]) ++d0;
        atomicAdd(&s_h[min(d0, kCfbDepthBins - 1)], 1);
        a.depth[b] = d0;
    }
    __syncthreads();
    if (a.dhist && threadIdx.x < kCfbDepthBins && s_h[threadIdx.x])
        atomicAdd(&a.dhist[threadIdx.x], s_h[threadIdx.x]);
    if (!in) return;
    int q, c;
    cfb_node(a, b, q, c);
    const size_t o = (size_t)q * a.row_cap;
    const int d = a.depth[b];
    a.open[b] = 1;
    atomicMax(a.maxdepth, d);
    int none = 0;
    if (c > 0) {
        const int p = a.tr.parent[o + c];
        const CfPose from{a.tr.x[o + c], a.tr.y[o + c], a.tr.yaw[o + c]};
        const CfPose to{a.tr.x[o + p], a.tr.y[o + p], a.tr.yaw[o + p]};
        none = cf_npoint(sc, from, to) == 0 ? 1 : 0;
    }
    a.tnone[cfb_memo_row(a, q) + c] = (unsigned char)none;
}

// tnone_up[c]: any tree edge from c down to the root has a None steer
__global__ __launch_bounds__(256) void cfb_tnone_up_kernel(CfbArgs a) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= a.nitems + a.Q) return;
    int q, c;
    cfb_node(a, b, q, c);
    const size_t o = (size_t)q * a.row_cap;
    int any = 0;
    const size_t m = cfb_memo_row(a, q);
    for (int k = c; k > 0; k = a.tr.parent[o + k]) any |= a.tnone[m + k];
    a.tnone_up[m + c] = (unsigned char)any;
}

// a thread's task count -> its first task index: one atomic per 256-thread workgroup on the
// round's counter (per wave, ~9k waves contending for one address cost ~0.2 ms a round).  Every
// thread of the workgroup must call it.
__device__ inline int cfb_reserve(int* counter, int cnt, int* wsum) {
    __shared__ int s_wt[4], s_base;
    const int lane = __lane_id(), w = threadIdx.x >> 6;
    const int incl = wave_incl_scan(cnt);
    if (lane == 63) s_wt[w] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int tot = s_wt[0] + s_wt[1] + s_wt[2] + s_wt[3];
        s_base = tot ? atomicAdd(counter, tot) : 0;
        if (wsum && tot) atomicAdd(wsum, tot);
    }
    __syncthreads();
    int wb = s_base;
    for (int k = 0; k < w; ++k) wb += s_wt[k];
    return wb + incl - cnt;
}

// phase A round r: the next `span` candidates (depth m0 .. m0 + span - 1, root first) of every open
// node, as explicit (child, parent pose) tasks: child = the node's position (compute_yaw toward
// the candidate, as Node::new does), parent = the candidate's stored pose
__global__ __launch_bounds__(256) void cfb_emit_a_kernel(CfbArgs a, int m0, int span) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    int cnt = 0, q = 0, c = 0, d = 0;
    if (b < a.nitems + a.Q && a.open[b]) {
        cfb_node(a, b, q, c);
        d = a.depth[b];
        cnt = min(span, d + 1 - m0);
        if (cnt < 0) cnt = 0;
    }
    const int t0 = cfb_reserve(&a.st->W, cnt, a.wsum);
    if (b < a.nitems + a.Q) {
        a.tfirst[b] = t0;
        a.tcnt[b] = cnt;
    }
    if (cnt == 0) return;
    const size_t o = (size_t)q * a.row_cap;
    const double x = a.tr.x[o + c], y = a.tr.y[o + c];
    // climb to depth m0 + cnt - 1, then emit the candidates downward to depth m0
    int k = c;
    for (int dd = d; dd > m0 + cnt - 1; --dd) k = a.tr.parent[o + k];
    for (int i = cnt - 1; i >= 0; --i) {
        const int t = t0 + i;
        SteerTask tk;
        tk.x = x;
        tk.y = y;
        tk.px = a.tr.x[o + k];
        tk.py = a.tr.y[o + k];
        tk.pyaw = a.tr.yaw[o + k];
        tk.pnode = k;
        tk.literal = 0;
        a.tasks[t] = tk;
        a.tnode[t] = b;
        if (i > 0) k = a.tr.parent[o + k];
    }
}

// phase A round r, after the walk: a node settles at its first candidate (in order) that is not
// rejected — accepted: ftab = 2 + depth (| 1 << 30 for a None steer, finalize's panic); literal
// path or error: left unknown for check_finish_kernel — or when its last candidate was rejected:
// ftab = 1 (no candidate)
__global__ __launch_bounds__(256) void cfb_consume_a_kernel(CfbArgs a, int m0) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b == 0) a.st->W = 0;  // the next round's counter (every reader of W has finished)
    if (b >= a.nitems + a.Q) return;
    const int cnt = a.tcnt[b];
    if (cnt == 0) return;
    int q, c;
    cfb_node(a, b, q, c);
    const int t0 = a.tfirst[b];
    for (int i = 0; i < cnt; ++i) {
        const int s = a.status[t0 + i];
        if (s == kReject) continue;
        if (s == kAccept) {
            const int fnone = a.none[t0 + i];
            a.ftab[cfb_memo_row(a, q) + c] = (2 + m0 + i) | (fnone << 30);
        }
        a.open[b] = 0;
        return;
    }
    if (m0 + cnt > a.depth[b]) {
        a.ftab[cfb_memo_row(a, q) + c] = 1;
        a.open[b] = 0;
    }
}

// an item's optimize chain from ftab (check_finish_kernel's level loop): n[0] = the item's node,
// n[l + 1] = its level-l candidate (pos[l] = that node's depth); false when an entry on the way
// is unknown
__device__ inline bool cfb_chain(const CfbArgs& a, size_t o, size_t mr, int c, int d, int* n,
                                 int* pos, int& s, int& fnone) {
    s = 0;
    fnone = 0;
    n[0] = c;
    int cur = c, curd = d;
    for (int level = 0; level < kCfLevels; ++level) {
        const int fm = a.ftab[mr + cur];
        if (fm == 0) return false;
        if (fm == 1) break;
        const int found = (fm & 0x3fffffff) - 2;
        fnone = fm >> 30;
        pos[level] = found;
        s = level + 1;
        if (curd == 0) {  // a level at the root: root copies to the recursion limit
            for (int l2 = level + 1; l2 < kCfLevels; ++l2) pos[l2] = 0;
            for (int l2 = level + 1; l2 <= kCfLevels; ++l2) n[l2] = cur;
            s = kCfLevels;
            break;
        }
        while (curd > found) {
            cur = a.tr.parent[o + cur];
            --curd;
        }
        n[level + 1] = cur;
    }
    return true;
}

// phase B: every item's goal edge, and the copy edges of its chain that no other item claimed
__global__ __launch_bounds__(256) void cfb_emit_b_kernel(CfbArgs a) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    int n[kCfLevels + 1], pos[kCfLevels];
    int s = 0, fnone = 0, cnt = 0, q = 0, c = 0;
    size_t o = 0, mr = 0;
    bool ok = false;
    unsigned claimed = 0;  // bit e: this item steers copy edge e (1 <= e < s)
    if (b < a.nitems) {
        cfb_node(a, b, q, c);
        o = (size_t)q * a.row_cap;
        mr = cfb_memo_row(a, q);
        ok = cfb_chain(a, o, mr, c, a.depth[b], n, pos, s, fnone);
        if (ok) {
            cnt = 1;
            // (a plain L2 read first: the edges near a query's root are claimed once and read by
            // most of its items — an exchange each serialised on those few addresses)
            for (int e = 1; e < s; ++e)
                if (__hip_atomic_load(&a.gclaim[mr + n[e - 1]], __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT) == 0 &&
                    atomicExch(&a.gclaim[mr + n[e - 1]], 1) == 0) {
                    claimed |= 1u << e;
                    ++cnt;
                }
        }
    }
    const int t0 = cfb_reserve(&a.st->W, cnt, a.wsum);
    if (!ok) return;
    const double* X = a.tr.x + o;
    const double* Y = a.tr.y + o;
    // the goal edge: Node::new_goal (the goal keeps its yaw: the planner's optimised yaw when
    // optimize succeeded, rrt.rs:489-501) into pose 1 — the copy at the node toward n[1], or
    // the node's stored pose when the chain is empty
    const double gyaw = a.goals[3 * q + 2];
    SteerTask tk;
    tk.x = a.goals[3 * q];
    tk.y = a.goals[3 * q + 1];
    if (s > 0) {
        tk.px = X[c];
        tk.py = Y[c];
        tk.pyaw = cf_atan2(Y[n[1]] - Y[c], X[n[1]] - X[c]);
    } else {
        tk.px = X[c];
        tk.py = Y[c];
        tk.pyaw = a.tr.yaw[o + c];
    }
    tk.pnode = 0;
    tk.literal = 0;
    a.tasks[t0] = tk;
    StarTaskExt ex{};
    ex.own_yaw = 1;
    ex.cyaw = gyaw;
    a.ext[t0] = ex;
    a.tnode[t0] = b;
    int t = t0 + 1;
    for (int e = 1; e < s; ++e) {
        if (!((claimed >> e) & 1u)) continue;
        // copy edge e: from the copy at v = n[e - 1] toward n[e] (compute_yaw) to the copy at
        // n[e] toward n[e + 1]
        const int v = n[e - 1], w = n[e], w2 = n[e + 1];
        SteerTask ct;
        ct.x = X[v];
        ct.y = Y[v];
        ct.px = X[w];
        ct.py = Y[w];
        ct.pyaw = cf_atan2(Y[w2] - Y[w], X[w2] - X[w]);
        ct.pnode = w;
        ct.literal = 0;
        a.tasks[t] = ct;
        a.ext[t] = StarTaskExt{};
        a.tnode[t] = -1 - (int)(mr + v);
        ++t;
    }
}

// phase B, after the walk: the verdicts into gotab / gtab (a None steer: finalize's panic; a
// literal-path or error verdict stays unknown)
__global__ __launch_bounds__(256) void cfb_store_b_kernel(CfbArgs a) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.st->W) return;
    int s = a.status[t];
    if (a.none[t]) s = kCfPanic;
    else if (s != kAccept && s != kReject) return;
    const int n = a.tnode[t];
    if (n >= 0)
        a.gotab[n] = s + 1;
    else
        a.gtab[-1 - n] = s + 1;
}

// after a rounds walk: the literal-path tasks (the trim cases steer_walk hands back, e.g. the
// zero-length copy edges at a root, whose points are all 0.0) re-run by steer_collide_literal,
// as mq_insert does for the extend tasks, so their verdicts reach the memo instead of punting
// every item whose chain holds them to check_finish_kernel.  The list first, then one wave per
// listed task (wave w owns scratch slot w: no locks), so the serial generations run side by side
__global__ __launch_bounds__(256) void cfb_lit_list_kernel(CfbArgs a, int* __restrict__ list,
                                                           int* __restrict__ count) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < a.st->W && a.status[t] == kLiteral) list[atomicAdd(count, 1)] = t;
}

// steer_collide_literal with the literal course generated by the whole wave: the word of
// dubins_path_planning(child → parent) as cf_npoint_steer chooses it, then line_edge_wave (the
// line kernel's lane-parallel restatement of dubins_literal: the same points, the same trim), then
// the same chunk test.  A long trim-case course (thousands of points) no longer runs on one lane.
__device__ int steer_collide_literal_wave(const SceneDev& sc, double x, double y, double yaw,
                                          double px, double py, double pyaw, double* bx,
                                          double* by) {
    const int lane = __lane_id();
    Steer st;
    (void)cf_npoint_steer(sc, CfPose{x, y, yaw}, CfPose{px, py, pyaw}, st);
    const double w[4] = {(double)st.word, st.t, st.p, st.q};
    int n = 0;
    const int r = line_edge_wave(x, y, yaw, w, sc.turn_radius, sc.step_size, bx, by,
                                 kLiteralCap - 1, lane, &n);
    if (r == kSteerOverflow) return kError;
    if (lane == 0) {
        if (r == kSteerNone) {  // polyline [(x, y), (px, py)] (rrt.rs:313)
            bx[0] = x;
            by[0] = y;
            n = 1;
        }
        bx[n] = px;
        by[n] = py;
    }
    if (r == kSteerNone) n = 1;
    __threadfence_block();  // the wave's points before it reads them back
    const int np = n + 1;   // the junction point is bounds-checked too
    for (int base = 0; base == 0 || base + 1 < np; base += 63) {
        const int i = base + lane;
        const bool has = i < np;
        const double qx = has ? bx[i] : x, qy = has ? by[i] : y;
        if (chunk_rejects<false>(sc, has, has && (lane >= 1 || base == 0), has && lane >= 1, qx, qy))
            return kReject;
    }
    return kAccept;
}

__global__ __launch_bounds__(256) void cfb_lit_run_kernel(CfbArgs a, SceneDev sc,
                                                          const int* __restrict__ list,
                                                          const int* __restrict__ count,
                                                          double* __restrict__ lit_scratch) {
    const int lane = __lane_id();
    const int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int nw = (int)((gridDim.x * blockDim.x) >> 6);
    double* bx = lit_scratch + (size_t)gw * 3 * kLiteralCap;
    const int n = *count;
    for (int i = gw; i < n; i += nw) {
        const int t = list[i];
        const SteerTask tk = a.tasks[t];
        const int r = steer_collide_literal_wave(sc, tk.x, tk.y, a.yaw[t], tk.px, tk.py, tk.pyaw,
                                                 bx, bx + kLiteralCap);
        if (lane == 0) a.status[t] = r;
    }
}

hipError_t launch_cfb_literal(hipStream_t s, const SceneDev& sc, const CfbArgs& a, int max_tasks,
                              int* list, int* count, double* lit_scratch) {
    if (max_tasks <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(count, 0, sizeof(int), s);
    if (e != hipSuccess) return e;
    cfb_lit_list_kernel<<<(max_tasks + 255) / 256, 256, 0, s>>>(a, list, count);
    cfb_lit_run_kernel<<<kLiteralWaves / 4, 256, 0, s>>>(a, sc, list, count, lit_scratch);
    return hipGetLastError();
}

// one lane per item: finalize's verdict from the memo (check_finish_kernel's order and
// precedence), its outputs or its line item; an item with an unknown verdict goes to plist
__global__ __launch_bounds__(256) void cfb_assemble_kernel(CfbArgs a, int* __restrict__ ok_out,
                                                           double* __restrict__ len_out,
                                                           int* __restrict__ npts_out,
                                                           int* __restrict__ err,
                                                           int* __restrict__ items,
                                                           int* __restrict__ plist) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= a.nitems) return;
    int q, c;
    cfb_node(a, b, q, c);
    const size_t o = (size_t)q * a.row_cap, mr = cfb_memo_row(a, q);
    int n[kCfLevels + 1], pos[kCfLevels];
    int s = 0, fnone = 0;
    bool known = cfb_chain(a, o, mr, c, a.depth[b], n, pos, s, fnone);
    // verdicts in finalize's order: 0 accept, 1 reject, 2 panic (the first non-accepted decides,
    // a None steer anywhere wins over a rejection)
    int first = 0;
    bool any_none = false;
    if (known) {
        const int g = a.gotab[b];
        known = g == 1 + kAccept || g == 1 + kReject || g == 1 + kCfPanic;
        if (known && g != 1 + kAccept) first = g == 1 + kReject ? 1 : 2;
        any_none = g == 1 + kCfPanic;
    }
    for (int e = 1; known && e < s; ++e) {
        const int g = a.gtab[mr + n[e - 1]];
        known = g == 1 + kAccept || g == 1 + kReject || g == 1 + kCfPanic;
        if (known && g != 1 + kAccept && first == 0) first = g == 1 + kReject ? 1 : 2;
        any_none |= g == 1 + kCfPanic;
    }
    if (!known) {
        plist[atomicAdd(&a.pcount[0], 1)] = b;
        return;
    }
    if (s >= 1 && fnone) {  // edge s: the last level's accepted candidate edge
        any_none = true;
        if (first == 0) first = 2;
    }
    const bool tree_none = a.tnone_up[mr + n[s]] != 0;  // edges s + 1 .. E - 1
    int bad = 0;
    bool vok = false;
    if (first == 2) {
        bad = 2;
    } else if (first == 1) {
        if (any_none || tree_none) bad = 2;
    } else {
        vok = true;
        if (tree_none) bad = 2;
    }
    if (vok && bad == 0) {
        const int it = atomicAdd(&items[0], 1);
        int* ob = items + 1 + (size_t)it * kCfItem;
        ob[0] = b;
        ob[1] = s;
        ob[2] = 1;
        ob[3] = 0;
        for (int i = 0; i < kCfLevels; ++i) ob[4 + i] = i < s ? pos[i] : 0;
    } else {
        ok_out[b] = 0;
        len_out[b] = 0.0;
        npts_out[b] = 0;
        if (bad) atomicOr(err, bad);
    }
}

hipError_t launch_cfb(hipStream_t s, const SceneDev& sc, CfbArgs a, int phase, int round,
                      int* ok, double* len, int* npts, int* err, int* items, int* plist) {
    const int nn = a.nitems + a.Q;
    const int g = (nn + 255) / 256;
    switch (phase) {
        case kCfbDepth:
            cfb_depth_kernel<<<g, 256, 0, s>>>(a, sc);
            cfb_tnone_up_kernel<<<g, 256, 0, s>>>(a);
            break;
        case kCfbEmitA:
            cfb_emit_a_kernel<<<g, 256, 0, s>>>(a, round, a.span);  // round: the first depth m0
            break;
        case kCfbConsumeA:
            cfb_consume_a_kernel<<<g, 256, 0, s>>>(a, round);
            break;
        case kCfbEmitB:
            cfb_emit_b_kernel<<<(a.nitems + 255) / 256, 256, 0, s>>>(a);
            break;
        case kCfbStoreB:
            cfb_store_b_kernel<<<(round + 255) / 256, 256, 0, s>>>(a);  // round: the task bound
            break;
        case kCfbAssemble:
            cfb_assemble_kernel<<<(a.nitems + 255) / 256, 256, 0, s>>>(a, ok, len, npts, err,
                                                                        items, plist);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// the steer rounds' records in chunks of `cap` tasks: chunk [base, base + cap) of the round's
// a.st->W tasks gets its own task count (cfb_chunk_begin), and after its walk the None flags of
// its records (consume A / store B read them once every chunk's record is overwritten)
__global__ void cfb_chunk_begin_kernel(const DevState* __restrict__ all, DevState* __restrict__ chunk,
                                       int base, int cap) {
    const int w = all->W - base;
    chunk->W = w < 0 ? 0 : (w < cap ? w : cap);
    chunk->ncomp = 0;
    chunk->alist = nullptr;
}

__global__ __launch_bounds__(256) void cfb_chunk_none_kernel(const DevState* __restrict__ chunk,
                                                             const PrepRec* __restrict__ rec,
                                                             unsigned char* __restrict__ none) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < chunk->W) none[t] = rec[t].state == kPrepNone ? 1 : 0;
}

hipError_t launch_cfb_chunk(hipStream_t s, const DevState* all, DevState* chunk, int base,
                            int cap, bool begin, const PrepRec* rec, unsigned char* none) {
    if (begin)
        cfb_chunk_begin_kernel<<<1, 1, 0, s>>>(all, chunk, base, cap);
    else
        cfb_chunk_none_kernel<<<(cap + 255) / 256, 256, 0, s>>>(chunk, rec, none);
    return hipGetLastError();
}

// a steer round over the tasks the emit kernel counted in st->W (the query batch's kernels)
hipError_t launch_cfb_steer(hipStream_t s, const SceneDev& sc, const CfbArgs& a, int max_tasks,
                            bool own_yaw, long long* wg_points) {
    if (max_tasks <= 0) return hipSuccess;
    const int pb = std::min((max_tasks + 31) / 32, 8192);
    steer_prep_kernel<<<pb, kPrepThreads, 0, s>>>(a.st, sc, nullptr, nullptr, nullptr, nullptr,
                                                  a.rec, a.yaw, a.tasks, nullptr,
                                                  own_yaw ? a.ext : nullptr);
    const int wb = std::min(std::max(1, (max_tasks + kWalkThreads / 64 - 1) / (kWalkThreads / 64)),
                            std::min(kWalkMaxWG, walk_grid_cap<kWalkMinWBatch, 4, true>(sc)));
    launch_walk<kWalkMinWBatch, true>(s, wb, a.st, sc, a.rec, nullptr, a.status, nullptr, nullptr,
                                      wg_points);
    return hipGetLastError();
}

// ------------------------------------------------- multi-query batch (config 3)
//
// One lockstep step advances every query by one plan_one extend iteration (rrt.rs:583-589):
//   mq_sample_nn   one wave per query: rand_point (the query's own seeded stream) and the exact
//                  f64 brute-force nearest node of its tree (lanes stride the SoA rows, lowest
//                  index on ties) — each step streams every tree once: the HBM-read-bound NN of
//                  SURVEY §8d
//   steer_prep / steer_walk   the window pipeline's kernels on the Q explicit tasks
//   mq_insert      the verdict (literal path for the measure-zero trim cases), append, it += 1
// Queries are independent, so there is no speculation and no resolve.
// One query's window of the lockstep step (one wave, all 64 lanes): lane l serves window slot
// k = l % K over node group g = l / K (nodes i = g mod 64/K), so every node row is loaded once per
// wave, not once per slot.  Space::rand_point of iteration it[q] + k on stream q (rrt.rs:139-146,
// Q7), the obstacle pre-test, the exact nearest node of tree q as the step found it (rrt.rs:378-391,
// Q9: lanes stride the rows, lowest index on ties), the verdict cache; the task into
// tasks[q K + k].
__device__ __forceinline__ bool mq_nn_query(const MqDev& mq, double minx, double maxx, double miny,
                                            double maxy, SteerTask* __restrict__ tasks,
                                            const SceneDev* __restrict__ scp, int q, int lane,
                                            SteerTask& tko) {
    const int K = mq.K, G = 64 / K;
    const int k = lane & (K - 1), g = lane / K;
    const int64_t it = mq.it[q] + k;
    const bool live = it < mq.target[q];
    const uint64_t seed = mq.seed[q];
    // the verdict cache: the task region still holds the previous step's window, which
    // started Tp iterations before this one, so iteration it sat in old slot k + Tp; its
    // parent, verdict and yaw are read before any lane overwrites the region.  Lane k reads slot
    // k + Tp, which lane k + Tp of the SAME wave rewrites below (tasks, status, tyaw of slot t):
    // that is ordered only because all K slots of a query are served by one wave (K <= 64, one
    // query per K lanes) and every load is issued before the first store: the wave barrier
    // keeps the compiler from sinking a load past the stores, and one wave's vector memory
    // requests to an address are served in issue order.  Serving a query's slots from more than
    // one wave would need a grid-wide ordering instead.
    int opn = -1, ost = -1;
    double oyw = 0.0;
    if (mq.it_prev && g == 0) {
        const int64_t Tp = mq.it[q] - mq.it_prev[q];
        if (Tp >= 0 && Tp < K && k + Tp < K) {
            const int to = q * K + k + (int)Tp;
            opn = tasks[to].pnode;
            ost = mq.status[to];
            if (mq.tyaw) oyw = mq.tyaw[to];
        }
    }
    __builtin_amdgcn_wave_barrier();
    double x = 0.0, y = 0.0;
    if (live) {
        x = gen_range(seed, 2 * (uint64_t)it, minx, maxx);
        y = gen_range(seed, 2 * (uint64_t)it + 1, miny, maxy);
    }
    // the pre-test first (its loads overlap the scan; its result is used after it)
    const bool blocked = live && scp && point_blocked<false, kSceneAny>(*scp, x, y);
    const int n = mq.n[q];
    const size_t row = (size_t)q * mq.cap;
    const double* __restrict__ X = mq.x + row;
    const double* __restrict__ Y = mq.y + row;
    double bd = __builtin_inf();
    int bi = 0x7fffffff;
#pragma unroll 4
    for (int i = g; i < n; i += G) {
        const double dx = x - X[i], dy = y - Y[i];
        const double d2 = dx * dx + dy * dy;
        if (d2 < bd) {
            bd = d2;
            bi = i;
        }
    }
    for (int m = K; m < 64; m <<= 1) {  // the G lanes of slot k
        if (m == 16)
            argmin_swap<false>(bd, bi);
        else if (m == 32)
            argmin_swap<true>(bd, bi);
        else
            argmin_pair(bd, bi, __shfl_xor(bd, m), __shfl_xor(bi, m));
    }
    bool need = false;  // the slot needs steer_prep + steer_walk
    const int t = q * K + k;
    if (g == 0) {
        if (!live) {
            tasks[t].pnode = -1;
        } else if (blocked) {
            // the sample lies in an obstacle: rejected whatever its parent (pnode -2: no steer,
            // and the insert never cuts the window there)
            tasks[t].x = x;
            tasks[t].y = y;
            tasks[t].pnode = -2;
            if (mq.alist) mq.status[t] = kReject;
        } else {
            // the same child (the counter RNG redraws it) and the same parent pose (rows are
            // never rewritten) as a task the previous step walked: its verdict (kReject 0 /
            // kAccept 1, as 2 + verdict) — settled here with the old slot's yaw (the same
            // compute_yaw of the same poses) when the batch lists its active tasks, else
            // steer_prep writes it as decided
            const int cached = (opn == bi && (ost == kAccept || ost == kReject)) ? 2 + ost : 0;
            tko = SteerTask{x, y, X[bi], Y[bi], mq.yaw[row + bi], bi, cached};
            tasks[t] = tko;
            mq.nnd2[t] = bd;
            if (mq.alist && cached) {
                mq.status[t] = cached - 2;
                mq.tyaw[t] = oyw;
            } else {
                need = true;
            }
        }
    }
    if (mq.it_prev && lane == 0) mq.it_prev[q] = mq.it[q];
    return need;
}

// The listed tasks take one reservation per workgroup (its waves' counts summed in LDS): one
// atomic per query on the batch's one counter serialised the 8192-query step (642 -> 612 M
// it/s).  NT: 1024 threads (16 queries) for large sub-batches, 256 for small ones, whose
// workgroups would otherwise crowd onto a few CUs (a 512-query sub-batch: 32 workgroups).
template <int NT>
__global__ __launch_bounds__(NT) void mq_sample_nn_kernel(MqDev mq, double minx,
                                                                    double maxx, double miny,
                                                                    double maxy,
                                                                    SteerTask* __restrict__ tasks,
                                                                    const SceneDev* __restrict__ scp) {
    constexpr int kMqNnWaves = NT / 64;
    __shared__ int s_cnt[kMqNnWaves];
    __shared__ int s_base;
    const int lane = __lane_id();
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    // (every wave of the workgroup makes the same trips: the barriers below)
    for (int qb = (int)blockIdx.x * kMqNnWaves; qb < mq.Q; qb += (int)gridDim.x * kMqNnWaves) {
        const int q = qb + wave;
        SteerTask tk{};
        const bool need =
            q < mq.Q && mq_nn_query(mq, minx, maxx, miny, maxy, tasks, scp, q, lane, tk);
        if (mq.alist) {
            const uint64_t nm = __ballot(need);
            if (lane == 0) s_cnt[wave] = __popcll(nm);
            __syncthreads();
            if (threadIdx.x == 0) {
                int tot = 0;
                for (int w = 0; w < kMqNnWaves; ++w) {
                    const int c = s_cnt[w];
                    s_cnt[w] = tot;
                    tot += c;
                }
                s_base = tot ? atomicAdd(&mq.st->W, tot) : 0;
            }
            __syncthreads();
            if (need) {
                const int i = s_base + s_cnt[wave] + __popcll(nm & ((1ull << lane) - 1ull));
                mq.alist[i] = q * mq.K + lane;  // (need: lane = slot k, node group 0)
                mq.status[q * mq.K + lane] = -2 - i;  // (the walk's verdict: lstat[i])
                tk.literal = 0;
                mq.ctask[i] = tk;
            }
            __syncthreads();  // (s_cnt / s_base: the next trip)
        }
    }
}

// the iteration targets of one pp_batch_extend call: n_steps more iterations, at most max_iter
__global__ __launch_bounds__(256) void mq_target_kernel(MqDev mq, int64_t n_steps,
                                                        int64_t* __restrict__ target) {
    const int q = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (q >= mq.Q) return;
    const int64_t t = mq.it[q] + n_steps;
    target[q] = t < mq.max_iter ? t : mq.max_iter;
}

__global__ __launch_bounds__(256) void mq_insert_kernel(MqDev mq, SceneDev sc,
                                                        const SteerTask* __restrict__ tasks,
                                                        int* __restrict__ status,
                                                        const double* __restrict__ yaw,
                                                        double* __restrict__ lit_scratch,
                                                        int* __restrict__ lit_locks,
                                                        int* __restrict__ err) {
    // a wave serves 64 / K queries, K lanes each (lane = g * K + k: the window's iteration
    // it[q] + k of its g-th query; K a power of two <= kMqMaxK = 64, automatically 32, halved
    // while Q * K > 262144).  Literal-path re-runs first (rare, the wave's one scratch buffer), then each query's in-order replay: iteration k keeps its
    // speculative verdict unless an accepted window sample k' < k is strictly nearer than its
    // snapshot NN (snapshot nodes have lower indices and win ties) — the window stops there and
    // the next step resumes at it; the accepted samples before it are appended in order
    // (rrt.rs:586-589).
    const int lane = __lane_id();
    const int gw = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
    const int nw = (int)((gridDim.x * blockDim.x) >> 6);
    // the step's steer kernels are done: the next step's mq_sample_nn lists afresh
    if (mq.alist && gw == 0 && lane == 0) mq.st->W = 0;
    const int K = mq.K, G = 64 / K;
    const int g = lane / K, k = lane - g * K, g0 = g * K;
    const uint64_t gmask = (K == 64 ? ~0ull : ((1ull << K) - 1ull)) << g0;
    for (int base = gw * G; base < mq.Q; base += nw * G) {
        const int q = base + g;
        const bool in = q < mq.Q;
        const int t = q * K + k;
        SteerTask tk{};
        int st = kReject;
        double yw = 0.0, d2nn = 0.0;
        if (in) {
            tk = tasks[t];
            st = status[t];
            yw = yaw[t];
            if (st <= -2) {  // a listed slot: the walk's verdict, kept for the next step's cache
                const int i = -2 - st, lg = mq.st->lgrid;
                st = mq.lstat[(i % lg) * mq.st->lper + i / lg];
                status[t] = st;
            }
        }
        const bool live = in && tk.pnode != -1;  // (pnode -2: a sample in an obstacle)
        const bool act = in && tk.pnode >= 0;
        if (act) d2nn = mq.nnd2[t];
        if (uint64_t lit = __ballot(act && st == kLiteral)) {
            const int slot = lit_acquire(lit_locks, gw);
            double* bx = lit_scratch + (size_t)slot * 3 * kLiteralCap;
            for (; lit; lit &= lit - 1) {
                const int l = __builtin_ctzll(lit);
                const double x = __shfl(tk.x, l), y = __shfl(tk.y, l), w = __shfl(yw, l);
                const double px = __shfl(tk.px, l), py = __shfl(tk.py, l);
                const double pw = __shfl(tk.pyaw, l);
                const int r = steer_collide_literal(sc, x, y, w, px, py, pw, bx, bx + kLiteralCap,
                                                    bx + 2 * kLiteralCap);
                if (lane == l) st = r;
            }
            lit_release(lit_locks, slot);
        }
        const bool blocked = in && mq.blocked && mq.blocked[q];
        const uint64_t accm = __ballot(act && st == kAccept && !blocked);
        bool cut = !live;
        for (int j = 0; j < K; ++j) {  // slot j of every query against its later slots
            const double xj = __shfl(tk.x, g0 + j), yj = __shfl(tk.y, g0 + j);
            if (((accm >> (g0 + j)) & 1ull) && k > j && act) {
                const double dx = tk.x - xj, dy = tk.y - yj;
                if (dx * dx + dy * dy < d2nn) cut = true;
            }
        }
        const uint64_t cutm = __ballot(in && cut) & gmask;
        const int T = cutm ? (int)__builtin_ctzll(cutm) - g0 : K;  // iterations consumed
        const uint64_t keep = accm & gmask & ((T >= 64 ? ~0ull : ((1ull << T) - 1ull)) << g0);
        const bool bad = __ballot(k < T && act && st == kError) & gmask;
        const int n = in ? mq.n[q] : 0;
        const int before = __popcll(keep & ((1ull << lane) - 1ull));
        if (!bad && k < T && ((keep >> lane) & 1ull)) {
            const size_t o = (size_t)q * mq.cap + n + before;
            mq.x[o] = tk.x;
            mq.y[o] = tk.y;
            mq.yaw[o] = yw;
            mq.parent[o] = tk.pnode;
        }
        // NN node-distance evaluations of the sequential spec: iteration k scans the tree as it
        // stands then (n + the window samples accepted before it)
        int64_t ev = (in && k < T) ? (int64_t)(n + before) : 0;
        for (int o = 1; o < K; o <<= 1) ev += __shfl_xor(ev, o);
        if (in && k == 0 && T > 0) {
            if (bad) {
                atomicOr(err, 1);
            } else {
                mq.n[q] = n + __popcll(keep);
                mq.it[q] += T;
                mq.evals[q] += ev;
            }
        }
    }
}

// roots of a new batch (RRT::new, rrt.rs:344-346): row 0 of every tree
__global__ __launch_bounds__(256) void mq_init_kernel(MqDev mq, const double* __restrict__ starts) {
    const int q = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (q >= mq.Q) return;
    const size_t o = (size_t)q * mq.cap;
    mq.x[o] = starts[3 * q];
    mq.y[o] = starts[3 * q + 1];
    mq.yaw[o] = starts[3 * q + 2];
    mq.parent[o] = -1;
    mq.n[q] = 1;
    mq.it[q] = 0;
    mq.evals[q] = 0;
}

hipError_t launch_mq_init(hipStream_t s, const MqDev& mq, const double* starts) {
    mq_init_kernel<<<(mq.Q + 255) / 256, 256, 0, s>>>(mq, starts);
    return hipGetLastError();
}

hipError_t launch_mq_target(hipStream_t s, const MqDev& mq, int64_t n_steps, int64_t* target) {
    mq_target_kernel<<<(mq.Q + 255) / 256, 256, 0, s>>>(mq, n_steps, target);
    return hipGetLastError();
}

// tasks per step (per sub-batch) from which the batch walk runs at 6 waves per SIMD: with its
// spill down to 20 B (round 5) the 1024-query shard's 16k-task sub-batch steps gain too
// (276.8 -> 283.0 M it/s, gpurun_out/r05occ; 3 workgroups per CU instead of 2: no gain)
constexpr int kBigStepTasks = 16384;

hipError_t launch_mq_steps(hipStream_t s, const MqArgs& a, int steps) {
    const int Q = a.mq.Q;
    const int T = Q * a.mq.K;  // tasks per step
    // one wave per query: 16 per workgroup from 2048 queries (a sub-batch of the full batch), 4 below
    const bool big_nn = Q >= 2048;
    const int nn_waves = big_nn ? 16 : 4;
    const int nn_blocks = std::min((Q + nn_waves - 1) / nn_waves, 4096);
    const int prep_blocks = std::min((T + kPrepThreads / 8 - 1) / (kPrepThreads / 8), 2048);
    // the grid cap of the instantiation this step size launches (below)
    const int walk_cap = T >= kBigStepTasks ? walk_grid_cap<kWalkMinWBatch, 2, true>(a.sc)
                                            : walk_grid_cap<kWalkMinWBatch - 1, 2, true>(a.sc);
    const int walk_blocks = std::min((T + kWalkThreads / 64 - 1) / (kWalkThreads / 64),
                                     std::min(kWalkMaxWG, walk_cap));
    const int ins_blocks = std::min((Q + 4 * (64 / a.mq.K) - 1) / (4 * (64 / a.mq.K)), 4096);
    int* wstat = a.mq.alist ? a.mq.lstat : a.status;  // the walk's verdicts (list order)

    for (int k = 0; k < steps; ++k) {
        hipEvent_t* ev = a.ev ? a.ev + 5 * k : nullptr;
        if (ev) (void)hipEventRecord(ev[0], s);
        if (big_nn)
            mq_sample_nn_kernel<1024><<<nn_blocks, 1024, 0, s>>>(a.mq, a.sc.minx, a.sc.maxx,
                                                                a.sc.miny, a.sc.maxy, a.tasks, a.scp);
        else
            mq_sample_nn_kernel<256><<<nn_blocks, 256, 0, s>>>(a.mq, a.sc.minx, a.sc.maxx,
                                                              a.sc.miny, a.sc.maxy, a.tasks, a.scp);
        if (ev) (void)hipEventRecord(ev[1], s);
        // (the listed tasks, compacted by mq_sample_nn)
        steer_prep_kernel<<<prep_blocks, kPrepThreads, 0, s>>>(a.st, a.sc, nullptr, nullptr,
                                                              nullptr, nullptr, a.rec, a.yaw,
                                                              a.mq.alist ? a.mq.ctask : a.tasks);
        if (ev) (void)hipEventRecord(ev[2], s);
        // with the analytic straight segments (s_classify).  Steps of >= kBigStepTasks tasks
        // walk at 6 waves per SIMD (80 VGPRs, 20 B of spill), smaller ones at 5 (96 VGPRs, no
        // spill); the 8192-query batch at 5 waves: 641 -> 623 M it/s (round 5, one box)
        if (T >= kBigStepTasks)
            launch_walk<kWalkMinWBatch, true>(s, walk_blocks, a.st, a.sc, a.rec, nullptr, wstat,
                                              nullptr, nullptr, a.wg_points);
        else
            launch_walk<kWalkMinWBatch - 1, true>(s, walk_blocks, a.st, a.sc, a.rec, nullptr,
                                                  wstat, nullptr, nullptr, a.wg_points);
        if (ev) (void)hipEventRecord(ev[3], s);
        mq_insert_kernel<<<ins_blocks, 256, 0, s>>>(a.mq, a.sc, a.tasks, a.status, a.yaw,
                                                    a.lit_scratch, a.lit_locks, a.err);
        if (ev) (void)hipEventRecord(ev[4], s);
    }
    return hipGetLastError();
}

// ------------------------------------------------------- RRT* query batch (config 5, §3.7)
//
// One lockstep step = one RRT* iteration of every query (oracle/pp_oracle.c orc_star_extend):
//   star_sample    one wave per query: rand_point, the exact nearest node, Steer(eta) and the
//                  gate task (new → nearest)                                      → round A
//   star_knn       gated queries: X_near = the k nearest nodes of the new point (exact f64,
//                  (d2, index) order, distances cached in LDS), one choose-parent task per
//                  X_near node other than the nearest                               → round B
//   star_insert    the first strict minimum of cost(p) + edge cost over the feasible candidates
//                  (nearest first), the append, one rewire task per X_near node that could
//                  still get cheaper (cost(new) < cost(m))                          → round C
//   star_rewire    the rewires in X_near order against the costs as they stand, each followed by
//                  a level-synchronous recomputation of the rewired node's subtree costs
// Rounds A/B/C are the window pipeline's steer_prep / steer_walk on explicit tasks; their task
// counts live in DevState W (stA: Q, stB / stC: counted on the device), so a step needs no host
// round trip.
constexpr int kKnnWaves = 4;
constexpr int kKnnCache = 2048;  // d2 values cached per wave (LDS: 4 x 16 KB)

__device__ __forceinline__ bool star_feasible(int status, double e) {
    return status == kAccept && e <= 1.7976931348623157e308;  // Some and verified (finite cost)
}

// Bitonic sort of one (d, i) pair per lane across the wave, ascending in (d, i) lexicographic
// order (lane r ends up with the r-th smallest): 21 compare-exchange stages over __shfl_xor.
struct Kv {
    double d;
    int i;
};
__device__ __forceinline__ Kv bitonic64(double d, int lane, int i = 0) {
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            const double od = __shfl_xor(d, stride);
            const int oi = __shfl_xor(i, stride);
            const bool other_less = od < d || (od == d && oi < i);
            const bool keep_min = ((lane & stride) == 0) == ((lane & size) == 0 || size == 64);
            if (keep_min == other_less) {
                d = od;
                i = oi;
            }
        }
    }
    return Kv{d, i};
}

// exact lower bound of an edge's Dubins cost (normalised by the turn radius): the chord, with a
// slack far above the rounding of both (prunes only what cannot win, so results are unchanged)
__device__ __forceinline__ double star_chord_lb(double d2, double curv) {
    return sqrt(d2) * curv * (1.0 - 1e-9) - 1e-9;
}

__global__ __launch_bounds__(256) void star_sample_kernel(StarDev sd, double minx, double maxx,
                                                          double miny, double maxy,
                                                          SteerTask* __restrict__ tasks) {
    const int lane = __lane_id();
    const int gw = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
    const int nw = (int)((gridDim.x * blockDim.x) >> 6);
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // the step's round-B / round-C task counters
        sd.stB->W = 0;
        sd.stC->W = 0;
    }
    const MqDev& mq = sd.mq;
    for (int q = gw; q < mq.Q; q += nw) {
        const int64_t it = mq.it[q];
        if (it >= mq.target[q]) {
            if (lane == 0) {
                tasks[q].pnode = -1;
                sd.pn[q] = -1;
            }
            continue;
        }
        const uint64_t seed = mq.seed[q];
        double x = gen_range(seed, 2 * (uint64_t)it, minx, maxx);      // rrt.rs:139-146 (Q7)
        double y = gen_range(seed, 2 * (uint64_t)it + 1, miny, maxy);
        const int n = mq.n[q];
        const size_t row = (size_t)q * mq.cap;
        const double* __restrict__ X = mq.x + row;
        const double* __restrict__ Y = mq.y + row;
        double bd = __builtin_inf();
        int bi = 0x7fffffff;
#pragma unroll 4
        for (int i = lane; i < n; i += 64) {  // rrt.rs:378-391 (Q9: exact, lowest index on ties)
            const double dx = x - X[i], dy = y - Y[i];
            const double d2 = dx * dx + dy * dy;
            if (d2 < bd) {
                bd = d2;
                bi = i;
            }
        }
        wave_argmin(bd, bi);
        const double nx = X[bi], ny = Y[bi];
        if (sd.eta > 0.0 && bd > sd.eta * sd.eta) {  // Steer(x_nearest, x_rand)
            const double f = sd.eta / sqrt(bd);
            x = nx + (x - nx) * f;
            y = ny + (y - ny) * f;
        }
        if (lane == 0) {
            SteerTask tk{};
            tk.x = x;
            tk.y = y;
            tk.px = nx;
            tk.py = ny;
            tk.pyaw = mq.yaw[row + bi];
            tk.pnode = bi;
            tasks[q] = tk;
            sd.px[q] = x;
            sd.py[q] = y;
            sd.pn[q] = bi;
        }
    }
}

__global__ __launch_bounds__(256) void star_knn_kernel(StarDev sd, const int* __restrict__ statusA,
                                                       const double* __restrict__ costA,
                                                       SteerTask* __restrict__ tasksB,
                                                       StarTaskExt* __restrict__ extB,
                                                       int* __restrict__ err) {
    __shared__ double s_d2[kKnnWaves][kKnnCache];
    __shared__ double s_cd[kKnnWaves][64];
    __shared__ int s_ci[kKnnWaves][64];
    const int lane = __lane_id(), wave = threadIdx.x >> 6;
    double* cand_d = s_cd[wave];
    int* cand_i = s_ci[wave];
    const MqDev& mq = sd.mq;
    double* cache = s_d2[wave];
    __shared__ int s_cnt[kKnnWaves], s_base;
    // wave w of workgroup b serves queries b * kKnnWaves + w (+ the grid's stride): every wave of
    // a workgroup runs the same iterations, so the round-B task reservation is one atomic per
    // workgroup instead of one per query (one counter address for the whole launch)
    for (int qb = (int)blockIdx.x * kKnnWaves; qb < mq.Q; qb += (int)gridDim.x * kKnnWaves) {
        const int q = qb + wave;
        const int p = q < mq.Q ? sd.pn[q] : -1;
        bool live = p >= 0;
        int n = 0, st = kReject;
        if (live) {
            n = mq.n[q];
            st = statusA[q];
            // the gate: the edge new → nearest (a literal-path verdict is settled by star_insert)
            const bool gate = (st == kLiteral || star_feasible(st, costA[q])) &&
                              !(mq.blocked && mq.blocked[q]);
            if (!gate) {
                if (lane == 0) {
                    if (st == kError) atomicOr(err, 1);  // n_point overflow: the reference panics
                    sd.nnear[q] = -1;
                    mq.it[q] += 1;
                    mq.evals[q] += n;
                }
                live = false;
            }
        }
        double x = 0.0, y = 0.0, c0 = 0.0;
        size_t row = 0;
        int k = 0, mine = -1;
        bool want = false;
        uint64_t bm = 0;
        const double* __restrict__ X = mq.x;
        const double* __restrict__ Y = mq.y;
        if (live) {
            x = sd.px[q];
            y = sd.py[q];
            row = (size_t)q * mq.cap;
            X = mq.x + row;
            Y = mq.y + row;
            k = sd.ksched[n];
            const bool cached = n <= kKnnCache;
            bool done = false;
            if (cached) {
                double lmin = __builtin_inf();
#pragma unroll 8
                for (int i = lane; i < n; i += 64) {
                    const double dx = x - X[i], dy = y - Y[i];
                    const double d2 = dx * dx + dy * dy;
                    cache[i] = d2;
                    lmin = fmin(lmin, d2);
                }
                // T = the k-th smallest lane minimum: k distinct nodes lie within it, so the k
                // nearest are among the nodes with d2 <= T (usually k..2k of them)
                const double T = readlane_f64(bitonic64(lmin, lane).d, k - 1);
                int c = 0;
                for (int i = lane; i < n; i += 64) c += cache[i] <= T;
                int off = wave_incl_scan(c);  // inclusive prefix over the lanes
                const int C = __builtin_amdgcn_readlane(off, 63);
                if (C <= 64) {  // gather them into one (d2, index) pair per lane and sort the wave
                    off -= c;
                    for (int i = lane; i < n; i += 64)
                        if (cache[i] <= T) {
                            cand_d[off] = cache[i];
                            cand_i[off] = i;
                            ++off;
                        }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    Kv kv{__builtin_inf(), 0x7fffffff};
                    if (lane < C) kv = Kv{cand_d[lane], cand_i[lane]};
                    kv = bitonic64(kv.d, lane, kv.i);
                    mine = lane < k ? kv.i : -1;
                    done = true;
                    __builtin_amdgcn_wave_barrier();  // the list is reused by the next query
                }
            }
            if (!done) {
                // k rounds of the lexicographic (d2, index) successor of the previous winner
                double pd = -1.0;
                int pi = -1;
                for (int r = 0; r < k; ++r) {
                    double bd = __builtin_inf();
                    int bi = 0x7fffffff;
                    for (int i = lane; i < n; i += 64) {
                        double d2;
                        if (cached) {
                            d2 = cache[i];
                        } else {
                            const double dx = x - X[i], dy = y - Y[i];
                            d2 = dx * dx + dy * dy;
                        }
                        if ((d2 > pd || (d2 == pd && i > pi)) && d2 < bd) {
                            bd = d2;
                            bi = i;
                        }
                    }
                    wave_argmin(bd, bi);
                    pd = bd;
                    pi = bi;
                    if (lane == r) mine = bi;
                }
            }
            const bool has = lane < k;
            if (has) sd.near[(size_t)q * kStarKMax + lane] = mine;
            // candidates that could still beat the nearest's cost c0 (chord lower bound): the
            // others can never be the first strict minimum, so they are not steered
            c0 = sd.cost[row + p] + costA[q];
            want = has && mine != p;
            if (want) {
                const double dx = x - X[mine], dy = y - Y[mine];
                want = sd.cost[row + mine] + star_chord_lb(dx * dx + dy * dy, sd.curv) < c0;
            }
            bm = __ballot(want);
        }
        const int cnt = __popcll(bm);
        if (lane == 0) s_cnt[wave] = cnt;
        __syncthreads();
        if (threadIdx.x == 0) {
            int tot = 0;
            for (int w = 0; w < kKnnWaves; ++w) tot += s_cnt[w];
            s_base = tot > 0 ? atomicAdd(&sd.stB->W, tot) : 0;
        }
        __syncthreads();
        if (live) {
            int slot = s_base;
            for (int w = 0; w < wave; ++w) slot += s_cnt[w];
            slot = cnt > 0 ? slot : 0;
            if (lane == 0) {
                sd.nnear[q] = k;
                sd.bmask[q] = bm;
                sd.bslot[q] = slot;
            }
            if (want) {  // X_near order
                const int idx = __popcll(bm & ((1ull << lane) - 1ull));
                SteerTask tk{};
                tk.x = x;
                tk.y = y;
                tk.px = X[mine];
                tk.py = Y[mine];
                tk.pyaw = mq.yaw[row + mine];
                tk.pnode = mine;
                tasksB[slot + idx] = tk;
                StarTaskExt ex{};
                ex.cull = 1;  // only a candidate strictly cheaper than the nearest's can win
                ex.cbase = sd.cost[row + mine];
                ex.climit = c0;
                extB[slot + idx] = ex;
            }
        }
        __syncthreads();  // s_cnt / s_base are rewritten by the next iteration
    }
}

// settle literal-path verdicts of a wave's lanes (the measure-zero trim cases), one at a time
__device__ __forceinline__ int star_settle(const SceneDev& sc, int st, bool act, double x, double y,
                                           double yaw, double px, double py, double pyaw,
                                           double* lit_scratch, int* locks, int hint) {
    const int lane = __lane_id();
    uint64_t lit = __ballot(act && st == kLiteral);
    if (!lit) return st;
    const int slot = lit_acquire(locks, hint);
    double* bx = lit_scratch + (size_t)slot * 3 * kLiteralCap;
    for (; lit; lit &= lit - 1) {
        const int l = __builtin_ctzll(lit);
        const int r = steer_collide_literal(sc, __shfl(x, l), __shfl(y, l), __shfl(yaw, l),
                                            __shfl(px, l), __shfl(py, l), __shfl(pyaw, l), bx,
                                            bx + kLiteralCap, bx + 2 * kLiteralCap);
        if (lane == l) st = r;
    }
    lit_release(locks, slot);
    return st;
}

__global__ __launch_bounds__(256) void star_insert_kernel(
    StarDev sd, SceneDev sc, const int* __restrict__ statusA, const double* __restrict__ yawA,
    const double* __restrict__ costA, const SteerTask* __restrict__ tasksB,
    const int* __restrict__ statusB, const double* __restrict__ yawB,
    const double* __restrict__ costB, SteerTask* __restrict__ tasksC,
    StarTaskExt* __restrict__ extC, double* __restrict__ lit_scratch, int* __restrict__ err) {
    const int lane = __lane_id();
    const int gw = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
    const MqDev& mq = sd.mq;
    const int wave = threadIdx.x >> 6;
    __shared__ int s_cnt[4], s_base;
    // every wave of a workgroup runs the same iterations (queries b * 4 + w, + the grid's
    // stride), so the round-C task reservation is one atomic per workgroup
    for (int qb = (int)blockIdx.x * 4; qb < mq.Q; qb += (int)gridDim.x * 4) {
        const int q = qb + wave;
        bool live = q < mq.Q && sd.pn[q] >= 0;
        const int k = live ? sd.nnear[q] : -1;
        live = live && k >= 0;  // (k < 0: no insert this step, settled by star_knn)
        const int p = live ? sd.pn[q] : 0;
        const int n = live ? mq.n[q] : 0;
        const size_t row = (size_t)(live ? q : 0) * mq.cap;
        double x = 0.0, y = 0.0, cb = 0.0, yb = 0.0;
        int mine = -1;
        uint64_t wm = 0;
        bool want = false;
        if (live) {
            x = sd.px[q];
            y = sd.py[q];
            mine = lane < k ? sd.near[(size_t)q * kStarKMax + lane] : -1;
            // the nearest, then the X_near nodes star_knn steered (the pruned ones cannot win)
            const int ncand = 1 + __popcll(sd.bmask[q]);
            const bool act = lane < ncand;
            int node = p, st = kReject;
            double yaw = 0.0, e = __builtin_inf();
            if (lane == 0) {
                st = statusA[q];
                yaw = yawA[q];
                e = costA[q];
            } else if (act) {
                const int t = sd.bslot[q] + lane - 1;
                node = tasksB[t].pnode;
                st = statusB[t];
                yaw = yawB[t];
                e = costB[t];
            }
            const double nx = mq.x[row + node], ny = mq.y[row + node], nyaw = mq.yaw[row + node];
            st = star_settle(sc, st, act, x, y, yaw, nx, ny, nyaw, lit_scratch, sd.lit_locks, gw);
            if (__ballot(act && st == kError)) {
                if (lane == 0) atomicOr(err, 1);
                live = false;
            } else {
                const bool feas = act && star_feasible(st, e);
                if (!__shfl((int)feas, 0)) {  // the gate failed on the literal path
                    if (lane == 0) {
                        sd.nnear[q] = -1;
                        mq.it[q] += 1;
                        mq.evals[q] += n;
                    }
                    live = false;
                } else {
                    // choose parent: the first strict minimum of cost(node) + edge cost in
                    // candidate order
                    double c = feas ? sd.cost[row + node] + e : __builtin_inf();
                    int bl = lane;
                    wave_argmin(c, bl);
                    const int best = __shfl(node, bl);
                    yb = __shfl(yaw, bl);
                    const double eb = __shfl(e, bl);
                    cb = c;
                    if (lane == 0) {
                        const size_t o = row + n;
                        mq.x[o] = x;
                        mq.y[o] = y;
                        mq.yaw[o] = yb;
                        mq.parent[o] = best;
                        sd.cost[o] = cb;
                        sd.elen[o] = eb;
                        mq.n[q] = n + 1;
                        mq.it[q] += 1;
                        mq.evals[q] += n;
                        sd.cb[q] = cb;
                    }
                    // rewire tasks: X_near nodes other than the parent that could still get
                    // cheaper (cost(new) + e >= cost(new) >= cost(m) otherwise; costs only
                    // decrease)
                    want = lane < k && mine != best;
                    if (want) {  // chord lower bound of the rewire edge (prunes only what cannot rewire)
                        const double dx = x - mq.x[row + mine], dy = y - mq.y[row + mine];
                        want = cb + star_chord_lb(dx * dx + dy * dy, sd.curv) < sd.cost[row + mine];
                    }
                    wm = __ballot(want);
                }
            }
        }
        const int cnt = __popcll(wm);
        if (lane == 0) s_cnt[wave] = cnt;
        __syncthreads();
        if (threadIdx.x == 0) {
            const int tot = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
            s_base = tot > 0 ? atomicAdd(&sd.stC->W, tot) : 0;
        }
        __syncthreads();
        if (live) {
            int slot = s_base;
            for (int w = 0; w < wave; ++w) slot += s_cnt[w];
            slot = cnt > 0 ? slot : -1;
            if (lane == 0) {
                sd.cslot[q] = slot;
                sd.cmask[q] = wm;
            }
            if (want) {
                SteerTask tk{};
                tk.x = mq.x[row + mine];
                tk.y = mq.y[row + mine];
                tk.px = x;
                tk.py = y;
                tk.pyaw = yb;
                tk.pnode = n;  // the new node (the edge's parent)
                const int tc = slot + __popcll(wm & ((1ull << lane) - 1ull));
                tasksC[tc] = tk;
                StarTaskExt ex{};
                ex.cyaw = mq.yaw[row + mine];
                ex.own_yaw = 1;
                ex.node = mine;
                ex.cull = 1;  // only a strictly cheaper path through the new node matters
                ex.cbase = cb;
                ex.climit = sd.cost[row + mine];
                extC[tc] = ex;
            }
        }
        __syncthreads();  // s_cnt / s_base are rewritten by the next iteration
    }
}

constexpr int kRwReg = 16;  // rewire propagation: node rows per lane and batch of gathers
__global__ __launch_bounds__(256) void star_rewire_kernel(
    StarDev sd, SceneDev sc, const SteerTask* __restrict__ tasksC,
    const StarTaskExt* __restrict__ extC, const int* __restrict__ statusC,
    const double* __restrict__ costC, double* __restrict__ lit_scratch, int* __restrict__ err) {
    const int lane = __lane_id();
    const int gw = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
    const int nw = (int)((gridDim.x * blockDim.x) >> 6);
    const MqDev& mq = sd.mq;
    for (int q = gw; q < mq.Q; q += nw) {
        if (sd.pn[q] < 0 || sd.nnear[q] < 0) continue;
        const int slot = sd.cslot[q];
        if (slot < 0) continue;
        const int cnt = __popcll(sd.cmask[q]);
        const bool act = lane < cnt;
        SteerTask tk{};
        StarTaskExt ex{};
        int st = kReject;
        double e = __builtin_inf();
        if (act) {
            tk = tasksC[slot + lane];
            ex = extC[slot + lane];
            st = statusC[slot + lane];
            e = costC[slot + lane];
        }
        st = star_settle(sc, st, act, tk.x, tk.y, ex.cyaw, tk.px, tk.py, tk.pyaw, lit_scratch,
                         sd.lit_locks, gw);
        if (__ballot(act && st == kError)) {
            if (lane == 0) atomicOr(err, 1);
            continue;
        }
        const uint64_t fm = __ballot(act && star_feasible(st, e));
        const size_t row = (size_t)q * mq.cap;
        const int n = mq.n[q];
        const int nwn = n - 1;  // the node star_insert appended
        const double cb = sd.cb[q];
        double* __restrict__ cost = sd.cost + row;
        double* __restrict__ elen = sd.elen + row;
        int* __restrict__ par = mq.parent + row;
        int* __restrict__ mark = sd.mark + row;
        int s = sd.stamp[q];
        int64_t rw = 0;
        for (uint64_t f = fm; f; f &= f - 1) {  // X_near order
            const int i = __builtin_ctzll(f);
            const int m = __shfl(ex.node, i);
            const double em = __shfl(e, i);
            const double cn = cb + em;
            if (!(cn < cost[m])) continue;
            if (lane == 0) {
                par[m] = nwn;
                elen[m] = em;
                cost[m] = cn;
                mark[m] = s;
            }
            ++rw;
            // this wave alone reads and writes query q's rows in this kernel, so its lanes
            // exchange them through the CU's own cache: a workgroup-scope fence (the stores
            // complete) orders them, with no L2 writeback or L1 invalidation per pass
            __threadfence_block();
            // the subtree of m, level by level: a node's parent is final one pass earlier
            // (lane l holds nodes l, l + 64, ...; a pass loads kRwReg rows of parents per lane,
            // then issues all of their mark gathers at once, instead of one dependent pair per
            // 64 nodes)
            for (;;) {
                bool any = false;
                for (int j0 = 0; j0 < n; j0 += 64 * kRwReg) {
                    int pr[kRwReg], mk[kRwReg];
#pragma unroll
                    for (int r = 0; r < kRwReg; ++r) {
                        const int j = j0 + lane + 64 * r;
                        pr[r] = j < n ? par[j] : -1;
                    }
#pragma unroll
                    for (int r = 0; r < kRwReg; ++r) mk[r] = pr[r] >= 0 ? mark[pr[r]] : 0;
#pragma unroll
                    for (int r = 0; r < kRwReg; ++r) {
                        if (pr[r] >= 0 && mk[r] == s) {
                            const int j = j0 + lane + 64 * r;
                            cost[j] = cost[pr[r]] + elen[j];
                            mark[j] = s + 1;
                            any = true;
                        }
                    }
                }
                __threadfence_block();
                ++s;
                if (!__ballot(any)) break;
            }
        }
        if (lane == 0) {
            sd.stamp[q] = s;
            sd.rewires[q] += rw;
        }
    }
}

hipError_t launch_star_steps(hipStream_t s, const StarArgs& a, int steps) {
    const int Q = a.sd.mq.Q;
    const int TB = Q * kStarKMax;  // task capacity of rounds B and C
    const int qb = std::min((Q + 3) / 4, 4096);
    const int knn_blocks = std::min((Q + kKnnWaves - 1) / kKnnWaves, 4096);
    const int lit_blocks = std::min((Q + 3) / 4, 4096);  // literal scratch: slot locks
    const int prepA = std::min((Q + kPrepThreads / 8 - 1) / (kPrepThreads / 8), 2048);
    const int prepB = std::min((TB + kPrepThreads / 8 - 1) / (kPrepThreads / 8), 2048);
    const int walkA = std::min((Q + kWalkThreads / 64 - 1) / (kWalkThreads / 64),
                               std::min(kWalkMaxWG, walk_grid_cap<kWalkMinWStar, 4, true>(a.sc)));
    const int lds = a.sc.lds_bytes;
    // a scene read from global memory (no LDS image) makes the walk latency-bound: fill every
    // wave slot the walk's 48 VGPRs allow (4 workgroups of 8 waves per CU)
    const int walk_cap = lds > 0 ? std::min(kWalkMaxWG, walk_grid_cap<kWalkMinWStar, 4, true>(a.sc)) : 1024;
    const int walkB = std::min((TB + kWalkThreads / 64 - 1) / (kWalkThreads / 64), walk_cap);
    // ev (profiling): 8 per step — around star_sample, then around each round's walk
    auto round = [&](DevState* st, int pb, int wb, const SteerTask* t, const StarTaskExt* ext,
                     int* status, double* yaw, double* cost, hipEvent_t* ev) {
        steer_prep_kernel<<<pb, kPrepThreads, 0, s>>>(st, a.sc, nullptr, nullptr, nullptr, nullptr,
                                                      a.rec, yaw, t, cost, ext);
        if (ev) (void)hipEventRecord(ev[0], s);
        // (the analytic straight segments, s_classify: config 5 21.9 -> 25.1 M it/s, same digest)
        launch_walk<kWalkMinWStar, true>(s, wb, st, a.sc, a.rec, nullptr, status, nullptr, nullptr,
                                         a.wg_points);
        if (ev) (void)hipEventRecord(ev[1], s);
    };
    for (int k = 0; k < steps; ++k) {
        hipEvent_t* ev = a.ev ? a.ev + 8 * k : nullptr;
        if (ev) (void)hipEventRecord(ev[0], s);
        star_sample_kernel<<<qb, 256, 0, s>>>(a.sd, a.sc.minx, a.sc.maxx, a.sc.miny, a.sc.maxy,
                                              a.tA);
        if (ev) (void)hipEventRecord(ev[1], s);
        round(a.sd.stA, prepA, walkA, a.tA, nullptr, a.sA, a.yA, a.cA, ev ? ev + 2 : nullptr);
        star_knn_kernel<<<knn_blocks, 64 * kKnnWaves, 0, s>>>(a.sd, a.sA, a.cA, a.tB, a.eB,
                                                              a.err);
        round(a.sd.stB, prepB, walkB, a.tB, a.eB, a.sB, a.yB, a.cB, ev ? ev + 4 : nullptr);
        star_insert_kernel<<<lit_blocks, 256, 0, s>>>(a.sd, a.sc, a.sA, a.yA, a.cA, a.tB, a.sB,
                                                      a.yB, a.cB, a.tC, a.eC, a.lit_scratch,
                                                      a.err);
        round(a.sd.stC, prepB, walkB, a.tC, a.eC, a.sC, a.yC, a.cC, ev ? ev + 6 : nullptr);
        star_rewire_kernel<<<lit_blocks, 256, 0, s>>>(a.sd, a.sc, a.tC, a.eC, a.sC, a.cC,
                                                      a.lit_scratch, a.err);
    }
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void star_init_kernel(StarDev sd) {
    const int q = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (q >= sd.mq.Q) return;
    const size_t o = (size_t)q * sd.mq.cap;
    sd.cost[o] = 0.0;
    sd.elen[o] = 0.0;
    sd.stamp[q] = 1;
    sd.rewires[q] = 0;
}

hipError_t launch_star_init(hipStream_t s, const StarArgs& a, const double* starts) {
    hipError_t e = launch_mq_init(s, a.sd.mq, starts);
    if (e != hipSuccess) return e;
    star_init_kernel<<<(a.sd.mq.Q + 255) / 256, 256, 0, s>>>(a.sd);
    return hipGetLastError();
}

// --------------------------------------------------------------------------- launch wrappers

namespace {
SamplesArgs samples_args(const WindowArgs& a) {
    SamplesArgs g;
    g.K = a.K;
    g.target = a.target;
    g.seed = a.seed;
    g.minx = a.sc.minx;
    g.maxx = a.sc.maxx;
    g.miny = a.sc.miny;
    g.maxy = a.sc.maxy;
    for (int q = 0; q < 2; ++q) {
        g.wsx[q] = a.wsx + (size_t)q * a.Kcap;
        g.wsy[q] = a.wsy + (size_t)q * a.Kcap;
        g.wsx32[q] = a.wsx32 + (size_t)q * a.Kcap;
        g.wsy32[q] = a.wsy32 + (size_t)q * a.Kcap;
        g.perm[q] = a.perm + (size_t)q * a.Kcap;
        g.cofs[q] = a.cofs + (size_t)q * 257;
        g.sxy[q] = a.sxy + (size_t)q * a.Kcap;
        g.ssx[q] = a.ssx + (size_t)q * a.Kcap;
        g.ssy[q] = a.ssy + (size_t)q * a.Kcap;
        g.ob[q] = a.ob + (size_t)q * (kMaxWindow / kQPB);
        g.sq[q] = a.sq + (size_t)q * a.Kcap;
        g.ipos[q] = a.ipos + (size_t)q * a.Kcap;
        g.blk[q] = a.blk ? a.blk + (size_t)q * a.Kcap : nullptr;
    }
    g.scp = a.scp;
    g.hsx = a.hsx;
    g.hsy = a.hsy;
    g.hs_base = a.hrec.base;
    return g;
}
PairGrid pair_grid(const SamplesArgs& g, int p, double eps_coord) {
    PairGrid r;
    r.perm = g.perm[p];
    r.cofs = g.cofs[p];
    r.sxy = g.sxy[p];
    r.ssx = g.ssx[p];
    r.ssy = g.ssy[p];
    r.minx = g.minx;
    r.miny = g.miny;
    r.fx = 16.0 / (g.maxx - g.minx);  // samples_role's factors, bit for bit
    r.fy = 16.0 / (g.maxy - g.miny);
    // f32 rounding of both samples' coordinates (and of the distance arithmetic)
    r.slack = (float)(5.0e-4 + 4.0 * eps_coord);
    return r;
}

WinKArgs win_args(const WindowArgs& a, int p, int gen, int resolve, int scan, int64_t seq) {
    WinKArgs k;
    k.st = a.st;
    k.sc = a.sc;
    k.tr = a.tr;
    k.K = a.K;
    k.Kcap = a.Kcap;
    k.nqb = (a.K + kQPB - 1) / kQPB;
    k.chunks = scan_chunks(a.K);
    k.p = p;
    k.gen = gen;
    k.resolve = resolve;
    k.scan = scan;
    k.seq = seq;
    k.target = a.target;
    k.seed = a.seed;
    k.wsx[0] = a.wsx;
    k.wsx[1] = a.wsx + a.Kcap;
    k.wsy[0] = a.wsy;
    k.wsy[1] = a.wsy + a.Kcap;
    k.wsx32[0] = a.wsx32;
    k.wsx32[1] = a.wsx32 + a.Kcap;
    k.wsy32[0] = a.wsy32;
    k.wsy32[1] = a.wsy32 + a.Kcap;
    k.perm[0] = a.perm;
    k.perm[1] = a.perm + a.Kcap;
    k.sq[0] = a.sq;
    k.sq[1] = a.sq + a.Kcap;
    k.pbest = a.pbest;
    k.psecond = a.psecond;
    k.pidx = a.pidx;
    k.nn_idx = a.nn_idx;
    k.cand_cnt = a.cand_cnt;
    k.cand = a.cand;
    k.pend = a.pend;
    k.snap_status = a.snap_status;
    k.snap_yaw = a.snap_yaw;
    k.fin_par = a.fin_par;
    k.rs = a.rs;
    k.lit_scratch = a.lit_scratch;
    k.gen_next = gen && scan;
    k.g = samples_args(a);
    k.hrec = a.hrec;
    return k;
}
}  // namespace


hipError_t launch_window(hipStream_t s, const WindowArgs& a, hipEvent_t* ev, int64_t seq,
                         int resolve_prev) {
    const int K = a.K;
    const int p = (int)(seq & 1);
    const WinKArgs wk = win_args(a, p, 1, resolve_prev, 1, seq);
    if (!resolve_prev)  // the batch's first window: its samples (later: the previous window's draw)
        window_samples_kernel<<<1, 1024, 0, s>>>(a.st, wk.g, p);
    double* wsx = a.wsx + (size_t)p * a.Kcap;
    double* wsy = a.wsy + (size_t)p * a.Kcap;
    if (ev) (void)hipEventRecord(ev[0], s);
    // (the screen's geometry is decided on the device, from the samples not in an obstacle:
    // every workgroup past it returns at once)
    window_kernel<<<1 + kScanGrid, kScanThreads, 0, s>>>(wk);
    if (resolve_prev && !kWinRepair) resolve_tail_kernel<<<1, kResolveThreads, 0, s>>>(wk);
    if (ev) (void)hipEventRecord(ev[1], s);
    // one workgroup past the samples' draws the next window's samples
    nn_finalize_kernel<<<(K + kFinSamples - 1) / kFinSamples + 1, kFinThreads, 0, s>>>(
        a.st, p, seq, wk.chunks, a.pbest, a.psecond, a.pidx, a.Kcap, wsx, wsy, a.tr.x32, a.tr.y32,
        a.tr.x, a.tr.y, a.tr.yaw, a.eps_coord, a.nn_idx, a.nn_d2, a.snap_pose,
        pair_grid(wk.g, p, a.eps_coord), a.cand_cnt, a.cand, a.pend, wk.sq[p], wk.g.ipos[p], wk.g,
        1, wk.g.blk[p]);
    if (ev) (void)hipEventRecord(ev[2], s);
    // snapshot and candidate tasks together: prep covers 2K tasks per pass, walk 4 per workgroup
    const int prep_blocks = (2 * K + kPrepThreads / 8 - 1) / (kPrepThreads / 8);
    steer_prep_kernel<<<prep_blocks, kPrepThreads, 0, s>>>(a.st, a.sc, wsx, wsy, a.snap_pose, a.cand,
                                                  a.rec, a.snap_yaw, nullptr, nullptr, nullptr,
                                                  wk.g.blk[p]);
    if (ev) (void)hipEventRecord(ev[3], s);
    // snapshot tasks plus the usual few candidate tasks in one round of waves
    const int nwg = std::min((K + K / 4 + kWalkThreads / 64 - 1) / (kWalkThreads / 64),
                             std::min(kWalkMaxWG, walk_grid_cap(a.sc)));
    launch_walk<kWalkMinWWindow>(s, nwg, a.st, a.sc, a.rec, a.cand, a.snap_status, a.cand_cnt,
                                 a.pend, a.wg_points);
    if (ev) (void)hipEventRecord(ev[4], s);
    return hipGetLastError();
}

hipError_t launch_drain(hipStream_t s, const WindowArgs& a, int64_t seq_next) {
    const WinKArgs wk = win_args(a, (int)(seq_next & 1), 1, 1, 0, seq_next);
    window_kernel<<<1, kScanThreads, 0, s>>>(wk);
    if (!kWinRepair) resolve_tail_kernel<<<1, kResolveThreads, 0, s>>>(wk);
    return hipGetLastError();
}

hipError_t launch_nearest(hipStream_t s, const WindowArgs& a) {
    const int K = a.K;
    const WinKArgs wk = win_args(a, 0, 0, 0, 1, 0);
    window_kernel<<<1 + wk.nqb * wk.chunks, kScanThreads, 0, s>>>(wk);
    nn_finalize_kernel<<<(K + kFinSamples - 1) / kFinSamples, kFinThreads, 0, s>>>(
        a.st, 0, 0, wk.chunks, a.pbest, a.psecond, a.pidx, a.Kcap, a.wsx, a.wsy, a.tr.x32,
        a.tr.y32, a.tr.x, a.tr.y, a.tr.yaw, a.eps_coord, a.nn_idx, a.nn_d2, nullptr, PairGrid{},
        nullptr, nullptr, nullptr, nullptr, nullptr, wk.g, 0, nullptr);
    return hipGetLastError();
}

// Space::verify (rrt.rs:124-137) of whole polylines, one wave per line: chunks of 63 points
// (lane 0 carries the previous chunk's last point) through the walk's chunk test — every point
// in bounds (and in a free cell, config 4), every segment clear of the discs / edge buffers; a
// one-point line is its degenerate segment.  Polygon mode: point 0 outside every obstacle
// polygon (Q10p: with no segment meeting an edge buffer the line is on one side).
__global__ __launch_bounds__(256) void verify_lines_kernel(SceneDev sc, const double* __restrict__ X,
                                                          const double* __restrict__ Y,
                                                          const int64_t* __restrict__ off, int k,
                                                          uint8_t* __restrict__ ok) {
    const int lane = __lane_id();
    const int gw = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int nw = (int)((gridDim.x * blockDim.x) >> 6);
    for (int i = gw; i < k; i += nw) {
        const int64_t a = off[i], n = off[i + 1] - a;
        bool good = true;
        if (n > 0) {
            if (n == 1) {
                const bool has = lane == 0;
                good = !chunk_rejects<false>(sc, has, has, has, X[a], Y[a]);
            } else {
                // lane l holds point c0 + l; lane 0 is the previous chunk's last point (checked)
                for (int64_t c0 = 0; c0 + 1 < n && good; c0 += 63) {
                    const int64_t j = c0 + lane;
                    const bool has = j < n;
                    const double qx = has ? X[a + j] : 0.0, qy = has ? Y[a + j] : 0.0;
                    good = !chunk_rejects<false>(sc, has, has && (lane >= 1 || c0 == 0),
                                                 has && lane >= 1, qx, qy);
                }
            }
            if (good && sc.ne > 0 &&
                in_obstacle(sc.ne, sc.ex0, sc.ey0, sc.ex1, sc.ey1, sc.epoly, X[a], Y[a]))
                good = false;
        }
        if (lane == 0) ok[i] = good ? 1 : 0;
    }
}

hipError_t launch_verify_lines(hipStream_t st, const SceneDev& sc, const double* X,
                               const double* Y, const int64_t* off, int k, uint8_t* ok) {
    if (k <= 0) return hipSuccess;
    const int waves = std::min(k, 16384);
    verify_lines_kernel<<<(waves + 3) / 4, 256, 0, st>>>(sc, X, Y, off, k, ok);
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

hipError_t launch_dubins_origin(hipStream_t st, const double* conf, int n, int cap, double* px,
                                double* py, double* pyaw, int* n_out, int* word_out,
                                double* cost_out, int* status_out) {
    if (n <= 0) return hipSuccess;
    dubins_origin_kernel<<<(n + 63) / 64, 64, 0, st>>>(conf, n, cap, px, py, pyaw, n_out, word_out,
                                                       cost_out, status_out);
    return hipGetLastError();
}

hipError_t launch_dubins_words(hipStream_t st, const double* abd, int n, double* tpq, int* ok) {
    if (n <= 0) return hipSuccess;
    dubins_words_kernel<<<(n + 63) / 64, 64, 0, st>>>(abd, n, tpq, ok);
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
