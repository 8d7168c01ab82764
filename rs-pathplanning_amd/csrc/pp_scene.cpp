// pp_scene.cpp — host-side scene building (see pp_scene.h).  No HIP: the library uploads what
// these functions return; tests/sanitize/ runs them under ASan/UBSan on the CPU.
#include "pp_scene.h"

#include <algorithm>
#include <cmath>
#include <cstring>

#include "../../include/pathplanning_amd.h"

namespace ppamd {
namespace scene {

namespace {
int fail(std::string* err, int code, const char* msg) {
    if (err) *err = msg;
    return code;
}

void push_item(Items& it, double bx0, double bx1, double by0, double by1, CullDisc d) {
    it.bx0.push_back(bx0);
    it.bx1.push_back(bx1);
    it.by0.push_back(by0);
    it.by1.push_back(by1);
    it.d4.push_back(d);
}

// a ring's vertices without a closing repeat of the first one (geo closes rings itself)
void ring(const double* xy, int n, std::vector<double>& vx, std::vector<double>& vy) {
    if (n > 1 && xy[0] == xy[2 * (n - 1)] && xy[1] == xy[2 * (n - 1) + 1]) --n;
    vx.resize((size_t)std::max(n, 0));
    vy.resize((size_t)std::max(n, 0));
    for (int i = 0; i < n; ++i) {
        vx[i] = xy[2 * i];
        vy[i] = xy[2 * i + 1];
    }
}
}  // namespace

float cull_slack_for(double mx) {
    // the rounding of coordinates of magnitude <= mx to f32 (both ends of a difference, both
    // axes) with a wide margin; never below the 1e-3 that covers |c| <= 2^10
    return (float)std::max(1.0e-3, 16.0 * mx * std::ldexp(1.0, -24));
}

int disc_scene(double x0, double y0, double x1, double y1, double robot_width, const double* cx,
               const double* cy, const double* r, int m, DiscScene* out, std::string* err) {
    if (m < 0 || (m > 0 && (!cx || !cy || !r)))
        return fail(err, PP_ERR_INVALID_ARGUMENT, "bad obstacle arrays");
    // Space::new, rrt.rs:82-111: bounds offset by -width/2, obstacles by +width/2
    const double half = robot_width / 2.0;
    DiscScene& s = *out;
    s.minx = x0 + half;
    s.maxx = x1 - half;
    s.miny = y0 + half;
    s.maxy = y1 - half;
    if (!(s.minx < s.maxx) || !(s.miny < s.maxy))  // gen_range asserts low < high (rrt.rs:142-143)
        return fail(err, PP_ERR_INVALID_ARGUMENT, "shrunken bounds are empty");
    s.r2.resize((size_t)m);
    s.rcull.resize((size_t)m);
    s.items = Items{};
    double mx = std::max({std::fabs(s.minx), std::fabs(s.maxx), std::fabs(s.miny), std::fabs(s.maxy)});
    for (int k = 0; k < m; ++k) {
        if (!std::isfinite(cx[k]) || !std::isfinite(cy[k]) || !std::isfinite(r[k]))
            return fail(err, PP_ERR_INVALID_ARGUMENT, "non-finite obstacle disc");
        const double reff = r[k] + half;
        const double rc = reff * (1.0 + 1e-9) + 1e-9;
        s.r2[k] = reff * reff;
        s.rcull[k] = rc;
        // f32 cull copy: the radius rounded up (the cull only ever over-includes); w is the
        // radius for the walk's f32 decision band
        push_item(s.items, cx[k] - rc, cx[k] + rc, cy[k] - rc, cy[k] + rc,
                  CullDisc{(float)cx[k], (float)cy[k], std::nextafter((float)rc, 1e30f), (float)reff});
        mx = std::max({mx, std::fabs(cx[k]) + rc, std::fabs(cy[k]) + rc});
    }
    s.items.mx = mx;
    return 0;
}

int polygon_scene(const double* bounds_xy, int nb, const double* obs_xy, const int32_t* obs_off,
                  int n_obs, double robot_width, PolygonScene* out, std::string* err) {
    if (!bounds_xy || nb < 3 || n_obs < 0 || (n_obs > 0 && (!obs_xy || !obs_off)))
        return fail(err, PP_ERR_INVALID_ARGUMENT, "bad polygon arrays (bounds need >= 3 vertices)");
    PolygonScene& s = *out;
    ring(bounds_xy, nb, s.bvx, s.bvy);
    if (s.bvx.size() < 3) return fail(err, PP_ERR_INVALID_ARGUMENT, "bounds ring has < 3 vertices");
    for (size_t i = 0; i < s.bvx.size(); ++i)
        if (!std::isfinite(s.bvx[i]) || !std::isfinite(s.bvy[i]))
            return fail(err, PP_ERR_INVALID_ARGUMENT, "non-finite bounds vertex");
    // Space::new, rrt.rs:82-106: rand_point samples the bbox of the shrunken bounds — here the
    // bounds' bbox shrunk by width/2, which contains the eroded polygon (Q10p)
    const double half = robot_width / 2.0;
    s.minx = *std::min_element(s.bvx.begin(), s.bvx.end()) + half;
    s.maxx = *std::max_element(s.bvx.begin(), s.bvx.end()) - half;
    s.miny = *std::min_element(s.bvy.begin(), s.bvy.end()) + half;
    s.maxy = *std::max_element(s.bvy.begin(), s.bvy.end()) - half;
    if (!(s.minx < s.maxx) || !(s.miny < s.maxy))
        return fail(err, PP_ERR_INVALID_ARGUMENT, "shrunken bounds are empty");
    double mx = 0.0;
    for (size_t i = 0; i < s.bvx.size(); ++i) mx = std::max({mx, std::fabs(s.bvx[i]), std::fabs(s.bvy[i])});
    // obstacle edges (rrt.rs:108-111: every obstacle buffered by width/2)
    s.ex0.clear();
    s.ey0.clear();
    s.ex1.clear();
    s.ey1.clear();
    s.epoly.clear();
    s.items = Items{};
    const double rcull = half * (1.0 + 1e-9) + 1e-9;
    std::vector<double> vx, vy;
    for (int o = 0; o < n_obs; ++o) {
        const int a = obs_off[o], b = obs_off[o + 1];
        if (a < 0 || b < a) return fail(err, PP_ERR_INVALID_ARGUMENT, "bad obstacle offsets");
        ring(obs_xy + 2 * (size_t)a, b - a, vx, vy);
        const int n = (int)vx.size();
        for (int i = 0; i < n; ++i) {
            if (!std::isfinite(vx[i]) || !std::isfinite(vy[i]))
                return fail(err, PP_ERR_INVALID_ARGUMENT, "non-finite obstacle vertex");
            const int j = i + 1 == n ? 0 : i + 1;
            s.ex0.push_back(vx[i]);
            s.ey0.push_back(vy[i]);
            s.ex1.push_back(vx[j]);
            s.ey1.push_back(vy[j]);
            s.epoly.push_back(o);
            // f32 cull disc: the midpoint, half the length + h, rounded up generously
            const double hl = 0.5 * std::hypot(vx[j] - vx[i], vy[j] - vy[i]);
            const double rr = (hl + rcull) * (1.0 + 1e-7) + 1e-9;
            push_item(s.items, std::min(vx[i], vx[j]) - rcull, std::max(vx[i], vx[j]) + rcull,
                      std::min(vy[i], vy[j]) - rcull, std::max(vy[i], vy[j]) + rcull,
                      CullDisc{(float)(0.5 * (vx[i] + vx[j])), (float)(0.5 * (vy[i] + vy[j])),
                               std::nextafter((float)rr, 1e30f), 0.0f});
            mx = std::max({mx, std::fabs(vx[i]), std::fabs(vy[i])});
        }
    }
    s.items.mx = mx + half;
    return 0;
}

ItemGrid build_item_grid(double minx, double maxx, double miny, double maxy, const Items& items,
                         int part_budget) {
    // square cells, about one cell per item; a scene whose LDS image [goff | items | d4] does not
    // fit gets the image without the cull discs (read from global memory), at a coarser grid if
    // that is what it takes
    part_budget = std::max(0, std::min(part_budget, kLdsImage));
    const int m = (int)items.d4.size();
    const double spanx = maxx - minx, spany = maxy - miny;
    const double span = std::max(spanx, spany);
    auto al = [](size_t b) { return (int)((b + 15) & ~(size_t)15); };
    ItemGrid g;
    g.x0 = minx;
    g.y0 = miny;
    const int per0 = std::max(1, std::min(256, (int)std::ceil(std::sqrt((double)std::max(m, 1)))));
    std::vector<int> count;
    for (int per_axis = per0;; per_axis = per_axis * 3 / 4) {
        const double cell = span / per_axis;
        g.gnx = std::max(1, std::min(256, (int)std::ceil(spanx / cell)));
        g.gny = std::max(1, std::min(256, (int)std::ceil(spany / cell)));
        g.ginv = 1.0 / cell;
        auto cell_of = [&](double v, double v0, int n) {
            const double f = std::floor((v - v0) * g.ginv);
            return f < 0.0 ? 0 : (f >= (double)(n - 1) ? n - 1 : (int)f);
        };
        // two passes (count, then fill) over the items' cell ranges
        const size_t cells = (size_t)g.gnx * g.gny;
        count.assign(cells, 0);
        for (int pass = 0; pass < 2; ++pass) {
            if (pass == 1) {
                g.goff.assign(cells + 1, 0);
                for (size_t q = 0; q < cells; ++q) g.goff[q + 1] = g.goff[q] + count[q];
                g.gitems.assign((size_t)g.goff[cells], 0);
                std::fill(count.begin(), count.end(), 0);
            }
            for (int k = 0; k < m; ++k) {
                const int x0c = cell_of(items.bx0[k], minx, g.gnx), x1c = cell_of(items.bx1[k], minx, g.gnx);
                const int y0c = cell_of(items.by0[k], miny, g.gny), y1c = cell_of(items.by1[k], miny, g.gny);
                for (int gy = y0c; gy <= y1c; ++gy)
                    for (int gx = x0c; gx <= x1c; ++gx) {
                        const size_t q = (size_t)gy * g.gnx + gx;
                        if (pass == 1) g.gitems[(size_t)g.goff[q] + count[q]] = k;
                        ++count[q];
                    }
            }
        }
        g.o_goff = 0;
        g.o_items = g.o_goff + al(g.goff.size() * sizeof(int));
        const int grid_bytes = g.o_items + al(g.gitems.size() * sizeof(int));
        const int full = grid_bytes + al((size_t)m * sizeof(CullDisc));
        if (full <= kLdsImage) {  // everything in LDS
            g.lds_total = full;
            g.o_d4 = grid_bytes;
            break;
        }
        if (grid_bytes <= part_budget && m > 4096) {  // the grid in LDS, the cull discs in L2
            g.lds_total = grid_bytes;
            g.o_d4 = -1;
            break;
        }
        if (per_axis <= 8 || m <= 4096) {  // no LDS image: the walk reads the scene from L2
            g.lds_total = 0;
            g.o_d4 = -1;
            break;
        }
    }
    if (g.lds_total > 0) {  // the image, contiguous in global memory (stage_scene copies it whole)
        g.image.assign((size_t)g.lds_total, 0);
        std::memcpy(g.image.data() + g.o_goff, g.goff.data(), g.goff.size() * sizeof(int));
        if (!g.gitems.empty())
            std::memcpy(g.image.data() + g.o_items, g.gitems.data(), g.gitems.size() * sizeof(int));
        if (g.o_d4 >= 0 && m > 0)
            std::memcpy(g.image.data() + g.o_d4, items.d4.data(), (size_t)m * sizeof(CullDisc));
    }
    return g;
}

InsideBits inside_bitmap(double minx, double maxx, double miny, double maxy, const double* cx,
                         const double* cy, const std::vector<double>& r2, int n) {
    InsideBits ib;
    const int m = (int)r2.size();
    if (n <= 0 || (n & 31) || m == 0 || !(maxx > minx) || !(maxy > miny)) return ib;
    const double span = std::max(maxx - minx, maxy - miny);
    const double cell = span / n;
    ib.n = n;
    ib.x0 = minx;
    ib.y0 = miny;
    ib.inv = 1.0 / cell;
    const int words = n / 32;
    ib.bits.assign((size_t)n * words, 0u);
    // a point maps to cell floor((v - v0) * inv): the corners are widened by a margin far above
    // that rounding, so every point the device maps into the cell lies in the tested square
    const double eps = 1e-6 * cell + 1e-9 * (std::fabs(minx) + std::fabs(miny) + span);
    for (int k = 0; k < m; ++k) {
        const double r = std::sqrt(r2[k]);
        const int i0 = std::max(0, (int)std::floor((cx[k] - r - minx) / cell));
        const int i1 = std::min(n - 1, (int)std::floor((cx[k] + r - minx) / cell));
        const int j0 = std::max(0, (int)std::floor((cy[k] - r - miny) / cell));
        const int j1 = std::min(n - 1, (int)std::floor((cy[k] + r - miny) / cell));
        const double lim = r2[k] * (1.0 - 1e-9);
        for (int j = j0; j <= j1; ++j) {
            const double ya = miny + j * cell - eps - cy[k], yb = miny + (j + 1) * cell + eps - cy[k];
            const double dy2 = std::max(ya * ya, yb * yb);
            for (int i = i0; i <= i1; ++i) {
                const double xa = minx + i * cell - eps - cx[k], xb = minx + (i + 1) * cell + eps - cx[k];
                const double dx2 = std::max(xa * xa, xb * xb);
                if (dx2 + dy2 < lim) ib.bits[(size_t)j * words + (i >> 5)] |= 1u << (i & 31);
            }
        }
    }
    return ib;
}

}  // namespace scene
}  // namespace ppamd
