// TEST INFRASTRUCTURE ONLY: the CPU sanitizer driver (tests/test_sanitize.py builds it with
// -fsanitize=address,undefined).  It exercises the two host-side C/C++ parts that never run on
// the GPU:
//   * the library's scene building (rs-pathplanning_amd/csrc/pp_scene.cpp: Space::new's shrunken
//     bounds and buffered obstacles, rrt.rs:81-122, the item grid CSR and its LDS image), checked
//     against a brute-force recount of every item's cells;
//   * the C oracle (oracle/pp_oracle.c): extend with and without the full re-verify, check_finish,
//     plan, RRT*, the threaded query pool, on the same scenes.
// Input: the scene file tests/test_sanitize.py writes.  Output: one JSON object per scene, which
// the test compares with the unsanitized oracle (oracle/liboracle.so) run in-process.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../rs-pathplanning_amd/csrc/pp_scene.h"

// mirrors of oracle/pp_oracle.c's structs (as oracle/oracle.py mirrors them in ctypes)
extern "C" {
struct orc_scene {
    double minx, maxx, miny, maxy;
    int m;
    const double* cx;
    const double* cy;
    const double* r2;
    double turn_radius, step_size;
    const uint32_t* bits;
    int bw, bh, bwords;
    double bx0, by0, binv;
    int nbv;
    const double* bvx;
    const double* bvy;
    int ne;
    const double *ex0, *ey0, *ex1, *ey1;
    const int* epoly;
    double h2;
};
struct orc_tree {
    double* x;
    double* y;
    double* yaw;
    int32_t* parent;
    int cap, n;
};
int64_t orc_rrt_extend(const orc_scene*, orc_tree*, uint64_t, int64_t, int64_t, int, int32_t*,
                       int8_t*);
int orc_check_finish(const orc_scene*, const orc_tree*, int, double, double, double, int, double*,
                     double*, int, int*, double*, int*, int*);
int64_t orc_plan(const orc_scene*, orc_tree*, uint64_t, int64_t, int64_t, double, double, double,
                 int, int*, double*, int32_t*);
int64_t orc_queries(const orc_scene*, const double*, const uint64_t*, int, int64_t, int, int);
int64_t orc_star_extend(const orc_scene*, orc_tree*, double*, double*, uint64_t, int64_t, int64_t,
                        int, double, int64_t*, int32_t*, int8_t*);
int64_t orc_star_queries(const orc_scene*, const double*, const uint64_t*, int, int64_t, int,
                         double, int, int64_t*);
}

namespace sc = ppamd::scene;

static void die(const char* what) {
    std::fprintf(stderr, "san_driver: %s\n", what);
    std::exit(2);
}

struct Reader {
    FILE* f;
    double d() {
        double v;
        if (std::fscanf(f, "%lf", &v) != 1) die("short input");
        return v;
    }
    long long i() {
        long long v;
        if (std::fscanf(f, "%lld", &v) != 1) die("short input");
        return v;
    }
    std::string s() {
        char buf[128];
        if (std::fscanf(f, "%127s", buf) != 1) return std::string();
        return buf;
    }
};

// brute-force recount of the CSR: item k must be listed exactly once in every cell of its
// clamped cull-box range and nowhere else; the LDS image must hold the same words
static long check_grid(const sc::ItemGrid& g, const sc::Items& it) {
    const size_t cells = (size_t)g.gnx * g.gny;
    if (g.goff.size() != cells + 1 || g.goff[0] != 0) die("goff shape");
    for (size_t q = 0; q < cells; ++q)
        if (g.goff[q + 1] < g.goff[q]) die("goff not monotone");
    if ((size_t)g.goff[cells] != g.gitems.size()) die("gitems size");
    auto cell_of = [&](double v, double v0, int n) {
        const double f = std::floor((v - v0) * g.ginv);
        return f < 0.0 ? 0 : (f >= (double)(n - 1) ? n - 1 : (int)f);
    };
    std::vector<int> seen(it.d4.size(), 0);
    long expect = 0;
    for (size_t k = 0; k < it.d4.size(); ++k) {
        const int x0 = cell_of(it.bx0[k], g.x0, g.gnx), x1 = cell_of(it.bx1[k], g.x0, g.gnx);
        const int y0 = cell_of(it.by0[k], g.y0, g.gny), y1 = cell_of(it.by1[k], g.y0, g.gny);
        expect += (long)(x1 - x0 + 1) * (y1 - y0 + 1);
        for (int gy = y0; gy <= y1; ++gy)
            for (int gx = x0; gx <= x1; ++gx) {
                const size_t q = (size_t)gy * g.gnx + gx;
                int hits = 0;
                for (int e = g.goff[q]; e < g.goff[q + 1]; ++e) hits += g.gitems[e] == (int)k;
                if (hits != 1) die("item not listed exactly once in a covered cell");
            }
    }
    if (expect != (long)g.gitems.size()) die("extra grid entries");
    for (size_t q = 0; q < cells; ++q)
        for (int e = g.goff[q] + 1; e < g.goff[q + 1]; ++e)
            if (g.gitems[e] <= g.gitems[e - 1]) die("cell list not ascending");
    if (g.lds_total > 0) {
        if ((int)g.image.size() != g.lds_total || g.lds_total > sc::kLdsImage) die("image size");
        if (std::memcmp(g.image.data() + g.o_goff, g.goff.data(), g.goff.size() * 4)) die("image goff");
        if (!g.gitems.empty() &&
            std::memcmp(g.image.data() + g.o_items, g.gitems.data(), g.gitems.size() * 4))
            die("image items");
        if (g.o_d4 >= 0 && !it.d4.empty() &&
            std::memcmp(g.image.data() + g.o_d4, it.d4.data(), it.d4.size() * sizeof(sc::CullDisc)))
            die("image discs");
    }
    return expect;
}

struct TreeBuf {
    std::vector<double> x, y, yaw, cost, elen;
    std::vector<int32_t> parent;
    orc_tree t;
    TreeBuf(double sx, double sy, double syaw, int cap)
        : x(cap), y(cap), yaw(cap), cost(cap), elen(cap), parent(cap, -1) {
        x[0] = sx;
        y[0] = sy;
        yaw[0] = syaw;
        t = orc_tree{x.data(), y.data(), yaw.data(), parent.data(), cap, 1};
    }
};

static void print_tree(const char* key, const TreeBuf& b) {
    long long psum = 0;
    for (int i = 0; i < b.t.n; ++i) psum += b.parent[i];
    const int l = b.t.n - 1;
    std::printf("\"%s\": [%d, %lld, %.17g, %.17g, %.17g], ", key, b.t.n, psum, b.x[l], b.y[l], b.yaw[l]);
}

int main(int argc, char** argv) {
    if (argc != 2) die("usage: san_driver SCENES");
    Reader in{std::fopen(argv[1], "r")};
    if (!in.f) die("cannot open input");
    std::printf("[");
    bool first = true;
    for (std::string tag = in.s(); !tag.empty(); tag = in.s()) {
        if (tag != "scene") die("expected 'scene'");
        const std::string name = in.s(), kind = in.s();
        sc::DiscScene ds;
        sc::PolygonScene ps;
        std::string err;
        int rc = 0;
        double width, turn, step;
        std::vector<double> c3, bxy, oxy;
        std::vector<int32_t> off;
        if (kind == "discs") {
            const double x0 = in.d(), y0 = in.d(), x1 = in.d(), y1 = in.d();
            width = in.d();
            turn = in.d();
            step = in.d();
            const int m = (int)in.i();
            c3.resize((size_t)m * 3);
            for (auto& v : c3) v = in.d();
            std::vector<double> cx(m), cy(m), r(m);
            for (int k = 0; k < m; ++k) {
                cx[k] = c3[3 * k];
                cy[k] = c3[3 * k + 1];
                r[k] = c3[3 * k + 2];
            }
            rc = sc::disc_scene(x0, y0, x1, y1, width, cx.data(), cy.data(), r.data(), m, &ds, &err);
        } else if (kind == "polygons") {
            width = in.d();
            turn = in.d();
            step = in.d();
            const int nb = (int)in.i();
            bxy.resize((size_t)nb * 2);
            for (auto& v : bxy) v = in.d();
            const int n_obs = (int)in.i();
            off.resize((size_t)n_obs + 1);
            for (auto& v : off) v = (int32_t)in.i();
            const int nv = (int)in.i();
            oxy.resize((size_t)std::max(nv, 0) * 2);
            for (auto& v : oxy) v = in.d();
            rc = sc::polygon_scene(bxy.data(), nb, oxy.data(), off.data(), n_obs, width, &ps, &err);
        } else {
            die("unknown scene kind");
        }
        const double sx = in.d(), sy = in.d(), syaw = in.d(), gx = in.d(), gy = in.d(), gyaw = in.d();
        const long long seed = in.i(), iters = in.i();
        std::printf("%s{\"name\": \"%s\", \"rc\": %d", first ? "" : ", ", name.c_str(), rc);
        first = false;
        if (rc) {
            std::printf(", \"err\": \"%s\"}", err.c_str());
            continue;
        }
        const bool poly = kind == "polygons";
        const sc::Items& items = poly ? ps.items : ds.items;
        const double minx = poly ? ps.minx : ds.minx, maxx = poly ? ps.maxx : ds.maxx;
        const double miny = poly ? ps.miny : ds.miny, maxy = poly ? ps.maxy : ds.maxy;
        std::printf(", \"box\": [%.17g, %.17g, %.17g, %.17g], \"grids\": [", minx, maxx, miny, maxy);
        const int budgets[] = {sc::kLdsImage, 16 * 1024, 0, 1 << 30, -5};
        for (int b = 0; b < 5; ++b) {
            const sc::ItemGrid g = sc::build_item_grid(minx, maxx, miny, maxy, items, budgets[b]);
            const long entries = check_grid(g, items);
            std::printf("%s[%d, %d, %ld, %d, %d]", b ? ", " : "", g.gnx, g.gny, entries, g.lds_total, g.o_d4);
        }
        std::printf("], \"cull_slack\": %.9g, ", (double)sc::cull_slack_for(items.mx));
        if (!poly) {  // the inside bitmap: every point a set cell maps to is inside some disc
            const int m = (int)ds.r2.size();
            std::vector<double> bx(m), by(m);
            for (int k = 0; k < m; ++k) {
                bx[k] = c3[3 * k];
                by[k] = c3[3 * k + 1];
            }
            const sc::InsideBits ib = sc::inside_bitmap(minx, maxx, miny, maxy, bx.data(), by.data(), ds.r2, 256);
            long set = 0, bad = 0;
            for (int j = 0; j < ib.n; ++j)
                for (int i = 0; i < ib.n; ++i) {
                    if (!((ib.bits[(size_t)j * (ib.n / 32) + (i >> 5)] >> (i & 31)) & 1u)) continue;
                    ++set;
                    for (int u = 0; u <= 4; ++u)
                        for (int v = 0; v <= 4; ++v) {
                            // points across the cell, its edges pushed to the last double that
                            // still maps into it (the device's floor((x - x0) * inv))
                            double x = ib.x0 + (i + u / 4.0) / ib.inv, y = ib.y0 + (j + v / 4.0) / ib.inv;
                            while (std::floor((x - ib.x0) * ib.inv) > i) x = std::nextafter(x, -1e300);
                            while (std::floor((x - ib.x0) * ib.inv) < i) x = std::nextafter(x, 1e300);
                            while (std::floor((y - ib.y0) * ib.inv) > j) y = std::nextafter(y, -1e300);
                            while (std::floor((y - ib.y0) * ib.inv) < j) y = std::nextafter(y, 1e300);
                            bool in = false;
                            for (int k = 0; k < m && !in; ++k) {
                                const double dx = x - bx[k], dy = y - by[k];
                                in = dx * dx + dy * dy < ds.r2[k] * (1.0 - 1e-9);
                            }
                            bad += !in;
                        }
                }
            std::printf("\"inside\": [%ld, %ld], ", set, bad);
        }
        // the oracle on the same scene
        std::vector<double> cx, cy;
        orc_scene o{};
        o.minx = minx;
        o.maxx = maxx;
        o.miny = miny;
        o.maxy = maxy;
        o.turn_radius = turn;
        o.step_size = step;
        if (poly) {
            o.nbv = (int)ps.bvx.size();
            o.bvx = ps.bvx.data();
            o.bvy = ps.bvy.data();
            o.ne = (int)ps.ex0.size();
            o.ex0 = ps.ex0.data();
            o.ey0 = ps.ey0.data();
            o.ex1 = ps.ex1.data();
            o.ey1 = ps.ey1.data();
            o.epoly = ps.epoly.data();
            o.h2 = (width / 2.0) * (width / 2.0);
        } else {
            const int m = (int)ds.r2.size();
            cx.resize(m);
            cy.resize(m);
            for (int k = 0; k < m; ++k) {
                cx[k] = c3[3 * k];
                cy[k] = c3[3 * k + 1];
            }
            o.m = m;
            o.cx = cx.data();
            o.cy = cy.data();
            o.r2 = ds.r2.data();
        }
        const int cap = (int)iters + 2;
        TreeBuf a(sx, sy, syaw, cap), b(sx, sy, syaw, cap);
        std::vector<int32_t> lnn(iters);
        std::vector<int8_t> lacc(iters);
        const int64_t acc_a = orc_rrt_extend(&o, &a.t, (uint64_t)seed, 0, iters, 0, lnn.data(), lacc.data());
        const int64_t acc_b = orc_rrt_extend(&o, &b.t, (uint64_t)seed, 0, iters, 1, nullptr, nullptr);
        std::printf("\"extend\": [%lld, %lld], ", (long long)acc_a, (long long)acc_b);
        print_tree("tree", a);
        // check_finish on a few nodes, with the line copied out
        std::printf("\"finish\": [");
        std::vector<double> lx(1 << 16), ly(1 << 16);
        for (int j = 0; j < 4; ++j) {
            const int node = a.t.n > 1 ? (int)((long long)(a.t.n - 1) * j / 3) : 0;
            int n = 0, chain[16], nch = 0;
            double len = 0.0;
            const int r = orc_check_finish(&o, &a.t, node, gx, gy, gyaw, 0, lx.data(), ly.data(),
                                           (int)lx.size(), &n, &len, chain, &nch);
            std::printf("%s[%d, %d, %d, %.17g, %d]", j ? ", " : "", node, r, n, r == 1 ? len : 0.0, nch);
        }
        int best = -1;
        double blen = 0.0;
        TreeBuf p(sx, sy, syaw, cap);
        std::vector<int32_t> flog(iters);
        const int64_t pr = orc_plan(&o, &p.t, (uint64_t)seed, 0, iters, gx, gy, gyaw, 0, &best, &blen, flog.data());
        std::printf("], \"plan\": [%lld, %d, %.17g], ", (long long)pr, best, best >= 0 ? blen : -1.0);
        TreeBuf s(sx, sy, syaw, cap);
        int64_t rew = 0;
        const int64_t sacc = orc_star_extend(&o, &s.t, s.cost.data(), s.elen.data(), (uint64_t)seed,
                                             0, iters, 0, 0.0, &rew, nullptr, nullptr);
        std::printf("\"star\": [%lld, %lld], ", (long long)sacc, (long long)rew);
        print_tree("star_tree", s);
        // the threaded pools (4 queries on 2 threads)
        double starts[12];
        uint64_t seeds[4];
        for (int q = 0; q < 4; ++q) {
            starts[3 * q] = sx;
            starts[3 * q + 1] = sy;
            starts[3 * q + 2] = syaw;
            seeds[q] = (uint64_t)seed + 1000u * (uint64_t)q;
        }
        const int64_t qa = orc_queries(&o, starts, seeds, 4, iters / 4, 0, 2);
        int64_t qrw = 0;
        const int64_t qs = orc_star_queries(&o, starts, seeds, 4, iters / 4, 0, 0.0, 2, &qrw);
        std::printf("\"queries\": [%lld, %lld, %lld]}", (long long)qa, (long long)qs, (long long)qrw);
    }
    std::printf("]\n");
    std::fclose(in.f);
    return 0;
}
