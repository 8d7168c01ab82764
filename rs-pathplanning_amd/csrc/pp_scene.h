// pp_scene.h — host-side scene building of the C ABI (pp_space_new, pp_space_new_polygons):
// Space::new's shrunken bounds and buffered obstacles (rrt.rs:81-122) turned into the device
// layout — the collision items (discs, or polygon edges in polygon mode), their cull boxes and
// f32 cull discs, and the uniform item grid (CSR) with its LDS image.  Plain C++ with no HIP
// dependency, so the same code is compiled into the library and, with -fsanitize=address,undefined,
// into the CPU sanitizer driver (tests/sanitize/).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace ppamd {
namespace scene {

// f32 cull disc of one collision item, layout-identical to HIP's float4 (x, y, r, w)
struct CullDisc {
    float x, y, r, w;
};

// the items of a scene: the closed cull box of item k is [bx0, bx1] x [by0, by1]
struct Items {
    std::vector<double> bx0, bx1, by0, by1;
    std::vector<CullDisc> d4;
    double mx = 0.0;  // largest coordinate magnitude reached (f32 cull slack)
};

// disc mode (rrt.rs:108-111 with create_circle discs): radii grown by half = width/2
struct DiscScene {
    double minx, maxx, miny, maxy;
    std::vector<double> r2, rcull;  // (r + half)^2 and the cull radius (rounded up)
    Items items;
};

// polygon mode (Q10p): rings without the closing repeat, obstacle edges with their polygon id
struct PolygonScene {
    double minx, maxx, miny, maxy;
    std::vector<double> bvx, bvy;
    std::vector<double> ex0, ey0, ex1, ey1;
    std::vector<int> epoly;
    Items items;
};

// the uniform item grid: cell (gx, gy) lists items gitems[goff[c] .. goff[c+1]) with
// c = gy * gnx + gx; cells cover the sampling box from (x0, y0) at 1/ginv per cell.
// LDS image layout [goff | items | d4] at byte offsets o_goff, o_items, o_d4 (-1: the cull discs
// stay in global memory), lds_total bytes (0: no image, the walk reads the scene from L2).
struct ItemGrid {
    std::vector<int> goff, gitems;
    int gnx = 1, gny = 1;
    double x0 = 0.0, y0 = 0.0, ginv = 1.0;
    int lds_total = 0, o_goff = 0, o_items = 0, o_d4 = -1;
    std::vector<char> image;  // lds_total bytes
};

constexpr int kLdsImage = 64 * 1024;  // 2 workgroups per CU fit in 160 KB

// Each returns 0 or a PP_ERR_* code with *err set.
int disc_scene(double x0, double y0, double x1, double y1, double robot_width, const double* cx,
               const double* cy, const double* r, int m, DiscScene* out, std::string* err);
int polygon_scene(const double* bounds_xy, int nb, const double* obs_xy, const int32_t* obs_off,
                  int n_obs, double robot_width, PolygonScene* out, std::string* err);
// part_budget: the LDS budget for a grid-only image (bytes, clamped to kLdsImage)
ItemGrid build_item_grid(double minx, double maxx, double miny, double maxy, const Items& items,
                         int part_budget);
// f32 cull slack for coordinates of magnitude <= mx
float cull_slack_for(double mx);

// The cells of an n x n grid over the sampling box (square cells of the larger span, from
// (minx, miny), 1 / inv per cell) that lie wholly inside an inflated disc — every corner,
// widened by a rounding margin, at d2 < r2 (1 - 1e-9): bit i % 32 of word j * (n / 32) + i / 32
// for cell (i, j).  A sample in such a cell is inside the disc (convexity), so its line is
// rejected whatever its parent (point_blocked); cells the boundary crosses stay clear.
struct InsideBits {
    std::vector<uint32_t> bits;
    int n = 0;
    double x0 = 0.0, y0 = 0.0, inv = 1.0;
};
InsideBits inside_bitmap(double minx, double maxx, double miny, double maxy, const double* cx,
                         const double* cy, const std::vector<double>& r2, int n);

}  // namespace scene
}  // namespace ppamd
