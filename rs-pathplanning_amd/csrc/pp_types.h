// pp_types.h — POD types shared by the host planner and the HIP kernels.
#pragma once

#include <stdint.h>

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

// Window-level constants.
constexpr int kCandCap = 16;        // in-window nearer-sample list per sample
constexpr int kSlots = 1 + kCandCap;  // steer slots per sample: snapshot parent + candidates
constexpr int kMaxChunks = 64;      // node chunks of the NN scan (partials per query)
constexpr int kLiteralCap = 16384;  // points per literal-path scratch buffer
constexpr int kLiteralWaves = 256;  // concurrent literal-path waves (scratch buffers)

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
};

// Tree in device memory: f32 SoA for the NN screen, f64 SoA for everything exact.
struct TreeDev {
    const float* x32;
    const float* y32;
    const double* x;
    const double* y;
    const double* yaw;
    int n;
};

// An explicit steer task: child (x, y) steered toward its parent — tree node `pnode` when
// pnode >= 0, else the explicit pose (px, py, pyaw).
struct SteerTask {
    double x, y, px, py, pyaw;
    int pnode;
    int literal;  // 1 = take the literal (single-lane) path
};

// A window sample i < j that is strictly nearer to sample j than j's snapshot NN.
struct CandEntry {
    int j, i;
    double d2;
};

// An accepted window sample to append: parent = tree node `parent`, or nn_idx[j] when -1.
struct CommitEntry {
    int j, parent;
    double yaw;
};

}  // namespace ppamd
