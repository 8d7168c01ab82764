// pp_kernels.h — host-side launch wrappers of the HIP kernels (pp_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "pp_types.h"

namespace ppamd {

// Nearest tree node of each of nq samples (exact f64 argmin of dx*dx+dy*dy, lowest index on ties)
// via the f32 screen + exact rescan of the flagged near-ties.  Partials need n_chunks*stride.
hipError_t launch_nn(hipStream_t st, const TreeDev& tr, const double* qx, const double* qy,
                     int nq, int stride, float* pbest, float* psecond, int* pidx, double eps_coord,
                     int* out_idx, double* out_d2, int* flag_list, int* flag_count,
                     hipEvent_t ev_scan0, hipEvent_t ev_scan1);

hipError_t launch_pairs(hipStream_t st, const double* wsx, const double* wsy, const double* nn_d2,
                        int W, int* cand_cnt, CandEntry* cand, int* ncomp);

hipError_t launch_steer_window(hipStream_t st, const SceneDev& sc, const TreeDev& tr,
                               const double* wsx, const double* wsy, const int* nn_idx,
                               const CandEntry* cand, const int* ncomp, int W, int* snap_status,
                               double* snap_yaw, int* spec_status, double* spec_yaw);

hipError_t launch_steer_tasks(hipStream_t st, const SceneDev& sc, const TreeDev& tr,
                              const SteerTask* tasks, int n, int* out_status, double* out_yaw,
                              double* scratch);

hipError_t launch_sample(hipStream_t st, uint64_t seed, int64_t it0, int W, double minx,
                         double maxx, double miny, double maxy, double* wsx, double* wsy);

hipError_t launch_append(hipStream_t st, const CommitEntry* ents, int n_new, int n0,
                         const double* wsx, const double* wsy, const int* nn_idx, float* x32,
                         float* y32, double* X, double* Y, double* YAW, int* PAR);

hipError_t launch_dubins_batch(hipStream_t st, const double* conf, int n, int cap, double* px,
                               double* py, double* pyaw, int* n_out, int* word_out,
                               double* cost_out, int* status_out);

}  // namespace ppamd
