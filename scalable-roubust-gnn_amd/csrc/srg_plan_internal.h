// srg_plan_internal.h -- library-internal entry points between the one-GPU planner (srg_plan.hip: the
// layout, its lifetime, the C-ABI over plans) and the kernels' translation unit (srg_spmm.hip: the
// launch loops).  Not part of the C-ABI (include/srgnn_hip.h).
#ifndef SRG_PLAN_INTERNAL_H_
#define SRG_PLAN_INTERNAL_H_

#include <cstdint>

#include "srgnn_hip.h"

extern "C" {

// srg_spmm.hip: thread-local srg_last_error
void srg_set_error(int code, const char* msg);

// One fp32 hop over a plan's launches (X -> Y), the aggregation epilogue on the launches agg_on marks.
int srg_run_plan_hop(const srg_hop_launch* launches, int32_t n_launch, int32_t join_hub, const float* X,
                     int64_t ldx, float* Y, int64_t ldy, int32_t d, const uint8_t* agg_on, float* agg,
                     int64_t lda, float w, int32_t agg_init, void* stream);

// Roles of a plan's launches in an fp64 Chebyshev step (srg_run_plan_cheby_f64)
#define SRG_CHEBY64_FIRST 0x1   /* the launch's rows' chains start here (block 0) */
#define SRG_CHEBY64_LAST 0x2    /* ... and end here (block 0's whole rows, the last block) */
#define SRG_CHEBY64_HUBS 0x4    /* the whole hub rows: hub workgroups on the side stream */

// One fp64 Chebyshev step (k_cheby's recurrence and epilogue) over a plan's launches with their roles;
// `values` are fp64 values at the plan's entry positions (a SRG_PLAN_SPANS plan over the caller's arrays).
int srg_run_plan_cheby_f64(const srg_hop_launch* launches, const uint8_t* roles, int32_t n_launch,
                           const int64_t* indptr, const int32_t* indices, const double* values, const double* Tc,
                           const double* To, double* Tn, int64_t ld, int32_t d, int mode, double a1, double a2,
                           const double* coef_prev, const double* coef, int32_t n_scales, double* R,
                           int64_t r_stride, void* stream);

}  // extern "C"

#endif  // SRG_PLAN_INTERNAL_H_
