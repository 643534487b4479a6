// One kernel per translation unit, selected at build time (pntf/build.py):
//   -DPNTF_KIND=0..4 -DPNTF_DIM=3|6   field_kernel<DIM, KIND>
//   -DPNTF_KIND=0..4 -DPNTF_DIM=3|6 -DPNTF_SPLIT_FIELD   field_split_kernel<DIM, KIND>
//   -DPNTF_KIND=0..4 -DPNTF_DIM=3|6 -DPNTF_WIDE_FIELD    wide_field_kernel<DIM, KIND> (pntf_wide.h)
//   -DPNTF_PLAN -DPNTF_DIM=3|6         plan_kernel<DIM>
//   -DPNTF_PLAN_SPLIT -DPNTF_DIM=3|6   plan_split_kernel<DIM> (pntf_split.h)
//   -DPNTF_RESIDUAL -DPNTF_DIM=3|6     residual_kernel<DIM> (Taylor mode, pntf_taylor.h)
//   -DPNTF_KIND=0..4 -DPNTF_DIM=3|6 -DPNTF_QUAD_FIELD    field_quad_kernel<DIM, KIND> (pntf_quad.h)
//   -DPNTF_PLAN_QUAD -DPNTF_QSOLO=0|1 -DPNTF_DIM=3|6   plan_quad_kernel<DIM, SOLO> (pntf_quad.h)
//   -DPNTF_UTIL                        pack_kernel, copy_kernel, sum_kernel, wide / quad packing
#include "pntf_quad.h"
#include "pntf_split.h"
#include "pntf_taylor.h"
#include "pntf_wide.h"

namespace pntf {
#if defined(PNTF_KIND) && defined(PNTF_QUAD_FIELD)
template __global__ void field_quad_kernel<PNTF_DIM, PNTF_KIND>(FieldArgs);
#elif defined(PNTF_PLAN_QUAD)
template __global__ void plan_quad_kernel<PNTF_DIM, PNTF_QSOLO>(PlanArgs);
#elif defined(PNTF_KIND) && defined(PNTF_WIDE_FIELD)
template __global__ void wide_field_kernel<PNTF_DIM, PNTF_KIND, false>(FieldArgs);
template __global__ void wide_field_kernel<PNTF_DIM, PNTF_KIND, true>(FieldArgs);
#elif defined(PNTF_KIND) && defined(PNTF_SPLIT_FIELD)
template __global__ void field_split_kernel<PNTF_DIM, PNTF_KIND>(FieldArgs);
#elif defined(PNTF_KIND)
template __global__ void field_kernel<PNTF_DIM, PNTF_KIND>(FieldArgs);
#elif defined(PNTF_PLAN)
template __global__ void plan_kernel<PNTF_DIM>(PlanArgs);
#elif defined(PNTF_PLAN_SPLIT)
template __global__ void plan_split_kernel<PNTF_DIM>(PlanArgs);
#elif defined(PNTF_RESIDUAL)
template __global__ void residual_kernel<PNTF_DIM>(ResidualArgs);
#endif
}  // namespace pntf
