// One kernel per translation unit, selected at build time (pntf/build.py):
//   -DPNTF_KIND=0..4 -DPNTF_DIM=3|6   field_kernel<DIM, KIND>
//   -DPNTF_PLAN -DPNTF_DIM=3|6         plan_kernel<DIM>
//   -DPNTF_UTIL                        pack_kernel, copy_kernel
#include "pntf_field.h"

namespace pntf {
#if defined(PNTF_KIND)
template __global__ void field_kernel<PNTF_DIM, PNTF_KIND>(FieldArgs);
#elif defined(PNTF_PLAN)
template __global__ void plan_kernel<PNTF_DIM>(PlanArgs);
#endif
}  // namespace pntf
