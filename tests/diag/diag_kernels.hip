// Diagnostic builds of the τ+∇τ kernel body under other launch bounds / workgroup shapes.
// Not part of libpntf.so; built by hand with hipcc -shared into tests/diag/libdiag.so.
#include "pntf_field.h"

namespace pntf {
template <int LB>
__global__ __launch_bounds__(256, LB) void diag_fk256(FieldArgs a) {
  field_body<3, K_TAU_GRAD>(a, blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6),
                            gridDim.x * 4);
}
__global__ __launch_bounds__(512, 1) void diag_fk512(FieldArgs a) {
  field_body<3, K_TAU_GRAD>(a, blockIdx.x * 8 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6),
                            gridDim.x * 8);
}
}  // namespace pntf

extern "C" int diag_tau_grad(int variant, int grid, const float* P, const float* xp, int64_t n,
                             const float* Btab, float* tau, float* dtau, float* ws) {
  using namespace pntf;
  FieldArgs a{P, xp, Btab, nullptr, n, 1, 0, tau, dtau, ws};
  if (variant == 0) hipLaunchKernelGGL(diag_fk256<2>, dim3(grid), dim3(256), 0, 0, a);
  if (variant == 1) hipLaunchKernelGGL(diag_fk256<1>, dim3(grid), dim3(256), 0, 0, a);
  if (variant == 2) hipLaunchKernelGGL(diag_fk512, dim3(grid), dim3(512), 0, 0, a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
