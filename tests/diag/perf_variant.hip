// Perf-variant builds of the τ+∇τ kernel (dim 3, exact mode) under other weight-stream
// parameters (-DPNTF_PF_STEPS, -DPNTF_NO1).  Diagnostics only; built by
// tests/diag/build_perf.sh into tests/diag/libperf_<name>.so and timed by perf_variants.py.
#ifdef PERF_WIDE
#define PNTF_UTIL   // pack_x6_kernel
#include "pntf_wide.h"
#elif defined(PERF_SPLIT)
#include "pntf_split.h"
#elif defined(PERF_QUAD)
#include "pntf_quad.h"
#else
#include "pntf_field.h"
#endif

extern "C" int perf_split_width() {
#ifdef PERF_QUAD
  return -4;   // quad tiles: 4 pairs per workgroup
#elif defined(PERF_SPLIT)
  return pntf::SPLIT;
#else
  return 0;
#endif
}

extern "C" int perf_tau_grad(int grid, const float* P, const float* xp, int64_t n,
                             const float* Btab, float* tau, float* dtau, float* ws,
                             hipStream_t stream) {
  using namespace pntf;
  FieldArgs a{P, xp, Btab, nullptr, n, 1, 0, tau, dtau, ws};
#ifdef PERF_WIDE
#ifndef PERF_WBL
#define PERF_WBL 0
#endif
  hipLaunchKernelGGL((wide_field_kernel<3, K_TAU_GRAD, PERF_WBL>), dim3(grid), dim3(256), 0,
                     stream, a);
#elif defined(PERF_QUAD)    // one workgroup per 4-pair tile
  hipLaunchKernelGGL((field_quad_kernel<3, K_TAU_GRAD>), dim3(grid), dim3(64 * Q_WAVES), 0,
                     stream, a);
#elif defined(PERF_SPLIT)   // one workgroup per 16-pair tile; ws: SPLIT slots per workgroup
  hipLaunchKernelGGL((field_split_kernel<3, K_TAU_GRAD>), dim3(grid), dim3(64 * SPLIT), 0,
                     stream, a);
#else
  hipLaunchKernelGGL((field_kernel<3, K_TAU_GRAD>), dim3(grid), dim3(256), 0, stream, a);
#endif
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

#ifdef PERF_WIDE
// floats of the blob this build reads, and the split-bf16 region of an x6 build: P holds that
// many floats, the first PACKED_TOTAL of them the production blob
extern "C" long long perf_packed_total() {
  return PNTF_WIDE_X6 ? pntf::PACKED_TOTAL_X6 : pntf::PACKED_TOTAL;
}
extern "C" int perf_pack_x6(float* P, hipStream_t stream) {
  using namespace pntf;
  const int64_t n = (int64_t)(2 * SZ_DIR / 1024) * 2 * 64;
  for (int bm = 0; bm < 2; ++bm)
    hipLaunchKernelGGL(pack_x6_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                       P + OFF_WIDE, reinterpret_cast<uint16_t*>(P + (bm ? OFF_X6BM : OFF_X6)),
                       bm);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
#endif

#ifdef PNTF_DEBUG_DUMP
extern "C" int perf_set_dbg(float* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(pntf::pntf_dbg), &p, sizeof(p)) == hipSuccess ? 0 : 1;
}
#endif

#ifdef PNTF_DEBUG_STAMPS
extern "C" int perf_set_stamps(unsigned long long* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(pntf::pntf_stamps), &p, sizeof(p)) == hipSuccess ? 0 : 1;
}
#endif

#ifdef PERF_QUAD
// C5-shaped planner launch of this build's quad kernels, the way pntf_plan_ex AUTO runs them:
// the 4-query MFMA tiles with the tail hand-off, then the SOLO resume launch (tail = ws, 8 + 8q
// bytes, zeroed by the caller).  dim 6, exact mode.
extern "C" int perf_plan6(int grid, int cus, const float* P, const float* xp0, int64_t q,
                          const float* Btab, float step, float tol, int max_iter, float* path,
                          int32_t* steps, int32_t* tail, hipStream_t stream) {
  using namespace pntf;
  PlanArgs a{P, xp0, Btab, nullptr, q, 1, 0, step, tol, max_iter, path, steps, nullptr, tail,
             (int32_t)cus};
  dim3 b(64 * Q_WAVES);
  hipLaunchKernelGGL((plan_quad_kernel<6, false>), dim3(grid), b, 0, stream, a);
  if (tail)
    hipLaunchKernelGGL((plan_quad_kernel<6, true>), dim3(q < cus ? q : cus), b, 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
#endif
