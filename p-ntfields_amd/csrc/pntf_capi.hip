// C ABI of libpntf.so (declared in include/pntf.h): argument checks, launch geometry,
// error reporting.  Device code lives in pntf_field.hip.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>

#include "pntf.h"

#include "pntf_common.h"

// Kernels are compiled one per translation unit (pntf_kernels.hip, PNTF_DIM/PNTF_KIND) so
// the build parallelises; here they are only declared.
namespace pntf {
template <int DIM, int KIND>
__global__ void field_kernel(FieldArgs a);
template <int DIM, int KIND>
__global__ void field_split_kernel(FieldArgs a);
template <int DIM, int KIND, bool BL>
__global__ void wide_field_kernel(FieldArgs a);
template <int DIM>
__global__ void plan_kernel(PlanArgs a);
template <int DIM>
__global__ void plan_split_kernel(PlanArgs a);
template <int DIM, int KIND>
__global__ void field_quad_kernel(FieldArgs a);
template <int DIM, bool SOLO>
__global__ void plan_quad_kernel(PlanArgs a);
template <int DIM>
__global__ void residual_kernel(ResidualArgs a);
__global__ void sum_kernel(const float* __restrict__ x, int64_t n, double* __restrict__ out);
__global__ void pack_kernel(const float* __restrict__ src, int rows, int cols, int ld,
                            int trans, float* __restrict__ dst);
__global__ void copy_kernel(const float* __restrict__ src, int n, float* __restrict__ dst);
__global__ void pack_wide_kernel(const float* __restrict__ src, int rows, int cols, int ld,
                                 int trans, float scale, float* __restrict__ dst);
__global__ void pack_wide_aux_kernel(const float* __restrict__ plain, float* __restrict__ wide);
__global__ void pack_x6_kernel(const float* __restrict__ wide, uint16_t* __restrict__ x6, int bm);
__global__ void pack_nx6_kernel(const float* __restrict__ src, int rows, int cols,
                                uint16_t* __restrict__ dst);
__global__ void pack_quad_kernel(const float* __restrict__ src, int rows, int cols, int dir,
                                 float* __restrict__ dst);
__global__ void pack_quad_aux_kernel(const float* __restrict__ plain, float* __restrict__ quad);
}  // namespace pntf

using namespace pntf;

static thread_local char g_err[512] = "";

static int fail(int code, const char* fmt, const char* detail = "") {
  snprintf(g_err, sizeof(g_err), fmt, detail);
  return code;
}

static int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return PNTF_ERR_HIP;
  }
  return PNTF_OK;
}

static int num_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    return 256;
  return cus;
}

static constexpr size_t SLOT_BYTES = (size_t)SCRATCH_FLOATS_PER_WAVE * sizeof(float);
static constexpr size_t WSLOT_BYTES = (size_t)WSCRATCH_FLOATS_PER_WAVE * sizeof(float);

// persistent grid: one 4-wave workgroup per CU at most, never more than the tiles need
static int64_t grid_for(int64_t n) {
  int64_t ntiles = (n + TILE - 1) / TILE;
  int64_t wgs = (ntiles + WAVES - 1) / WAVES;
  int64_t cap = (int64_t)num_cus() * WG_PER_CU;
  return wgs < cap ? (wgs < 1 ? 1 : wgs) : cap;
}

// split-tile grid (pntf_split.h): one 4-wave workgroup per pair tile, at most one per CU
static int64_t split_grid_for(int64_t n) {
  int64_t ntiles = (n + TILE - 1) / TILE;
  int64_t cap = (int64_t)num_cus() * WG_PER_CU;
  return ntiles < cap ? (ntiles < 1 ? 1 : ntiles) : cap;
}

// wide grid (pntf_wide.h): 32-pair tiles, one 4-wave workgroup per CU at most
static int64_t wide_grid_for(int64_t n) {
  int64_t ntiles = (n + WTILE - 1) / WTILE;
  int64_t wgs = (ntiles + WAVES - 1) / WAVES;
  int64_t cap = (int64_t)num_cus() * WG_PER_CU;
  return wgs < cap ? (wgs < 1 ? 1 : wgs) : cap;
}

// quad grid (pntf_quad.h): 4-pair tiles, one Q_WAVES-wave workgroup per tile, at most one per CU
static int64_t quad_grid_for(int64_t n) {
  int64_t ntiles = (n + 3) / 4;
  int64_t cap = (int64_t)num_cus();
  return ntiles < cap ? (ntiles < 1 ? 1 : ntiles) : cap;
}

// Quad tiles while every tile gets a CU of its own: a planner step of a 4-pair tile is bound
// by the CU's weight stream, not by its MFMAs.
// PNTF_QSOLO=0 in the environment (read once) runs batches of at most one query per CU on
// the MFMA quad layers instead of the VALU SOLO layers (to compare the two).
static bool solo_enabled() {
  static const int on = [] {
    const char* e = getenv("PNTF_QSOLO");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return on != 0;
}

static bool use_quad(int64_t n, int schedule) {
  if (schedule == PNTF_SCHED_QUAD_TILE) return true;
  if (schedule != PNTF_SCHED_AUTO) return false;
  return (n + 3) / 4 <= (int64_t)num_cus();
}

static int grid_with_ws(int64_t n, size_t ws_bytes, int64_t* grid, bool split = false,
                        bool wide = false) {
  int64_t g = split ? split_grid_for(n) : wide ? wide_grid_for(n) : grid_for(n);
  int64_t fit = (int64_t)(ws_bytes / ((wide ? WSLOT_BYTES : SLOT_BYTES) *
                                      (split ? SPLIT_WAVES : WAVES)));
  if (fit < 1) return fail(PNTF_ERR_WORKSPACE, "workspace too small (%s)", "need >= 4 slots");
  *grid = g < fit ? g : fit;
  return PNTF_OK;
}

// Split tiles (pntf_split.h) while every tile still gets a CU of its own or shares one with
// at most one other: a split tile takes ~1/3 of the one-wave time, and the one-wave kernels
// win once the tiles fill every SIMD.
static bool use_split(int64_t n, int schedule) {
  if (schedule == PNTF_SCHED_SPLIT_TILE) return true;
  if (schedule == PNTF_SCHED_WAVE_TILE || schedule == PNTF_SCHED_WIDE_TILE) return false;
  return (n + TILE - 1) / TILE <= 2 * (int64_t)num_cus();
}

// Default schedule of the field entry points without an explicit one
// (pntf_set_field_schedule); pntf_field_ex takes the schedule per call instead.
static int g_field_schedule = PNTF_SCHED_AUTO;

static bool valid_schedule(int s) {
  return s == PNTF_SCHED_AUTO || s == PNTF_SCHED_WAVE_TILE || s == PNTF_SCHED_SPLIT_TILE ||
         s == PNTF_SCHED_WIDE_TILE || s == PNTF_SCHED_QUAD_TILE;
}

// wide_field_kernel keeps its tile index in a 32-bit SGPR (pntf_wide.h): the first pair of the
// last tile, tile * WTILE, must stay below 2^31.  Larger batches run the wave-tile kernel
// (int64 tile index) whatever schedule was asked for.
static constexpr int64_t WIDE_MAX_PAIRS = (int64_t)0x7fffffff - WTILE + 1;

// The kernel family a field call of n pairs runs (PNTF_SCHED_QUAD/SPLIT/WIDE/WAVE_TILE).
static int resolve_field_schedule(int64_t n, int schedule) {
  if (use_quad(n, schedule)) return PNTF_SCHED_QUAD_TILE;
  if (use_split(n, schedule)) return PNTF_SCHED_SPLIT_TILE;
  if (schedule == PNTF_SCHED_WAVE_TILE || n > WIDE_MAX_PAIRS) return PNTF_SCHED_WAVE_TILE;
  return PNTF_SCHED_WIDE_TILE;
}

#ifndef PNTF_BUILD_INFO
#define PNTF_BUILD_INFO "unstamped"
#endif

// An empty batch is valid whatever the data pointers are (torch hands out NULL for empty
// tensors); callers return PNTF_OK right after this check when n == 0.
static int check_common(const float* packed, int dim, const float* xp, int64_t n,
                        const float* Btab, int32_t n_env) {
  if (dim != 3 && dim != 6) return fail(PNTF_ERR_ARG, "dim must be 3 or 6%s");
  if (n < 0) return fail(PNTF_ERR_ARG, "negative batch%s");
  if (n == 0) return PNTF_OK;
  if (!packed || !xp || !Btab) return fail(PNTF_ERR_ARG, "null pointer argument%s");
  if (n_env < 1) return fail(PNTF_ERR_ARG, "n_env must be >= 1%s");
  return PNTF_OK;
}

template <int DIM>
static void launch_quad(int kind, int64_t grid, const FieldArgs& a, hipStream_t s) {
  dim3 g((unsigned)grid), b(64 * Q_WAVES);
  switch (kind) {
    case K_TAU: hipLaunchKernelGGL((field_quad_kernel<DIM, K_TAU>), g, b, 0, s, a); break;
    case K_TAU_GRAD: hipLaunchKernelGGL((field_quad_kernel<DIM, K_TAU_GRAD>), g, b, 0, s, a); break;
    case K_VELOCITY: hipLaunchKernelGGL((field_quad_kernel<DIM, K_VELOCITY>), g, b, 0, s, a); break;
    case K_SPEED: hipLaunchKernelGGL((field_quad_kernel<DIM, K_SPEED>), g, b, 0, s, a); break;
    default: hipLaunchKernelGGL((field_quad_kernel<DIM, K_TRAVEL>), g, b, 0, s, a); break;
  }
}

template <int DIM, bool BL>
static void launch_wide(int kind, dim3 g, dim3 b, const FieldArgs& a, hipStream_t s) {
  switch (kind) {
    case K_TAU: hipLaunchKernelGGL((wide_field_kernel<DIM, K_TAU, BL>), g, b, 0, s, a); break;
    case K_TAU_GRAD:
      hipLaunchKernelGGL((wide_field_kernel<DIM, K_TAU_GRAD, BL>), g, b, 0, s, a);
      break;
    case K_VELOCITY:
      hipLaunchKernelGGL((wide_field_kernel<DIM, K_VELOCITY, BL>), g, b, 0, s, a);
      break;
    case K_SPEED: hipLaunchKernelGGL((wide_field_kernel<DIM, K_SPEED, BL>), g, b, 0, s, a); break;
    default: hipLaunchKernelGGL((wide_field_kernel<DIM, K_TRAVEL, BL>), g, b, 0, s, a); break;
  }
}

template <int DIM>
static void launch_field(int kind, int64_t grid, const FieldArgs& a, hipStream_t s,
                         bool split, bool wide) {
  dim3 g((unsigned)grid), b(split ? 64 * SPLIT_WAVES : 256);
  if (wide) {
    // the env-B table in LDS when it fits (identical values, so identical results)
    if ((int64_t)a.n_env * DIM * H <= WBL_FLOATS) launch_wide<DIM, true>(kind, g, b, a, s);
    else launch_wide<DIM, false>(kind, g, b, a, s);
    return;
  }
  if (split) {
    switch (kind) {
      case K_TAU: hipLaunchKernelGGL((field_split_kernel<DIM, K_TAU>), g, b, 0, s, a); break;
      case K_TAU_GRAD:
        hipLaunchKernelGGL((field_split_kernel<DIM, K_TAU_GRAD>), g, b, 0, s, a);
        break;
      case K_VELOCITY:
        hipLaunchKernelGGL((field_split_kernel<DIM, K_VELOCITY>), g, b, 0, s, a);
        break;
      case K_SPEED: hipLaunchKernelGGL((field_split_kernel<DIM, K_SPEED>), g, b, 0, s, a); break;
      default: hipLaunchKernelGGL((field_split_kernel<DIM, K_TRAVEL>), g, b, 0, s, a); break;
    }
    return;
  }
  switch (kind) {
    case K_TAU: hipLaunchKernelGGL((field_kernel<DIM, K_TAU>), g, b, 0, s, a); break;
    case K_TAU_GRAD: hipLaunchKernelGGL((field_kernel<DIM, K_TAU_GRAD>), g, b, 0, s, a); break;
    case K_VELOCITY: hipLaunchKernelGGL((field_kernel<DIM, K_VELOCITY>), g, b, 0, s, a); break;
    case K_SPEED: hipLaunchKernelGGL((field_kernel<DIM, K_SPEED>), g, b, 0, s, a); break;
    default: hipLaunchKernelGGL((field_kernel<DIM, K_TRAVEL>), g, b, 0, s, a); break;
  }
}

static int run_field(int kind, const float* packed, int dim, const float* xp, int64_t n,
                     const float* Btab, const int32_t* env, int32_t n_env, int mode,
                     float* out0, float* out1, void* ws, size_t ws_bytes, int schedule,
                     hipStream_t s) {
  int st = check_common(packed, dim, xp, n, Btab, n_env);
  if (st) return st;
  if (kind < K_TAU || kind > K_TRAVEL) return fail(PNTF_ERR_ARG, "unknown field kind%s");
  if (!valid_schedule(schedule)) return fail(PNTF_ERR_ARG, "unknown schedule%s");
  if (mode != PNTF_GRAD_EXACT && mode != PNTF_GRAD_BACKGRAD_COMPAT)
    return fail(PNTF_ERR_ARG, "unknown gradient mode%s");
  if (n == 0) return PNTF_OK;
  if (!out0 || (kind == K_TAU_GRAD && !out1)) return fail(PNTF_ERR_ARG, "null output%s");
  const bool grad = kind != K_TAU && kind != K_TRAVEL;
  const int resolved = resolve_field_schedule(n, schedule);
  if (resolved == PNTF_SCHED_QUAD_TILE) {   // σ10 stays in LDS: no workspace
    FieldArgs a{packed, xp, Btab, env, n, n_env, mode, out0, out1, (float*)ws};
    if (dim == 3) launch_quad<3>(kind, quad_grid_for(n), a, s);
    else launch_quad<6>(kind, quad_grid_for(n), a, s);
    return check_launch("field_quad_kernel");
  }
  const bool split = resolved == PNTF_SCHED_SPLIT_TILE;
  const bool wide = resolved == PNTF_SCHED_WIDE_TILE;
  int64_t grid = split ? split_grid_for(n) : wide ? wide_grid_for(n) : grid_for(n);
  if (grad) {
    if (!ws) return fail(PNTF_ERR_WORKSPACE, "null workspace%s");
    st = grid_with_ws(n, ws_bytes, &grid, split, wide);
    if (st) return st;
  }
  FieldArgs a{packed, xp, Btab, env, n, n_env, mode, out0, out1, (float*)ws};
  if (dim == 3) launch_field<3>(kind, grid, a, s, split, wide);
  else launch_field<6>(kind, grid, a, s, split, wide);
  return check_launch(split ? "field_split_kernel" : wide ? "wide_field_kernel" : "field_kernel");
}

extern "C" {

int pntf_abi_version(void) { return PNTF_ABI_VERSION; }

const char* pntf_status_string(int status) {
  switch (status) {
    case PNTF_OK: return "ok";
    case PNTF_ERR_ARG: return "invalid argument";
    case PNTF_ERR_WORKSPACE: return "workspace too small";
    case PNTF_ERR_HIP: return "HIP runtime error";
    default: return "unknown status";
  }
}

const char* pntf_last_error(void) { return g_err; }

size_t pntf_packed_floats(void) { return (size_t)PACKED_TOTAL_NX6; }

const char* pntf_build_info(void) { return PNTF_BUILD_INFO; }

int pntf_set_field_schedule(int schedule) {
  if (!valid_schedule(schedule)) return fail(PNTF_ERR_ARG, "unknown schedule%s");
  g_field_schedule = schedule;
  return PNTF_OK;
}

int pntf_field_schedule_for(int64_t n, int schedule) {
  if (n < 0 || !valid_schedule(schedule)) return -1;
  return resolve_field_schedule(n, schedule);
}

size_t pntf_workspace_bytes(int64_t n) {
  if (n <= 0) n = 1;
  int64_t g = grid_for(n), gs = split_grid_for(n);
  size_t narrow = (size_t)g * WAVES * SLOT_BYTES, split = (size_t)gs * SPLIT_WAVES * SLOT_BYTES;
  if (split > narrow) narrow = split;
  size_t wide = (size_t)wide_grid_for(n) * WAVES * WSLOT_BYTES;
  return narrow > wide ? narrow : wide;
}

int pntf_pack_weights(const float* const* params, int n_params, float* packed,
                      hipStream_t stream) {
  if (!params || !packed) return fail(PNTF_ERR_ARG, "null pointer argument%s");
  if (n_params != 30) return fail(PNTF_ERR_ARG, "expected 30 state-dict tensors%s");
  for (int i = 0; i < 30; ++i)
    if (i != 8 && i != 9 && !params[i]) return fail(PNTF_ERR_ARG, "null state-dict tensor%s");
  // state-dict index of each packed matrix (pntf_common.h order) and its shape
  struct M { int idx, rows, cols, off; };
  const M mats[] = {
      {0, 128, 256, OFF_E0},                                  // encoder.0
      {2, 128, 128, OFF_EBLK + 0 * SZ_E},                     // encoder.1
      {10, 128, 128, OFF_EBLK + 1 * SZ_E},                    // encoder1.1
      {4, 128, 128, OFF_EBLK + 2 * SZ_E},                     // encoder.2
      {12, 128, 128, OFF_EBLK + 3 * SZ_E},                    // encoder1.2
      {6, 128, 128, OFF_E3},                                  // encoder.3
      {14, 256, 256, OFF_GBLK + 0 * SZ_G},                    // generator.0
      {24, 256, 256, OFF_GBLK + 1 * SZ_G},                    // generator1.0
      {16, 256, 256, OFF_GBLK + 2 * SZ_G},                    // generator.1
      {26, 256, 256, OFF_GBLK + 3 * SZ_G},                    // generator1.1
      {18, 256, 256, OFF_GBLK + 4 * SZ_G},                    // generator.2
      {28, 256, 256, OFF_GBLK + 5 * SZ_G},                    // generator1.2
      {20, 128, 256, OFF_G3},                                 // generator.3
  };
  hipMemsetAsync(packed, 0, sizeof(float) * PACKED_TOTAL_NX6, stream);
  for (int m = 0; m < (int)(sizeof(mats) / sizeof(mats[0])); ++m) {
    const M& d = mats[m];
    int64_t cnt = (int64_t)d.rows * d.cols;
    unsigned blocks = (unsigned)((cnt + 255) / 256);
    // forward: A = W (rows x cols); backward: A = W^T (cols x rows)
    hipLaunchKernelGGL(pack_kernel, dim3(blocks), dim3(256), 0, stream, params[d.idx], d.rows,
                       d.cols, d.cols, 0, packed + OFF_FWD + d.off);
    hipLaunchKernelGGL(pack_kernel, dim3(blocks), dim3(256), 0, stream, params[d.idx], d.cols,
                       d.rows, d.cols, 1, packed + OFF_BWD + d.off);
    // the wide (32x32x2) fragment order of the same two matrices
    // (forward encoder[0] times κ: the wide kernels carry κ-scaled activations, pntf_wide.h)
    hipLaunchKernelGGL(pack_wide_kernel, dim3(blocks), dim3(256), 0, stream, params[d.idx],
                       d.rows, d.cols, d.cols, 0, d.off == OFF_E0 ? WIDE_KAPPA : 1.f,
                       packed + OFF_WIDE + OFF_FWD + d.off);
    hipLaunchKernelGGL(pack_wide_kernel, dim3(blocks), dim3(256), 0, stream, params[d.idx],
                       d.cols, d.rows, d.cols, 1, 1.f, packed + OFF_WIDE + OFF_BWD + d.off);
    // the residual kernel's split-bf16 Taylor layers (16x16x32 step order, forward only)
    hipLaunchKernelGGL(pack_nx6_kernel, dim3((unsigned)((cnt / 8 + 255) / 256)), dim3(256), 0,
                       stream, params[d.idx], d.rows, d.cols,
                       reinterpret_cast<uint16_t*>(packed + OFF_NX6 + d.off / 2 * 3));
  }
  // the quad streams: every layer of both directions in planner-step order
  for (int L = 0; L < Q_NL; ++L) {
    const M& d = mats[Q_LAYERS[L].mat];
    unsigned blocks = (unsigned)(((int64_t)d.rows * d.cols + 255) / 256);
    hipLaunchKernelGGL(pack_quad_kernel, dim3(blocks), dim3(256), 0, stream, params[d.idx],
                       d.rows, d.cols, Q_LAYERS[L].dir, packed + OFF_QUAD + q_layer_off(L));
  }
  struct Bc { int idx, n, off; };
  const Bc bs[] = {
      {1, 128, B_E0},           {3, 128, B_EBLK + 0},     {11, 128, B_EBLK + 128},
      {5, 128, B_EBLK + 256},   {13, 128, B_EBLK + 384},  {7, 128, B_E3},
      {15, 256, B_GBLK + 0},    {25, 256, B_GBLK + 256},  {17, 256, B_GBLK + 512},
      {27, 256, B_GBLK + 768},  {19, 256, B_GBLK + 1024}, {29, 256, B_GBLK + 1280},
      {21, 128, B_G3},          {22, 128, B_G4W},         {23, 1, B_G4B}};
  for (int i = 0; i < (int)(sizeof(bs) / sizeof(bs[0])); ++i)
    hipLaunchKernelGGL(copy_kernel, dim3(1), dim3(256), 0, stream, params[bs[i].idx], bs[i].n,
                       packed + OFF_BIAS + bs[i].off);
  const int aux = W_SZ_BCOL + W_SZ_G4W + 4;
  hipLaunchKernelGGL(pack_wide_aux_kernel, dim3((aux + 255) / 256), dim3(256), 0, stream,
                     packed + OFF_BIAS, packed + OFF_WIDE);
  hipLaunchKernelGGL(pack_quad_aux_kernel, dim3(Q_WAVES * Q_NAUX), dim3(256), 0, stream,
                     packed + OFF_BIAS, packed + OFF_QUAD);
  // the wide kernels' split-bf16 layers read a regrouped, pre-split copy of both directions
  const int64_t nx6 = (int64_t)(2 * SZ_DIR / 1024) * 2 * 64;
  for (int bm = 0; bm < 2; ++bm)
    hipLaunchKernelGGL(pack_x6_kernel, dim3((unsigned)((nx6 + 255) / 256)), dim3(256), 0, stream,
                       packed + OFF_WIDE,
                       reinterpret_cast<uint16_t*>(packed + (bm ? OFF_X6BM : OFF_X6)), bm);
  return check_launch("pack_weights");
}

// ---- handle form: the library owns the packed weights
struct pntf_net {
  float* packed;
};

pntf_net* pntf_net_create(const float* const* params, int n_params, hipStream_t stream) {
  float* p = nullptr;
  if (hipMalloc(&p, sizeof(float) * PACKED_TOTAL_NX6) != hipSuccess) {
    fail(PNTF_ERR_HIP, "pntf_net_create: hipMalloc of the packed weights failed%s");
    return nullptr;
  }
  if (pntf_pack_weights(params, n_params, p, stream) != PNTF_OK) {
    hipFree(p);
    return nullptr;
  }
  pntf_net* net = new (std::nothrow) pntf_net{p};
  if (!net) {
    hipFree(p);
    fail(PNTF_ERR_ARG, "pntf_net_create: out of host memory%s");
  }
  return net;
}

int pntf_net_update(pntf_net* net, const float* const* params, int n_params,
                    hipStream_t stream) {
  if (!net) return fail(PNTF_ERR_ARG, "pntf_net_update: null handle%s");
  return pntf_pack_weights(params, n_params, net->packed, stream);
}

const float* pntf_net_packed(const pntf_net* net) { return net ? net->packed : nullptr; }

void pntf_net_destroy(pntf_net* net) {
  if (!net) return;
  hipFree(net->packed);
  delete net;
}

int pntf_tau(const float* packed, int dim, const float* xp, int64_t n, const float* Btab,
             const int32_t* env, int32_t n_env, float* tau, hipStream_t stream) {
  return run_field(K_TAU, packed, dim, xp, n, Btab, env, n_env, 0, tau, nullptr, nullptr, 0,
                   g_field_schedule, stream);
}

int pntf_tau_grad(const float* packed, int dim, const float* xp, int64_t n,
                  const float* Btab, const int32_t* env, int32_t n_env, int mode, float* tau,
                  float* dtau, void* ws, size_t ws_bytes, hipStream_t stream) {
  return run_field(K_TAU_GRAD, packed, dim, xp, n, Btab, env, n_env, mode, tau, dtau, ws,
                   ws_bytes, g_field_schedule, stream);
}

int pntf_path_velocity(const float* packed, int dim, const float* xp, int64_t n,
                       const float* Btab, const int32_t* env, int32_t n_env, int mode,
                       float* vel, float* tau, void* ws, size_t ws_bytes,
                       hipStream_t stream) {
  return run_field(K_VELOCITY, packed, dim, xp, n, Btab, env, n_env, mode, vel, tau, ws,
                   ws_bytes, g_field_schedule, stream);
}

int pntf_speed(const float* packed, int dim, const float* xp, int64_t n, const float* Btab,
               const int32_t* env, int32_t n_env, float* speed, void* ws, size_t ws_bytes,
               hipStream_t stream) {
  return run_field(K_SPEED, packed, dim, xp, n, Btab, env, n_env, PNTF_GRAD_EXACT, speed,
                   nullptr, ws, ws_bytes, g_field_schedule, stream);
}

int pntf_travel_time(const float* packed, int dim, const float* xp, int64_t n,
                     const float* Btab, const int32_t* env, int32_t n_env, float* tt,
                     hipStream_t stream) {
  return run_field(K_TRAVEL, packed, dim, xp, n, Btab, env, n_env, 0, tt, nullptr, nullptr, 0,
                   g_field_schedule, stream);
}

int pntf_field_ex(int kind, const float* packed, int dim, const float* xp, int64_t n,
                  const float* Btab, const int32_t* env, int32_t n_env, int mode, float* out0,
                  float* out1, void* ws, size_t ws_bytes, int schedule, hipStream_t stream) {
  return run_field(kind, packed, dim, xp, n, Btab, env, n_env, mode, out0, out1, ws, ws_bytes,
                   schedule, stream);
}

int pntf_plan(const float* packed, int dim, const float* xp0, int64_t q, const float* Btab,
              const int32_t* env, int32_t n_env, int mode, float step, float tol,
              int32_t max_iter, float* path, int32_t* steps, void* ws, size_t ws_bytes,
              hipStream_t stream) {
  return pntf_plan_ex(packed, dim, xp0, q, Btab, env, n_env, mode, step, tol, max_iter, path,
                      steps, ws, ws_bytes, PNTF_SCHED_AUTO, stream);
}

int pntf_plan_ex(const float* packed, int dim, const float* xp0, int64_t q, const float* Btab,
                 const int32_t* env, int32_t n_env, int mode, float step, float tol,
                 int32_t max_iter, float* path, int32_t* steps, void* ws, size_t ws_bytes,
                 int schedule, hipStream_t stream) {
  int st = check_common(packed, dim, xp0, q, Btab, n_env);
  if (st) return st;
  if (max_iter < 0) return fail(PNTF_ERR_ARG, "max_iter must be >= 0%s");
  if (mode != PNTF_GRAD_EXACT && mode != PNTF_GRAD_BACKGRAD_COMPAT)
    return fail(PNTF_ERR_ARG, "unknown gradient mode%s");
  if (!valid_schedule(schedule)) return fail(PNTF_ERR_ARG, "unknown schedule%s");
  if (q == 0) return PNTF_OK;
  if (!path || !steps) return fail(PNTF_ERR_ARG, "null output%s");
  PlanArgs a{packed, xp0, Btab, env, q, n_env, mode, step, tol, max_iter, path, steps,
             (float*)ws, nullptr, 0};
  if (use_quad(q, schedule)) {
    const int64_t cus = num_cus();
    dim3 g((unsigned)quad_grid_for(q)), b(64 * Q_WAVES);
    if (schedule == PNTF_SCHED_AUTO && q <= cus && solo_enabled()) {
      // one query per CU (the reference's Q = 1 loop, small batches): VALU SOLO layers
      dim3 gs((unsigned)q);
      if (dim == 3) hipLaunchKernelGGL((plan_quad_kernel<3, true>), gs, b, 0, stream, a);
      else hipLaunchKernelGGL((plan_quad_kernel<6, true>), gs, b, 0, stream, a);
      return check_launch("plan_quad_kernel<solo>");
    }
    // AUTO with a workspace: the 4-query tiles hand the last <= CUs active queries off to a
    // SOLO launch (pntf_quad.h "Tail hand-off"; bit-identical results, QUAD_TILE runs without)
    const bool hand_off = schedule == PNTF_SCHED_AUTO && solo_enabled() && ws &&
                          ws_bytes >= sizeof(int32_t) * (size_t)(2 + 2 * q);
    if (hand_off) {
      a.tail = (int32_t*)ws;
      a.yield_at = (int32_t)cus;
      if (hipMemsetAsync(ws, 0, 2 * sizeof(int32_t), stream) != hipSuccess)
        return check_launch("plan tail reset");
    }
    if (dim == 3) hipLaunchKernelGGL((plan_quad_kernel<3, false>), g, b, 0, stream, a);
    else hipLaunchKernelGGL((plan_quad_kernel<6, false>), g, b, 0, stream, a);
    st = check_launch("plan_quad_kernel");
    if (st || !hand_off) return st;
    dim3 gs((unsigned)(q < cus ? q : cus));
    if (dim == 3) hipLaunchKernelGGL((plan_quad_kernel<3, true>), gs, b, 0, stream, a);
    else hipLaunchKernelGGL((plan_quad_kernel<6, true>), gs, b, 0, stream, a);
    return check_launch("plan_quad_kernel<solo, resume>");
  }
  if (!ws) return fail(PNTF_ERR_WORKSPACE, "null workspace%s");
  const bool split = use_split(q, schedule);
  int64_t grid;
  st = grid_with_ws(q, ws_bytes, &grid, split);
  if (st) return st;
  dim3 g((unsigned)grid), b(256);
  if (split) {
    b = dim3(64 * SPLIT_WAVES);
    if (dim == 3) hipLaunchKernelGGL((plan_split_kernel<3>), g, b, 0, stream, a);
    else hipLaunchKernelGGL((plan_split_kernel<6>), g, b, 0, stream, a);
    return check_launch("plan_split_kernel");
  }
  if (dim == 3) hipLaunchKernelGGL((plan_kernel<3>), g, b, 0, stream, a);
  else hipLaunchKernelGGL((plan_kernel<6>), g, b, 0, stream, a);
  return check_launch("plan_kernel");
}

int pntf_eikonal_residual(const float* packed, int dim, const float* xp, const float* yobs,
                          int64_t n, const float* Btab, const int32_t* env, int32_t n_env,
                          float gamma, float* tau, float* dtau, float* ltau, float* diff,
                          void* ws, size_t ws_bytes, hipStream_t stream) {
  int st = check_common(packed, dim, xp, n, Btab, n_env);
  if (st) return st;
  if (n == 0) return PNTF_OK;
  if (diff && !yobs) return fail(PNTF_ERR_ARG, "diff requested without yobs%s");
  if (!ws) return fail(PNTF_ERR_WORKSPACE, "null workspace%s");
  int64_t grid;
  st = grid_with_ws(n, ws_bytes, &grid);
  if (st) return st;
  ResidualArgs a{packed, xp, yobs, Btab, env, n, n_env, gamma, tau, dtau, ltau, diff,
                 (float*)ws};
  if (dim == 3)
    hipLaunchKernelGGL((residual_kernel<3>), dim3((unsigned)grid), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL((residual_kernel<6>), dim3((unsigned)grid), dim3(256), 0, stream, a);
  return check_launch("residual_kernel");
}

int pntf_sum(const float* x, int64_t n, double* out, hipStream_t stream) {
  if (!out || n < 0 || (n > 0 && !x)) return fail(PNTF_ERR_ARG, "bad pntf_sum arguments%s");
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(1024), 0, stream, x, n, out);
  return check_launch("sum_kernel");
}

}  // extern "C"
