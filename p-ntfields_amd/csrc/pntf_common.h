// Shared device-side definitions for the P-NTFields MI355X kernels.
//
// Data layout of the fused τ/∇τ kernels ("transposed" MFMA formulation):
//   * one wave owns a tile of 16 (start, goal) pairs; the pair index is the MFMA column
//     t = lane & 15, so the four lane groups g = lane >> 4 all belong to the same pair;
//   * an activation vector of 16*k features is k f32x4 "tiles": lane (t, g) holds feature
//     rows 4 g + s, s = 0..3, of column t — exactly the C/D layout of
//     v_mfma_f32_16x16x4_f32, so a layer's output tile is the next layer's B operand with
//     no data movement (k-step s takes register s; lane group g supplies k = g, i.e. row
//     4 g + s);
//   * the weights are the A operand, pre-packed ("fragment order") so that one
//     global_load_dwordx4 per lane fetches the A operands of the 4 k-steps of one input
//     tile and each wave-instruction reads 1 KiB contiguous:
//        P[((ot*KT + kt)*64 + lane)*4 + s] = W[16 ot + (lane & 15)][16 kt + 4 (lane >> 4) + s]
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pntf {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Split-bf16 layers (pntf_wide.h wx6_split, pntf_taylor.h nx6_split): PNTF_X6_DOT = 1 takes
// the residual x - bf16(x) of a split stage as one v_dot2c_f32_bf16 per element (x + p.lo·(-1)
// + p.hi·0: the product is exact and so is the difference, an RNE residual being
// representable) instead of an unpack and a subtract.
#ifndef PNTF_X6_DOT
#define PNTF_X6_DOT 0
#endif
typedef __bf16 x6bf16x2 __attribute__((ext_vector_type(2)));
typedef float x6f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ x6f32x2 x6_resid(x6f32x2 x, x6bf16x2 p) {
  // (-1, -0) and (-0, -1) as 32-bit literals: the plain (-1, 0) would be encoded as the inline
  // constant -1.0, which the hardware does not read as the bf16 pair (-1, 0)
  const x6bf16x2 nlo = __builtin_bit_cast(x6bf16x2, 0x8000bf80u), nhi = __builtin_bit_cast(x6bf16x2, 0xbf808000u);
  x6f32x2 r;
  r[0] = __builtin_amdgcn_fdot2_f32_bf16(p, nlo, x[0], false);
  r[1] = __builtin_amdgcn_fdot2_f32_bf16(p, nhi, x[1], false);
  return r;
}

constexpr int H = 128;              // hidden width (model_res_sigmoid_multi.py:134)
constexpr int TILE = 16;            // pairs per wave
constexpr int WAVES = 4;            // waves per workgroup (one per SIMD)
// Waves per workgroup of the split-tile kernels (pntf_split.h): 8, two per SIMD, so one
// wave's LDS exchange and epilogue run beside the other's MFMAs (4: one per SIMD).  The 8-wave
// build returned wrong ∇τ in pair columns 12-15 until the store-data hazard was found and
// padded (pntf_field.h bstore).
#ifndef PNTF_SPLIT
#define PNTF_SPLIT 8
#endif
constexpr int SPLIT_WAVES = PNTF_SPLIT;
// One wave per SIMD: the wave-tile / wide kernels need up to 512 VGPRs to stay spill-free
// (at two waves per SIMD, 256 VGPRs, hipcc spills to scratch).
#ifndef PNTF_WAVES_PER_SIMD
#define PNTF_WAVES_PER_SIMD 1
#endif
constexpr int WAVES_PER_SIMD = PNTF_WAVES_PER_SIMD;
constexpr int WG_PER_CU = WAVES_PER_SIMD;
constexpr float TWO_PI = 6.283185307179586f;

// ---------------------------------------------------------------- packed weight blob
// One direction (forward A = W, backward A = W^T) holds 15 matrices in this order.
constexpr int SZ_E0 = 128 * 256, SZ_E = 128 * 128, SZ_G = 256 * 256, SZ_G3 = 128 * 256;
constexpr int OFF_E0 = 0;
constexpr int OFF_EBLK = OFF_E0 + SZ_E0;      // (encoder.1, encoder1.1, encoder.2, encoder1.2)
constexpr int OFF_E3 = OFF_EBLK + 4 * SZ_E;
constexpr int OFF_GBLK = OFF_E3 + SZ_E;       // (generator.i, generator1.i) for i = 0..2
constexpr int OFF_G3 = OFF_GBLK + 6 * SZ_G;
constexpr int SZ_DIR = OFF_G3 + SZ_G3;
constexpr int OFF_FWD = 0;
constexpr int OFF_BWD = SZ_DIR;
constexpr int OFF_BIAS = 2 * SZ_DIR;
// bias block (plain order)
constexpr int B_E0 = 0;
constexpr int B_EBLK = 128;                   // 4 x 128 in the EBLK order above
constexpr int B_E3 = B_EBLK + 4 * 128;
constexpr int B_GBLK = B_E3 + 128;            // 6 x 256 in the GBLK order above
constexpr int B_G3 = B_GBLK + 6 * 256;
constexpr int B_G4W = B_G3 + 128;             // generator.4.weight (1 x 128)
constexpr int B_G4B = B_G4W + 128;            // generator.4.bias (padded to 4)
constexpr int SZ_BIAS = B_G4B + 4;
constexpr int PACKED_FLOATS = OFF_BIAS + SZ_BIAS;   // the 16x16 ("narrow") blob
// Wide blob (pntf_wide.h, v_mfma_f32_32x32x2_f32), packed right after the narrow one: the
// same 13 matrices in both directions in wide fragment order (same OFF_* offsets), the bias
// columns (one fragment per 4 out tiles of 32, bias in lanes 0-31), the head vector in the
// 32-row register order, and the head bias.
constexpr int OFF_WIDE = PACKED_FLOATS;
constexpr int W_OFF_BCOL = 2 * SZ_DIR;
constexpr int W_SZ_BCOL = (B_G4W / 128) * 256;
constexpr int W_OFF_G4W = W_OFF_BCOL + W_SZ_BCOL;
constexpr int W_SZ_G4W = 16 * 256;
constexpr int W_OFF_G4B = W_OFF_G4W + W_SZ_G4W;
constexpr int W_SZ = W_OFF_G4B + 4;
// Quad blob (pntf_quad.h, v_mfma_f32_4x4x1_16b_f32 on 4-pair tiles), packed after the wide
// one: per wave of a workgroup, the fragments of its share (1/Q_WAVES) of every layer's out
// rows in the order a planner step consumes them (13 forward layers, then the 13 reverse
// ones), so the weight ring is one linear stream; then per wave 14 bias vectors (the 13
// forward layers' biases and the head row, in the wave's compact row order).
// Q_WAVES = 8 (two per SIMD): one CU streams L2/MALL at ~130 GB/s with 8 waves loading
// against ~103 GB/s with 4 (tests/diag/stream_probe2.hip), and a planner step is bound by
// that stream (quad tiles).
#ifndef PNTF_QWAVES
#define PNTF_QWAVES 8
#endif
constexpr int Q_WAVES = PNTF_QWAVES;
static_assert(Q_WAVES == 4 || Q_WAVES == 8, "quad layers: 4 or 8 waves per workgroup");
constexpr int Q_NL = 26;
constexpr int Q_STREAM = 2 * SZ_DIR / Q_WAVES;      // floats of one wave's fragment stream
constexpr int Q_NF_FWD = SZ_DIR / Q_WAVES / 256;    // 1 KiB fragments of its forward part
// the wide kernels carry their activations times 10 / ln 2 (pntf_wide.h WKAPPA; the packer
// scales encoder[0]'s forward fragments and the forward bias columns by it)
constexpr float WIDE_KAPPA = 14.4269504088896341f;
// env-B table staged in LDS by the wide kernels when n_env · dim · 128 floats fit (pntf_wide.h
// WBt<true>): 20 KiB, i.e. dim 3 up to 13 environments, dim 6 up to 6
constexpr int WBL_FLOATS = 5120;
constexpr int Q_NAUX = 14;
constexpr int OFF_QUAD = (OFF_WIDE + W_SZ + 63) / 64 * 64;
constexpr int Q_OFF_AUX = Q_WAVES * Q_STREAM;
constexpr int Q_SZ = Q_OFF_AUX + Q_WAVES * Q_NAUX * 256;
constexpr int PACKED_TOTAL = OFF_QUAD + Q_SZ;
// Split-bf16 wide fragments (pntf_wide.h, PNTF_WIDE_X6): the wide region's two directions
// regrouped per 32 x 32 step into 2 k blocks x 3 bf16 terms (1.5x the fp32 bytes; a matrix at
// fp32 wide offset o sits at 1.5 o here)
constexpr int OFF_X6 = (PACKED_TOTAL + 63) / 64 * 64;
constexpr int X6_SZ = 3 * SZ_DIR;
// the same in block-major step order for the two-column (encoder) layers (pntf_wide.h
// wx6_block_major; other layers' order is unchanged)
constexpr int OFF_X6BM = OFF_X6 + X6_SZ;
constexpr int PACKED_TOTAL_X6 = OFF_X6BM + X6_SZ;
// Split-bf16 narrow fragments (pntf_taylor.h, the residual kernel's Taylor directions on
// v_mfma_f32_16x16x32_bf16, round 6): the forward direction regrouped per (16-row out tile,
// 32-feature k block) into 3 bf16 terms of 1 KiB each, in taylor_layer_x6's step order (out
// tiles in groups of NX6_G sharing one split of the input block: 16 = every layer's out tiles
// in one group, the residual kernel accumulating in its out bank); a matrix at forward offset o
// sits at 1.5 o here.
constexpr int NX6_G = 16;
constexpr int OFF_NX6 = (PACKED_TOTAL_X6 + 63) / 64 * 64;
constexpr int NX6_SZ = 3 * SZ_DIR / 2;
constexpr int PACKED_TOTAL_NX6 = OFF_NX6 + NX6_SZ;
// Quad layer list in stream order: packed matrix (0..12, the OFF_* order above), direction
// (0: A = W, 1: A = W^T), out rows, in features, plain bias offset (forward layers).
struct QLayer {
  int mat, dir, out, in, bias;
};
constexpr QLayer Q_LAYERS[Q_NL] = {
    {0, 0, 128, 256, B_E0},          {1, 0, 128, 128, B_EBLK},
    {2, 0, 128, 128, B_EBLK + 128},  {3, 0, 128, 128, B_EBLK + 256},
    {4, 0, 128, 128, B_EBLK + 384},  {5, 0, 128, 128, B_E3},
    {6, 0, 256, 256, B_GBLK},        {7, 0, 256, 256, B_GBLK + 256},
    {8, 0, 256, 256, B_GBLK + 512},  {9, 0, 256, 256, B_GBLK + 768},
    {10, 0, 256, 256, B_GBLK + 1024}, {11, 0, 256, 256, B_GBLK + 1280},
    {12, 0, 128, 256, B_G3},
    {12, 1, 256, 128, -1}, {11, 1, 256, 256, -1}, {10, 1, 256, 256, -1},
    {9, 1, 256, 256, -1},  {8, 1, 256, 256, -1},  {7, 1, 256, 256, -1},
    {6, 1, 256, 256, -1},  {5, 1, 128, 128, -1},  {4, 1, 128, 128, -1},
    {3, 1, 128, 128, -1},  {2, 1, 128, 128, -1},  {1, 1, 128, 128, -1},
    {0, 1, 256, 128, -1}};
// Start of layer L in a wave's stream (floats).
constexpr int q_layer_off(int L) {
  int o = 0;
  for (int i = 0; i < L; ++i) o += Q_LAYERS[i].out * Q_LAYERS[i].in / Q_WAVES;
  return o;
}
static_assert(q_layer_off(Q_NL) == Q_STREAM, "quad stream covers both directions");
static_assert(q_layer_off(13) == Q_NF_FWD * 256, "forward part of the quad stream");

// ---------------------------------------------------------------- per-wave scratch (saved σ10)
// Each saved "tile" is 16 feature rows x 16 pairs = 256 floats, stored lane-major
// (64 lanes x float4) so every store/load instruction moves 1 KiB contiguous.
constexpr int T_E0 = 0;                       // 2 cols x 8 tiles
constexpr int T_EBLK = 16;                    // block b (0,1): +32b: y1 (16 tiles), y2 (16 tiles)
constexpr int T_S0 = 80;                      // merge switch s0 = σ10(zs - zg), 8 tiles
constexpr int T_GBLK = 88;                    // block i (0..2): +32i: y1 (16), y2 (16)
constexpr int T_G3 = 184;                     // 8 tiles
constexpr int SCRATCH_TILES = 192;
constexpr int SCRATCH_FLOATS_PER_WAVE = SCRATCH_TILES * 256;
// Wide kernels: 32 pairs per wave; a saved tile is 32 features x 32 pairs = 4 KiB, index
// c·OT + t for 2-point layers.
constexpr int WTILE = 32;
constexpr int WT_E0 = 0;                      // 2 points x 4 tiles
constexpr int WT_EBLK = 8;                    // block b: +16b: y1 (8 tiles), y2 (8 tiles)
constexpr int WT_S0 = 40;                     // merge switch, 4 tiles
constexpr int WT_GBLK = 44;                   // block i: +16i: y1 (8), y2 (8)
constexpr int WT_G3 = 92;                     // 4 tiles
constexpr int WSCRATCH_TILES = 96;
constexpr int WSCRATCH_FLOATS_PER_WAVE = WSCRATCH_TILES * 1024;

// ---------------------------------------------------------------- kernel arguments
enum Kind { K_TAU = 0, K_TAU_GRAD = 1, K_VELOCITY = 2, K_SPEED = 3, K_TRAVEL = 4 };

struct FieldArgs {
  const float* P;        // packed weights
  const float* xp;       // (n, 2*DIM)
  const float* Btab;     // (n_env, DIM, 128)
  const int32_t* env;    // (n) or null
  int64_t n;
  int32_t n_env;
  int32_t compat;
  float* out0;           // tau / velocity / speed / travel time
  float* out1;           // dtau (K_TAU_GRAD), tau (K_VELOCITY, optional)
  float* ws;             // scratch, SCRATCH_FLOATS_PER_WAVE per slot
};

struct PlanArgs {
  const float* P;
  const float* xp0;      // (q, 2*DIM)
  const float* Btab;
  const int32_t* env;
  int64_t q;
  int32_t n_env;
  int32_t compat;
  float step, tol;
  int32_t max_iter;      // the loop body runs at most max_iter + 1 times
  float* path;           // (q, max_iter + 2, 2*DIM)
  int32_t* steps;        // (q)
  float* ws;
  // Tail hand-off of the quad planner (pntf_quad.h; NULL = off): tail[0] = queries done,
  // tail[1] = queries handed off, tail[2 .. 2+q) = their indices, tail[2+q .. 2+2q) = the
  // iteration each resumes at.  The 4-query tiles yield once at most `yield_at` queries of the
  // batch are still active; a SOLO launch with the same `tail` resumes the handed-off ones.
  int32_t* tail;
  int32_t yield_at;
};

struct ResidualArgs {
  const float* P;
  const float* xp;       // (n, 2*DIM)
  const float* yobs;     // (n, 2) observed speeds (may be null when diff is null)
  const float* Btab;
  const int32_t* env;
  int64_t n;
  int32_t n_env;
  float gamma;           // viscosity weight of the Laplacian term (Model.Loss :937)
  float* tau;            // (n)        optional
  float* dtau;           // (n, 2*DIM) optional
  float* ltau;           // (n, 2*DIM) optional: diagonal second derivatives
  float* diff;           // (n)        optional: per-pair residual
  float* ws;
};

}  // namespace pntf
