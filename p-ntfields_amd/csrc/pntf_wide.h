#pragma once
// Wide τ / ∇τ kernels: 32 (start, goal) pairs per wave on v_mfma_f32_32x32x2_f32
// ("wide kernels").
//
// Why: beside fp32 MFMAs on gfx950 every vector-memory instruction steals MFMA issue cycles
// (tests/diag/vmem_probe.hip, mfma32_probe.hip: ~5-15 cycles per buffer_load_dwordx4 beside
// v_mfma_f32_16x16x4_f32, ~1 beside v_mfma_f32_32x32x2_f32), and the 16-pair kernel of
// pntf_field.h loads one 1 KiB weight fragment per 4-8 of its MFMAs.  With 32 pairs as the
// MFMA's N dimension one fragment feeds 4 (32x32x2) MFMAs of 64 cycles, so the weight stream
// costs half the loads per pair and almost no issue time.
//
// Layout (same "transposed" formulation as pntf_field.h, 32-row tiles):
//   * lane l = (j, h), j = l & 31 the pair, h = l >> 5; a 32-feature activation tile is one
//     f32x16 per lane, register r holding feature row(r, h) = (r & 3) + 8 (r >> 2) + 4 h —
//     exactly the C/D layout of v_mfma_f32_32x32x2_f32;
//   * a layer's output tile is the next layer's B operand as is: instruction (kt, r) takes
//     B = in[kt][r] (k-pair rows row(r, 0), row(r, 1)) and A = the weight column pair of the
//     same rows, packed ("wide fragment order", pntf_pack_weights) so that one
//     buffer_load_dwordx4 per lane fetches the A operands of 4 consecutive registers:
//        P[(((ot·KT + kt)·4 + u)·64 + l)·4 + s] = M[32 ot + (l & 31)][32 kt + 8 u + 4 (l >> 5) + s]
//   * the bias enters as one extra MFMA per out tile (A = the bias column on the h = 0 lanes,
//     B = 1), and a residual as that MFMA's C operand, so neither costs VALU work;
//   * activations live in two banks X[8], Y[8] (256 features, or 2 points x 128 features);
//     saved σ10 tiles (4 KiB per 32-feature tile and point) go to a per-wave scratch slot.
#include "pntf_field.h"
#include "pntf_stamp.h"

namespace pntf {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}

// ---------------------------------------------------------------- split-bf16 layers (x6)
// PNTF_WIDE_X6 = 1: the generic layers (wlayer: the encoder and generator blocks, encoder[-1],
// generator[-2] and their transposes, 90 % of the MFMA work) run each fp32 product as six
// v_mfma_f32_32x32x16_bf16 on three-term bf16 splits of both operands (the training GEMMs'
// scheme, pntf_gemm.hip x6_split: 2.67x the fp32 MFMA rate).  A 32-feature tile's registers
// 8b..8b+7 are the B operand of k block b as they are (lane (j, h) holds feature rows
// wrow(8b + i, h), i = 0..7); the weights are pre-split in the same k order (OFF_X6,
// pack_x6_kernel).  encoder[0] runs split-bf16 as well (PNTF_X6_E0, default 1); only the
// Fourier fold (encoder[0]^T fused with the Fourier Jacobian) stays on fp32 MFMA.
#ifndef PNTF_WIDE_X6
#define PNTF_WIDE_X6 0
#endif
constexpr int WNL = PNTF_WIDE_X6 ? 6 : 4;   // weight fragments per wlayer step
static_assert(WNL <= RING_NL, "x6 layers read 6 fragments per step: build with PNTF_RING_NL=6");
typedef __bf16 wbf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 wbf16x2 __attribute__((ext_vector_type(2)));
typedef float wf32x2 __attribute__((ext_vector_type(2)));
// three-term RNE split of registers 8b..8b+7 of a tile (x = x0 + x1 + x2, each bf16)
template <bool OPAQUE = false>
__device__ __forceinline__ void wx6_split(const f32x16& v, int b, wbf16x8 (&s)[3]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    wf32x2 x = {v[8 * b + 2 * i], v[8 * b + 2 * i + 1]};
    // per step: the split is not shared between the out tiles of a layer (that would keep a
    // whole split input bank live, 192 registers)
    if constexpr (OPAQUE) asm volatile("" : "+v"(x));
    const wbf16x2 p0 = __builtin_convertvector(x, wbf16x2);
#ifdef PNTF_ABL_NOSPLIT   // diagnostics only (tests/diag ablations): one term, wrong results
    s[0][2 * i] = s[1][2 * i] = s[2][2 * i] = p0[0];
    s[0][2 * i + 1] = s[1][2 * i + 1] = s[2][2 * i + 1] = p0[1];
    continue;
#endif
#if PNTF_X6_DOT
    const wf32x2 r1 = x6_resid(x, p0);
    const wbf16x2 p1 = __builtin_convertvector(r1, wbf16x2);
    const wf32x2 r2 = x6_resid(r1, p1);
#else
    const wf32x2 r1 = x - __builtin_convertvector(p0, wf32x2);
    const wbf16x2 p1 = __builtin_convertvector(r1, wbf16x2);
    const wf32x2 r2 = r1 - __builtin_convertvector(p1, wf32x2);
#endif
    const wbf16x2 p2 = __builtin_convertvector(r2, wbf16x2);
    s[0][2 * i] = p0[0]; s[0][2 * i + 1] = p0[1];
    s[1][2 * i] = p1[0]; s[1][2 * i + 1] = p1[1];
    s[2][2 * i] = p2[0]; s[2][2 * i + 1] = p2[1];
  }
}
// out tiles per group of an x6 layer: G accumulators of NC tiles live
// PNTF_X6_ACC = 1 (round 6, the default): the out bank is the accumulator and every layer's
// out tiles form one group (xlayer below); the split copy is then in (kt, ot) step order for
// every layer (0: round 5's engine, wlayer, and its order — diagnostic builds only)
#ifndef PNTF_X6_ACC
#define PNTF_X6_ACC 1
#endif
#ifndef PNTF_X6_G1
#define PNTF_X6_G1 (PNTF_X6_ACC ? 8 : 4)
#endif
#ifndef PNTF_X6_G2
#define PNTF_X6_G2 (PNTF_X6_ACC ? 4 : 1)
#endif
#ifndef PNTF_X6_G1BUF
#define PNTF_X6_G1BUF 1
#endif
#ifndef PNTF_X6_BM
#define PNTF_X6_BM 0
#endif
// two-column layers in block-major steps (wlayer x6, pack_x6_kernel)
constexpr bool wx6_block_major(int NC) { return PNTF_X6_BM && NC == 2; }
// the order pack_x6_kernel writes: block-major for two-column layers into the OFF_X6BM copy
constexpr int wx6_group(int OT, int NC) { return NC == 2 ? PNTF_X6_G2 : (OT < PNTF_X6_G1 ? OT : PNTF_X6_G1); }
// the six products of order >= 2^-16, the small ones first
__device__ __forceinline__ f32x16 wx6_mma(const f32x4& w0, const f32x4& w1, const f32x4& w2,
                                          const wbf16x8 (&x)[3], f32x16 acc) {
  const wbf16x8 a0 = __builtin_bit_cast(wbf16x8, w0), a1 = __builtin_bit_cast(wbf16x8, w1),
                a2 = __builtin_bit_cast(wbf16x8, w2);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a2, x[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, x[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, x[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, x[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, x[1], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, x[0], acc, 0, 0, 0);
}
// Activations carried pre-scaled by κ = 10/ln 2 (round 4).  The forward pass keeps
// y' = κ·y and h' = κ·h: encoder[0]'s weights and every forward bias column are packed times κ
// (pack_wide_kernel / pack_wide_aux_kernel), the interior layers' weights are not (W·h' + κ·b
// = κ·y), and the head row divides it out once per pair.  Then e^{-10|y|} = 2^{-|y'|} needs no
// scaling multiply and softplus₁₀'s log term no constant: κ·softplus₁₀(y) = max(y', 0) +
// log₂(1 + 2^{-|y'|}); σ(10 y) is unchanged, so the reverse sweep (σ tiles, unscaled Wᵀ) is
// as before.  One VALU op fewer per activation element (tests/diag ablation: -0.5 %).
constexpr float WKAPPA = WIDE_KAPPA;                  // 10 / ln 2
constexpr float WKAPPA_INV = 0.0693147180559945309f;  // ln 2 / 10
__device__ __forceinline__ SpSig wsp_sig(float y) {   // y = κ·(pre-activation)
#ifdef PNTF_ABL_CHEAPACT   // diagnostics only (tests/diag ablations): no transcendentals
  return SpSig{fmaxf(y, 0.f) * 0.5f + 0.01f, 0.5f};
#endif
  const float t = __builtin_amdgcn_exp2f(-fabsf(y));
  const float u = 1.f + t;
  const float r = __builtin_amdgcn_rcpf(u);
  const bool pos = y >= 0.f;
  SpSig o;
  o.sp = (pos ? y : 0.f) + __builtin_amdgcn_logf(u);   // κ·softplus₁₀ (log2: v_log_f32)
  o.sg = pos ? r : t * r;
  return o;
}

// feature row of register r in lane half h of a 32-row tile
__device__ __forceinline__ constexpr int wrow(int r, int h) {
  return (r & 3) + 8 * (r >> 2) + 4 * h;
}

// ---------------------------------------------------------------- scratch (saved σ10)
struct WScratch {
  Rsrc r;
};
__device__ __forceinline__ WScratch make_wscratch(float* p) {
  return WScratch{make_rsrc(p, p ? WSCRATCH_FLOATS_PER_WAVE * 4 : 0)};
}
#ifdef PNTF_ABL_HOTLOAD   // diagnostics only: σ reloads from a 16 KiB region no store touches
__device__ float pntf_abl_hot[4 * 1024];
#endif
// cache policy of the saved-σ stores (nt: they stream past the L2 that holds the weights)
#ifndef PNTF_WSTORE_AUX
#define PNTF_WSTORE_AUX AUX_NT
#endif
// tile t = 4 KiB: part q (registers 4q..4q+3) of all lanes is 1 KiB contiguous
__device__ __forceinline__ void wstore(WScratch sc, int t, int lane, const f32x16& v) {
#ifdef PNTF_ABL_NOSTORE   // diagnostics only: the σ stores are dropped (wrong results)
  asm volatile("" ::"v"(v[0]), "v"(v[5]), "v"(v[10]), "v"(v[15]));
  return;
#endif
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x4 p{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
    bstore<PNTF_WSTORE_AUX>(sc.r, p, lane * 16, t * 4096 + q * 1024);
  }
}
__device__ __forceinline__ f32x16 wload(WScratch sc, int t, int lane) {
  f32x16 v;
#ifdef PNTF_ABL_NOLOAD    // diagnostics only (tests/diag ablations)
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = 0.5f;
  return v;
#endif
#ifdef PNTF_ABL_L2LOAD    // diagnostics only: same loads, from a 16 KiB L2-resident region
  t &= 3;
#endif
#ifdef PNTF_ABL_HOTLOAD   // diagnostics only: same loads (nt, bypass L1) from an L2-hot region
  sc.r = make_rsrc(pntf_abl_hot, 16384);
  t = 0;
#endif
#ifdef PNTF_ABL_UNUSED    // diagnostics only: the loads issue, their data is not used
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x4 p = __builtin_bit_cast(
        f32x4, __builtin_amdgcn_raw_buffer_load_b128(sc.r, lane * 16, t * 4096 + q * 1024,
                                                     AUX_LOAD));
    asm volatile("" ::"v"(p));
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) v[r] = 0.5f;
  return v;
#endif
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x4 p = __builtin_bit_cast(
        f32x4, __builtin_amdgcn_raw_buffer_load_b128(sc.r, lane * 16, t * 4096 + q * 1024,
                                                     AUX_LOAD));
#pragma unroll
    for (int s = 0; s < 4; ++s) v[4 * q + s] = p[s];
  }
  return v;
}

// ---------------------------------------------------------------- LDS σ tiles
// The σ tiles the reverse sweep consumes at once when a phase starts — generator[-2]'s four
// (the head step, right after the forward -> reverse drain) and the merge switch's four (the
// merge Jacobian) — stay in LDS: 8 tiles x 4 KiB per wave, 128 KiB per workgroup (the kernel
// uses no other LDS).  From the scratch slot each of those reloads waited out a whole HBM
// round trip with nothing else in flight.  Layout as the scratch tiles: part q of a tile is
// 1 KiB contiguous (lane-major f32x4), so ds_write_b128 / ds_read_b128 are conflict-free.
typedef __attribute__((address_space(3))) f32x4 wlds_f4;
constexpr int WL_G3 = 0, WL_S0 = 4, WL_TILES = 8;
typedef __attribute__((address_space(3))) float wlds_f;
struct WLds {
  wlds_f4* p;          // this wave's region, offset by the lane
  const wlds_f* hw;    // the head row generator.4.weight (128 floats, staged once per workgroup)
};
__device__ __forceinline__ void lstore(WLds l, int t, const f32x16& v) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
    l.p[(t * 4 + q) * 64] = f32x4{v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]};
}
__device__ __forceinline__ f32x16 lload(WLds l, int t) {
  f32x16 v;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x4 p = l.p[(t * 4 + q) * 64];
#pragma unroll
    for (int s = 0; s < 4; ++s) v[4 * q + s] = p[s];
  }
  return v;
}

// ---------------------------------------------------------------- weight stream heads
constexpr int WF = (OFF_WIDE + OFF_FWD) * 4;   // byte base of the forward wide fragments
constexpr int WB = (OFF_WIDE + OFF_BWD) * 4;   // ... of the transposed ones
constexpr int WBC = (OFF_WIDE + W_OFF_BCOL) * 4;
constexpr int WHW = (OFF_WIDE + W_OFF_G4W) * 4;
constexpr int WG4B = (OFF_WIDE + W_OFF_G4B) * 4;

// standard layer: step st = ot·KT + kt reads fragments (ot, kt, u = l); base is the layer's
// byte offset in the fp32 wide region.  x6: fragments (ot, kt, 3b + term) of the split copy
// BMR: the block-major copy (OFF_X6BM) that two-column x6 layers read when PNTF_X6_BM
template <bool BMR>
struct WHeadT {
  int base;
  __device__ int operator()(int j, int l) const {
#if PNTF_WIDE_X6
    return (BMR ? OFF_X6BM : OFF_X6) * 4 + (base - OFF_WIDE * 4) / 2 * 3 + (j * 6 + l) * 1024;
#else
    return base + (j * 4 + l) * 1024;
#endif
  }
};
typedef WHeadT<false> WHead;
typedef WHeadT<PNTF_WIDE_X6 && PNTF_X6_BM && !PNTF_X6_ACC> WHeadE;   // an encoder layer (two columns)
// fragments per step of whatever a step sequence hands over to (a WHead is always a wlayer)
struct WE0Head;
struct WFoldHead;
template <class F>
constexpr int wnext_nl();
// encoder[0] on Fourier features, k-tile outer: step st = kt·4 + ot (KT = 8)
// x6 (PNTF_X6_E0): the split copy of encoder[0] (κ-scaled like its fp32 fragments), whose
// two-column per-tile order is (ot·KT + kt) as well (PNTF_X6_G2 = 1)
#ifndef PNTF_X6_E0
#define PNTF_X6_E0 1
#endif
constexpr bool WE0X6 = PNTF_WIDE_X6 && PNTF_X6_E0;
constexpr int WE0NL = WE0X6 ? 6 : 4;   // fragments per encoder[0] step
static_assert(!WE0X6 || PNTF_X6_G2 == 1 || PNTF_X6_G2 == 4,
              "encoder[0]'s split copy in per-tile (G2 = 1) or step (G2 = 4) order");
struct WE0Head {
  __device__ int operator()(int j, int l) const {
    if constexpr (WE0X6 && PNTF_X6_G2 == 4)   // (kt, ot) order: the step order itself
      return OFF_X6 * 4 + (WF + OFF_E0 * 4 - OFF_WIDE * 4) / 2 * 3 + (j * 6 + l) * 1024;
    else if constexpr (WE0X6)
      return OFF_X6 * 4 + (WF + OFF_E0 * 4 - OFF_WIDE * 4) / 2 * 3 +
             ((((j % 4) * 8 + j / 4) * 6 + l) * 1024);
    else
      return WF + OFF_E0 * 4 + ((((j % 4) * 8 + j / 4) * 4 + l) * 1024);
  }
};
// reverse sweep head: generator[-2]^T (OT 8, KT 4)
__device__ __forceinline__ WHead wbwd_head() { return WHead{WB + OFF_G3 * 4}; }
// Fourier fold (encoder[0]^T, OT 8, KT 4): step st = (o·4 + kt)·2 + half reads out tile
// o + 4·half (sin rows o, cos rows o + 4)
// x6 (PNTF_X6_FOLD): the split copy of encoder[0]^T (per-tile order, as encoder[0]'s)
#ifndef PNTF_X6_FOLD
#define PNTF_X6_FOLD 0
#endif
constexpr bool WFX6 = PNTF_WIDE_X6 && PNTF_X6_FOLD;
constexpr int WFNL = WFX6 ? 6 : 4;   // fragments per fold step
static_assert(!WFX6 || PNTF_X6_G2 == 1, "encoder[0]^T's split copy in per-tile order");
struct WFoldHead {
  __device__ int operator()(int j, int l) const {
    const int o = j / 8, kt = (j / 2) % 4, half = j % 2;
    if constexpr (WFX6)
      return OFF_X6 * 4 + (WB + OFF_E0 * 4 - OFF_WIDE * 4) / 2 * 3 +
             ((((o + 4 * half) * 4 + kt) * 6 + l) * 1024);
    else
      return WB + OFF_E0 * 4 + ((((o + 4 * half) * 4 + kt) * 4 + l) * 1024);
  }
};
// Fourier fold on split-bf16 in the accumulate engine (PNTF_X6_ACC, PNTF_XFOLD): step
// S = (p·4 + kt)·4 + ot_local over two passes p of 4 out tiles (sin/cos rows of feature tiles
// 2p, 2p + 1); the split copy of encoder[0]^T is packed in this order (pack_x6_kernel)
#ifndef PNTF_XFOLD
#define PNTF_XFOLD 1
#endif
constexpr bool XFOLD = PNTF_WIDE_X6 && PNTF_X6_ACC && PNTF_XFOLD;
struct WFoldXHead {
  __device__ int operator()(int j, int l) const {
    return OFF_X6 * 4 + (WB + OFF_E0 * 4 - OFF_WIDE * 4) / 2 * 3 + (j * 6 + l) * 1024;
  }
};
template <class F>
constexpr int wnext_nl() {
  if constexpr (std::is_same<F, WFoldXHead>::value) return 6;
  if constexpr (std::is_same<F, WE0Head>::value) return WE0NL;
  else if constexpr (std::is_same<F, WFoldHead>::value) return WFNL;
  else return std::is_same<F, WHead>::value || std::is_same<F, WHeadE>::value ? WNL : 4;
}

// ---------------------------------------------------------------- generic wide layer
#if !PNTF_WIDE_X6
// One Linear layer over OT out tiles x KT input tiles, NC columns (points) sharing the
// weights; bank index of column c, tile t is c·OT + t (out) / c·KT + t (in).  Step st =
// (ot, kt) runs 16·NC MFMAs on the 4 fragments of (ot, kt).  ly.init(ot, acc) starts out
// tile ot (its bias MFMA, residual as C); ly.epi(ot, acc) finishes it — when L::DEFER, only
// after the first step of the next out tile has issued its MFMAs (the last tile's at once).
template <int OT, int KT, int NC, int SITE, int NLN, class L, class PreF, class NextF>
__device__ __forceinline__ void wlayer(Ring& ring, Rsrc W, int wbase, const f32x16 (&in)[8],
                                       int lane, L& ly, PreF pre, NextF naddr) {
  static_assert(NC * KT <= 8 && NC * OT <= 8, "bank size");
  static_assert(NLN == 4, "the next step sequence's width comes from its head type");
  constexpr int STEPS = OT * KT;
  constexpr bool DEF = L::DEFER;          // epilogue deferred past the next tile's first step
  f32x16 acc[DEF ? 2 : 1][NC];
  run_steps<STEPS, 4, wnext_nl<NextF>(), SITE>(
      ring, W, lane * 16, WHead{wbase}, naddr, [&](auto st, const f32x4 (&a)[4]) {
        constexpr int S = decltype(st)::value;
        constexpr int ot = S / KT, kt = S % KT, p = DEF ? (ot & 1) : 0;
        if constexpr (S == 0) ly.start();
        pre(st);
        if constexpr (kt == 0) ly.init(ot, acc[p]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int c = 0; c < NC; ++c)
              acc[p][c] = mfma32(a[u][s], in[c * KT + kt][4 * u + s], acc[p][c]);
        if constexpr (DEF) {
          if constexpr (kt == 0 && ot > 0) ly.epi(ot - 1, acc[p ^ 1]);
          if constexpr (S == STEPS - 1) ly.epi(ot, acc[p]);
        } else if constexpr (kt == KT - 1) {
          ly.epi(ot, acc[p]);
        }
      });
}

#else
// x6 layer: out tiles in groups of G (wx6_group); step (g, kt, o) runs the six split products
// of k blocks 0 and 1 of input tile kt for out tile g·G + o, so input tile kt is split once
// per group (at o = 0) instead of once per out tile, and G accumulators are live.  The
// fragments are packed in this step order (pack_x6_kernel).  ly.init(ot) starts tile ot at
// its group's kt = 0 (bias MFMA, residual; a reverse layer's σ tile load into out[ot]);
// ly.epi(ot) runs one step after the tile's last MFMAs (the last tile's at once).
template <int OT, int KT, int NC, int SITE, int NLN, class L, class PreF, class NextF>
__device__ __forceinline__ void wlayer(Ring& ring, Rsrc W, int wbase, const f32x16 (&in)[8],
                                       int lane, L& ly, PreF pre, NextF naddr) {
  static_assert(NC * KT <= 8 && NC * OT <= 8, "bank size");
  static_assert(NLN == 4, "the next step sequence's width comes from its head type");
  if constexpr (wx6_block_major(NC)) {
    // two-column layers (the encoder): step (g, kt, b) splits k block b of input tile kt once
    // and runs it against the G = 2 out tiles of group g (fragments 3o + term), so a step
    // holds one block's split (12 registers per column) and the split is shared by 2 tiles
    constexpr int G = 2, STEPS = OT * KT;
    static_assert(OT % G == 0 && 3 * G == 6, "block-major groups");
    f32x16 acc[G][NC];
    run_steps<STEPS, 6, wnext_nl<NextF>(), SITE>(
        ring, W, lane * 16, WHeadE{wbase}, naddr, [&](auto st, const f32x4 (&a)[6]) {
          constexpr int S = decltype(st)::value;
          constexpr int g = S / (2 * KT), kt = (S / 2) % KT, b = S % 2;
          if constexpr (S == 0) ly.start();
          pre(st);
          if constexpr (kt == 0 && b == 0) {
#pragma unroll
            for (int o = 0; o < G; ++o) ly.init(g * G + o, acc[o]);
          }
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            wbf16x8 xs[3];
            wx6_split<true>(in[c * KT + kt], b, xs);
#pragma unroll
            for (int o = 0; o < G; ++o)
              acc[o][c] = wx6_mma(a[3 * o], a[3 * o + 1], a[3 * o + 2], xs, acc[o][c]);
          }
          if constexpr (kt == KT - 1 && b == 1) {
#pragma unroll
            for (int o = 0; o < G; ++o) ly.epi(g * G + o, acc[o]);
          }
        });
    return;
  }
  constexpr int G = wx6_group(OT, NC), STEPS = OT * KT;
  static_assert(OT % G == 0, "out tile groups");
  // accumulator buffers: one per tile of the group (G = 1 with PNTF_X6_G1BUF = 2: two,
  // alternating per tile, so the deferred epilogue of the previous tile reads the other one;
  // with 1 the previous tile's epilogue runs before the next tile starts)
  constexpr int NB = G == 1 ? PNTF_X6_G1BUF : G;
  f32x16 acc[NB][NC];
  wbf16x8 xs[NC][2][3];
  run_steps<STEPS, 6, wnext_nl<NextF>(), SITE>(
      ring, W, lane * 16, WHead{wbase}, naddr, [&](auto st, const f32x4 (&a)[6]) {
        constexpr int S = decltype(st)::value;
        constexpr int g = S / (KT * G), kt = (S / G) % KT, oo = S % G, ot = g * G + oo;
        // accumulator buffer of this tile and of the previous group's last tile
        constexpr int o = G == 1 ? (g % NB) : oo, last = G == 1 ? ((g + 1) % NB) : G - 1;
        if constexpr (NB == 1 && kt == 0 && g > 0) ly.epi(ot - 1, acc[0]);
        if constexpr (S == 0) ly.start();
        pre(st);
        if constexpr (oo == 0) {   // the group's first tile: split input tile kt
#pragma unroll
          for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int b = 0; b < 2; ++b) wx6_split<true>(in[c * KT + kt], b, xs[c][b]);
        }
        if constexpr (kt == 0) ly.init(ot, acc[o]);
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int c = 0; c < NC; ++c)
            acc[o][c] = wx6_mma(a[3 * b], a[3 * b + 1], a[3 * b + 2], xs[c][b], acc[o][c]);
        if constexpr (G > 1 && kt == KT - 1 && oo > 0) ly.epi(ot - 1, acc[o - 1]);
        if constexpr (NB > 1 && kt == 0 && oo == 0 && g > 0) ly.epi(ot - 1, acc[last]);
        if constexpr (S == STEPS - 1) ly.epi(ot, acc[o]);
      });
}
#endif

// bias-column operands of a layer: fragment g holds out tiles 4g..4g+3 (lanes 0-31)
template <int OT>
struct BiasCols {
  f32x4 v[(OT + 3) / 4];
  __device__ __forceinline__ void load(Rsrc W, int lane, int plain_off) {
#pragma unroll
    for (int g = 0; g < (OT + 3) / 4; ++g)
      v[g] = bload(W, lane * 16, WBC + ((plain_off / 128 + g) * 64) * 16);
  }
  __device__ __forceinline__ float operator()(int ot) const { return v[ot / 4][ot % 4]; }
};

// forward Linear + softplus10: out = sp(A·in + b (+ out if RES)); σ10 saved when SAVE (to
// the scratch slot, or to LDS tiles sc0.. when IN_LDS)
template <int OT_, int KT_, int NC_, bool RES, bool SAVE, bool IN_LDS = false>
struct WFwdAct {
  static constexpr int OT = OT_, KT = KT_, NC = NC_;
  static constexpr bool DEFER = true;
  f32x16 (&out)[8];
  WScratch sc;
  int sc0, lane;
  BiasCols<OT_> bc;   // loaded by the caller one layer ahead
  WLds wl;
  __device__ __forceinline__ void start() {}
  __device__ __forceinline__ void init(int ot, f32x16 (&acc)[NC]) {
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = mfma32(bc(ot), 1.f, RES ? out[c * OT + ot] : zero16());
  }
  __device__ __forceinline__ void epi(int ot, const f32x16 (&acc)[NC]) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      f32x16 h, g;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        SpSig q = wsp_sig(acc[c][r]);
        h[r] = q.sp;
        g[r] = q.sg;
      }
      out[c * OT + ot] = h;
      if (SAVE && IN_LDS) lstore(wl, sc0 + c * OT + ot, g);
      else if (SAVE) wstore(sc, sc0 + c * OT + ot, lane, g);
    }
  }
};

// forward Linear without activation (encoder[-1], :234)
template <int OT_, int KT_, int NC_>
struct WFwdLin {
  static constexpr int OT = OT_, KT = KT_, NC = NC_;
  static constexpr bool DEFER = true;
  f32x16 (&out)[8];
  BiasCols<OT_> bc;
  __device__ __forceinline__ void start() {}
  __device__ __forceinline__ void init(int ot, f32x16 (&acc)[NC]) {
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[c] = mfma32(bc(ot), 1.f, zero16());
  }
  __device__ __forceinline__ void epi(int ot, const f32x16 (&acc)[NC]) {
#pragma unroll
    for (int c = 0; c < NC; ++c) out[c * OT + ot] = acc[c];
  }
};

// reverse: out = (A^T·in (+ out if RES)) ⊙ σ tile (if MUL).  Both banks are full here, so
// the σ tile is loaded into the out tile's own registers when the tile starts (its old value,
// the residual, is dead once it is the accumulator's start), KT steps of MFMAs before the
// epilogue multiplies it in place.  Not deferred (no second accumulator).  (Loading all of a
// layer's σ tiles at its start measured slower.)
template <int OT_, int KT_, int NC_, bool RES, bool MUL>
struct WBwd {
  static constexpr int OT = OT_, KT = KT_, NC = NC_;
  static constexpr bool DEFER = false;
  f32x16 (&out)[8];
  WScratch sc;
  int mul0, lane;
  __device__ __forceinline__ void start() {}
  __device__ __forceinline__ void init(int ot, f32x16 (&acc)[NC]) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      acc[c] = RES ? out[c * OT + ot] : zero16();
      if (MUL) out[c * OT + ot] = wload(sc, mul0 + c * OT + ot, lane);
    }
  }
  __device__ __forceinline__ void epi(int ot, const f32x16 (&acc)[NC]) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
      out[c * OT + ot] = MUL ? acc[c] * out[c * OT + ot] : acc[c];
  }
};

// env B reads (Fourier projections and fold) and head-row reads, each behind a hook for
// the tests/diag ablations (PNTF_ABL_NOBW / PNTF_ABL_NOHW: register stand-ins, wrong results)
__device__ __forceinline__ f32x4 wbw_load(const float* p) {
#ifdef PNTF_ABL_NOBW
  float v = 1e-3f * (float)(reinterpret_cast<uintptr_t>(p) & 255);
  asm volatile("v_mov_b32 %0, %0" : "+v"(v));
  return f32x4{v, v + 1e-4f, v + 2e-4f, v + 3e-4f};
#else
  return ld4(p);
#endif
}
// Where a lane reads its environment's B rows: global memory (any table), or the table staged
// in LDS once per workgroup when it fits (WBL_FLOATS; pntf_capi.hip picks the kernel).  The LDS
// reads take the Fourier projections' and the fold's B loads off the in-order vmcnt queue.
template <bool BL>
struct WBt {
  __device__ __forceinline__ f32x4 load(const PairIO& io, int i) const {
    return wbw_load(io.Bw + i);
  }
};
template <>
struct WBt<true> {
  const wlds_f* t;   // this lane's environment in the staged table
  __device__ __forceinline__ f32x4 load(const PairIO&, int i) const {
#ifdef PNTF_ABL_NOBW
    return wbw_load(reinterpret_cast<const float*>(static_cast<uintptr_t>(i)));
#else
    return *reinterpret_cast<const wlds_f4*>(t + i);
#endif
  }
};

// head-row features 32 t + 8 u + 4 h .. + 3 (the rows of registers 4u..4u+3 of tile t): an
// LDS broadcast read (half the lanes share each address).  From the packed blob these 16
// loads per pass were sunk to their use and each waited out an L2 round trip with the whole
// weight ring (vmcnt(0)); tests/diag ablation: -0.5 % kernel time.
__device__ __forceinline__ f32x4 whw_load(const WLds& wl, int t, int u, int h) {
#ifdef PNTF_ABL_NOHW
  float v = 1e-3f * (float)((t * 4 + u + h) & 255);
  asm volatile("v_mov_b32 %0, %0" : "+v"(v));
  return f32x4{v, v + 1e-4f, v + 2e-4f, v + 3e-4f};
#else
  return *reinterpret_cast<const wlds_f4*>(wl.hw + 32 * t + 8 * u + 4 * h);
#endif
}

// ---------------------------------------------------------------- Fourier projections
// q[c][r] = x_c · 2πB[:, 32 kt + row(r, h)] for the lane's 16 feature rows of Fourier tile
// kt, both points; the B rows come from the pair's environment (io.Bw, dim x 128).
template <int DIM, class BT>
__device__ __forceinline__ void wfourier_q(const PairIO& io, const BT& bt, int kt, int h,
                                           f32x16 (&q)[2]) {
#pragma unroll
  for (int c = 0; c < 2; ++c) q[c] = zero16();
#pragma unroll
  for (int d = 0; d < DIM; ++d)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      f32x4 b = bt.load(io, d * H + 32 * kt + 8 * u + 4 * h);
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int s = 0; s < 4; ++s) q[c][4 * u + s] = fmaf(io.x[c][d], TWO_PI * b[s], q[c][4 * u + s]);
    }
}

// ---------------------------------------------------------------- forward pass
// NN.out on 32 pairs.  GRAD: save σ tiles.  On entry the ring holds WE0Head; on return the
// first PF steps of `after`.  Returns τ of the lane's pair (same in both lane halves).
template <int DIM, bool GRAD, class BT, class AfterF>
__device__ __forceinline__ float wide_forward(Ring& ring, Rsrc W, const PairIO& io, BT bt,
                                              f32x16 (&X)[8], f32x16 (&Y)[8], WScratch sc,
                                              WLds wl, int compat, int lane, AfterF after) {
  const int h = lane >> 5;
  const float cm = compat ? 1.f : 0.f;

  // ---- encoder[0] (:186-190, :227), k-tile outer: X[c·4 + ot] accumulate 4 out tiles x 2
  // points; sin tiles (kt < 4) are computed at step (kt, 0), their cos partners (kt + 4)
  // kept in Y[c·4 + kt] until then.
  BiasCols<4> be0, a0bc;
  BiasCols<8> gbc;
  be0.load(W, lane, B_E0);
  {
    f32x16 q[2], sn[2];
    wfourier_q<DIM>(io, bt, 0, h, q);
    run_steps<32, WE0NL, WNL, SITE_FWD_E0>(
        ring, W, lane * 16, WE0Head{}, WHeadE{WF + OFF_EBLK * 4},
        [&](auto st, const f32x4 (&a)[WE0NL]) {
          constexpr int S = decltype(st)::value;
          constexpr int kt = S / 4, ot = S % 4;
          if constexpr (ot == 0 && kt < 4) {
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
              for (int r = 0; r < 16; ++r) {
                float x0, x1;
                sincos_fast(q[c][r], x0, x1);
                sn[c][r] = x0;
                Y[c * 4 + kt][r] = x1;
              }
          }
          if constexpr (kt == 0) {
#pragma unroll
            for (int c = 0; c < 2; ++c) X[c * 4 + ot] = mfma32(be0(ot), 1.f, zero16());
          }
          if constexpr (WE0X6) {
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
              for (int b = 0; b < 2; ++b) {
                wbf16x8 xs[3];
                wx6_split<true>(kt < 4 ? sn[c] : Y[c * 4 + (kt & 3)], b, xs);
                X[c * 4 + ot] = wx6_mma(a[3 * b], a[3 * b + 1], a[3 * b + 2], xs, X[c * 4 + ot]);
              }
          } else {
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
              for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                  float b;
                  if constexpr (kt < 4) b = sn[c][4 * u + s];
                  else b = Y[c * 4 + kt - 4][4 * u + s];
                  X[c * 4 + ot] = mfma32(a[u][s], b, X[c * 4 + ot]);
                }
          }
          // next sin/cos tile's projections, after this tile's MFMAs are issued
          if constexpr (ot == 3 && kt < 3) wfourier_q<DIM>(io, bt, kt + 1, h, q);
          if constexpr (S == 16) a0bc.load(W, lane, B_EBLK);
        });
  }
  // bias, softplus, σ (compat: the out_backgrad quirk :435-438 stores σ10(softplus(y)))
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    f32x16 s, g;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      SpSig v = wsp_sig(X[t][r]);
      s[r] = v.sp;
      g[r] = fmaf(cm, __builtin_amdgcn_rcpf(2.f - v.sg) - v.sg, v.sg);
    }
    X[t] = s;
    if (GRAD) wstore(sc, WT_E0 + t, lane, g);
  }

  // ---- encoder residual blocks (:228-232); X = h (2 points x 4 tiles).  Each layer's bias
  // columns are fetched at the first step of the layer before it.
  const int WE = WF + OFF_EBLK * 4;
  {
    WFwdAct<4, 4, 2, false, GRAD> a0{Y, sc, WT_EBLK, lane, {}};
    WFwdAct<4, 4, 2, true, GRAD> b0{X, sc, WT_EBLK + 8, lane, {}};
    WFwdAct<4, 4, 2, false, GRAD> a1{Y, sc, WT_EBLK + 16, lane, {}};
    WFwdAct<4, 4, 2, true, GRAD> b1{X, sc, WT_EBLK + 24, lane, {}};
    WFwdLin<4, 4, 2> e3{Y, {}};
    a0.bc = a0bc;
    wlayer<4, 4, 2, SITE_FWD_ENC, 4>(ring, W, WE, X, lane, a0,
                                     at<0>([&] { b0.bc.load(W, lane, B_EBLK + 128); }),
                                     WHeadE{WE + SZ_E * 4});
    wlayer<4, 4, 2, SITE_FWD_ENC, 4>(ring, W, WE + SZ_E * 4, Y, lane, b0,
                                     at<0>([&] { a1.bc.load(W, lane, B_EBLK + 256); }),
                                     WHeadE{WE + 2 * SZ_E * 4});
    wlayer<4, 4, 2, SITE_FWD_ENC, 4>(ring, W, WE + 2 * SZ_E * 4, X, lane, a1,
                                     at<0>([&] { b1.bc.load(W, lane, B_EBLK + 384); }),
                                     WHeadE{WE + 3 * SZ_E * 4});
    wlayer<4, 4, 2, SITE_FWD_ENC, 4>(ring, W, WE + 3 * SZ_E * 4, Y, lane, b1,
                                     at<0>([&] { e3.bc.load(W, lane, B_E3); }),
                                     WHeadE{WF + OFF_E3 * 4});
    // ---- encoder[-1] (:234) -> Y (zs = Y[0..3], zg = Y[4..7])
    wlayer<4, 4, 2, SITE_FWD_ENC, 4>(ring, W, WF + OFF_E3 * 4, X, lane, e3,
                                     at<0>([&] { gbc.load(W, lane, B_GBLK); }),
                                     WHead{WF + OFF_GBLK * 4});
  }

  // ---- symmetric smooth max / min merge (:236-244) -> X (u = [M | m], 8 tiles)
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    f32x16 s0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float zs = Y[t][r], zg = Y[4 + t][r];   // κ-scaled
      float d = zs - zg;
      float e = __builtin_amdgcn_exp2f(-fabsf(d));    // e^{-10|zs - zg|}
      float cc = __builtin_amdgcn_logf(1.f + e);      // κ·0.1·ln(1 + e)
      X[t][r] = fmaxf(zs, zg) + cc;
      X[4 + t][r] = fminf(zs, zg) - cc;
      float rr = __builtin_amdgcn_rcpf(1.f + e);
      s0[r] = (d >= 0.f) ? rr : e * rr;
    }
    if (GRAD) lstore(wl, WL_S0 + t, s0);
  }

  // ---- generator residual blocks (:246-249); X = u (8 tiles); gbc carries the next
  // layer's bias columns across the loop
#pragma unroll 1
  for (int i = 0; i < 3; ++i) {
    const int wa = opaque(WF + (OFF_GBLK + (2 * i) * SZ_G) * 4);
    const int wb = opaque(WF + (OFF_GBLK + (2 * i + 1) * SZ_G) * 4);
    const int wn = opaque(i < 2 ? WF + (OFF_GBLK + (2 * i + 2) * SZ_G) * 4 : WF + OFF_G3 * 4);
    const int bo = opaque(B_GBLK + (2 * i) * 256);
    const int bn = opaque(i < 2 ? B_GBLK + (2 * i + 2) * 256 : B_G3);
    WFwdAct<8, 8, 1, false, GRAD> ga{Y, sc, WT_GBLK + 16 * i, lane, gbc};
    WFwdAct<8, 8, 1, true, GRAD> gb{X, sc, WT_GBLK + 16 * i + 8, lane, {}};
    wlayer<8, 8, 1, SITE_FWD_GEN, 4>(ring, W, wa, X, lane, ga,
                                     at<0>([&] { gb.bc.load(W, lane, bo + 256); }),
                                     WHead{wb});
    wlayer<8, 8, 1, SITE_FWD_GEN, 4>(ring, W, wb, Y, lane, gb,
                                     at<0>([&] { gbc.load(W, lane, bn); }), WHead{wn});
  }
  // ---- generator[-2] + act (:251-252) -> Y[0..3] (its bias columns: gbc's first 4 tiles)
  {
    WFwdAct<4, 8, 1, false, GRAD, true> g3{Y, sc, WL_G3, lane, {}, wl};
    g3.bc.v[0] = gbc.v[0];
    wlayer<4, 8, 1, SITE_FWD_GEN, 4>(ring, W, WF + OFF_G3 * 4, X, lane, g3, NoPre{}, after);
  }
  // ---- head generator[-1] + sigmoid(0.1 y) (:254-255)
  float part = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      f32x4 w = whw_load(wl, t, u, h);
#pragma unroll
      for (int s = 0; s < 4; ++s) part = fmaf(w[s], Y[t][4 * u + s], part);
    }
  part += __shfl_xor(part, 32);
  const float y4 = fmaf(part, WKAPPA_INV, bload(W, 0, WG4B)[0]);   // part = κ·(g4w·h3)
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-0.144269504088896341f * y4));
}

// ---- encoder[0]^T (256 x 128: OT 8, KT 4) fused with the Fourier Jacobian (:639-645), the
// last phase of the reverse sweep; Y holds dL/d(encoder[0] output) (2 points x 4 tiles).
template <int DIM, class BT, class AfterF>
__device__ __forceinline__ void wide_fold(Ring& ring, Rsrc W, const PairIO& io, BT bt,
                                          const f32x16 (&Y)[8], int lane, float (&ds)[DIM],
                                          float (&dg)[DIM], AfterF after) {
  const int h = lane >> 5;
  // Feature tile o pairs sin rows (out tile o) with cos rows (out tile o + 4) of the same q;
  // step (o, kt, half) accumulates half's out tile; after (o, 3, 1) the tile pair folds
  //   dτ/dx_c += Σ_rows 2πB[:, f] (dφ_sin cos q_f - dφ_cos sin q_f)
  float acc[2][DIM];
#pragma unroll
  for (int d = 0; d < DIM; ++d) acc[0][d] = acc[1][d] = 0.f;
  f32x16 ph[2][2];   // [sin | cos rows][point]
  run_steps<32, WFNL, wnext_nl<AfterF>(), SITE_FOLD>(
      ring, W, lane * 16, WFoldHead{}, after, [&](auto st, const f32x4 (&a)[WFNL]) {
        constexpr int S = decltype(st)::value;
        constexpr int o = S / 8, kt = (S / 2) % 4, half = S % 2;
        if constexpr (kt == 0) {
#pragma unroll
          for (int c = 0; c < 2; ++c) ph[half][c] = zero16();
        }
        if constexpr (WFX6) {
          // (split per step: keeping it for the second half spills)
#pragma unroll
          for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
              wbf16x8 xs[3];
              wx6_split<true>(Y[c * 4 + kt], b, xs);
              ph[half][c] = wx6_mma(a[3 * b], a[3 * b + 1], a[3 * b + 2], xs, ph[half][c]);
            }
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
              for (int c = 0; c < 2; ++c)
                ph[half][c] = mfma32(a[u][s], Y[c * 4 + kt][4 * u + s], ph[half][c]);
        }
        if constexpr (kt == 3 && half == 1) {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            f32x4 bw[DIM];
#pragma unroll
            for (int d = 0; d < DIM; ++d) bw[d] = TWO_PI * bt.load(io, d * H + 32 * o + 8 * u + 4 * h);
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
              for (int s = 0; s < 4; ++s) {
                float q = 0.f;
#pragma unroll
                for (int d = 0; d < DIM; ++d) q = fmaf(io.x[c][d], bw[d][s], q);
                float sn, cs;
                sincos_fast(q, sn, cs);
                const int r = 4 * u + s;
                float gg = ph[0][c][r] * cs - ph[1][c][r] * sn;
#pragma unroll
                for (int d = 0; d < DIM; ++d) acc[c][d] = fmaf(bw[d][s], gg, acc[c][d]);
              }
          }
        }
      });
#pragma unroll
  for (int d = 0; d < DIM; ++d) {
    ds[d] = acc[0][d] + __shfl_xor(acc[0][d], 32);
    dg[d] = acc[1][d] + __shfl_xor(acc[1][d], 32);
  }
}

// ---------------------------------------------------------------- reverse sweep
// Exact reverse mode (or out_backgrad when the forward stored the quirk).  On entry the ring
// holds wbwd_head(); on return the first PF steps of `after`.  ds/dg: dτ/dxs, dτ/dxg of the
// lane's pair (same in both halves).
template <int DIM, class BT, class AfterF>
__device__ __forceinline__ void wide_backward(Ring& ring, Rsrc W, const PairIO& io, BT bt,
                                              float tau, f32x16 (&X)[8], f32x16 (&Y)[8],
                                              WScratch sc,
                                              WLds wl, int lane, float (&ds)[DIM],
                                              float (&dg)[DIM], AfterF after) {
  const int h = lane >> 5;
  // ---- head and generator[-2] (:592-613): Y[t] = d · g4w ⊙ σ10(y3)
  const float dd = 0.1f * tau * (1.f - tau);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    f32x16 s3 = lload(wl, WL_G3 + t);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      f32x4 w = whw_load(wl, t, u, h);
#pragma unroll
      for (int s = 0; s < 4; ++s) Y[t][4 * u + s] = (dd * w[s]) * s3[4 * u + s];
    }
  }
  // du = G3^T dv ⊙ σ10(y2 of generator block 2) -> X   (G3^T: 256 x 128, OT 8, KT 4)
  {
    WBwd<8, 4, 1, false, true> l{X, sc, WT_GBLK + 16 * 2 + 8, lane};
    wlayer<8, 4, 1, SITE_BWD_GEN, 4>(ring, W, WB + OFF_G3 * 4, Y, lane, l, NoPre{},
                                     WHead{WB + (OFF_GBLK + 5 * SZ_G) * 4});
  }
  // ---- generator blocks, reverse (:615-618): blocks 2 and 1 in a loop, block 0 peeled (its
  // second layer multiplies by no σ and hands over to encoder[-1]^T)
#pragma unroll 1
  for (int i = 2; i >= 1; --i) {
    const int wa = opaque(WB + (OFF_GBLK + (2 * i) * SZ_G) * 4);
    const int wb = opaque(WB + (OFF_GBLK + (2 * i + 1) * SZ_G) * 4);
    const int wn = opaque(WB + (OFF_GBLK + (2 * i - 1) * SZ_G) * 4);
    // da = (G1_i^T dr) ⊙ σ10(y1_i) -> Y
    WBwd<8, 8, 1, false, true> lb{Y, sc, WT_GBLK + 16 * i, lane};
    wlayer<8, 8, 1, SITE_BWD_GEN, 4>(ring, W, wb, X, lane, lb, NoPre{}, WHead{wa});
    // du = G_i^T da + dr, then ⊙ σ10(y2_{i-1})
    WBwd<8, 8, 1, true, true> la{X, sc, WT_GBLK + 16 * (i - 1) + 8, lane};
    wlayer<8, 8, 1, SITE_BWD_GEN, 4>(ring, W, wa, Y, lane, la, NoPre{}, WHead{wn});
  }
  {
    WBwd<8, 8, 1, false, true> lb{Y, sc, WT_GBLK, lane};
    wlayer<8, 8, 1, SITE_BWD_GEN, 4>(ring, W, WB + (OFF_GBLK + 1 * SZ_G) * 4, X, lane, lb,
                                     NoPre{}, WHead{WB + OFF_GBLK * 4});
    WBwd<8, 8, 1, true, false> la{X, sc, 0, lane};
    wlayer<8, 8, 1, SITE_BWD_GEN, 4>(ring, W, WB + OFF_GBLK * 4, Y, lane, la, NoPre{},
                                     WHeadE{WB + OFF_E3 * 4});
  }
  // ---- merge Jacobian (:620-627): X[0..3] = dzs, X[4..7] = dzg
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    f32x16 s0 = lload(wl, WL_S0 + t);
    f32x16 s1 = 1.f - s0;
    f32x16 dM = X[t], dm = X[4 + t];
    X[t] = s0 * dM + s1 * dm;
    X[4 + t] = s1 * dM + s0 * dm;
  }
  // ---- encoder[-1]^T ⊙ σ10(y2 of encoder block 1), then the blocks, reverse (:629-636)
  const int WE = WB + OFF_EBLK * 4;
  {
    WBwd<4, 4, 2, false, true> e3{Y, sc, WT_EBLK + 24, lane};
    wlayer<4, 4, 2, SITE_BWD_ENC, 4>(ring, W, WB + OFF_E3 * 4, X, lane, e3, NoPre{},
                                     WHeadE{WE + 3 * SZ_E * 4});
    WBwd<4, 4, 2, false, true> b1{X, sc, WT_EBLK + 16, lane};
    wlayer<4, 4, 2, SITE_BWD_ENC, 4>(ring, W, WE + 3 * SZ_E * 4, Y, lane, b1, NoPre{},
                                     WHeadE{WE + 2 * SZ_E * 4});
    WBwd<4, 4, 2, true, true> a1{Y, sc, WT_EBLK + 8, lane};
    wlayer<4, 4, 2, SITE_BWD_ENC, 4>(ring, W, WE + 2 * SZ_E * 4, X, lane, a1, NoPre{},
                                     WHeadE{WE + 1 * SZ_E * 4});
    WBwd<4, 4, 2, false, true> b0{X, sc, WT_EBLK, lane};
    wlayer<4, 4, 2, SITE_BWD_ENC, 4>(ring, W, WE + 1 * SZ_E * 4, Y, lane, b0, NoPre{},
                                     WHeadE{WE});
    WBwd<4, 4, 2, true, true> a0{Y, sc, WT_E0, lane};
    wlayer<4, 4, 2, SITE_BWD_ENC, 4>(ring, W, WE, X, lane, a0, NoPre{}, WFoldHead{});
  }

  // ---- encoder[0]^T (256 x 128: OT 8, KT 4) fused with the Fourier Jacobian (:639-645).
  // Feature tile o pairs sin rows (out tile o) with cos rows (out tile o + 4) of the same q;
  // step (o, kt, half) accumulates half's out tile; after (o, 3, 1) the tile pair folds
  //   dτ/dx_c += Σ_rows 2πB[:, f] (dφ_sin cos q_f - dφ_cos sin q_f)
  float acc[2][DIM];
#pragma unroll
  for (int d = 0; d < DIM; ++d) acc[0][d] = acc[1][d] = 0.f;
  f32x16 ph[2][2];   // [sin | cos rows][point]
  run_steps<32, WFNL, wnext_nl<AfterF>(), SITE_FOLD>(
      ring, W, lane * 16, WFoldHead{}, after, [&](auto st, const f32x4 (&a)[WFNL]) {
        constexpr int S = decltype(st)::value;
        constexpr int o = S / 8, kt = (S / 2) % 4, half = S % 2;
        if constexpr (kt == 0) {
#pragma unroll
          for (int c = 0; c < 2; ++c) ph[half][c] = zero16();
        }
        if constexpr (WFX6) {
          // (split per step: keeping it for the second half spills)
#pragma unroll
          for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int b = 0; b < 2; ++b) {
              wbf16x8 xs[3];
              wx6_split<true>(Y[c * 4 + kt], b, xs);
              ph[half][c] = wx6_mma(a[3 * b], a[3 * b + 1], a[3 * b + 2], xs, ph[half][c]);
            }
        } else {
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
              for (int c = 0; c < 2; ++c)
                ph[half][c] = mfma32(a[u][s], Y[c * 4 + kt][4 * u + s], ph[half][c]);
        }
        if constexpr (kt == 3 && half == 1) {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            f32x4 bw[DIM];
#pragma unroll
            for (int d = 0; d < DIM; ++d) bw[d] = TWO_PI * bt.load(io, d * H + 32 * o + 8 * u + 4 * h);
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
              for (int s = 0; s < 4; ++s) {
                float q = 0.f;
#pragma unroll
                for (int d = 0; d < DIM; ++d) q = fmaf(io.x[c][d], bw[d][s], q);
                float sn, cs;
                sincos_fast(q, sn, cs);
                const int r = 4 * u + s;
                float gg = ph[0][c][r] * cs - ph[1][c][r] * sn;
#pragma unroll
                for (int d = 0; d < DIM; ++d) acc[c][d] = fmaf(bw[d][s], gg, acc[c][d]);
              }
          }
        }
      });
#pragma unroll
  for (int d = 0; d < DIM; ++d) {
    ds[d] = acc[0][d] + __shfl_xor(acc[0][d], 32);
    dg[d] = acc[1][d] + __shfl_xor(acc[1][d], 32);
  }
}

#if PNTF_WIDE_X6 && PNTF_X6_ACC
// ================================================================ accumulate-in-bank layers
// Round 6.  The round-5 x6 layers issued their VALU in bursts the MFMAs
// could not shadow: each group's input split right before the MFMAs that read it, and each out
// tile's whole softplus/σ epilogue in one step (gfx950: a v_mfma_f32_32x32x16_bf16 leaves 24 of
// its 32 cycles to independent VALU of the same wave, MI355X_MICROARCH.md; a step whose VALU
// exceeds that serialises).  Here:
//   * the out bank is the accumulator: out tile ot of the layer IS the MFMA C/D (the residual
//     is its initial value, the bias one fp32 MFMA at kt = 0), so no accumulator registers are
//     needed beside the two banks and every layer's out tiles form ONE group — each input tile
//     is split once per layer (round 5: twice in the generator, 2-4 times in the encoder);
//   * steps (kt, ot), ot fastest; the split of input tile kt + 1 (one-column layers) runs
//     inside the OT steps of tile kt, one k block at a time, into the other half of a double
//     buffer;
//   * the epilogue runs in CHUNKS (4 registers of one out tile and column: the softplus/σ of 4
//     elements and their 16-byte σ store, or the reverse sweep's σ multiply with its 16-byte
//     σ load issued PDS steps ahead), CPS chunks per step from the step after the first out
//     tile is final; the chunks that do not fit in the layer's last steps run in the first
//     steps of the NEXT layer (its pre hook, XPend), each before that layer splits the tile.
// Chunk j (tile t = j / (4 NC), column c = (j / 4) % NC, part q = j % 4) runs at step
// E(j) = STEPS - OT + 1 + j / CPS of the layer (>= STEPS: the next layer's step E - STEPS).
template <class L>
struct XSched {
  static constexpr int STEPS = L::OT * L::KT;
  static constexpr int E(int j) { return STEPS - L::OT + 1 + j / L::CPS; }
  static constexpr int P(int j) { return E(j) - L::PDS; }   // its σ prefetch (reverse)
};
// the chunks (and prefetches) of layer ly due at its step S (S >= STEPS: in the next layer)
template <class L, int S>
__device__ __forceinline__ void xdue(L& ly) {
  if constexpr (L::NCH > 0) {
    static_for<0, L::NCH>([&](auto jj) {
      constexpr int j = decltype(jj)::value;
      if constexpr (L::PF && XSched<L>::P(j) == S) ly.prefetch(j);
    });
    static_for<0, L::NCH>([&](auto jj) {
      constexpr int j = decltype(jj)::value;
      if constexpr (XSched<L>::E(j) == S) ly.chunk(j);
    });
  }
}
// the previous layer's pending chunks as the next layer's pre hook
// diagnostics (PNTF_XNOPEND bit 0: forward layers, bit 1: reverse layers): no chunk crosses into
// the next layer (xlayer flushes its pending chunks at its end)
#ifndef PNTF_XNOPEND
#define PNTF_XNOPEND 0
#endif
template <class L>
struct XPend {
  L& ly;
  template <class ST>
  __device__ __forceinline__ void operator()(ST) const {
    if constexpr (!(PNTF_XNOPEND & (L::PF ? 2 : 1))) xdue<L, XSched<L>::STEPS + ST::value>(ly);
  }
};
// ... or all at once (before a phase that reads the whole bank): the remaining virtual steps
// in order, so that the σ prefetch ring never holds more than its NSLOT quads (issuing every
// pending prefetch first overwrote slots before their chunks read them)
template <class L>
__device__ __forceinline__ void xflush(L& ly) {
  if constexpr (L::NCH > 0) {
    constexpr int S0 = XSched<L>::STEPS, S1 = XSched<L>::E(L::NCH - 1) + 1;
    if constexpr (S1 > S0)
      static_for<S0, S1>([&](auto ss) { xdue<L, decltype(ss)::value>(ly); });
  }
}

// split double buffer of one-column layers, and where in the OT steps of input tile kt the
// two k blocks of tile kt + 1 are split
#ifndef PNTF_X6_PIPE
#define PNTF_X6_PIPE 0
#endif
// encoder[0]: its input tile split once per kt and shared by the 4 out tiles (0: per step)
#ifndef PNTF_XE0SHARE
#define PNTF_XE0SHARE 1
#endif
// Banks in the AGPR file: each accumulated out tile passes an empty asm with an AGPR operand
// (the VGPR file then holds the ring, the splits and the epilogue's temporaries; the chunks
// and splits read a bank through v_accvgpr_read).  Both banks VALU-written in the VGPR file,
// as the compiler otherwise chooses, leaves no VGPRs for the rest (spills).
#ifndef PNTF_XAGPR
#define PNTF_XAGPR 2
#endif
__device__ __forceinline__ void xagpr(f32x16& t) {
#if PNTF_XAGPR
  asm("" : "+a"(t));
#endif
}
__device__ __forceinline__ void xvgpr(f32x16& t) { asm("" : "+v"(t)); }
// Each input tile is split once per layer here, so nothing invites the compiler to keep a
// split bank live; the opaque copy of wx6_split (round 5) only costs moves (PNTF_XOPQ = 1 keeps it)
#ifndef PNTF_XOPQ
#define PNTF_XOPQ 0
#endif
constexpr bool XOPQ = PNTF_XOPQ;
// sched_group_barrier interleave per step: (1 MFMA, XIGLP VALU) x MFMAs (0: off)
#ifndef PNTF_XIGLP
#define PNTF_XIGLP 0
#endif

// One Linear layer on split-bf16 MFMA, accumulating in ly.out (bank index c·OT + ot), input
// bank `in` (c·KT + kt).  ly.init(ot) starts out tile ot at kt = 0 (bias MFMA / residual /
// zero); ly's chunks run as above; pre(st) runs first in every step (the previous layer's
// pending chunks, loads for the next layer).
template <int OT, int KT, int NC, int SITE, bool IN_X, class L, class PreF, class NextF>
__device__ __forceinline__ void xlayer(Ring& ring, Rsrc W, int wbase, f32x16 (&in)[8],
                                       int lane, L& ly, PreF pre, NextF naddr) {
  static_assert(NC * KT <= 8 && NC * OT <= 8, "bank size");
  static_assert(L::OT == OT && L::KT == KT && L::NC == NC, "layer object shape");
  constexpr int STEPS = OT * KT;
  constexpr bool PIPE = NC == 1 && PNTF_X6_PIPE;
  constexpr int SB0 = OT / 4, SB1 = (3 * OT) / 4;   // split steps of blocks 0 / 1 of tile kt+1
  wbf16x8 xs[PIPE ? 2 : 1][NC][2][3];
  run_steps<STEPS, 6, wnext_nl<NextF>(), SITE>(
      ring, W, lane * 16, WHead{wbase}, naddr, [&](auto st, const f32x4 (&a)[6]) {
        constexpr int S = decltype(st)::value;
        constexpr int kt = S / OT, ot = S % OT, p = PIPE ? (kt & 1) : 0;
        pre(st);
        if constexpr (ot == 0 && (kt == 0 || !PIPE)) {
#pragma unroll
          for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int b = 0; b < 2; ++b) wx6_split<XOPQ>(in[c * KT + kt], b, xs[p][c][b]);
        }
        if constexpr (kt == 0) ly.init(ot);
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int c = 0; c < NC; ++c)
            ly.out[c * OT + ot] = wx6_mma(a[3 * b], a[3 * b + 1], a[3 * b + 2], xs[p][c][b],
                                          ly.out[c * OT + ot]);
#if PNTF_XAGPR != 3
#pragma unroll
        for (int c = 0; c < NC; ++c) xagpr(ly.out[c * OT + ot]);
#endif
#if PNTF_XAGPR == 2
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          xagpr(in[t]);
          xagpr(ly.out[t]);
        }
#elif PNTF_XAGPR == 3
        // bank X in the VGPR file, bank Y in the AGPR file: a layer reading X splits without
        // AGPR reads, one accumulating into X runs its epilogue chunks without AGPR moves
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          if constexpr (IN_X) {
            xvgpr(in[t]);
            xagpr(ly.out[t]);
          } else {
            xagpr(in[t]);
            xvgpr(ly.out[t]);
          }
        }
#endif
        if constexpr (PIPE && kt + 1 < KT) {
          if constexpr (ot == SB0) wx6_split<XOPQ>(in[kt + 1], 0, xs[p ^ 1][0][0]);
          if constexpr (ot == SB1) wx6_split<XOPQ>(in[kt + 1], 1, xs[p ^ 1][0][1]);
        }
        xdue<L, S>(ly);
#if PNTF_XIGLP > 0
        static_for<0, 12 * NC>([&](auto) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, PNTF_XIGLP, 0);
        });
#endif
      });
  if constexpr ((PNTF_XNOPEND & (L::PF ? 2 : 1)) != 0) xflush(ly);
}

// ---- layer objects: OT, KT, NC; CPS chunks per step; NCH chunks; PF/PDS: σ prefetch
// forward Linear + softplus10: out = sp(A·in + b (+ out if RES)); σ10 saved when SAVE (scratch
// tile sc0 + c·OT + t, or LDS tiles when IN_LDS); ACT0: encoder[0]'s compat quirk (:435-438)
template <int OT_, int KT_, int NC_, bool RES, bool SAVE, bool IN_LDS = false, bool ACT0 = false>
struct XFwdAct {
  static constexpr int OT = OT_, KT = KT_, NC = NC_, CPS = NC_, NCH = NC_ * OT_ * 4, PDS = 0;
  static constexpr bool PF = false;
  f32x16 (&out)[8];
  WScratch sc;
  int sc0, lane;
  BiasCols<OT_> bc;
  WLds wl;
  float cm;   // ACT0: 1 in compat mode
  __device__ __forceinline__ void init(int ot) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
      out[c * OT + ot] = mfma32(bc(ot), 1.f, RES ? out[c * OT + ot] : zero16());
  }
  __device__ __forceinline__ void prefetch(int) {}
  __device__ __forceinline__ void chunk(int j) {
    const int t = j / (4 * NC), c = (j / 4) % NC, q = j % 4;
    f32x4 g;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const SpSig v = wsp_sig(out[c * OT + t][4 * q + s]);
      out[c * OT + t][4 * q + s] = v.sp;
      g[s] = ACT0 ? fmaf(cm, __builtin_amdgcn_rcpf(2.f - v.sg) - v.sg, v.sg) : v.sg;
    }
    if constexpr (SAVE && IN_LDS) wl.p[((sc0 + c * OT + t) * 4 + q) * 64] = g;
    else if constexpr (SAVE) bstore<PNTF_WSTORE_AUX>(sc.r, g, lane * 16, (sc0 + c * OT + t) * 4096 + q * 1024);
  }
};
// forward Linear without activation (encoder[-1], :234): nothing pending
template <int OT_, int KT_, int NC_>
struct XFwdLin {
  static constexpr int OT = OT_, KT = KT_, NC = NC_, CPS = 1, NCH = 0, PDS = 0;
  static constexpr bool PF = false;
  f32x16 (&out)[8];
  BiasCols<OT_> bc;
  __device__ __forceinline__ void init(int ot) {
#pragma unroll
    for (int c = 0; c < NC; ++c) out[c * OT + ot] = mfma32(bc(ot), 1.f, zero16());
  }
  __device__ __forceinline__ void prefetch(int) {}
  __device__ __forceinline__ void chunk(int) {}
};
// reverse: out = (A^T·in (+ out if RES)) ⊙ σ tile mul0 + c·OT + t (if MUL); each chunk's σ part
// is loaded PDS steps ahead into a ring of NSLOT registers quads
#ifndef PNTF_XPDS
#define PNTF_XPDS 3
#endif
template <int OT_, int KT_, int NC_, bool RES, bool MUL>
struct XBwd {
  static constexpr int OT = OT_, KT = KT_, NC = NC_, CPS = NC_, NCH = MUL ? NC_ * OT_ * 4 : 0;
  static constexpr int PDS = PNTF_XPDS, NSLOT = CPS * (PDS + 1);
  static constexpr bool PF = MUL;
  f32x16 (&out)[8];
  WScratch sc;
  int mul0, lane;
  f32x4 sg[NSLOT];
  __device__ __forceinline__ void init(int ot) {
    if constexpr (!RES) {
#pragma unroll
      for (int c = 0; c < NC; ++c) out[c * OT + ot] = zero16();
    }
  }
  __device__ __forceinline__ void prefetch(int j) {
    const int t = j / (4 * NC), c = (j / 4) % NC, q = j % 4;
    sg[j % NSLOT] = __builtin_bit_cast(
        f32x4, __builtin_amdgcn_raw_buffer_load_b128(sc.r, lane * 16,
                                                     (mul0 + c * OT + t) * 4096 + q * 1024,
                                                     AUX_LOAD));
  }
  __device__ __forceinline__ void chunk(int j) {
    const int t = j / (4 * NC), c = (j / 4) % NC, q = j % 4;
#pragma unroll
    for (int s = 0; s < 4; ++s) out[c * OT + t][4 * q + s] *= sg[j % NSLOT][s];
  }
};

// the split-bf16 fold in the kernels that stage the env-B table in LDS (the headline's); the
// global-table instantiations keep the fp32 fold, whose registers fit beside their B pointers
template <class BT>
constexpr bool xfold() { return XFOLD && std::is_same<BT, WBt<true>>::value; }

// ---------------------------------------------------------------- Fourier fold (x6 acc)
// encoder[0]^T on split-bf16 MFMA fused with the Fourier Jacobian (:639-645).  Two passes; in
// pass p the four out tiles sin(o), cos(o) for o = 2p, 2p + 1 accumulate in X (dead here:
// X[c·4 + ot_local]) over the 4 input tiles of Y, each input tile split once per pass and
// shared by the 4 tiles; after the pass the two feature tiles fold into dτ/dx_c as wide_fold.
template <int DIM, class BT, class AfterF>
__device__ __forceinline__ void wide_fold_x(Ring& ring, Rsrc W, const PairIO& io, BT bt,
                                            f32x16 (&X)[8], f32x16 (&Y)[8], int lane,
                                            float (&ds)[DIM], float (&dg)[DIM], AfterF after) {
  const int h = lane >> 5;
  float acc[2][DIM];
#pragma unroll
  for (int d = 0; d < DIM; ++d) acc[0][d] = acc[1][d] = 0.f;
  wbf16x8 xs[2][2][3];
  run_steps<32, 6, wnext_nl<AfterF>(), SITE_FOLD>(
      ring, W, lane * 16, WFoldXHead{}, after, [&](auto st, const f32x4 (&a)[6]) {
        constexpr int S = decltype(st)::value;
        constexpr int p = S / 16, kt = (S / 4) % 4, otl = S % 4;
        if constexpr (otl == 0) {
#pragma unroll
          for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int b = 0; b < 2; ++b) wx6_split<XOPQ>(Y[c * 4 + kt], b, xs[c][b]);
        }
        if constexpr (kt == 0) {
#pragma unroll
          for (int c = 0; c < 2; ++c) X[c * 4 + otl] = zero16();
        }
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int c = 0; c < 2; ++c)
            X[c * 4 + otl] = wx6_mma(a[3 * b], a[3 * b + 1], a[3 * b + 2], xs[c][b], X[c * 4 + otl]);
#if PNTF_XAGPR == 3
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          xvgpr(X[t]);
          xagpr(Y[t]);
        }
#else
#pragma unroll
        for (int c = 0; c < 2; ++c) xagpr(X[c * 4 + otl]);
#endif
#if PNTF_XAGPR == 2
#pragma unroll
        for (int t = 0; t < 8; ++t) xagpr(Y[t]);   // both banks in the AGPR file (as xlayer)
#endif
        // after the pass: feature tiles o = 2p + ol, sin rows X[c·4 + 2 ol], cos X[c·4 + 2 ol + 1]
        if constexpr (kt == 3 && otl == 3) {
#pragma unroll
          for (int ol = 0; ol < 2; ++ol) {
            const int o = 2 * p + ol;
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              f32x4 bw[DIM];
#pragma unroll
              for (int d = 0; d < DIM; ++d)
                bw[d] = TWO_PI * bt.load(io, d * H + 32 * o + 8 * u + 4 * h);
#pragma unroll
              for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                  float q = 0.f;
#pragma unroll
                  for (int d = 0; d < DIM; ++d) q = fmaf(io.x[c][d], bw[d][s], q);
                  float sn, cs;
                  sincos_fast(q, sn, cs);
                  const int r = 4 * u + s;
                  const float gg = X[c * 4 + 2 * ol][r] * cs - X[c * 4 + 2 * ol + 1][r] * sn;
#pragma unroll
                  for (int d = 0; d < DIM; ++d) acc[c][d] = fmaf(bw[d][s], gg, acc[c][d]);
                }
            }
          }
        }
      });
#pragma unroll
  for (int d = 0; d < DIM; ++d) {
    ds[d] = acc[0][d] + __shfl_xor(acc[0][d], 32);
    dg[d] = acc[1][d] + __shfl_xor(acc[1][d], 32);
  }
}

// ---------------------------------------------------------------- forward pass (x6 acc)
// As wide_forward; the encoder[0] epilogue and every layer's run as chunks (above).
template <int DIM, bool GRAD, class BT, class AfterF>
__device__ __forceinline__ float wide_forward_x(Ring& ring, Rsrc W, const PairIO& io, BT bt,
                                                f32x16 (&X)[8], f32x16 (&Y)[8], WScratch sc,
                                                WLds wl, int compat, int lane, AfterF after) {
  const int h = lane >> 5;
  // ---- encoder[0] (:186-190, :227), k-tile outer: X[c·4 + ot] accumulate 4 out tiles x 2
  // points; sin tiles (kt < 4) are computed at step (kt, 0), their cos partners (kt + 4)
  // kept in Y[c·4 + kt] until then; the input tile (sin or cos) is split once per kt and
  // shared by the 4 out tiles
  XFwdAct<4, 8, 2, false, GRAD, false, true> e0{X, sc, WT_E0, lane, {}, wl, compat ? 1.f : 0.f};
  e0.bc.load(W, lane, B_E0);
  XFwdAct<4, 4, 2, false, GRAD> a0{Y, sc, WT_EBLK, lane, {}, wl, 0.f};
  {
    f32x16 q[2], sn[2];
    wbf16x8 xs[2][2][3];
    wfourier_q<DIM>(io, bt, 0, h, q);
    run_steps<32, WE0NL, WNL, SITE_FWD_E0>(
        ring, W, lane * 16, WE0Head{}, WHead{WF + OFF_EBLK * 4},
        [&](auto st, const f32x4 (&a)[WE0NL]) {
          constexpr int S = decltype(st)::value;
          constexpr int kt = S / 4, ot = S % 4;
          if constexpr (ot == 0 && kt < 4) {
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
              for (int r = 0; r < 16; ++r) {
                float x0, x1;
                sincos_fast(q[c][r], x0, x1);
                sn[c][r] = x0;
                Y[c * 4 + kt][r] = x1;
              }
          }
          if constexpr (ot == 0 || !PNTF_XE0SHARE) {
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
              for (int b = 0; b < 2; ++b)
                wx6_split<XOPQ>(kt < 4 ? sn[c] : Y[c * 4 + (kt & 3)], b, xs[c][b]);
          }
          if constexpr (kt == 0) e0.init(ot);
#pragma unroll
          for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int c = 0; c < 2; ++c)
              X[c * 4 + ot] = wx6_mma(a[3 * b], a[3 * b + 1], a[3 * b + 2], xs[c][b], X[c * 4 + ot]);
#if PNTF_XAGPR == 3
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            xvgpr(X[t]);
            if (kt >= 4 || t % 4 < kt) xagpr(Y[t]);
          }
#endif
#if PNTF_XAGPR != 3
#pragma unroll
          for (int c = 0; c < 2; ++c) xagpr(X[c * 4 + ot]);
#endif
#if PNTF_XAGPR == 2
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            xagpr(X[t]);
            if (kt >= 4 || t % 4 < kt) xagpr(Y[t]);   // the cos tiles already computed
          }
#endif
          // next sin/cos tile's projections, after this tile's MFMAs are issued
          if constexpr (ot == 3 && kt < 3) wfourier_q<DIM>(io, bt, kt + 1, h, q);
          if constexpr (S == 16) a0.bc.load(W, lane, B_EBLK);
          xdue<decltype(e0), S>(e0);
        });
  }

  // ---- encoder residual blocks (:228-232); X = h (2 points x 4 tiles).  Each layer's bias
  // columns are fetched at the first step of the layer before it.
  const int WE = WF + OFF_EBLK * 4;
  {
    XFwdAct<4, 4, 2, true, GRAD> b0{X, sc, WT_EBLK + 8, lane, {}, wl, 0.f};
    XFwdAct<4, 4, 2, false, GRAD> a1{Y, sc, WT_EBLK + 16, lane, {}, wl, 0.f};
    XFwdAct<4, 4, 2, true, GRAD> b1{X, sc, WT_EBLK + 24, lane, {}, wl, 0.f};
    XFwdLin<4, 4, 2> e3{Y, {}};
    xlayer<4, 4, 2, SITE_FWD_ENC, true>(ring, W, WE, X, lane, a0,
                                  both(XPend<decltype(e0)>{e0},
                                       at<0>([&] { b0.bc.load(W, lane, B_EBLK + 128); })),
                                  WHead{WE + SZ_E * 4});
    xlayer<4, 4, 2, SITE_FWD_ENC, false>(ring, W, WE + SZ_E * 4, Y, lane, b0,
                                  both(XPend<decltype(a0)>{a0},
                                       at<0>([&] { a1.bc.load(W, lane, B_EBLK + 256); })),
                                  WHead{WE + 2 * SZ_E * 4});
    xlayer<4, 4, 2, SITE_FWD_ENC, true>(ring, W, WE + 2 * SZ_E * 4, X, lane, a1,
                                  both(XPend<decltype(b0)>{b0},
                                       at<0>([&] { b1.bc.load(W, lane, B_EBLK + 384); })),
                                  WHead{WE + 3 * SZ_E * 4});
    xlayer<4, 4, 2, SITE_FWD_ENC, false>(ring, W, WE + 3 * SZ_E * 4, Y, lane, b1,
                                  both(XPend<decltype(a1)>{a1},
                                       at<0>([&] { e3.bc.load(W, lane, B_E3); })),
                                  WHead{WF + OFF_E3 * 4});
    // ---- encoder[-1] (:234) -> Y (zs = Y[0..3], zg = Y[4..7])
    xlayer<4, 4, 2, SITE_FWD_ENC, true>(ring, W, WF + OFF_E3 * 4, X, lane, e3, XPend<decltype(b1)>{b1},
                                  WHead{WF + OFF_GBLK * 4});
  }

  // ---- symmetric smooth max / min merge (:236-244) -> X (u = [M | m], 8 tiles)
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    f32x16 s0;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float zs = Y[t][r], zg = Y[4 + t][r];   // κ-scaled
      float d = zs - zg;
      float e = __builtin_amdgcn_exp2f(-fabsf(d));    // e^{-10|zs - zg|}
      float cc = __builtin_amdgcn_logf(1.f + e);      // κ·0.1·ln(1 + e)
      X[t][r] = fmaxf(zs, zg) + cc;
      X[4 + t][r] = fminf(zs, zg) - cc;
      float rr = __builtin_amdgcn_rcpf(1.f + e);
      s0[r] = (d >= 0.f) ? rr : e * rr;
    }
    if (GRAD) lstore(wl, WL_S0 + t, s0);
  }

  // ---- generator residual blocks (:246-249), rotated so that one loop body carries a
  // layer's pending chunks into the next: ga0; (gb_i, ga_{i+1}) for i = 0, 1; gb2; g3
  XFwdAct<8, 8, 1, false, GRAD> ga{Y, sc, WT_GBLK, lane, {}, wl, 0.f};
  XFwdAct<8, 8, 1, true, GRAD> gb{X, sc, WT_GBLK + 8, lane, {}, wl, 0.f};
  ga.bc.load(W, lane, B_GBLK);
  xlayer<8, 8, 1, SITE_FWD_GEN, true>(ring, W, WF + OFF_GBLK * 4, X, lane, ga,
                                at<0>([&] { gb.bc.load(W, lane, B_GBLK + 256); }),
                                WHead{WF + (OFF_GBLK + SZ_G) * 4});
#pragma unroll 1
  for (int i = 0; i < 2; ++i) {
    const int wb = opaque(WF + (OFF_GBLK + (2 * i + 1) * SZ_G) * 4);
    const int wa = opaque(WF + (OFF_GBLK + (2 * i + 2) * SZ_G) * 4);
    const int wn = opaque(WF + (OFF_GBLK + (2 * i + 3) * SZ_G) * 4);
    const int ba = opaque(B_GBLK + (2 * i + 2) * 256);
    gb.sc0 = opaque(WT_GBLK + 16 * i + 8);
    xlayer<8, 8, 1, SITE_FWD_GEN, false>(ring, W, wb, Y, lane, gb,
                                  both(XPend<decltype(ga)>{ga},
                                       at<0>([&] { ga.bc.load(W, lane, ba); })),
                                  WHead{wa});
    ga.sc0 = opaque(WT_GBLK + 16 * i + 16);
    xlayer<8, 8, 1, SITE_FWD_GEN, true>(ring, W, wa, X, lane, ga,
                                  both(XPend<decltype(gb)>{gb},
                                       at<0>([&] { gb.bc.load(W, lane, ba + 256); })),
                                  WHead{wn});
  }
  // ---- generator block 2's second layer, then generator[-2] + act (:251-252) -> Y[0..3]
  XFwdAct<4, 8, 1, false, GRAD, true> g3{Y, sc, WL_G3, lane, {}, wl, 0.f};
  gb.sc0 = WT_GBLK + 16 * 2 + 8;
  xlayer<8, 8, 1, SITE_FWD_GEN, false>(ring, W, WF + (OFF_GBLK + 5 * SZ_G) * 4, Y, lane, gb,
                                both(XPend<decltype(ga)>{ga},
                                     at<0>([&] { g3.bc.load(W, lane, B_G3); })),
                                WHead{WF + OFF_G3 * 4});
  xlayer<4, 8, 1, SITE_FWD_GEN, true>(ring, W, WF + OFF_G3 * 4, X, lane, g3, XPend<decltype(gb)>{gb},
                                after);
  xflush(g3);
  // ---- head generator[-1] + sigmoid(0.1 y) (:254-255)
  float part = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      f32x4 w = whw_load(wl, t, u, h);
#pragma unroll
      for (int s = 0; s < 4; ++s) part = fmaf(w[s], Y[t][4 * u + s], part);
    }
  part += __shfl_xor(part, 32);
  const float y4 = fmaf(part, WKAPPA_INV, bload(W, 0, WG4B)[0]);   // part = κ·(g4w·h3)
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-0.144269504088896341f * y4));
}

// ---------------------------------------------------------------- reverse sweep (x6 acc)
template <int DIM, class BT, class AfterF>
__device__ __forceinline__ void wide_backward_x(Ring& ring, Rsrc W, const PairIO& io, BT bt,
                                                float tau, f32x16 (&X)[8], f32x16 (&Y)[8],
                                                WScratch sc, WLds wl, int lane,
                                                float (&ds)[DIM], float (&dg)[DIM],
                                                AfterF after) {
  const int h = lane >> 5;
  // ---- head and generator[-2] (:592-613): Y[t] = d · g4w ⊙ σ10(y3)
  const float dd = 0.1f * tau * (1.f - tau);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    f32x16 s3 = lload(wl, WL_G3 + t);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      f32x4 w = whw_load(wl, t, u, h);
#pragma unroll
      for (int s = 0; s < 4; ++s) Y[t][4 * u + s] = (dd * w[s]) * s3[4 * u + s];
    }
  }
#if defined(PNTF_XMIXB) && PNTF_XMIXB == 2   // diagnostics: the round-5 generator layers
  // du = G3^T dv ⊙ σ10(y2 of generator block 2) -> X   (G3^T: 256 x 128, OT 8, KT 4)
  {
    WBwd<8, 4, 1, false, true> l{X, sc, WT_GBLK + 16 * 2 + 8, lane};
    wlayer<8, 4, 1, SITE_BWD_GEN, 4>(ring, W, WB + OFF_G3 * 4, Y, lane, l, NoPre{},
                                     WHead{WB + (OFF_GBLK + 5 * SZ_G) * 4});
  }
  // ---- generator blocks, reverse (:615-618): blocks 2 and 1 in a loop, block 0 peeled (its
  // second layer multiplies by no σ and hands over to encoder[-1]^T)
#pragma unroll 1
  for (int i = 2; i >= 1; --i) {
    const int wa = opaque(WB + (OFF_GBLK + (2 * i) * SZ_G) * 4);
    const int wb = opaque(WB + (OFF_GBLK + (2 * i + 1) * SZ_G) * 4);
    const int wn = opaque(WB + (OFF_GBLK + (2 * i - 1) * SZ_G) * 4);
    // da = (G1_i^T dr) ⊙ σ10(y1_i) -> Y
    WBwd<8, 8, 1, false, true> lb{Y, sc, WT_GBLK + 16 * i, lane};
    wlayer<8, 8, 1, SITE_BWD_GEN, 4>(ring, W, wb, X, lane, lb, NoPre{}, WHead{wa});
    // du = G_i^T da + dr, then ⊙ σ10(y2_{i-1})
    WBwd<8, 8, 1, true, true> la{X, sc, WT_GBLK + 16 * (i - 1) + 8, lane};
    wlayer<8, 8, 1, SITE_BWD_GEN, 4>(ring, W, wa, Y, lane, la, NoPre{}, WHead{wn});
  }
  {
    WBwd<8, 8, 1, false, true> lb{Y, sc, WT_GBLK, lane};
    wlayer<8, 8, 1, SITE_BWD_GEN, 4>(ring, W, WB + (OFF_GBLK + 1 * SZ_G) * 4, X, lane, lb,
                                     NoPre{}, WHead{WB + OFF_GBLK * 4});
    WBwd<8, 8, 1, true, false> la{X, sc, 0, lane};
    wlayer<8, 8, 1, SITE_BWD_GEN, 4>(ring, W, WB + OFF_GBLK * 4, Y, lane, la, NoPre{},
                                     WHeadE{WB + OFF_E3 * 4});
  }
#else
  // du = G3^T dv ⊙ σ10(y2 of generator block 2) -> X   (G3^T: 256 x 128, OT 8, KT 4)
  XBwd<8, 4, 1, false, true> l3{X, sc, WT_GBLK + 16 * 2 + 8, lane, {}};
  xlayer<8, 4, 1, SITE_BWD_GEN, false>(ring, W, WB + OFF_G3 * 4, Y, lane, l3, NoPre{},
                                WHead{WB + (OFF_GBLK + 5 * SZ_G) * 4});
  // ---- generator blocks, reverse (:615-618), rotated: lb_2; (la_i, lb_{i-1}) for i = 2, 1;
  // la_0 (no σ: it hands over to encoder[-1]^T)
  XBwd<8, 8, 1, false, true> lb{Y, sc, WT_GBLK + 16 * 2, lane, {}};
  XBwd<8, 8, 1, true, true> la{X, sc, 0, lane, {}};
  xlayer<8, 8, 1, SITE_BWD_GEN, true>(ring, W, WB + (OFF_GBLK + 5 * SZ_G) * 4, X, lane, lb,
                                XPend<decltype(l3)>{l3}, WHead{WB + (OFF_GBLK + 4 * SZ_G) * 4});
#pragma unroll 1
  for (int i = 2; i >= 1; --i) {
    const int wa = opaque(WB + (OFF_GBLK + (2 * i) * SZ_G) * 4);
    const int wb = opaque(WB + (OFF_GBLK + (2 * i - 1) * SZ_G) * 4);
    const int wn = opaque(WB + (OFF_GBLK + (2 * i - 2) * SZ_G) * 4);
    // du = G_i^T da + dr, then ⊙ σ10(y2_{i-1})
    la.mul0 = opaque(WT_GBLK + 16 * (i - 1) + 8);
    xlayer<8, 8, 1, SITE_BWD_GEN, false>(ring, W, wa, Y, lane, la, XPend<decltype(lb)>{lb}, WHead{wb});
    // da = (G1_{i-1}^T dr) ⊙ σ10(y1_{i-1}) -> Y
    lb.mul0 = opaque(WT_GBLK + 16 * (i - 1));
    xlayer<8, 8, 1, SITE_BWD_GEN, true>(ring, W, wb, X, lane, lb, XPend<decltype(la)>{la}, WHead{wn});
  }
  {
    XBwd<8, 8, 1, true, false> l0{X, sc, 0, lane, {}};
    xlayer<8, 8, 1, SITE_BWD_GEN, false>(ring, W, WB + OFF_GBLK * 4, Y, lane, l0,
                                  XPend<decltype(lb)>{lb}, WHead{WB + OFF_E3 * 4});
  }
#endif
  // ---- merge Jacobian (:620-627): X[0..3] = dzs, X[4..7] = dzg
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    f32x16 s0 = lload(wl, WL_S0 + t);
    f32x16 s1 = 1.f - s0;
    f32x16 dM = X[t], dm = X[4 + t];
    X[t] = s0 * dM + s1 * dm;
    X[4 + t] = s1 * dM + s0 * dm;
  }
#if defined(PNTF_XMIXB) && PNTF_XMIXB == 1   // diagnostics: the round-5 encoder layers
  // ---- encoder[-1]^T ⊙ σ10(y2 of encoder block 1), then the blocks, reverse (:629-636)
  const int WE = WB + OFF_EBLK * 4;
  {
    WBwd<4, 4, 2, false, true> e3{Y, sc, WT_EBLK + 24, lane};
    wlayer<4, 4, 2, SITE_BWD_ENC, 4>(ring, W, WB + OFF_E3 * 4, X, lane, e3, NoPre{},
                                     WHeadE{WE + 3 * SZ_E * 4});
    WBwd<4, 4, 2, false, true> b1{X, sc, WT_EBLK + 16, lane};
    wlayer<4, 4, 2, SITE_BWD_ENC, 4>(ring, W, WE + 3 * SZ_E * 4, Y, lane, b1, NoPre{},
                                     WHeadE{WE + 2 * SZ_E * 4});
    WBwd<4, 4, 2, true, true> a1{Y, sc, WT_EBLK + 8, lane};
    wlayer<4, 4, 2, SITE_BWD_ENC, 4>(ring, W, WE + 2 * SZ_E * 4, X, lane, a1, NoPre{},
                                     WHeadE{WE + 1 * SZ_E * 4});
    WBwd<4, 4, 2, false, true> b0{X, sc, WT_EBLK, lane};
    wlayer<4, 4, 2, SITE_BWD_ENC, 4>(ring, W, WE + 1 * SZ_E * 4, Y, lane, b0, NoPre{},
                                     WHeadE{WE});
    WBwd<4, 4, 2, true, true> a0{Y, sc, WT_E0, lane};
    wlayer<4, 4, 2, SITE_BWD_ENC, 4>(ring, W, WE, X, lane, a0, NoPre{}, WFoldHead{});
  }

  wide_fold<DIM>(ring, W, io, bt, Y, lane, ds, dg, after);
  return;
#else
  // ---- encoder[-1]^T ⊙ σ10(y2 of encoder block 1), then the blocks, reverse (:629-636)
  const int WE = WB + OFF_EBLK * 4;
  {
    XBwd<4, 4, 2, false, true> e3{Y, sc, WT_EBLK + 24, lane, {}};
    XBwd<4, 4, 2, false, true> b1{X, sc, WT_EBLK + 16, lane, {}};
    XBwd<4, 4, 2, true, true> a1{Y, sc, WT_EBLK + 8, lane, {}};
    XBwd<4, 4, 2, false, true> b0{X, sc, WT_EBLK, lane, {}};
    XBwd<4, 4, 2, true, true> a0{Y, sc, WT_E0, lane, {}};
#if defined(PNTF_XENCFLUSH)   // diagnostics: every reverse encoder layer finishes its chunks
    xlayer<4, 4, 2, SITE_BWD_ENC, true>(ring, W, WB + OFF_E3 * 4, X, lane, e3, NoPre{},
                                  WHead{WE + 3 * SZ_E * 4});
    xflush(e3);
    xlayer<4, 4, 2, SITE_BWD_ENC, false>(ring, W, WE + 3 * SZ_E * 4, Y, lane, b1, NoPre{},
                                  WHead{WE + 2 * SZ_E * 4});
    xflush(b1);
    xlayer<4, 4, 2, SITE_BWD_ENC, true>(ring, W, WE + 2 * SZ_E * 4, X, lane, a1, NoPre{},
                                  WHead{WE + 1 * SZ_E * 4});
    xflush(a1);
    xlayer<4, 4, 2, SITE_BWD_ENC, false>(ring, W, WE + 1 * SZ_E * 4, Y, lane, b0, NoPre{}, WHead{WE});
    xflush(b0);
    xlayer<4, 4, 2, SITE_BWD_ENC, true>(ring, W, WE, X, lane, a0, NoPre{}, WFoldHead{});
#else
    xlayer<4, 4, 2, SITE_BWD_ENC, true>(ring, W, WB + OFF_E3 * 4, X, lane, e3, NoPre{},
                                  WHead{WE + 3 * SZ_E * 4});
    xlayer<4, 4, 2, SITE_BWD_ENC, false>(ring, W, WE + 3 * SZ_E * 4, Y, lane, b1, XPend<decltype(e3)>{e3},
                                  WHead{WE + 2 * SZ_E * 4});
    xlayer<4, 4, 2, SITE_BWD_ENC, true>(ring, W, WE + 2 * SZ_E * 4, X, lane, a1, XPend<decltype(b1)>{b1},
                                  WHead{WE + 1 * SZ_E * 4});
    xlayer<4, 4, 2, SITE_BWD_ENC, false>(ring, W, WE + 1 * SZ_E * 4, Y, lane, b0, XPend<decltype(a1)>{a1},
                                  WHead{WE});
    if constexpr (xfold<BT>())
      xlayer<4, 4, 2, SITE_BWD_ENC, true>(ring, W, WE, X, lane, a0, XPend<decltype(b0)>{b0},
                                    WFoldXHead{});
    else
      xlayer<4, 4, 2, SITE_BWD_ENC, true>(ring, W, WE, X, lane, a0, XPend<decltype(b0)>{b0},
                                    WFoldHead{});
#endif
    xflush(a0);
  }
#endif
  if constexpr (xfold<BT>()) wide_fold_x<DIM>(ring, W, io, bt, X, Y, lane, ds, dg, after);
  else wide_fold<DIM>(ring, W, io, bt, Y, lane, ds, dg, after);
}
#endif  // PNTF_WIDE_X6 && PNTF_X6_ACC

// ---------------------------------------------------------------- kernel
template <int DIM, int KIND, bool BL>
__global__ __launch_bounds__(256, 1) void wide_field_kernel(FieldArgs a) {
  PNTF_CLOCK_SCOPE;
  constexpr bool GRAD = KIND != K_TAU && KIND != K_TRAVEL;
  const int lane = threadIdx.x & 63;
  const int slot = blockIdx.x * WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nslots = gridDim.x * WAVES;
  // tile indices are wave-uniform 32-bit values (kept in SGPRs): tile * WTILE must stay below
  // 2^31, so the host sends batches above 2^31 - 32 pairs to the wave-tile kernel instead
  // (pntf_capi.hip WIDE_MAX_PAIRS)
  const int ntiles = (int)((a.n + WTILE - 1) / WTILE);
  const WScratch sc =
      make_wscratch(GRAD ? a.ws + (int64_t)slot * WSCRATCH_FLOATS_PER_WAVE : nullptr);
  const Rsrc W = make_rsrc(a.P, (PNTF_WIDE_X6 ? PACKED_TOTAL_X6 : PACKED_TOTAL) * 4);
  __shared__ f32x4 wsig[GRAD ? WAVES * WL_TILES * 4 * 64 : 1];
  // each wave keeps its own copy of the head row (no workgroup barrier: a wave's LDS reads
  // follow its own writes in order)
  __shared__ f32x4 whead[WAVES * H / 4];
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const WLds wl{(wlds_f4*)wsig + (GRAD ? wv * (WL_TILES * 4 * 64) + lane : 0),
                (const wlds_f*)(whead + wv * (H / 4))};
  ((wlds_f*)(whead + wv * (H / 4)))[lane] = a.P[OFF_BIAS + B_G4W + lane];
  ((wlds_f*)(whead + wv * (H / 4)))[lane + 64] = a.P[OFF_BIAS + B_G4W + lane + 64];
  __shared__ f32x4 wbtab[BL ? WBL_FLOATS / 4 : 1];
  if constexpr (BL) {   // the host checked n_env · DIM · H <= WBL_FLOATS
    const int nb4 = a.n_env * (DIM * H / 4);
    for (int i = threadIdx.x; i < nb4; i += 256)
      wbtab[i] = *reinterpret_cast<const f32x4*>(a.Btab + 4 * i);
  }
  Ring ring;
  ring_fill<WE0NL>(ring, W, lane * 16, WE0Head{});
  if constexpr (BL) __syncthreads();
  for (int tile = slot; tile < ntiles; tile += nslots) {
    f32x16 X[8], Y[8];
    // the pair column, re-derived per tile from the lane·16 byte offset every load keeps
    // live (through an opaque copy, so it is not hoisted): a separate loop-invariant copy was
    // the one value that spilled
    int v16 = lane * 16;
    asm volatile("" : "+v"(v16));
    const int64_t pair = (int64_t)(tile * WTILE + ((v16 >> 4) & 31));
    PairIO io;
    const bool ok = load_pair<DIM>(a.xp, a.Btab, a.env, a.n, a.n_env, pair, io);
    WBt<BL> bt;
    if constexpr (BL) bt.t = (const wlds_f*)wbtab + (io.Bw - a.Btab);
    float tau;
#if PNTF_WIDE_X6 && PNTF_X6_ACC && defined(PNTF_XMIX) && PNTF_XMIX == 1   // diagnostics
#define PNTF_WFWD wide_forward_x
#define PNTF_WBWD wide_backward
#elif PNTF_WIDE_X6 && PNTF_X6_ACC && defined(PNTF_XMIX) && PNTF_XMIX == 2
#define PNTF_WFWD wide_forward
#define PNTF_WBWD wide_backward_x
#elif PNTF_WIDE_X6 && PNTF_X6_ACC
#define PNTF_WFWD wide_forward_x
#define PNTF_WBWD wide_backward_x
#else
#define PNTF_WFWD wide_forward
#define PNTF_WBWD wide_backward
#endif
    if constexpr (GRAD)
      tau = PNTF_WFWD<DIM, true>(ring, W, io, bt, X, Y, sc, wl, a.compat, lane, wbwd_head());
    else
      tau = PNTF_WFWD<DIM, false>(ring, W, io, bt, X, Y, sc, wl, a.compat, lane, WE0Head{});
    float ds[DIM], dg[DIM];
    if constexpr (GRAD) {
      drain_stores();
      PNTF_WBWD<DIM>(ring, W, io, bt, tau, X, Y, sc, wl, lane, ds, dg, WE0Head{});
    }
#undef PNTF_WFWD
#undef PNTF_WBWD
    const bool store = lane < 32 && pair < a.n;
    store_field<DIM, KIND>(a, pair, ok, store, tau, io, ds, dg);
  }
}

#if defined(PNTF_UTIL)
// ---------------------------------------------------------------- wide weight packing
// dst[(((ot·KT + kt)·4 + u)·64 + l)·4 + s] = M[32 ot + (l & 31)][32 kt + 8 u + 4 (l >> 5) + s]
// with M = src (rows x cols, row stride ld) or M = src^T (trans).
__global__ void pack_wide_kernel(const float* __restrict__ src, int rows, int cols, int ld,
                                 int trans, float scale, float* __restrict__ dst) {
  int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= (int64_t)rows * cols) return;
  int s = o & 3;
  int l = (o >> 2) & 63;
  int u = (o >> 8) & 3;
  int64_t rest = o >> 10;
  int KT = cols / 32;
  int kt = rest % KT;
  int ot = rest / KT;
  int n = 32 * ot + (l & 31);
  int k = 32 * kt + 8 * u + 4 * (l >> 5) + s;
  dst[o] = scale * (trans ? src[(int64_t)k * ld + n] : src[(int64_t)n * ld + k]);
}

// split-bf16 copy of the wide region's two directions (OFF_X6): step g = (matrix, ot, kt) of
// the fp32 region (1024 floats: fragments u = 0..3) becomes fragments 3b + term of k block b,
// whose element i is element i & 3 of fp32 fragment 2b + (i >> 2) of the same lane.
__global__ void pack_x6_kernel(const float* __restrict__ wide, uint16_t* __restrict__ x6, int bm) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // (step, block, lane)
  if (t >= (int64_t)(2 * SZ_DIR / 1024) * 2 * 64) return;
  const int lane = (int)(t & 63), b = (int)((t >> 6) & 1);
  const int gf = (int)(t >> 7);   // fp32 step: matrix base + ot·KT + kt
  // the matrix (offset and shape in the direction's OFF_* order; Wᵀ in the second direction)
  const int dir = gf >= SZ_DIR / 1024, f = gf * 1024 - dir * SZ_DIR;
  int m0, out, in, nc;
  if (f < OFF_EBLK) { m0 = OFF_E0; out = 128; in = 256; nc = 2; }
  else if (f < OFF_GBLK) { m0 = OFF_EBLK + (f - OFF_EBLK) / SZ_E * SZ_E; out = in = 128; nc = 2; }
  else if (f < OFF_G3) { m0 = OFF_GBLK + (f - OFF_GBLK) / SZ_G * SZ_G; out = in = 256; nc = 1; }
  else { m0 = OFF_G3; out = 128; in = 256; nc = 1; }
  if (dir) { const int x = out; out = in; in = x; }
  const int OT = out / 32, KT = in / 32;
  const int j = (f - m0) / 1024, ot = j / KT, kt = j % KT;
  // first fragment of (ot, kt, block b) in the x6 step order of wlayer; term p at + p
  int64_t fr;
  if (PNTF_X6_ACC && PNTF_XFOLD && !bm && dir && m0 == OFF_E0) {
    // encoder[0]^T for the accumulate engine's fold: pass p = (ot % 4) / 2 covers feature tiles
    // 2p, 2p + 1 with their sin (ot < 4) and cos (ot >= 4) rows; step (p, kt, ot_local),
    // ot_local = ((ot % 4) % 2)·2 + ot / 4, fragments 3b + term
    const int pp = (ot % 4) / 2, ol = ((ot % 4) % 2) * 2 + ot / 4;
    fr = ((int64_t)(gf - j) + (pp * KT + kt) * 4 + ol) * 6 + 3 * b;
  } else if (bm && nc == 2) {   // step (g, kt, b), fragments 3o + p
    fr = ((int64_t)(gf - j) + ((ot / 2) * KT + kt) * 2 + b) * 6 + (ot % 2) * 3;
  } else {                     // step (g, kt, o), fragments 3b + p
    const int G = wx6_group(OT, nc);
    fr = ((int64_t)(gf - j) + (ot / G) * KT * G + kt * G + ot % G) * 6 + 3 * b;
  }
  const float* src = wide + (int64_t)gf * 1024;
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = src[((2 * b + (i >> 2)) * 64 + lane) * 4 + (i & 3)];
  f32x16 tile;
#pragma unroll
  for (int i = 0; i < 16; ++i) tile[i] = v[i & 7];
  wbf16x8 s[3];
  wx6_split(tile, 0, s);
#pragma unroll
  for (int p = 0; p < 3; ++p)
    *reinterpret_cast<wbf16x8*>(x6 + ((fr + p) * 64 + lane) * 8) = s[p];
}

// bias columns, head vector and head bias of the wide region, from the plain bias block
__global__ void pack_wide_aux_kernel(const float* __restrict__ plain, float* __restrict__ wide) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  constexpr int NB = W_SZ_BCOL, NH = W_SZ_G4W;
  if (o < NB) {   // bias columns: fragment g, lane l, element s
    int s = o & 3, l = (o >> 2) & 63, g = o >> 8;
    wide[W_OFF_BCOL + o] = l < 32 ? WKAPPA * plain[128 * g + 32 * s + l] : 0.f;   // κ·bias
  } else if (o < NB + NH) {   // head vector: fragment (4t + u)
    int p = o - NB;
    int s = p & 3, l = (p >> 2) & 63, f = p >> 8;
    int t = f / 4, u = f % 4;
    wide[W_OFF_G4W + p] = plain[B_G4W + 32 * t + 8 * u + 4 * (l >> 5) + s];
  } else if (o < NB + NH + 4) {
    wide[W_OFF_G4B + (o - NB - NH)] = plain[B_G4B + (o - NB - NH)];
  }
}
#endif  // PNTF_UTIL

}  // namespace pntf
