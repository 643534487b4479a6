// Eikonal residual on MI355X: Taylor-mode (value, first and diagonal second derivative)
// evaluation of the P-NTFields MLP and the per-pair residual of Model.Loss.
//
// Reference: NN.out_laplace (models/model_res_sigmoid_multi.py:710-848, helpers :649-708)
// and Model.Loss (:897-951); restated in SURVEY.md Appendix A ("Taylor mode").
//
// Decomposition.  Per direction k (one coordinate of one endpoint) the Taylor rows
// (J_k, L_k) obey, layer by layer,
//     linear:  J' = A J,  L' = A L                        (+ residual J, L)
//     act:     J = σ(y) J',  L = σ'(y) J'^2 + σ(y) L'    with σ' = 10 σ (1 - σ)
// so directions never mix and need only σ(y) of the value pass.  The kernel therefore
// runs the value pass once (field kernel forward, σ tiles saved to the wave's scratch
// slot), then the 2·dim directions one after the other, each carrying (J_k, L_k) as two
// MFMA column sets (NC = 2: one weight fragment feeds both) through encoder (the one
// point the direction belongs to), merge, generator and head.  MACs per pair:
// 40·128² (value) + 2·dim·2·(7 + 26)·128² = 436·128² for dim 3.
#pragma once
#include "pntf_field.h"

namespace pntf {

// (J, L) <- [act](A·(J, L) (+ residual)) with σ tiles sig0 + ot of the value pass.
// in: J tiles in[0..KT), L tiles in[KT..2KT); out likewise with OT.  Epilogues are deferred
// into the next group (layer()); the σ tile of a group is fetched when the group starts.
template <int OT_, int KT_, bool RES, bool ACT, int NOUT>
struct TaylorL {
  static constexpr int OT = OT_, KT = KT_, NC = 2, NO = 1;
  static constexpr int EPS = EP_SPLIT, ROWS = 4 / EP_SPLIT;
  f32x4 (&out)[NOUT];
  Scratch sc;
  int sig0, lane;
  f32x4 g[2];
  f32x4 pend[1][2];
  __device__ __forceinline__ void init(int ot, f32x4 (&acc)[1][2]) {
    if (ACT) g[ot & 1] = load_tile(sc, sig0 + ot, lane);
#pragma unroll
    for (int c = 0; c < 2; ++c) acc[0][c] = RES ? out[c * OT + ot] : zero4();
  }
  __device__ __forceinline__ void epi(int t, int c, int h, const f32x4 (&v)[2]) {
    const f32x4 gg = g[t & 1];
#pragma unroll
    for (int r = h * ROWS; r < (h + 1) * ROWS; ++r) {
      const float J = v[0][r], L = v[1][r];
      if (!ACT)
        out[c * OT + t][r] = v[c][r];
      else if (c == 0)
        out[t][r] = gg[r] * J;                                                // :686
      else
        out[OT + t][r] = (10.f * gg[r] * (1.f - gg[r])) * J * J + gg[r] * L;  // :682-684
    }
  }
};

// ---------------------------------------------------------------- split-bf16 Taylor layers
// PNTF_TAYLOR_X6 = 1 (round 6): the direction passes' encoder / generator layers run each fp32
// product as six v_mfma_f32_16x16x32_bf16 on three-term bf16 splits of both operands (the
// headline's and the training GEMMs' scheme: x = x0 + x1 + x2 exactly, the three products of
// order < 2^-16 dropped, fp32 accumulation): 6 x 16 cycles where the fp32 step took 8 x 32.
// The activation layout is unchanged: for the 16x16x32 B operand lane (t, g) supplies k =
// 8 g + i, i.e. rows 4 g .. 4 g + 3 of input tiles 2 b (i < 4) and 2 b + 1 (i >= 4) — its own
// registers — and the weights are pre-split in that k order (OFF_NX6, pack_nx6_kernel).
#ifndef PNTF_TAYLOR_X6
#define PNTF_TAYLOR_X6 1
#endif
// 1: encoder[0] of the direction passes on split-bf16 as well, its J / L input rows built in TY
// (round 6 experiment: C3 77.9 ms against 77.8-79.4 across boxes, componentwise Δτ error
// 2.87e-4 against 2.55e-4, profiles/r06_c3_e0x6.txt: no measurable gain, so off); 0 (the
// default): fp32 MFMA on the Fourier Jacobian rows computed per step
#ifndef PNTF_TAYLOR_E0X6
#define PNTF_TAYLOR_E0X6 0
#endif
// accumulate in the out bank, every out tile in one group (NX6_G = 16, pntf_common.h)
#ifndef PNTF_TAYLOR_ACC
#define PNTF_TAYLOR_ACC 1
#endif
typedef __bf16 nbf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 nbf16x2 __attribute__((ext_vector_type(2)));
typedef float nf32x2 __attribute__((ext_vector_type(2)));
// three-term RNE split of the 8 k values (lo: rows of tile 2b, hi: of tile 2b + 1)
__device__ __forceinline__ void nx6_split(const f32x4& lo, const f32x4& hi, nbf16x8 (&s)[3]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    nf32x2 x = i < 2 ? nf32x2{lo[2 * i], lo[2 * i + 1]} : nf32x2{hi[2 * i - 4], hi[2 * i - 3]};
    asm volatile("" : "+v"(x));   // split here, not hoisted into a whole split bank
    const nbf16x2 p0 = __builtin_convertvector(x, nbf16x2);
#if PNTF_X6_DOT
    const nf32x2 r1 = x6_resid(x, p0);
    const nbf16x2 p1 = __builtin_convertvector(r1, nbf16x2);
    const nf32x2 r2 = x6_resid(r1, p1);
#else
    const nf32x2 r1 = x - __builtin_convertvector(p0, nf32x2);
    const nbf16x2 p1 = __builtin_convertvector(r1, nbf16x2);
    const nf32x2 r2 = r1 - __builtin_convertvector(p1, nf32x2);
#endif
    const nbf16x2 p2 = __builtin_convertvector(r2, nbf16x2);
    s[0][2 * i] = p0[0]; s[0][2 * i + 1] = p0[1];
    s[1][2 * i] = p1[0]; s[1][2 * i + 1] = p1[1];
    s[2][2 * i] = p2[0]; s[2][2 * i + 1] = p2[1];
  }
}
// the six products of order >= 2^-16, the small ones first
__device__ __forceinline__ f32x4 nx6_mma(const f32x4& w0, const f32x4& w1, const f32x4& w2,
                                         const nbf16x8 (&x)[3], f32x4 acc) {
  const nbf16x8 a0 = __builtin_bit_cast(nbf16x8, w0), a1 = __builtin_bit_cast(nbf16x8, w1),
                a2 = __builtin_bit_cast(nbf16x8, w2);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a2, x[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, x[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, x[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, x[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, x[1], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, x[0], acc, 0, 0, 0);
}
// out tiles of a group (one split of each input block per group)
template <int OT>
constexpr int nx6_group() { return OT < NX6_G ? OT : NX6_G; }

// (J, L) <- [act](A·(J, L) (+ residual)) as TaylorL, on split-bf16 MFMA.  Step (g, b, o) runs
// k block b (input tiles 2b, 2b + 1) of out tile g·G + o for both columns; the block is split
// at o = 0 and shared by the G tiles of the group.  A tile's σ tile is loaded when it starts
// (b = 0, NB steps of G before its epilogue) and the epilogue runs at its last step.
// wbase: the layer's byte offset in the forward fp32 direction (its split copy sits at 1.5x).
template <int OT, int KT, bool RES, bool ACT, int NIN, int NOUT>
__device__ __forceinline__ void taylor_layer_x6(Rsrc W, int wbase, const f32x4 (&in)[NIN],
                                                f32x4 (&out)[NOUT], Scratch sc, int sig0,
                                                int lane) {
  constexpr int NB = KT / 2, G = nx6_group<OT>(), STEPS = OT * NB;
  static_assert(KT % 2 == 0 && OT % G == 0 && 2 * KT <= NIN && 2 * OT <= NOUT, "layer shape");
  const int base = OFF_NX6 * 4 + wbase / 2 * 3;
  auto addr = [&](int st, int l) { return base + (st * 3 + l) * 1024; };
  Ring ring;
  ring_fill<3>(ring, W, lane * 16, addr);
#if PNTF_TAYLOR_ACC
  // the out bank is the accumulator (residual: its initial value), so the G = OT out tiles
  // share each input block's split (NX6_G covers every layer); tile ot's act epilogue runs
  // right after its last block's MFMAs
  {
    nbf16x8 xs[2][3];
    // σ tile of out tile t: loaded TSD steps before its epilogue (step (NB-1)·OT + t) into a
    // ring of TSD + 1 slots (a whole layer's σ tiles at once spilled in the dim-6 unit)
    constexpr int TSD = OT < 8 ? OT : 8, NGS = TSD + 1;
    f32x4 gs[NGS];
    run_steps<STEPS, 3, 0, SITE_TAYLOR>(
        ring, W, lane * 16, addr, NoNext{}, [&](auto st, const f32x4 (&a)[3]) {
          constexpr int S = decltype(st)::value;
          constexpr int o = S % G, b = (S / G) % NB, ot = (S / (G * NB)) * G + o;
          static_assert(G == OT, "one group");
          constexpr int LT = S + TSD - (NB - 1) * OT;   // the tile whose σ loads at this step
          if constexpr (ACT && LT >= 0 && LT < OT) gs[LT % NGS] = load_tile(sc, sig0 + LT, lane);
          if constexpr (o == 0) {
#pragma unroll
            for (int c = 0; c < 2; ++c)
              nx6_split(in[c * KT + 2 * b], in[c * KT + 2 * b + 1], xs[c]);
          }
          if constexpr (b == 0 && !RES) {
#pragma unroll
            for (int c = 0; c < 2; ++c) out[c * OT + ot] = zero4();
          }
#pragma unroll
          for (int c = 0; c < 2; ++c)
            out[c * OT + ot] = nx6_mma(a[0], a[1], a[2], xs[c], out[c * OT + ot]);
          if constexpr (ACT && b == NB - 1) {
            const f32x4 gg = gs[ot % NGS], J = out[ot], L = out[OT + ot];
            out[ot] = gg * J;                                                // :686
            out[OT + ot] = (10.f * gg * (1.f - gg)) * J * J + gg * L;        // :682-684
          }
        });
  }
  return;
#endif
  f32x4 acc[G][2], gs[G];
  nbf16x8 xs[2][3];
  run_steps<STEPS, 3, 0, SITE_TAYLOR>(
      ring, W, lane * 16, addr, NoNext{}, [&](auto st, const f32x4 (&a)[3]) {
        constexpr int S = decltype(st)::value;
        constexpr int o = S % G, b = (S / G) % NB, ot = (S / (G * NB)) * G + o;
        if constexpr (o == 0) {
#pragma unroll
          for (int c = 0; c < 2; ++c) nx6_split(in[c * KT + 2 * b], in[c * KT + 2 * b + 1], xs[c]);
        }
        if constexpr (b == 0) {
          if (ACT) gs[o] = load_tile(sc, sig0 + ot, lane);
#pragma unroll
          for (int c = 0; c < 2; ++c) acc[o][c] = RES ? out[c * OT + ot] : zero4();
        }
#pragma unroll
        for (int c = 0; c < 2; ++c) acc[o][c] = nx6_mma(a[0], a[1], a[2], xs[c], acc[o][c]);
        if constexpr (b == NB - 1) {
          if (!ACT) {
            out[ot] = acc[o][0];
            out[OT + ot] = acc[o][1];
          } else {
            const f32x4 gg = gs[o], J = acc[o][0], L = acc[o][1];
            out[ot] = gg * J;                                                // :686
            out[OT + ot] = (10.f * gg * (1.f - gg)) * J * J + gg * L;        // :682-684
          }
        }
      });
}

#if defined(PNTF_UTIL)
// Narrow split-bf16 copy of one forward matrix M (rows x cols, row-major; OFF_NX6): step
// st = (g·NB + b)·G + o of taylor_layer_x6 holds, for out tile ot = g·G + o and k block b, the
// three RNE bf16 terms of A[r][k] = M[16 ot + r][16 (2b + (i >> 2)) + 4 q + (i & 3)] at lane
// l = (r, q) = (l & 15, l >> 4), element i = k - 8 q; fragment 3 st + term, 1 KiB each.
__global__ void pack_nx6_kernel(const float* __restrict__ src, int rows, int cols,
                                uint16_t* __restrict__ dst) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;   // (step, lane)
  const int OT = rows / 16, NB = cols / 32, G = OT < NX6_G ? OT : NX6_G;
  if (t >= OT * NB * 64) return;
  const int l = t & 63, st = t >> 6;
  const int o = st % G, b = (st / G) % NB, ot = (st / (G * NB)) * G + o;
  const int r = l & 15, q = l >> 4;
  f32x4 lo, hi;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    lo[i] = src[(int64_t)(16 * ot + r) * cols + 16 * (2 * b) + 4 * q + i];
    hi[i] = src[(int64_t)(16 * ot + r) * cols + 16 * (2 * b + 1) + 4 * q + i];
  }
  nbf16x8 s[3];
  nx6_split(lo, hi, s);
#pragma unroll
  for (int p = 0; p < 3; ++p)
    *reinterpret_cast<nbf16x8*>(dst + ((int64_t)(st * 3 + p) * 64 + l) * 8) = s[p];
}
#endif  // PNTF_UTIL

template <int OT, int KT, bool RES, bool ACT, int NIN, int NOUT>
__device__ __forceinline__ void taylor_layer(Rsrc W, int wbase, const f32x4 (&in)[NIN],
                                             f32x4 (&out)[NOUT], Scratch sc, int sig0,
                                             int lane) {
  if constexpr (PNTF_TAYLOR_X6) {
    taylor_layer_x6<OT, KT, RES, ACT>(W, wbase, in, out, sc, sig0, lane);
    return;
  }
  TaylorL<OT, KT, RES, ACT, NOUT> ly{out, sc, sig0, lane};
  Ring ring;
  ring_fill<2>(ring, W, lane * 16, Head<KT, 2>{wbase});
  layer<OT, KT, 2, 2, SITE_TAYLOR, 0>(ring, W, wbase, in, lane, ly, NoPre{}, NoNext{});
  flush(ly);
}

// One direction k = p*DIM + d (p = 0 start, 1 goal point).  Returns (∂τ/∂x_k, ∂²τ/∂x_k²),
// identical in all four lane groups.  TX/TY: 32-tile banks (J tiles 0..15, L tiles 16..31
// in the generator; 0..7 / 8..15 in the encoder).
template <int DIM>
__device__ __forceinline__ void taylor_direction(Rsrc W, const PairIO& io, int p, int d,
                                                 float tau, f32x4 (&TX)[32], f32x4 (&TY)[32],
                                                 Scratch sc, int lane, float& Jt, float& Lt) {
  const int g = lane >> 4;
  constexpr int F = OFF_FWD * 4;
  constexpr int BB = OFF_BIAS * 4;
  float xp[DIM];
#pragma unroll
  for (int j = 0; j < DIM; ++j) xp[j] = p ? io.x[1][j] : io.x[0][j];

  // ---- encoder[0] on the Fourier Jacobian / Hessian rows (input_mapping_laplace :199-213)
#if PNTF_TAYLOR_E0X6
  // split-bf16 as the other layers: the J rows (js | jc) and L rows (ls | lc) of the 256
  // Fourier features are the layer's two input columns, built in TY (free until encoder[-1])
#pragma unroll
  for (int kt = 0; kt < 8; ++kt) {
    f32x4 q = zero4(), wd = zero4();
#pragma unroll
    for (int j = 0; j < DIM; ++j) {
      f32x4 wj = TWO_PI * ld4(io.Bw + j * H + 16 * kt + 4 * g);
      q += xp[j] * wj;
      wd = (j == d) ? wj : wd;
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float sn, cs;
      sincos_fast(q[s], sn, cs);
      TY[kt][s] = wd[s] * cs;
      TY[8 + kt][s] = -wd[s] * sn;
      TY[16 + kt][s] = -wd[s] * wd[s] * sn;
      TY[24 + kt][s] = -wd[s] * wd[s] * cs;
    }
  }
  // + act_laplace of encoder[0] (:729), σ tiles T_E0 + 8p + ot
  taylor_layer<8, 16, false, true>(W, F + OFF_E0 * 4, TY, TX, sc, T_E0 + p * 8, lane);
#else
#pragma unroll
  for (int i = 0; i < 16; ++i) TX[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    f32x4 js, jc, ls, lc;   // J/L rows of the sin part and the cos part of feature tile kt
    pipelined<64, 2, SITE_TAYLOR>(
        W, lane * 16,
        [&](int st, int l) { return frag<16>(F + OFF_E0 * 4, st % 8, st / 8 + 8 * l); },
        [&](auto st, const f32x4 (&a)[2]) {
          constexpr int kt = decltype(st)::value / 8, ot = decltype(st)::value % 8;
          if constexpr (ot == 0) {
            f32x4 q = zero4(), wd = zero4();
#pragma unroll
            for (int j = 0; j < DIM; ++j) {
              f32x4 wj = TWO_PI * ld4(io.Bw + j * H + 16 * kt + 4 * g);
              q += xp[j] * wj;
              wd = (j == d) ? wj : wd;
            }
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              float sn, cs;
              sincos_fast(q[s], sn, cs);
              js[s] = wd[s] * cs;
              jc[s] = -wd[s] * sn;
              ls[s] = -wd[s] * wd[s] * sn;
              lc[s] = -wd[s] * wd[s] * cs;
            }
          }
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            TX[ot] = mfma(a[0][s], js[s], TX[ot]);
            TX[8 + ot] = mfma(a[0][s], ls[s], TX[8 + ot]);
            TX[ot] = mfma(a[1][s], jc[s], TX[ot]);
            TX[8 + ot] = mfma(a[1][s], lc[s], TX[8 + ot]);
          }
        });
  }
#pragma unroll
  for (int ot = 0; ot < 8; ++ot) {   // act_laplace of encoder[0] (:729)
    const f32x4 gg = load_tile(sc, T_E0 + p * 8 + ot, lane);
    const f32x4 gp = 10.f * gg * (1.f - gg);
    const f32x4 J = TX[ot], L = TX[8 + ot];
    TX[ot] = gg * J;
    TX[8 + ot] = gp * J * J + gg * L;
  }
#endif

  // ---- encoder residual blocks (:731-746)
#pragma unroll 1
  for (int b = 0; b < 2; ++b) {
    const int wa = opaque(F + (OFF_EBLK + (2 * b) * SZ_E) * 4);
    const int wb = opaque(F + (OFF_EBLK + (2 * b + 1) * SZ_E) * 4);
    taylor_layer<8, 8, false, true>(W, wa, TX, TY, sc, T_EBLK + 32 * b + p * 8, lane);
    taylor_layer<8, 8, true, true>(W, wb, TY, TX, sc, T_EBLK + 32 * b + 16 + p * 8, lane);
  }
  // ---- encoder[-1], linear (:748-750) -> TY (J_z 0..7, L_z 8..15)
  taylor_layer<8, 8, false, false>(W, F + OFF_E3 * 4, TX, TY, sc, 0, lane);

  // ---- merge (:768-813): start directions take (s0, s1), goal directions (s1, s0)
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const f32x4 s0 = load_tile(sc, T_S0 + t, lane);
    const f32x4 s1 = 1.f - s0;
    const f32x4 c = 10.f * s0 * s1;                      // :790
    const f32x4 a = p ? s1 : s0, bb = p ? s0 : s1;
    const f32x4 J = TY[t], L = TY[8 + t];
    const f32x4 cj = c * J * J;
    TX[t] = a * J;               // J of the max half
    TX[8 + t] = bb * J;          // J of the min half
    TX[16 + t] = a * L + cj;     // L of the max half
    TX[24 + t] = bb * L - cj;    // L of the min half
  }

  // ---- generator residual blocks (:816-829)
#pragma unroll 1
  for (int i = 0; i < 3; ++i) {
    const int wa = opaque(F + (OFF_GBLK + (2 * i) * SZ_G) * 4);
    const int wb = opaque(F + (OFF_GBLK + (2 * i + 1) * SZ_G) * 4);
    taylor_layer<16, 16, false, true>(W, wa, TX, TY, sc, T_GBLK + 32 * i, lane);
    taylor_layer<16, 16, true, true>(W, wb, TY, TX, sc, T_GBLK + 32 * i + 16, lane);
  }
  // ---- generator[-2] + act (:832-835) -> TY (J_v 0..7, L_v 8..15)
  taylor_layer<8, 16, false, true>(W, F + OFF_G3 * 4, TX, TY, sc, T_G3, lane);

  // ---- head generator[-1] + actout_laplace (:837-840, :693-708)
  float jy = 0.f, ly = 0.f;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const f32x4 g4 = bload(W, g * 16, BB + (B_G4W + 16 * t) * 4);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      jy = fmaf(g4[s], TY[t][s], jy);
      ly = fmaf(g4[s], TY[8 + t][s], ly);
    }
  }
  jy += __shfl_xor(jy, 16);
  ly += __shfl_xor(ly, 16);
  jy += __shfl_xor(jy, 32);
  ly += __shfl_xor(ly, 32);
  const float dt = 0.1f * tau * (1.f - tau);
  const float ddt = 0.1f * dt * (1.f - 2.f * tau);
  Jt = dt * jy;
  Lt = ddt * jy * jy + dt * ly;
}

// Per-pair τ, ∇τ, Δ-rows and the Eikonal residual of Model.Loss (:914-946).
template <int DIM>
__device__ __forceinline__ void residual_body(const ResidualArgs& a, int slot, int nslots) {
  const int lane = threadIdx.x & 63;
  const int64_t ntiles = (a.n + TILE - 1) / TILE;
  const Scratch sc = make_scratch(a.ws + (int64_t)slot * SCRATCH_FLOATS_PER_WAVE);
  // the whole blob: the split-bf16 Taylor layers read the OFF_NX6 copy
  const Rsrc W = make_rsrc(a.P, PACKED_TOTAL_NX6 * 4);
  const float nan = __builtin_nanf("");
  for (int64_t tile = slot; tile < ntiles; tile += nslots) {
    const int64_t pair = tile * TILE + (lane & 15);
    PairIO io;
    const bool ok = load_pair<DIM>(a.xp, a.Btab, a.env, a.n, a.n_env, pair, io);
    const bool store = (lane < 16) && pair < a.n;
    float tau;
    {
      f32x4 X[16], Y[16];
      Carry cy;
      Ring ring;
      ring_fill<2>(ring, W, lane * 16, E0Head{});
      tau = forward_pass<DIM, true, 0>(ring, a.P, io, X, Y, cy, sc, 0, lane, NoNext{});
    }
    drain_stores();
    float D[DIM];
    float T0 = 0.f;
#pragma unroll
    for (int j = 0; j < DIM; ++j) {
      D[j] = io.x[1][j] - io.x[0][j];
      T0 = fmaf(D[j], D[j], T0);
    }
    float d2[2] = {0.f, 0.f}, dD[2] = {0.f, 0.f}, lap[2] = {0.f, 0.f};
#pragma unroll 1
    for (int k = 0; k < 2 * DIM; ++k) {
      const int p = k >= DIM ? 1 : 0;
      const int d = k - p * DIM;
      f32x4 TX[32], TY[32];
      float Jt, Lt;
      taylor_direction<DIM>(W, io, p, d, tau, TX, TY, sc, lane, Jt, Lt);
      float Dd = 0.f;
#pragma unroll
      for (int j = 0; j < DIM; ++j) Dd = (j == d) ? D[j] : Dd;
      // p is wave-uniform: select-accumulate keeps the arrays in registers
      d2[0] += p ? 0.f : Jt * Jt;
      d2[1] += p ? Jt * Jt : 0.f;
      dD[0] += p ? 0.f : Jt * Dd;
      dD[1] += p ? Jt * Dd : 0.f;
      lap[0] += p ? 0.f : Lt;
      lap[1] += p ? Lt : 0.f;
      if (store) {
        if (a.dtau) a.dtau[pair * 2 * DIM + k] = ok ? Jt : nan;
        if (a.ltau) a.ltau[pair * 2 * DIM + k] = ok ? Lt : nan;
      }
    }
    if (store) {
      if (a.tau) a.tau[pair] = ok ? tau : nan;
      if (a.diff) {
        const float T3 = tau * tau;
        const float S0 = T0 * d2[0] + 2.f * tau * dD[0] + T3;   // T01 - T02 + T3 (:925-933)
        const float S1 = T0 * d2[1] - 2.f * tau * dD[1] + T3;   // T11 - T12 + T3
        const float yp0 = 1.f / (sqrtf(S0) / T3 + a.gamma * lap[0]);   // :937-938
        const float yp1 = 1.f / (sqrtf(S1) / T3 + a.gamma * lap[1]);
        const float y0 = a.yobs[pair * 2], y1 = a.yobs[pair * 2 + 1];
        const float df = yp0 / y0 + y0 / yp0 + yp1 / y1 + y1 / yp1 - 4.f;   // :943-946
        a.diff[pair] = ok ? df : nan;
      }
    }
  }
}

template <int DIM>
__global__ __launch_bounds__(256, WAVES_PER_SIMD) void residual_kernel(ResidualArgs a) {
  residual_body<DIM>(a, blockIdx.x * WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6),
                     gridDim.x * WAVES);
}

}  // namespace pntf
