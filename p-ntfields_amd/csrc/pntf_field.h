#pragma once
// Fused τ / ∇τ kernels for the P-NTFields sigmoid-residual MLP on MI355X (gfx950).
//
// Reference math: models/model_res_sigmoid_multi.py  NN.out (:215-259), Model.gradient
// (:890-896), NN.out_backgrad (:402-647), Model.Gradient (:1218-1248), Model.Speed
// (:1195-1216), Model.TravelTimes (:1173-1186); planner loop test/gib_plan.py:74-86 and
// test/arm_plan.py:140-152.  Restated in SURVEY.md Appendix A; layout in pntf_common.h.
//
// One wave = 16 pairs.  All activations are register-resident in two banks X[16], Y[16]
// of f32x4 (64 VGPRs each); fp32 MFMA v_mfma_f32_16x16x4_f32 takes the streamed weights as
// the A operand and the previous layer's output tiles as the B operand.  The forward
// pass stores σ10(pre-activation) tiles to a per-wave scratch slot that the analytic
// reverse sweep reads back; nothing crosses waves, so there is no LDS and no barrier.
// Workgroups (4 waves) are persistent, two per CU (two waves per SIMD), and loop over
// pair tiles.
#include <type_traits>

#include "pntf_common.h"

namespace pntf {

// ---------------------------------------------------------------- elementwise math (A1)
// softplus_10 with torch's threshold (Softplus(beta=10), :140) and σ(10y) from one exp.
// Written with hardware v_exp/v_log/v_rcp and selects only: a branch (or an IEEE divide)
// here would split the unrolled MFMA stream and force spills.
__device__ __forceinline__ float exp_neg10abs(float y) {   // exp(-10|y|) in (0, 1]
  return __builtin_amdgcn_exp2f(-14.4269504088896341f * fabsf(y));
}
// log1p(t) for t in [0, 1] as log(1 + t): absolute error <= 2^-24, i.e. <= 6e-9 after the
// 1/10 of softplus_10 — far below the fp32 rounding of the activations it is added to.
__device__ __forceinline__ float log1p_small(float t) {
  return __builtin_amdgcn_logf(1.f + t) * 0.693147180559945309f;
}
struct SpSig {
  float sp, sg;
};
__device__ __forceinline__ SpSig sp_sig(float y) {
  float t = exp_neg10abs(y);
  float r = __builtin_amdgcn_rcpf(1.f + t);
  SpSig o;
  // torch returns y itself above 10y > 20; there 0.1*log1p(t) < 2.1e-10 < ulp(y)/2, so the
  // same expression rounds to exactly y without a select.
  o.sp = fmaxf(y, 0.f) + 0.1f * log1p_small(t);
  o.sg = (y >= 0.f) ? r : t * r;
  return o;
}

__device__ __forceinline__ float sig10(float y) {
  float t = exp_neg10abs(y);
  float r = __builtin_amdgcn_rcpf(1.f + t);
  return (y >= 0.f) ? r : t * r;
}

// Branch-free sincos for the Fourier features: Cody-Waite reduction by 2π (hi/lo split),
// then the hardware v_sin/v_cos on |r| <= π (input in revolutions).  The libm sincosf
// carries a Payne-Hanek slow path whose branches split the unrolled MFMA stream.
__device__ __forceinline__ void sincos_fast(float q, float& s, float& c) {
  const float inv2pi = 0.159154943091895336f;
  float k = rintf(q * inv2pi);
  float r = fmaf(-k, 6.28318548202514648f, q);      // fp32(2π)
  r = fmaf(-k, -1.74845553146951720e-7f, r);        // 2π - fp32(2π)
  float rev = r * inv2pi;
  s = __builtin_amdgcn_sinf(rev);
  c = __builtin_amdgcn_cosf(rev);
}

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------- weight stream
// Weight-stream prefetch depth (steps of the pipelined ring), step fences (bitmask of SITE_*
// call sites) and out tiles per MFMA group for single-column layers; overridable for the
// perf-variant diagnostics (tests/diag).
#ifndef PNTF_PF_STEPS
#define PNTF_PF_STEPS 3
#endif
#ifndef PNTF_STEP_FENCE
#define PNTF_STEP_FENCE 127
#endif
#ifndef PNTF_NO1
#define PNTF_NO1 4
#endif
// Packed weights are read through a buffer resource: per-lane voffset = lane*16 and a
// scalar byte offset per fragment, so address math stays on the SALU.
typedef __amdgpu_buffer_rsrc_t Rsrc;

__device__ __forceinline__ Rsrc make_rsrc(const float* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, bytes, 0x00020000);
}
__device__ __forceinline__ f32x4 bload(Rsrc r, int voff, int soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// Compile-time loop: f(std::integral_constant<int, I>) for I in [B, E).  Guarantees full
// unrolling (constant register-array indices) however long the layer's step sequence is.
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Software-pipelined step sequence: step st consumes NL weight fragments whose byte offsets
// are addr(st, l); fragments are prefetched PF steps ahead into a register ring so the
// L2/MALL latency of the stream hides behind the MFMAs of the previous PF steps.
template <int STEPS, int NL, int PF, int SITE, class AddrF, class BodyF>
__device__ __forceinline__ void pipelined(Rsrc r, int voff, AddrF addr, BodyF body) {
  f32x4 ring[PF][NL];
  static_for<0, (PF < STEPS ? PF : STEPS)>([&](auto p) {
#pragma unroll
    for (int l = 0; l < NL; ++l) ring[p][l] = bload(r, voff, addr(p(), l));
  });
  static_for<0, STEPS>([&](auto st) {
    constexpr int S = decltype(st)::value;
    f32x4 a[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l) a[l] = ring[S % PF][l];
    if constexpr (S + PF < STEPS) {
#pragma unroll
      for (int l = 0; l < NL; ++l) ring[S % PF][l] = bload(r, voff, addr(S + PF, l));
    }
    body(st, a);
    // Keep every load in the step that issues it: without the fence the scheduler sinks
    // prefetches next to their MFMA under register pressure, collapsing the ring.
    if constexpr ((PNTF_STEP_FENCE & SITE) != 0) __builtin_amdgcn_sched_barrier(0);
  });
}

// Hide a wave-uniform integer from the optimizer: inside the runtime block loops this keeps
// loop strength reduction from turning each of the ~100 fragment offsets of a layer into
// its own induction variable (which spilled >100 SGPRs); each offset becomes one s_add.
__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+s"(x));
  return x;
}

// Byte offset of fragment (ot, kt) of a packed (OT x KT) layer.
template <int KT>
__device__ __forceinline__ int frag(int base, int ot, int kt) {
  return base + ((ot * KT + kt) * 64) * 16;
}

__device__ __forceinline__ f32x4 ld4(const float* p) {
  return *reinterpret_cast<const f32x4*>(p);
}

// Per-wave scratch slot (saved σ10 tiles) through a buffer resource whose base is the
// wave's slot: voffset lane*16, scalar tile offset — one 1 KiB wave-instruction per tile,
// and no 64-bit per-tile VGPR addresses for the compiler to hoist.
// Both directions use the nt (streaming) policy.  For the loads it is a correctness
// requirement, not a hint: a persistent wave reuses its slot for every tile it owns, its
// stores of tile k+1 do not refresh the CU's vector L1, and a plain load would hit the L1
// lines of tile k (measured: ~3% stale ∇τ values at 262k pairs).  nt loads bypass L1
// (MI355X_MICROARCH.md, inter-workgroup visibility table).
constexpr int AUX_NT = 2;
struct Scratch {
  Rsrc r;
};
__device__ __forceinline__ Scratch make_scratch(float* sc) {
  return Scratch{make_rsrc(sc, sc ? SCRATCH_FLOATS_PER_WAVE * 4 : 0)};
}
__device__ __forceinline__ void store_tile(Scratch sc, int tile, int lane, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(
      __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), sc.r, lane * 16,
      tile * 1024, AUX_NT);
}
__device__ __forceinline__ f32x4 load_tile(Scratch sc, int tile, int lane) {
  return __builtin_bit_cast(
      f32x4, __builtin_amdgcn_raw_buffer_load_b128(sc.r, lane * 16, tile * 1024, AUX_NT));
}
// Between the forward sweep (stores) and the reverse sweep (loads of the same slot): wait
// until every store of this wave has been performed.  Without it the first reverse-sweep
// loads (the G3 σ tiles, stored a few hundred cycles earlier) can overtake their stores
// under full-chip load (measured: garbage ∇τ rows at 262k pairs, 2 workgroups per CU).
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Diagnostics only (tests/diag): -DPNTF_DEBUG_DUMP writes intermediate tiles of each wave's
// last pair tile to pntf_dbg[(wave*64 + idx)*256 + lane*4 ..].  Never in the shipped library.
#ifdef PNTF_DEBUG_DUMP
__device__ float* pntf_dbg;
__device__ __forceinline__ void dbg_tile(int idx, int lane, f32x4 v) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
  *reinterpret_cast<f32x4*>(pntf_dbg + ((size_t)w * 64 + idx) * 256 + lane * 4) = v;
}
#define PNTF_DBG(idx, v) dbg_tile(idx, lane, v)
#else
#define PNTF_DBG(idx, v)
#endif

constexpr int PF_STEPS = PNTF_PF_STEPS;
// Pipelined call sites (bits of PNTF_STEP_FENCE).
constexpr int SITE_FWD_E0 = 1, SITE_FWD_ENC = 2, SITE_FWD_GEN = 4, SITE_BWD_GEN = 8,
              SITE_BWD_ENC = 16, SITE_FOLD = 32, SITE_TAYLOR = 64;
template <int NC>
constexpr int out_group() { return NC == 1 ? PNTF_NO1 : 1; }

// Generic layer: out tiles processed NO at a time (NO*NC >= 2 independent MFMA chains).
//   init(ot, acc[o][c])  before the K loop of out-tile group starting at ot
//   epi(ot, acc)         after it
template <int OT, int KT, int NC, int SITE, int NIN, class InitF, class EpiF>
__device__ __forceinline__ void layer(Rsrc W, int wbase, const f32x4 (&in)[NIN], int lane,
                                      InitF init, EpiF epi) {
  constexpr int NO = out_group<NC>();
  constexpr int STEPS = (OT / NO) * KT;
  f32x4 acc[NO][NC];
  pipelined<STEPS, NO, PF_STEPS, SITE>(
      W, lane * 16,
      [&](int st, int l) { return frag<KT>(wbase, (st / KT) * NO + l, st % KT); },
      [&](auto st, const f32x4 (&a)[NO]) {
        constexpr int ot = (decltype(st)::value / KT) * NO, kt = decltype(st)::value % KT;
        if constexpr (kt == 0) init(ot, acc);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int o = 0; o < NO; ++o)
#pragma unroll
            for (int c = 0; c < NC; ++c) acc[o][c] = mfma(a[o][s], in[c * KT + kt][s], acc[o][c]);
        if constexpr (kt == KT - 1) epi(ot, acc);
      });
}

// ---------------------------------------------------------------- forward layers
// out[c*OT+ot] = softplus(A·in + bias (+ out[c*OT+ot] if RES)); σ10(pre) saved to scratch
// tile sc0 + c*OT + ot when SAVE.
template <int OT, int KT, int NC, bool RES, bool SAVE>
__device__ __forceinline__ void fwd_act_layer(Rsrc W, int wbase, int bias,
                                              const f32x4 (&in)[16], f32x4 (&out)[16],
                                              Scratch sc, int sc0, int lane) {
  constexpr int NO = out_group<NC>();
  const int g = lane >> 4;
  layer<OT, KT, NC, NC == 2 ? SITE_FWD_ENC : SITE_FWD_GEN>(
      W, wbase, in, lane,
      [&](int ot, f32x4 (&acc)[NO][NC]) {
#pragma unroll
        for (int o = 0; o < NO; ++o) {
          f32x4 b = bload(W, g * 16, bias + (16 * (ot + o)) * 4);
#pragma unroll
          for (int c = 0; c < NC; ++c) acc[o][c] = RES ? out[c * OT + ot + o] + b : b;
        }
      },
      [&](int ot, f32x4 (&acc)[NO][NC]) {
#pragma unroll
        for (int o = 0; o < NO; ++o)
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            f32x4 s, sg;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              SpSig v = sp_sig(acc[o][c][r]);
              s[r] = v.sp;
              sg[r] = v.sg;
            }
            out[c * OT + ot + o] = s;
            if (SAVE) store_tile(sc, sc0 + c * OT + ot + o, lane, sg);
          }
      });
}

// out[c*OT+ot] = A·in + bias, no activation (encoder[-1], :234).
template <int OT, int KT, int NC>
__device__ __forceinline__ void fwd_lin_layer(Rsrc W, int wbase, int bias,
                                              const f32x4 (&in)[16], f32x4 (&out)[16],
                                              int lane) {
  constexpr int NO = out_group<NC>();
  const int g = lane >> 4;
  layer<OT, KT, NC, NC == 2 ? SITE_FWD_ENC : SITE_FWD_GEN>(
      W, wbase, in, lane,
      [&](int ot, f32x4 (&acc)[NO][NC]) {
#pragma unroll
        for (int o = 0; o < NO; ++o) {
          f32x4 b = bload(W, g * 16, bias + (16 * (ot + o)) * 4);
#pragma unroll
          for (int c = 0; c < NC; ++c) acc[o][c] = b;
        }
      },
      [&](int ot, f32x4 (&acc)[NO][NC]) {
#pragma unroll
        for (int o = 0; o < NO; ++o)
#pragma unroll
          for (int c = 0; c < NC; ++c) out[c * OT + ot + o] = acc[o][c];
      });
}

// ---------------------------------------------------------------- backward layers
// out[c*OT+ot] = (A^T·in (+ out[c*OT+ot] if RES)) ⊙ scratch[mul0 + c*OT + ot] (if MUL)
template <int OT, int KT, int NC, bool RES, bool MUL>
__device__ __forceinline__ void bwd_layer(Rsrc W, int wbase, const f32x4 (&in)[16],
                                          f32x4 (&out)[16], Scratch sc,
                                          int mul0, int lane) {
  constexpr int NO = out_group<NC>();
  f32x4 m[NO][NC];
  layer<OT, KT, NC, NC == 2 ? SITE_BWD_ENC : SITE_BWD_GEN>(
      W, wbase, in, lane,
      [&](int ot, f32x4 (&acc)[NO][NC]) {
#pragma unroll
        for (int o = 0; o < NO; ++o)
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            if (MUL) m[o][c] = load_tile(sc, mul0 + c * OT + ot + o, lane);
            acc[o][c] = RES ? out[c * OT + ot + o] : f32x4{0.f, 0.f, 0.f, 0.f};
          }
      },
      [&](int ot, f32x4 (&acc)[NO][NC]) {
#pragma unroll
        for (int o = 0; o < NO; ++o)
#pragma unroll
          for (int c = 0; c < NC; ++c)
            out[c * OT + ot + o] = MUL ? acc[o][c] * m[o][c] : acc[o][c];
      });
}

// ---------------------------------------------------------------- one pair tile
struct PairIO {
  float x[2][6];    // [start|goal][dim]
  const float* Bw;  // this lane's env B (dim x 128), un-scaled
};

// q = x · (2π B) for the lane's 4 feature rows of Fourier tile kt, both columns.
template <int DIM>
__device__ __forceinline__ void fourier_tile(const PairIO& io, int kt, int g, f32x4 (&w)[DIM],
                                             f32x4 (&q)[2]) {
#pragma unroll
  for (int d = 0; d < DIM; ++d) w[d] = TWO_PI * ld4(io.Bw + d * H + 16 * kt + 4 * g);
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float acc = 0.f;
#pragma unroll
      for (int d = 0; d < DIM; ++d) acc = fmaf(io.x[c][d], w[d][s], acc);
      q[c][s] = acc;
    }
}

// Forward pass (NN.out).  GRAD: also save σ tiles for the reverse sweep.
// Returns τ for the lane's pair (identical in all four lane groups).
template <int DIM, bool GRAD>
__device__ __forceinline__ float forward_pass(const float* __restrict__ P, const PairIO& io,
                                              f32x4 (&X)[16], f32x4 (&Y)[16],
                                              Scratch sc, int compat, int lane) {
  const int g = lane >> 4;
  const Rsrc W = make_rsrc(P, PACKED_FLOATS * 4);
  constexpr int BB = OFF_BIAS * 4;  // byte base of biases / head
  constexpr int F = OFF_FWD * 4;   // byte base of the forward fragments

  const float cm = compat ? 1.f : 0.f;   // branch-free mode blend

  // ---- encoder[0] on Fourier features computed on the fly (:186-190, :227).
  // E0 is (128 x 256): OT = 8, KT = 16; input tiles 0..7 = sin q, 8..15 = cos q.
  // Step (kt, ot) loads fragments (ot, kt) and (ot, kt + 8).
#pragma unroll
  for (int ot = 0; ot < 8; ++ot) {
    f32x4 b = bload(W, g * 16, BB + (B_E0 + 16 * ot) * 4);
    X[ot] = b;
    X[8 + ot] = b;
  }
  {
    f32x4 sn[2], cs[2];
    pipelined<64, 2, PF_STEPS, SITE_FWD_E0>(
        W, lane * 16,
        [&](int st, int l) { return frag<16>(F + OFF_E0 * 4, st % 8, st / 8 + 8 * l); },
        [&](auto st, const f32x4 (&a)[2]) {
          constexpr int kt = decltype(st)::value / 8, ot = decltype(st)::value % 8;
          if constexpr (ot == 0) {
            f32x4 w[DIM], q[2];
            fourier_tile<DIM>(io, kt, g, w, q);
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
              for (int s = 0; s < 4; ++s) {
                float x0, x1;
                sincos_fast(q[c][s], x0, x1);
                sn[c][s] = x0;
                cs[c][s] = x1;
              }
          }
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
              X[c * 8 + ot] = mfma(a[0][s], sn[c][s], X[c * 8 + ot]);
              X[c * 8 + ot] = mfma(a[1][s], cs[c][s], X[c * 8 + ot]);
            }
        });
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    f32x4 s, sg;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      SpSig v = sp_sig(X[i][r]);
      s[r] = v.sp;
      sg[r] = cm * sig10(v.sp) + (1.f - cm) * v.sg;   // out_backgrad quirk (:435-438)
    }
    X[i] = s;
    if (GRAD) store_tile(sc, T_E0 + i, lane, sg);
    PNTF_DBG(i, sg);
    PNTF_DBG(16 + i, s);
  }

  // ---- encoder residual blocks (:228-232); X = h (2 cols x 8 tiles)
#pragma unroll 1
  for (int b = 0; b < 2; ++b) {
    const int wa = opaque(F + (OFF_EBLK + (2 * b) * SZ_E) * 4);
    const int wb = opaque(F + (OFF_EBLK + (2 * b + 1) * SZ_E) * 4);
    fwd_act_layer<8, 8, 2, false, GRAD>(W, wa, BB + (B_EBLK + (2 * b) * 128) * 4, X, Y, sc,
                                        T_EBLK + 32 * b, lane);
    fwd_act_layer<8, 8, 2, true, GRAD>(W, wb, BB + (B_EBLK + (2 * b + 1) * 128) * 4, Y, X, sc,
                                       T_EBLK + 32 * b + 16, lane);
  }
  // ---- encoder[-1] (:234) -> Y (zs = Y[0..7], zg = Y[8..15])
  fwd_lin_layer<8, 8, 2>(W, F + OFF_E3 * 4, BB + B_E3 * 4, X, Y, lane);

  // ---- symmetric smooth max / min merge (:236-244) -> X (u = [M | m], 16 tiles)
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    f32x4 s0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float zs = Y[t][r], zg = Y[8 + t][r];
      float d = zs - zg;
      float e = exp_neg10abs(d);
      float cc = 0.1f * log1p_small(e);
      X[t][r] = fmaxf(zs, zg) + cc;
      X[8 + t][r] = fminf(zs, zg) - cc;
      float rr = __builtin_amdgcn_rcpf(1.f + e);
      s0[r] = (d >= 0.f) ? rr : e * rr;
    }
    if (GRAD) store_tile(sc, T_S0 + t, lane, s0);
  }

  // ---- generator residual blocks (:246-249); X = u (16 tiles)
#pragma unroll 1
  for (int i = 0; i < 3; ++i) {
    const int wa = opaque(F + (OFF_GBLK + (2 * i) * SZ_G) * 4);
    const int wb = opaque(F + (OFF_GBLK + (2 * i + 1) * SZ_G) * 4);
    fwd_act_layer<16, 16, 1, false, GRAD>(W, wa, BB + (B_GBLK + (2 * i) * 256) * 4, X, Y, sc,
                                          T_GBLK + 32 * i, lane);
    fwd_act_layer<16, 16, 1, true, GRAD>(W, wb, BB + (B_GBLK + (2 * i + 1) * 256) * 4, Y, X, sc,
                                         T_GBLK + 32 * i + 16, lane);
  }
  // ---- generator[-2] + act (:251-252) -> Y[0..7]
  fwd_act_layer<8, 16, 1, false, GRAD>(W, F + OFF_G3 * 4, BB + B_G3 * 4, X, Y, sc, T_G3, lane);

  // ---- head generator[-1] + sigmoid(0.1 y) (:254-255)
  float part = 0.f;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    f32x4 g4 = bload(W, g * 16, BB + (B_G4W + 16 * t) * 4);
#pragma unroll
    for (int s = 0; s < 4; ++s) part = fmaf(g4[s], Y[t][s], part);
  }
  part += __shfl_xor(part, 16);
  part += __shfl_xor(part, 32);
  float y4 = part + bload(W, 0, BB + B_G4B * 4)[0];
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-0.144269504088896341f * y4));
}

// Reverse sweep: exact reverse mode, or NN.out_backgrad when the forward stored the quirk.
// Produces dτ/dxs (ds) and dτ/dxg (dg), identical in all four lane groups.
template <int DIM>
__device__ __forceinline__ void backward_pass(const float* __restrict__ P, const PairIO& io,
                                              float tau, f32x4 (&X)[16], f32x4 (&Y)[16],
                                              Scratch sc, int lane,
                                              float (&ds)[DIM], float (&dg)[DIM]) {
  const int g = lane >> 4;
  const Rsrc W = make_rsrc(P, PACKED_FLOATS * 4);
  constexpr int BB = OFF_BIAS * 4;  // byte base of biases / head
  constexpr int Bk = OFF_BWD * 4;  // byte base of the transposed fragments

  // ---- head and generator[-2] (:592-613): Y[t] = d * G4 ⊙ σ10(y3)
  const float dd = 0.1f * tau * (1.f - tau);
#pragma unroll
  for (int t = 0; t < 8; ++t)
    Y[t] = (dd * bload(W, g * 16, BB + (B_G4W + 16 * t) * 4)) * load_tile(sc, T_G3 + t, lane);
  // du = G3^T dv ⊙ σ10(y2 of generator block 2) -> X  (G3^T is 256 x 128: OT 16, KT 8)
  bwd_layer<16, 8, 1, false, true>(W, Bk + OFF_G3 * 4, Y, X, sc, T_GBLK + 32 * 2 + 16, lane);

  // ---- generator blocks, reverse (:615-618)
#pragma unroll 1
  for (int i = 2; i >= 0; --i) {
    const int wa = opaque(Bk + (OFF_GBLK + (2 * i) * SZ_G) * 4);
    const int wb = opaque(Bk + (OFF_GBLK + (2 * i + 1) * SZ_G) * 4);
    // da = (G1_i^T dr) ⊙ σ10(y1_i) -> Y
    bwd_layer<16, 16, 1, false, true>(W, wb, X, Y, sc, T_GBLK + 32 * i, lane);
    // du = G_i^T da + dr, then ⊙ σ10(y2_{i-1}) for the next block (none after block 0)
    if (i > 0)
      bwd_layer<16, 16, 1, true, true>(W, wa, Y, X, sc, T_GBLK + 32 * (i - 1) + 16, lane);
    else
      bwd_layer<16, 16, 1, true, false>(W, wa, Y, X, sc, 0, lane);
  }

  // ---- merge Jacobian (:620-627): X[0..7] = dzs, X[8..15] = dzg
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    f32x4 s0 = load_tile(sc, T_S0 + t, lane);
    f32x4 s1 = 1.f - s0;
    f32x4 dM = X[t], dm = X[8 + t];
    X[t] = s0 * dM + s1 * dm;
    X[8 + t] = s1 * dM + s0 * dm;
  }
  // ---- encoder[-1]^T, then ⊙ σ10(y2 of encoder block 1) -> Y
  bwd_layer<8, 8, 2, false, true>(W, Bk + OFF_E3 * 4, X, Y, sc, T_EBLK + 32 * 1 + 16, lane);
  // ---- encoder blocks, reverse (:633-636)
#pragma unroll 1
  for (int b = 1; b >= 0; --b) {
    const int wa = opaque(Bk + (OFF_EBLK + (2 * b) * SZ_E) * 4);
    const int wb = opaque(Bk + (OFF_EBLK + (2 * b + 1) * SZ_E) * 4);
    bwd_layer<8, 8, 2, false, true>(W, wb, Y, X, sc, T_EBLK + 32 * b, lane);
    // dh = E_i^T da + dr, then ⊙ σ10 of the layer below (block 0's y2, or encoder[0])
    bwd_layer<8, 8, 2, true, true>(W, wa, X, Y, sc, b > 0 ? T_EBLK + 16 : T_E0, lane);
  }

  // ---- encoder[0]^T (256 x 128: OT 16, KT 8) fused with the Fourier Jacobian (:639-645)
  // Step (kf, kt) loads fragments (kf, kt) [dφ_sin rows] and (kf + 8, kt) [dφ_cos rows].
  float acc[2][DIM];
#pragma unroll
  for (int i = 0; i < 16; ++i) PNTF_DBG(32 + i, Y[i]);
#pragma unroll
  for (int d = 0; d < DIM; ++d) acc[0][d] = acc[1][d] = 0.f;
  f32x4 ph[2][2];
  pipelined<64, 2, PF_STEPS, SITE_FOLD>(
      W, lane * 16,
      [&](int st, int l) { return frag<8>(Bk + OFF_E0 * 4, st / 8 + 8 * l, st % 8); },
      [&](auto st, const f32x4 (&a)[2]) {
        constexpr int kf = decltype(st)::value / 8, kt = decltype(st)::value % 8;
        if constexpr (kt == 0) {
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int c = 0; c < 2; ++c) ph[u][c] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            ph[0][c] = mfma(a[0][s], Y[c * 8 + kt][s], ph[0][c]);
            ph[1][c] = mfma(a[1][s], Y[c * 8 + kt][s], ph[1][c]);
          }
        if constexpr (kt == 7) {
          f32x4 w[DIM], q[2];
          fourier_tile<DIM>(io, kf, g, w, q);
#pragma unroll
          for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
              float sn, cs;
              sincos_fast(q[c][s], sn, cs);
              float gg = ph[0][c][s] * cs - ph[1][c][s] * sn;
#pragma unroll
              for (int d = 0; d < DIM; ++d) acc[c][d] = fmaf(w[d][s], gg, acc[c][d]);
            }
        }
      });
#pragma unroll
  for (int d = 0; d < DIM; ++d) {
    float a0 = acc[0][d], a1 = acc[1][d];
    PNTF_DBG(48 + d, (f32x4{a0, a1, 0.f, 0.f}));
    a0 += __shfl_xor(a0, 16);
    a1 += __shfl_xor(a1, 16);
    a0 += __shfl_xor(a0, 32);
    a1 += __shfl_xor(a1, 32);
    PNTF_DBG(56 + d, (f32x4{a0, a1, 0.f, 0.f}));
    ds[d] = a0;
    dg[d] = a1;
  }
}

// ---------------------------------------------------------------- epilogues (A9/A10)
// Model.Gradient (:1223-1248): v_e = -(σ_e D/(T0 τ) - (T0/τ²) ∇_eτ), v_e /= |v_e|²
template <int DIM>
__device__ __forceinline__ void path_velocity(const float (&x)[2][6], float tau,
                                              const float (&ds)[DIM], const float (&dg)[DIM],
                                              float (&vs)[DIM], float (&vg)[DIM]) {
  float D[DIM];
  float T0sq = 0.f;
#pragma unroll
  for (int d = 0; d < DIM; ++d) {
    D[d] = x[1][d] - x[0][d];
    T0sq = fmaf(D[d], D[d], T0sq);
  }
  float T0 = sqrtf(T0sq);
  float c1 = 1.f / (T0 * tau);
  float c2 = T0 / (tau * tau);
  float ns = 0.f, ng = 0.f;
#pragma unroll
  for (int d = 0; d < DIM; ++d) {
    vg[d] = -(c1 * D[d] - c2 * dg[d]);
    vs[d] = -(c1 * (-D[d]) - c2 * ds[d]);
    ng = fmaf(vg[d], vg[d], ng);
    ns = fmaf(vs[d], vs[d], ns);
  }
  float is = 1.f / ns, ig = 1.f / ng;
#pragma unroll
  for (int d = 0; d < DIM; ++d) {
    vs[d] *= is;
    vg[d] *= ig;
  }
}

template <int DIM>
__device__ __forceinline__ bool load_pair(const float* __restrict__ xp,
                                          const float* __restrict__ Btab,
                                          const int32_t* __restrict__ env, int64_t n,
                                          int32_t n_env, int64_t pair, PairIO& io) {
  int64_t pc = pair < n ? pair : n - 1;
  bool ok = pair < n;
  int e = env ? env[pc] : 0;
  if (e < 0 || e >= n_env) {
    ok = false;
    e = 0;
  }
  io.Bw = Btab + (int64_t)e * DIM * H;
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int d = 0; d < 6; ++d) io.x[c][d] = d < DIM ? xp[pc * 2 * DIM + c * DIM + d] : 0.f;
  return ok;
}

// ---------------------------------------------------------------- kernels
// Persistent body: wave `slot` of `nslots` takes tiles slot, slot + nslots, ...
template <int DIM, int KIND>
__device__ __forceinline__ void field_body(const FieldArgs& a, int slot, int nslots) {
  constexpr bool GRAD = KIND != K_TAU && KIND != K_TRAVEL;
  const int lane = threadIdx.x & 63;
  const int64_t ntiles = (a.n + TILE - 1) / TILE;
  const Scratch sc = make_scratch(GRAD ? a.ws + (int64_t)slot * SCRATCH_FLOATS_PER_WAVE : nullptr);
  const float nan = __builtin_nanf("");
  for (int64_t tile = slot; tile < ntiles; tile += nslots) {
    f32x4 X[16], Y[16];
    const int64_t pair = tile * TILE + (lane & 15);
    PairIO io;
    const bool ok = load_pair<DIM>(a.xp, a.Btab, a.env, a.n, a.n_env, pair, io);
    float tau = forward_pass<DIM, GRAD>(a.P, io, X, Y, sc, a.compat, lane);
    if (GRAD) drain_stores();
    const bool store = (lane < 16) && pair < a.n;
    if (!ok) tau = nan;
    if (KIND == K_TAU) {
      if (store) a.out0[pair] = tau;
    } else if (KIND == K_TRAVEL) {
      float T0sq = 0.f;
#pragma unroll
      for (int d = 0; d < DIM; ++d) {
        float D = io.x[1][d] - io.x[0][d];
        T0sq = fmaf(D, D, T0sq);
      }
      if (store) a.out0[pair] = sqrtf(T0sq) / tau;
    } else {
      float ds[DIM], dg[DIM];
      backward_pass<DIM>(a.P, io, tau, X, Y, sc, lane, ds, dg);
      if (KIND == K_TAU_GRAD) {
        if (store) {
          a.out0[pair] = tau;
#pragma unroll
          for (int d = 0; d < DIM; ++d) {
            a.out1[pair * 2 * DIM + d] = ok ? ds[d] : nan;
            a.out1[pair * 2 * DIM + DIM + d] = ok ? dg[d] : nan;
          }
        }
      } else if (KIND == K_VELOCITY) {
        float vs[DIM], vg[DIM];
        path_velocity<DIM>(io.x, tau, ds, dg, vs, vg);
        if (store) {
#pragma unroll
          for (int d = 0; d < DIM; ++d) {
            a.out0[pair * 2 * DIM + d] = vs[d];
            a.out0[pair * 2 * DIM + DIM + d] = vg[d];
          }
          if (a.out1) a.out1[pair] = tau;
        }
      } else {  // K_SPEED (Model.Speed, :1201-1213)
        float T0 = 0.f, gg = 0.f, gD = 0.f;
#pragma unroll
        for (int d = 0; d < DIM; ++d) {
          float D = io.x[1][d] - io.x[0][d];
          T0 = fmaf(D, D, T0);
          gg = fmaf(dg[d], dg[d], gg);
          gD = fmaf(dg[d], D, gD);
        }
        float S = T0 * gg - 2.f * tau * gD + tau * tau;
        if (store) a.out0[pair] = tau * tau / sqrtf(S);
      }
    }
  }
}

template <int DIM, int KIND>
__global__ __launch_bounds__(256, WAVES_PER_SIMD) void field_kernel(FieldArgs a) {
  field_body<DIM, KIND>(a, blockIdx.x * WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6),
                        gridDim.x * WAVES);
}

// Batched bidirectional planner: q independent copies of the batch-1 loop of
// test/gib_plan.py:74-86 (arm: test/arm_plan.py:140-152) with a per-query freeze.
template <int DIM>
__global__ __launch_bounds__(256, WAVES_PER_SIMD) void plan_kernel(PlanArgs a) {
  const int lane = threadIdx.x & 63;
  const int slot = blockIdx.x * WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nslots = gridDim.x * WAVES;
  const int64_t ntiles = (a.q + TILE - 1) / TILE;
  const Scratch sc = make_scratch(a.ws + (int64_t)slot * SCRATCH_FLOATS_PER_WAVE);
  const int cap = a.max_iter + 1;
  const int64_t rows = (int64_t)cap + 1;
  for (int64_t tile = slot; tile < ntiles; tile += nslots) {
    f32x4 X[16], Y[16];
    const int64_t qi = tile * TILE + (lane & 15);
    PairIO io;
    const bool ok = load_pair<DIM>(a.xp0, a.Btab, a.env, a.q, a.n_env, qi, io);
    const bool store = (lane < 16) && qi < a.q;
    float* prow = a.path + (store ? qi : 0) * rows * 2 * DIM;
    auto dist = [&]() {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < DIM; ++d) {
        float D = io.x[1][d] - io.x[0][d];
        s = fmaf(D, D, s);
      }
      return sqrtf(s);
    };
    bool active = ok && dist() > a.tol;
    if (store) {
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int d = 0; d < DIM; ++d) prow[c * DIM + d] = io.x[c][d];
    }
    int nsteps = 0;
    int it = 0;
    for (; it < cap; ++it) {
      if (!__any(active)) break;
      float tau = forward_pass<DIM, true>(a.P, io, X, Y, sc, a.compat, lane);
      drain_stores();
      float ds[DIM], dg[DIM], vs[DIM], vg[DIM];
      backward_pass<DIM>(a.P, io, tau, X, Y, sc, lane, ds, dg);
      path_velocity<DIM>(io.x, tau, ds, dg, vs, vg);
      if (active) {
#pragma unroll
        for (int d = 0; d < DIM; ++d) {
          io.x[0][d] = io.x[0][d] + a.step * vs[d];
          io.x[1][d] = io.x[1][d] + a.step * vg[d];
        }
        ++nsteps;
        if (!(dist() > a.tol)) active = false;
      }
      if (store) {
        float* pr = prow + (int64_t)(it + 1) * 2 * DIM;
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int d = 0; d < DIM; ++d) pr[c * DIM + d] = io.x[c][d];
      }
    }
    if (store) {
      for (int64_t r = it + 1; r < rows; ++r) {
        float* pr = prow + r * 2 * DIM;
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int d = 0; d < DIM; ++d) pr[c * DIM + d] = io.x[c][d];
      }
      a.steps[qi] = ok ? nsteps : -1;
    }
  }
}

#if defined(PNTF_UTIL)
// ---------------------------------------------------------------- weight packing
// dst[((ot*KT + kt)*64 + lane)*4 + s] = M[16 ot + (lane & 15)][16 kt + 4 (lane >> 4) + s]
// with M = src (rows x cols, row stride ld) or M = src^T (trans).
__global__ void pack_kernel(const float* __restrict__ src, int rows, int cols, int ld,
                            int trans, float* __restrict__ dst) {
  int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= (int64_t)rows * cols) return;
  int s = o & 3;
  int lane = (o >> 2) & 63;
  int64_t rest = o >> 8;
  int KT = cols / 16;
  int kt = rest % KT;
  int ot = rest / KT;
  int n = 16 * ot + (lane & 15);
  int k = 16 * kt + 4 * (lane >> 4) + s;
  dst[o] = trans ? src[(int64_t)k * ld + n] : src[(int64_t)n * ld + k];
}

__global__ void copy_kernel(const float* __restrict__ src, int n, float* __restrict__ dst) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

// Deterministic single-workgroup sum (fp64 accumulation) for loss_n.
__global__ __launch_bounds__(1024) void sum_kernel(const float* __restrict__ x, int64_t n,
                                                   double* __restrict__ out) {
  __shared__ double part[1024];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 1024) s += (double)x[i];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int w = 512; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = part[0];
}

#endif  // PNTF_UTIL

}  // namespace pntf
