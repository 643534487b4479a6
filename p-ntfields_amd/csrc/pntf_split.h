#pragma once
// Out-tile-split τ / ∇τ passes for latency-bound batches ("split kernels").
//
// The throughput kernels of pntf_field.h give one wave a whole 16-pair tile, so a batch of q
// pairs keeps only ceil(q/16) SIMDs busy: the 1024-query arm planner (BASELINE config C5)
// ran on 64 of the chip's 1024 SIMDs, and a batch-1 planner step (test/gib_plan.py, Q = 1)
// on one.  Here the four waves of a workgroup (one per SIMD) share one pair tile instead:
//   * wave w computes out tiles [w·OT/4, (w+1)·OT/4) of every layer (the packed fragments
//     of those tiles are contiguous, so the weight stream is the same ring as before with a
//     per-wave scalar base offset);
//   * its output tiles go to LDS, one s_barrier, and every wave reads the whole activation
//     back as the next layer's B operand (the register tile layout is the LDS layout:
//     1 KiB per tile, 16 B per lane, conflict-free ds_read_b128 / ds_write_b128);
//   * residual inputs are the wave's own slice of the block input, picked from the full
//     register bank before it is overwritten (uniform selects, no LDS);
//   * saved σ10 tiles stay per wave in its scratch slot: a feature tile is owned by the same
//     wave in the forward and the reverse sweep, so each wave reads back only what it wrote;
//   * the head dot product and the Fourier fold are reduced across the 4 waves through LDS
//     in a fixed order, so every wave holds the same τ and ∇τ (the planner's freeze test and
//     loop exit are wave-uniform and identical in all four waves).
// Per layer each wave does a quarter of the MFMAs plus one 16 KiB LDS read, so a planner
// step takes about a third of the one-wave time.
#include "pntf_field.h"

namespace pntf {

// Waves sharing a pair tile: SPLIT_WAVES = 8 (two per SIMD, so one wave's exchange and
// epilogue run beside the other's MFMAs) or 4 (one per SIMD); pntf_common.h PNTF_SPLIT.
constexpr int SPLIT = SPLIT_WAVES;
static_assert(SPLIT == 4 || SPLIT == 8, "split width");
constexpr int EOTL = 8 / SPLIT;    // local out tiles of an encoder layer (OT 8, 2 columns)
constexpr int GOTL = 16 / SPLIT;   // ... of a generator layer (OT 16)
constexpr int G3OTL = 8 / SPLIT;   // ... of generator[-2] (OT 8)
constexpr int FKL = 8 / SPLIT;     // Fourier feature tiles of the fold per wave (8 in all)
constexpr int GNL = GOTL < 4 ? GOTL : 4;   // weight fragments per step of a generator layer
constexpr int XBUF_FLOATS = 16 * 256;         // one activation: 16 tiles x 64 lanes x 4
constexpr int RED_FLOATS = SPLIT * 12 * 64;   // cross-wave partial sums (≤ 2·DIM per lane)
constexpr int SPLIT_LDS_FLOATS = 2 * XBUF_FLOATS + RED_FLOATS;

#ifdef PNTF_DEBUG_DUMP   // diagnostics only (tests/diag/split_dump.py)
__device__ float* pntf_dbg;
#ifndef PNTF_DUMP_WAVE
#define PNTF_DUMP_WAVE 0
#endif
#define PNTF_DUMPT(k, i, v)                                                            \
  if (blockIdx.x == 0 && sp.w == PNTF_DUMP_WAVE && pntf_dbg)                           \
    *reinterpret_cast<f32x4*>(pntf_dbg + (((k) * 16 + (i)) * 64 + sp.lane) * 4) = (v);
#define PNTF_DUMPW(k, i, v)                                                            \
  if (blockIdx.x == 0 && pntf_dbg)                                                     \
    *reinterpret_cast<f32x4*>(pntf_dbg + ((((k) + sp.w) * 16 + (i)) * 64 + sp.lane) * 4) = (v);
#define PNTF_DUMPX(k) \
  for (int i_ = 0; i_ < 16; ++i_) { PNTF_DUMPT(k, i_, X[i_]) }
#else
#define PNTF_DUMPT(k, i, v)
#define PNTF_DUMPW(k, i, v)
#define PNTF_DUMPX(k)
#endif

typedef __attribute__((address_space(3))) float lds_f;
typedef __attribute__((address_space(3))) f32x4 lds_f4;

// Diagnostics only (DESIGN.md §7.1 bisection, tests/diag): -DPNTF_DIAG_WAITS=<bit mask> puts a
// full s_waitcnt at the marked points of the split kernels.
#ifndef PNTF_DIAG_WAITS
#define PNTF_DIAG_WAITS 0
#endif
#define PNTF_DIAG_WAIT(bit)                                                                  \
  if constexpr ((PNTF_DIAG_WAITS >> (bit)) & 1) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

// Every wave's LDS writes done, then the workgroup barrier.  Written as one asm block with
// a memory clobber: the s_barrier builtin alone is not a compiler barrier for LDS accesses.
__device__ __forceinline__ void wg_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

struct Split {
  lds_f* lds;
  int w, lane;
  __device__ lds_f4* tile(int buf, int t) const {
    return reinterpret_cast<lds_f4*>(lds + buf * XBUF_FLOATS + t * 256 + lane * 4);
  }
  __device__ lds_f* red(int wave, int j) const {
    return lds + 2 * XBUF_FLOATS + (wave * 12 + j) * 64 + lane;
  }
};

// Local out tiles L[c·OTL + t] (global tile c·OTG + w·OTL + t) -> LDS buffer -> every
// wave's full bank X[0 .. NC·OTG).
template <int OTL, int NC>
__device__ __forceinline__ void exchange(const Split& sp, int buf, const f32x4 (&L)[16],
                                         f32x4 (&X)[16]) {
  constexpr int OTG = OTL * SPLIT;
  PNTF_DIAG_WAIT(0)
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int t = 0; t < OTL; ++t) {
#ifdef PNTF_DIAG_EXNOP   // diagnostics only (tests/diag split variants)
      asm volatile("s_nop 7\n\ts_nop 7" ::"v"(L[c * OTL + t]));
#endif
      *sp.tile(buf, c * OTG + sp.w * OTL + t) = L[c * OTL + t];
    }
  wg_sync();
#pragma unroll
  for (int i = 0; i < NC * OTG; ++i) {
    X[i] = *sp.tile(buf, i);
    if constexpr ((PNTF_DIAG_WAITS >> 5) & 1) {   // at most 8 LDS reads in flight
      if (i == 7) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
  PNTF_DIAG_WAIT(1)
#ifdef PNTF_DIAG_EXNOP
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_nop 7" ::: "memory");
#endif
}

// The wave's slice of a full bank: R[c·OTL + t] = X[c·OTG + w·OTL + t] (w is uniform).
template <int OTL, int NC>
__device__ __forceinline__ void slice(const f32x4 (&X)[16], int w, f32x4 (&R)[16]) {
  constexpr int OTG = OTL * SPLIT;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int t = 0; t < OTL; ++t) {
      f32x4 v = X[c * OTG + t];
#pragma unroll
      for (int q = 1; q < SPLIT; ++q) {
        // opaque condition: a select chain on w == q would otherwise be folded into a
        // runtime-indexed X[.], which sends the whole bank to scratch
        int m = w == q;
        asm volatile("" : "+v"(m));
        v = m ? X[c * OTG + q * OTL + t] : v;
      }
      R[c * OTL + t] = v;
    }
}

// Sum of one value per lane over the 4 waves, in wave order (identical in every wave).
template <int NV>
__device__ __forceinline__ void reduce_waves(const Split& sp, float (&v)[NV]) {
  PNTF_DIAG_WAIT(8)
#pragma unroll
  for (int j = 0; j < NV; ++j) *sp.red(sp.w, j) = v[j];
  wg_sync();
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    float s = *sp.red(0, j);
#pragma unroll
    for (int q = 1; q < SPLIT; ++q) s += *sp.red(q, j);
    v[j] = s;
  }
}

// Byte offset of wave w's first fragment in a packed (OTG x KT) layer.
template <int OTG, int KT>
__device__ __forceinline__ int wofs(int w) {
  return w * (OTG / SPLIT) * KT * 1024;
}

// Ring head of the split forward pass: encoder[0], local out tiles EOTL·w + o; step j reads
// fragments (local out tile j % EOTL, k tile j / EOTL + 8 l).
struct SE0Head {
  int base;
  __device__ int operator()(int j, int l) const {
    return base + (((j % EOTL) * 16 + j / EOTL + 8 * l) * 64) * 16;
  }
};
__device__ __forceinline__ SE0Head se0_head(int w) {
  return SE0Head{(OFF_FWD + OFF_E0) * 4 + wofs<8, 16>(w)};
}

struct SplitCarry {
  f32x4 sg3[8];       // σ10 of generator[-2], local tiles
  f32x4 g4w[G3OTL];   // generator[-1].weight rows of the local tiles
};

// Split forward pass (NN.out, :215-259).  X is the full bank; returns τ (same in all waves).
template <int DIM, bool GRAD, int NLA, class AfterF>
__device__ __forceinline__ float split_forward(Ring& ring, const float* __restrict__ P,
                                               const PairIO& io, f32x4 (&X)[16], SplitCarry& cy,
                                               Scratch sc, int compat, const Split& sp,
                                               AfterF after) {
  const int lane = sp.lane, g = lane >> 4, w = sp.w;
  const Rsrc W = make_rsrc(P, PACKED_FLOATS * 4);
  constexpr int BB = OFF_BIAS * 4;
  constexpr int F = OFF_FWD * 4;
  const float cm = compat ? 1.f : 0.f;
  f32x4 L[16], R[16];

  // ---- encoder[0] on Fourier features (:186-190, :227): local out tiles ol < EOTL of both
  // columns; every wave computes all 256 features (they are its B operand).
  f32x4 eb[EOTL];
#pragma unroll
  for (int i = 0; i < 2 * EOTL; ++i) L[i] = zero4();
  {
    f32x4 sn[2], cs[2];
    f32x4 bw[2][DIM];
#pragma unroll
    for (int d = 0; d < DIM; ++d) bw[0][d] = ld4(io.Bw + d * H + 4 * g);
    const int e0 = F + OFF_E0 * 4 + wofs<8, 16>(w);
    const int we = F + OFF_EBLK * 4 + wofs<8, 8>(w);
    run_steps<8 * EOTL, 2, 2, SITE_FWD_E0>(
        ring, W, lane * 16, SE0Head{e0}, Head<8, 2>{we},
        [&](auto st, const f32x4 (&a)[2]) {
          constexpr int S = decltype(st)::value;
          constexpr int kt = S / EOTL, ol = S % EOTL;
          if constexpr (S == 1) {
#pragma unroll
            for (int t = 0; t < EOTL; ++t)
              eb[t] = bload(W, g * 16, BB + (B_E0 + 16 * (EOTL * w + t)) * 4);
          }
          if constexpr (ol == 0) {
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
              for (int s = 0; s < 4; ++s) {
                float q = 0.f;
#pragma unroll
                for (int d = 0; d < DIM; ++d) q = fmaf(io.x[c][d], TWO_PI * bw[kt & 1][d][s], q);
                float x0, x1;
                sincos_fast(q, x0, x1);
                sn[c][s] = x0;
                cs[c][s] = x1;
              }
          }
          // the next Fourier tile's B rows (after this tile's projections)
          if constexpr (ol == EOTL - 1 && kt < 7) {
#pragma unroll
            for (int d = 0; d < DIM; ++d)
              bw[(kt + 1) & 1][d] = ld4(io.Bw + d * H + 16 * (kt + 1) + 4 * g);
          }
#pragma unroll
          for (int s = 0; s < 4; ++s) {
#pragma unroll
            for (int c = 0; c < 2; ++c) L[c * EOTL + ol] = mfma(a[0][s], sn[c][s], L[c * EOTL + ol]);
#pragma unroll
            for (int c = 0; c < 2; ++c) L[c * EOTL + ol] = mfma(a[1][s], cs[c][s], L[c * EOTL + ol]);
          }
        });
  }
  // bias, softplus, σ (compat: the out_backgrad quirk :435-438 stores σ10(softplus(y)))
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int i = 0; i < EOTL; ++i) {
      const int t = c * EOTL + i;
      f32x4 s, sg;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        SpSig v = sp_sig(L[t][r] + eb[i][r]);
        s[r] = v.sp;
        sg[r] = fmaf(cm, __builtin_amdgcn_rcpf(2.f - v.sg) - v.sg, v.sg);
      }
      L[t] = s;
      if (GRAD) store_tile(sc, T_E0 + t, lane, sg);
    }
  exchange<EOTL, 2>(sp, 0, L, X);
  PNTF_DUMPX(0)

  // ---- encoder residual blocks (:228-232)
  const int BE = BB + B_EBLK * 4 + w * EOTL * 16 * 4;
  const int WE = F + OFF_EBLK * 4 + wofs<8, 8>(w);
  {
    slice<EOTL, 2>(X, w, R);
    FwdAct<EOTL, 8, 2, false, GRAD> a0{W, BE, L, sc, T_EBLK, lane, cy.sg3};
    layer<EOTL, 8, 2, 2, SITE_FWD_ENC, 2>(ring, W, WE, X, lane, a0, NoPre{},
                                           Head<8, 2>{WE + SZ_E * 4});
    flush(a0);
    exchange<EOTL, 2>(sp, 1, L, X);
    PNTF_DUMPX(1)
#pragma unroll
    for (int i = 0; i < 2 * EOTL; ++i) L[i] = R[i];
    FwdAct<EOTL, 8, 2, true, GRAD> b0{W, BE + 128 * 4, L, sc, T_EBLK + 16, lane, cy.sg3};
    layer<EOTL, 8, 2, 2, SITE_FWD_ENC, 2>(ring, W, WE + SZ_E * 4, X, lane, b0, NoPre{},
                                           Head<8, 2>{WE + 2 * SZ_E * 4});
    flush(b0);
    exchange<EOTL, 2>(sp, 0, L, X);
    PNTF_DUMPX(2)
  }
  {
    slice<EOTL, 2>(X, w, R);
    FwdAct<EOTL, 8, 2, false, GRAD> a1{W, BE + 256 * 4, L, sc, T_EBLK + 32, lane, cy.sg3};
    layer<EOTL, 8, 2, 2, SITE_FWD_ENC, 2>(ring, W, WE + 2 * SZ_E * 4, X, lane, a1, NoPre{},
                                           Head<8, 2>{WE + 3 * SZ_E * 4});
    flush(a1);
    exchange<EOTL, 2>(sp, 1, L, X);
    PNTF_DUMPX(3)
#pragma unroll
    for (int i = 0; i < 2 * EOTL; ++i) L[i] = R[i];
    FwdAct<EOTL, 8, 2, true, GRAD> b1{W, BE + 384 * 4, L, sc, T_EBLK + 48, lane, cy.sg3};
    layer<EOTL, 8, 2, 2, SITE_FWD_ENC, 2>(ring, W, WE + 3 * SZ_E * 4, X, lane, b1, NoPre{},
                                           Head<8, 2>{F + OFF_E3 * 4 + wofs<8, 8>(w)});
    flush(b1);
    exchange<EOTL, 2>(sp, 0, L, X);
    PNTF_DUMPX(4)
  }
  // ---- encoder[-1] (:234) -> X = [zs | zg]
  {
    FwdLin<EOTL, 8, 2> e3{W, BB + (B_E3 + EOTL * 16 * w) * 4, L, lane};
    layer<EOTL, 8, 2, 2, SITE_FWD_ENC, GNL>(ring, W, F + OFF_E3 * 4 + wofs<8, 8>(w), X, lane, e3,
                                             NoPre{},
                                             Head<16>{F + OFF_GBLK * 4 + wofs<16, 16>(w)});
    flush(e3);
    exchange<EOTL, 2>(sp, 1, L, X);
    PNTF_DUMPX(5)
  }

  // ---- merge (:236-244), in place and redundantly in every wave: X = u = [M | m]
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    f32x4 s0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float zs = X[t][r], zg = X[8 + t][r];
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

  // ---- generator residual blocks (:246-249)
#pragma unroll 1
  for (int i = 0; i < 3; ++i) {
    const int wa = opaque(F + (OFF_GBLK + (2 * i) * SZ_G) * 4 + wofs<16, 16>(w));
    const int wb = opaque(F + (OFF_GBLK + (2 * i + 1) * SZ_G) * 4 + wofs<16, 16>(w));
    const int wn = opaque(i < 2 ? F + (OFF_GBLK + (2 * i + 2) * SZ_G) * 4 + wofs<16, 16>(w)
                                : F + OFF_G3 * 4 + wofs<8, 16>(w));
    const int bg = BB + (B_GBLK + (2 * i) * 256 + GOTL * 16 * w) * 4;
    slice<GOTL, 1>(X, w, R);
    FwdAct<GOTL, 16, 1, false, GRAD> ga{W, bg, L, sc, T_GBLK + 32 * i, lane, cy.sg3};
    layer<GOTL, 16, 1, 1, SITE_FWD_GEN, GNL>(ring, W, wa, X, lane, ga, NoPre{}, Head<16>{wb});
    flush(ga);
    exchange<GOTL, 1>(sp, 0, L, X);
    PNTF_DUMPX(6)
#pragma unroll
    for (int t = 0; t < GOTL; ++t) L[t] = R[t];
    FwdAct<GOTL, 16, 1, true, GRAD> gb{W, bg + 256 * 4, L, sc, T_GBLK + 32 * i + 16, lane,
                                       cy.sg3};
    // the last block hands over to generator[-2] (G3OTL local out tiles per step)
    if (i < 2)
      layer<GOTL, 16, 1, 1, SITE_FWD_GEN, GNL>(ring, W, wb, X, lane, gb, NoPre{}, Head<16>{wn});
    else
      layer<GOTL, 16, 1, 1, SITE_FWD_GEN, G3OTL>(ring, W, wb, X, lane, gb, NoPre{},
                                                  Head<16>{wn});
    flush(gb);
    exchange<GOTL, 1>(sp, 1, L, X);
    PNTF_DUMPX(7)
  }

  // ---- generator[-2] + act (:251-252): local tiles L[0..G3OTL), σ kept for the reverse sweep
#pragma unroll
  for (int t = 0; t < G3OTL; ++t)
    cy.g4w[t] = bload(W, g * 16, BB + (B_G4W + 16 * (G3OTL * w + t)) * 4);
  const float g4b = bload(W, 0, BB + B_G4B * 4)[0];
  {
    FwdAct<G3OTL, 16, 1, false, GRAD, GRAD> g3{W, BB + (B_G3 + G3OTL * 16 * w) * 4, L, sc, T_G3,
                                               lane, cy.sg3};
    layer<G3OTL, 16, 1, 1, SITE_FWD_GEN, NLA>(ring, W, F + OFF_G3 * 4 + wofs<8, 16>(w), X, lane,
                                               g3, NoPre{}, after);
    flush(g3);
  }
  // ---- head (:254-255): partial dot of the local tiles, summed over the waves
  float part[1] = {0.f};
#pragma unroll
  for (int t = 0; t < G3OTL; ++t)
#pragma unroll
    for (int s = 0; s < 4; ++s) part[0] = fmaf(cy.g4w[t][s], L[t][s], part[0]);
  part[0] += __shfl_xor(part[0], 16);
  part[0] += __shfl_xor(part[0], 32);
  reduce_waves<1>(sp, part);
  const float y4 = part[0] + g4b;
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-0.144269504088896341f * y4));
}

// Split reverse sweep (exact, or out_backgrad when the forward stored the quirk).  On entry
// the ring holds the G3^T head of this wave; on return the first PF steps of `after`.
template <int DIM, int NLA, class AfterF>
__device__ __forceinline__ void split_backward(Ring& ring, const float* __restrict__ P,
                                               const PairIO& io, float tau, f32x4 (&X)[16],
                                               const SplitCarry& cy, Scratch sc, const Split& sp,
                                               float (&ds)[DIM], float (&dg)[DIM],
                                               AfterF after) {
  const int lane = sp.lane, g = lane >> 4, w = sp.w;
  const Rsrc W = make_rsrc(P, PACKED_FLOATS * 4);
  constexpr int Bk = OFF_BWD * 4;
  f32x4 L[16], R[16];

  // ---- head and generator[-2] (:592-613): dv = d · G4 ⊙ σ10(y3), local tiles -> X[0..7]
  const float dd = 0.1f * tau * (1.f - tau);
  PNTF_DIAG_WAIT(2)
#pragma unroll
  for (int t = 0; t < G3OTL; ++t) L[t] = (dd * cy.g4w[t]) * cy.sg3[t];
  exchange<G3OTL, 1>(sp, 0, L, X);
  PNTF_DUMPX(20)
  // du = G3^T dv ⊙ σ10(y2 of generator block 2)   (G3^T: 256 x 128, OT 16, KT 8)
  {
    Bwd<GOTL, 8, 1, false, true> l{L, sc, T_GBLK + 32 * 2 + 16, lane};
    layer<GOTL, 8, 1, 1, SITE_BWD_GEN, GNL>(
        ring, W, Bk + OFF_G3 * 4 + wofs<16, 8>(w), X, lane, l, NoPre{},
        Head<16>{Bk + (OFF_GBLK + 5 * SZ_G) * 4 + wofs<16, 16>(w)});
    flush(l);
    exchange<GOTL, 1>(sp, 1, L, X);
    PNTF_DUMPX(21)
  }
  // ---- generator blocks, reverse (:615-618)
#pragma unroll 1
  for (int i = 2; i >= 0; --i) {
    const int wa = opaque(Bk + (OFF_GBLK + (2 * i) * SZ_G) * 4 + wofs<16, 16>(w));
    const int wb = opaque(Bk + (OFF_GBLK + (2 * i + 1) * SZ_G) * 4 + wofs<16, 16>(w));
    slice<GOTL, 1>(X, w, R);   // dr
    Bwd<GOTL, 16, 1, false, true> lb{L, sc, T_GBLK + 32 * i, lane};
    layer<GOTL, 16, 1, 1, SITE_BWD_GEN, GNL>(ring, W, wb, X, lane, lb, NoPre{}, Head<16>{wa});
    flush(lb);
    exchange<GOTL, 1>(sp, 0, L, X);
    PNTF_DUMPX(22)
#pragma unroll
    for (int t = 0; t < GOTL; ++t) L[t] = R[t];
    if (i > 0) {
      const int wn = opaque(Bk + (OFF_GBLK + (2 * i - 1) * SZ_G) * 4 + wofs<16, 16>(w));
      Bwd<GOTL, 16, 1, true, true> la{L, sc, T_GBLK + 32 * (i - 1) + 16, lane};
      layer<GOTL, 16, 1, 1, SITE_BWD_GEN, GNL>(ring, W, wa, X, lane, la, NoPre{}, Head<16>{wn});
      flush(la);
    } else {
      Bwd<GOTL, 16, 1, true, false> la{L, sc, 0, lane};
      layer<GOTL, 16, 1, 1, SITE_BWD_GEN, 2>(ring, W, wa, X, lane, la, NoPre{},
                                             Head<8, 2>{Bk + OFF_E3 * 4 + wofs<8, 8>(w)});
      flush(la);
    }
    exchange<GOTL, 1>(sp, 1, L, X);
    PNTF_DUMPX(23)
  }
  // ---- merge Jacobian (:620-627), redundantly in every wave: X = [dzs | dzg]
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    f32x4 s0 = load_tile(sc, T_S0 + t, lane);
    PNTF_DUMPT(30, t, s0)
    f32x4 s1 = 1.f - s0;
    f32x4 dM = X[t], dm = X[8 + t];
    X[t] = s0 * dM + s1 * dm;
    X[8 + t] = s1 * dM + s0 * dm;
  }
  PNTF_DIAG_WAIT(3)
#ifdef PNTF_DIAG_MERGENOP   // diagnostics only (tests/diag split variants)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#endif
  // ---- encoder[-1]^T, then ⊙ σ10(y2 of encoder block 1)
  const int WE = Bk + OFF_EBLK * 4 + wofs<8, 8>(w);
  {
    Bwd<EOTL, 8, 2, false, true> e3{L, sc, T_EBLK + 32 * 1 + 16, lane};
    layer<EOTL, 8, 2, 2, SITE_BWD_ENC, 2>(ring, W, Bk + OFF_E3 * 4 + wofs<8, 8>(w), X, lane, e3,
                                           NoPre{}, Head<8, 2>{WE + 3 * SZ_E * 4});
    flush(e3);
    PNTF_DIAG_WAIT(4)
#ifdef PNTF_DEBUG_DUMP
    for (int i_ = 0; i_ < 2 * EOTL; ++i_) { PNTF_DUMPW(40, i_, L[i_]) }
#endif
    exchange<EOTL, 2>(sp, 0, L, X);
    PNTF_DUMPX(24)
  }
  // ---- encoder blocks, reverse (:633-636)
  {
    slice<EOTL, 2>(X, w, R);
    Bwd<EOTL, 8, 2, false, true> b1{L, sc, T_EBLK + 32, lane};
    layer<EOTL, 8, 2, 2, SITE_BWD_ENC, 2>(ring, W, WE + 3 * SZ_E * 4, X, lane, b1, NoPre{},
                                           Head<8, 2>{WE + 2 * SZ_E * 4});
    flush(b1);
    exchange<EOTL, 2>(sp, 1, L, X);
    PNTF_DUMPX(25)
#pragma unroll
    for (int i = 0; i < 2 * EOTL; ++i) L[i] = R[i];
    Bwd<EOTL, 8, 2, true, true> a1{L, sc, T_EBLK + 16, lane};
    layer<EOTL, 8, 2, 2, SITE_BWD_ENC, 2>(ring, W, WE + 2 * SZ_E * 4, X, lane, a1, NoPre{},
                                           Head<8, 2>{WE + 1 * SZ_E * 4});
    flush(a1);
    exchange<EOTL, 2>(sp, 0, L, X);
    PNTF_DUMPX(26)
  }
  // local Fourier feature tiles kf = FKL·w + kl of the fold (sin rows kf, cos rows kf + 8)
  const int E0T = Bk + OFF_E0 * 4 + FKL * w * 8 * 1024;
  {
    slice<EOTL, 2>(X, w, R);
    Bwd<EOTL, 8, 2, false, true> b0{L, sc, T_EBLK, lane};
    layer<EOTL, 8, 2, 2, SITE_BWD_ENC, 2>(ring, W, WE + 1 * SZ_E * 4, X, lane, b0, NoPre{},
                                           Head<8, 2>{WE});
    flush(b0);
    exchange<EOTL, 2>(sp, 1, L, X);
    PNTF_DUMPX(27)
#pragma unroll
    for (int i = 0; i < 2 * EOTL; ++i) L[i] = R[i];
    Bwd<EOTL, 8, 2, true, true> a0{L, sc, T_E0, lane};
    layer<EOTL, 8, 2, 2, SITE_BWD_ENC, 2>(ring, W, WE, X, lane, a0, NoPre{},
                                           [=](int j, int l) {
                                             return E0T + ((j / 8 + 8 * l) * 8 + j % 8) * 1024;
                                           });
    flush(a0);
    exchange<EOTL, 2>(sp, 0, L, X);
    PNTF_DUMPX(28)
  }

  // ---- encoder[0]^T fused with the Fourier Jacobian (:639-645): this wave's feature tiles,
  // then the dim-vector summed over the waves.
  f32x4 ph[FKL][2][2];   // [kl][sin|cos rows][column]
#pragma unroll
  for (int kl = 0; kl < FKL; ++kl)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int c = 0; c < 2; ++c) ph[kl][u][c] = zero4();
  f32x4 bw[FKL][DIM];
#pragma unroll
  for (int kl = 0; kl < FKL; ++kl)
#pragma unroll
    for (int d = 0; d < DIM; ++d)
      bw[kl][d] = ld4(io.Bw + d * H + 16 * (FKL * w + kl) + 4 * g);
  run_steps<8 * FKL, 2, NLA, SITE_FOLD>(
      ring, W, lane * 16,
      [&](int st, int l) { return E0T + ((st / 8 + 8 * l) * 8 + st % 8) * 1024; }, after,
      [&](auto st, const f32x4 (&a)[2]) {
        constexpr int S = decltype(st)::value;
        constexpr int kl = S / 8, kt = S % 8;
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            ph[kl][0][c] = mfma(a[0][s], X[c * 8 + kt][s], ph[kl][0][c]);
            ph[kl][1][c] = mfma(a[1][s], X[c * 8 + kt][s], ph[kl][1][c]);
          }
      });
  float acc[2 * DIM];
#pragma unroll
  for (int j = 0; j < 2 * DIM; ++j) acc[j] = 0.f;
#pragma unroll
  for (int kl = 0; kl < FKL; ++kl)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        float q = 0.f;
#pragma unroll
        for (int d = 0; d < DIM; ++d) q = fmaf(io.x[c][d], TWO_PI * bw[kl][d][s], q);
        float sn, cs;
        sincos_fast(q, sn, cs);
#ifdef PNTF_DIAG_FOLDNOP   // diagnostics only (tests/diag split variants)
        asm volatile("s_nop 7\n\ts_nop 7" : "+v"(sn), "+v"(cs));
#endif
        float gg = ph[kl][0][c][s] * cs - ph[kl][1][c][s] * sn;
#pragma unroll
        for (int d = 0; d < DIM; ++d) acc[c * DIM + d] = fmaf(TWO_PI * bw[kl][d][s], gg, acc[c * DIM + d]);
      }
#pragma unroll
  for (int j = 0; j < 2 * DIM; ++j) {
    acc[j] += __shfl_xor(acc[j], 16);
    acc[j] += __shfl_xor(acc[j], 32);
  }
  reduce_waves<2 * DIM>(sp, acc);
#pragma unroll
  for (int d = 0; d < DIM; ++d) {
    ds[d] = acc[d];
    dg[d] = acc[DIM + d];
  }
}

// τ / ∇τ / epilogues on split tiles for small batches: one workgroup per 16-pair tile
// (grid-stride), same outputs as field_kernel<DIM, KIND>.
template <int DIM, int KIND>
__global__ __launch_bounds__(64 * SPLIT, 1) void field_split_kernel(FieldArgs a) {
  constexpr bool GRAD = KIND != K_TAU && KIND != K_TRAVEL;
  __shared__ float smem[SPLIT_LDS_FLOATS];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Split sp{(lds_f*)smem, w, lane};
  const int64_t ntiles = (a.n + TILE - 1) / TILE;
  const Scratch sc = make_scratch(
      GRAD ? a.ws + ((int64_t)blockIdx.x * SPLIT + w) * SCRATCH_FLOATS_PER_WAVE : nullptr);
  const Rsrc W = make_rsrc(a.P, PACKED_FLOATS * 4);
  const SE0Head e0h = se0_head(w);
  const Head<8> g3h{(OFF_BWD + OFF_G3) * 4 + wofs<16, 8>(w)};   // G3^T local out tiles
  Ring ring;
  ring_fill<2>(ring, W, lane * 16, e0h);
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    f32x4 X[16];
    SplitCarry cy;
    const int64_t pair = tile * TILE + (lane & 15);
    PairIO io;
    const bool ok = load_pair<DIM>(a.xp, a.Btab, a.env, a.n, a.n_env, pair, io);
    float tau;
    float ds[DIM], dg[DIM];
    if constexpr (GRAD) {
      tau = split_forward<DIM, true, GNL>(ring, a.P, io, X, cy, sc, a.compat, sp, g3h);
      drain_stores();
      split_backward<DIM, 2>(ring, a.P, io, tau, X, cy, sc, sp, ds, dg, e0h);
    } else {
      tau = split_forward<DIM, false, 2>(ring, a.P, io, X, cy, sc, a.compat, sp, e0h);
    }
    const bool store = w == 0 && (lane < 16) && pair < a.n;
    store_field<DIM, KIND>(a, pair, ok, store, tau, io, ds, dg);
  }
}

// Batched planner on split tiles: one workgroup per 16-query tile (grid-stride), the loop of
// plan_kernel (test/gib_plan.py:74-86, test/arm_plan.py:140-152) with per-query freeze.
// ws holds one scratch slot per wave (4 per workgroup).
template <int DIM>
__global__ __launch_bounds__(64 * SPLIT, 1) void plan_split_kernel(PlanArgs a) {
  __shared__ float smem[SPLIT_LDS_FLOATS];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const Split sp{(lds_f*)smem, w, lane};
  const int64_t ntiles = (a.q + TILE - 1) / TILE;
  const Scratch sc = make_scratch(a.ws + ((int64_t)blockIdx.x * SPLIT + w) * SCRATCH_FLOATS_PER_WAVE);
  const Rsrc W = make_rsrc(a.P, PACKED_FLOATS * 4);
  const int cap = a.max_iter + 1;
  const int64_t rows = (int64_t)cap + 1;
  const SE0Head e0h = se0_head(w);
  const Head<8> g3h{(OFF_BWD + OFF_G3) * 4 + wofs<16, 8>(w)};   // G3^T local out tiles
  Ring ring;
  ring_fill<2>(ring, W, lane * 16, e0h);
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    f32x4 X[16];
    SplitCarry cy;
    const int64_t qi = tile * TILE + (lane & 15);
    PairIO io;
    const bool ok = load_pair<DIM>(a.xp0, a.Btab, a.env, a.q, a.n_env, qi, io);
    const bool store = w == 0 && (lane < 16) && qi < a.q;
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
      float tau = split_forward<DIM, true, GNL>(ring, a.P, io, X, cy, sc, a.compat, sp, g3h);
      drain_stores();
      float ds[DIM], dg[DIM], vs[DIM], vg[DIM];
      split_backward<DIM, 2>(ring, a.P, io, tau, X, cy, sc, sp, ds, dg, e0h);
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

}  // namespace pntf
