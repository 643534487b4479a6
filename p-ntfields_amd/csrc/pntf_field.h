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
// Workgroups (4 waves, one per SIMD) are persistent and loop over pair tiles.
//
// Pipeline structure:
//   * one weight-fragment prefetch ring (Ring) flows through the whole pair tile: the last
//     PF steps of every layer prefetch the first PF steps of the layer after it, and the
//     last layer of a tile prefetches the first layer of the next tile;
//   * every layer's epilogue (bias, softplus, σ store / σ multiply) is deferred: the
//     epilogue of out-tile group g runs inside the first steps of group g+1, and the last
//     group's epilogue inside the first steps of the next layer where that layer does not
//     need it yet, so the VALU work issues in the shadow of MFMAs;
//   * a group's bias / saved-σ tiles are loaded when the group starts and consumed by its
//     deferred epilogue a group later (double-buffered by group parity), so no load is
//     consumed right after it issues.
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
#ifdef PNTF_ABL_CHEAPACT   // diagnostics only (tests/diag ablations): no transcendentals
  return SpSig{fmaxf(y, 0.f) * 0.5f + 0.01f, 0.5f};
#endif
  float t = exp_neg10abs(y);
  float u = 1.f + t;
  float r = __builtin_amdgcn_rcpf(u);
  bool pos = y >= 0.f;
  SpSig o;
  // softplus_10(y) = max(y, 0) + log(1 + e^{-10|y|}) / 10, with log2 → ln and the 1/10
  // folded into one constant.  torch returns y itself above 10y > 20; there the log term is
  // < 2.1e-10 < ulp(y)/2, so the same expression rounds to exactly y without a select.
  o.sp = fmaf(__builtin_amdgcn_logf(u), 0.0693147180559945309f, pos ? y : 0.f);
  o.sg = pos ? r : t * r;
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

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// ---------------------------------------------------------------- weight stream
// Weight-stream prefetch depth (steps of the ring), step fences (bitmask of SITE_* call
// sites) and out tiles per MFMA group for single-column layers; overridable for the
// perf-variant diagnostics (tests/diag).
#ifndef PNTF_PF_STEPS
#define PNTF_PF_STEPS 4
#endif
#ifndef PNTF_STEP_FENCE
#define PNTF_STEP_FENCE 127
#endif
#ifndef PNTF_NO1
#define PNTF_NO1 4
#endif
#ifndef PNTF_IGLP_V
#define PNTF_IGLP_V 0
#endif
#ifndef PNTF_IGLP_CLUSTER
#define PNTF_IGLP_CLUSTER 0
#endif
// Deferred epilogues after the step's MFMAs (1) or before them (0).  Before, the first unit
// of a group reads accumulators whose last MFMA was issued in the step just before, so the
// wave waits for that MFMA to drain (s_nop + dependency) with no MFMA of its own in flight.
#ifndef PNTF_EPI_LATE
#define PNTF_EPI_LATE 0
#endif
// Groups of lead for the saved-σ loads of the encoder's reverse layers (Bwd AH).
#ifndef PNTF_ENC_AH
#define PNTF_ENC_AH 1
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
// 16-byte buffer store.  On gfx950 an instruction that overwrites a 16-byte store's data VGPRs
// right after it corrupts the stored values in lanes 12-15 of every 16-lane row, and LLVM's
// hazard recognizer skips the wait state that needs for buffer stores with an SGPR soffset
// (DESIGN.md §7.1).  The s_nop reads the data, so nothing overwrites it before one wait state
// has passed; pntf/build.py's store-data guard checks every kernel's assembly.
template <int AUX>
__device__ __forceinline__ void bstore(Rsrc r, f32x4 v, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b128(
      __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), r, voff, soff, AUX);
#ifndef PNTF_BSTORE_UNGUARDED   // test only: tests/test_capi_host.py checks the guard fires
  asm volatile("s_nop 0" ::"v"(v));
#endif
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

constexpr int PF_STEPS = PNTF_PF_STEPS;
#ifndef PNTF_RING_NL
#define PNTF_RING_NL 4
#endif
constexpr int RING_NL = PNTF_RING_NL;   // fragments per step, at most (6: pntf_wide.h x6 layers)
// Pipelined call sites (bits of PNTF_STEP_FENCE).
constexpr int SITE_FWD_E0 = 1, SITE_FWD_ENC = 2, SITE_FWD_GEN = 4, SITE_BWD_GEN = 8,
              SITE_BWD_ENC = 16, SITE_FOLD = 32, SITE_TAYLOR = 64;

// The weight-fragment prefetch ring: slot j % PF holds the fragments of step j for the PF
// steps ahead of the one being computed.
struct Ring {
  f32x4 r[PF_STEPS][RING_NL];
};

// "Nothing follows": the ring drains at the end of the step sequence.
struct NoNext {
  __device__ int operator()(int, int) const { return 0; }
};
// First steps of a standard layer with KT input tiles and KS k-tiles per step: step j < PF
// reads fragment l = o*KS + ks = (out tile o, k tile j*KS + ks).
template <int KT, int KS = 1>
struct Head {
  int base;
  __device__ int operator()(int j, int l) const {
    return base + (((l / KS) * KT + j * KS + l % KS) * 64) * 16;
  }
};

// Byte offset of fragment (ot, kt) of a packed (OT x KT) layer.
template <int KT>
__device__ __forceinline__ int frag(int base, int ot, int kt) {
  return base + ((ot * KT + kt) * 64) * 16;
}

// Software-pipelined step sequence.  Step st consumes NL weight fragments whose byte offsets
// are addr(st, l).  On entry the ring holds steps 0..PF-1; the last PF steps refill it with
// the first PF steps of whatever follows (naddr, NLN fragments per step), so the L2 latency
// of the stream stays hidden across layer boundaries.
template <int STEPS, int NL, int NLN, int SITE, class AddrF, class NextF, class BodyF>
__device__ __forceinline__ void run_steps(Ring& ring, Rsrc r, int voff, AddrF addr,
                                          NextF naddr, BodyF body) {
  static_assert(STEPS % PF_STEPS == 0, "step count must be a multiple of the ring depth");
  static_assert(NL <= RING_NL && NLN <= RING_NL, "ring width");
  static_for<0, STEPS>([&](auto st) {
    constexpr int S = decltype(st)::value;
    constexpr int slot = S % PF_STEPS;
    f32x4 a[NL];
#pragma unroll
    for (int l = 0; l < NL; ++l) a[l] = ring.r[slot][l];
    if constexpr (S + PF_STEPS < STEPS) {
#pragma unroll
      for (int l = 0; l < NL; ++l) ring.r[slot][l] = bload(r, voff, addr(S + PF_STEPS, l));
    } else {
#pragma unroll
      for (int l = 0; l < NLN; ++l)
        ring.r[slot][l] = bload(r, voff, naddr(S + PF_STEPS - STEPS, l));
    }
#ifdef PNTF_RING_AGPR   // the weight ring in the AGPR file (an MFMA reads its A operand there)
#pragma unroll
    for (int l = 0; l < RING_NL; ++l) asm("" : "+a"(ring.r[slot][l]));
#endif
    body(st, a);
#if PNTF_IGLP_CLUSTER == 1
    // One VALU cluster per step: beside f32 MFMAs every gap that carries vector work pays a
    // switch cost (tests/diag/coexec_probe.hip: ~12-17 cycles for the first VALU op in a
    // gap, 4-8 for each further one), so the step's loads go first, then its MFMAs, then all
    // its VALU work in one gap (data dependencies still order a pre hook's VALU before the
    // MFMAs that read its results).
    __builtin_amdgcn_sched_group_barrier(0x020, 16, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 64, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, 512, 0);
    __builtin_amdgcn_sched_group_barrier(0x040, 16, 0);
#elif PNTF_IGLP_CLUSTER == 2
    // VALU first, then loads and MFMAs
    __builtin_amdgcn_sched_group_barrier(0x002, 512, 0);
    __builtin_amdgcn_sched_group_barrier(0x020, 16, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 64, 0);
    __builtin_amdgcn_sched_group_barrier(0x040, 16, 0);
#endif
#if PNTF_IGLP_V > 0
    // Interleave the step as (1 MFMA, PNTF_IGLP_V VALU) x 16 so dependent VALU chains of the
    // deferred epilogues sit between MFMAs instead of stalling the wave's in-order issue.
    static_for<0, 16>([&](auto) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, PNTF_IGLP_V, 0);
    });
#endif
    // Keep every load in the step that issues it: without the fence the scheduler sinks
    // prefetches next to their MFMA under register pressure, collapsing the ring.
    if constexpr ((PNTF_STEP_FENCE & SITE) != 0) __builtin_amdgcn_sched_barrier(0);
  });
}

template <int NL, class AddrF>
__device__ __forceinline__ void ring_fill(Ring& ring, Rsrc r, int voff, AddrF addr) {
#pragma unroll
  for (int p = 0; p < PF_STEPS; ++p)
#pragma unroll
    for (int l = 0; l < NL; ++l) ring.r[p][l] = bload(r, voff, addr(p, l));
}

// Standalone step sequence with its own ring (filled on entry, drained at the end).
template <int STEPS, int NL, int SITE, class AddrF, class BodyF>
__device__ __forceinline__ void pipelined(Rsrc r, int voff, AddrF addr, BodyF body) {
  Ring ring;
  ring_fill<NL>(ring, r, voff, addr);
  run_steps<STEPS, NL, 0, SITE>(ring, r, voff, addr, NoNext{}, body);
}

// Hide a wave-uniform integer from the optimizer: inside the runtime block loops this keeps
// loop strength reduction from turning each of the ~100 fragment offsets of a layer into
// its own induction variable (which spilled >100 SGPRs); each offset becomes one s_add.
__device__ __forceinline__ int opaque(int x) {
  asm volatile("" : "+s"(x));
  return x;
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
#ifndef PNTF_SCRATCH_LOAD_AUX  // overridden only by the build-guard test (tests/test_capi_host.py)
#define PNTF_SCRATCH_LOAD_AUX 2
#endif
constexpr int AUX_NT = 2;
constexpr int AUX_LOAD = PNTF_SCRATCH_LOAD_AUX;
struct Scratch {
  Rsrc r;
};
__device__ __forceinline__ Scratch make_scratch(float* sc) {
  return Scratch{make_rsrc(sc, sc ? SCRATCH_FLOATS_PER_WAVE * 4 : 0)};
}
__device__ __forceinline__ void store_tile(Scratch sc, int tile, int lane, f32x4 v) {
#ifdef PNTF_ABL_NOSTORE   // diagnostics only (tests/diag ablations)
  asm volatile("" ::"v"(v));
  return;
#endif
#ifdef PNTF_DIAG_STORENOP  // diagnostics only (tests/diag split variants)
  asm volatile("s_nop 7\n\ts_nop 7" ::"v"(v));
#endif
  bstore<AUX_NT>(sc.r, v, lane * 16, tile * 1024);
#if defined(PNTF_DIAG_WAITS) && (PNTF_DIAG_WAITS >> 6) & 1   // diagnostics only
  asm volatile("s_waitcnt expcnt(0)" ::: "memory");
#endif
#if defined(PNTF_DIAG_WAITS) && (PNTF_DIAG_WAITS >> 7) & 1
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
}
__device__ __forceinline__ f32x4 load_tile(Scratch sc, int tile, int lane) {
#ifdef PNTF_ABL_NOLOAD    // diagnostics only (tests/diag ablations)
  return f32x4{0.5f, 0.5f, 0.5f, 0.5f};
#endif
  return __builtin_bit_cast(
      f32x4, __builtin_amdgcn_raw_buffer_load_b128(sc.r, lane * 16, tile * 1024, AUX_LOAD));
}
// Between the forward sweep (stores) and the reverse sweep (loads of the same slot): wait
// until every store of this wave has been performed.  Without it the first reverse-sweep
// loads (stored a few hundred cycles earlier) can overtake their stores under full-chip
// load (measured: garbage ∇τ rows at 262k pairs, 2 workgroups per CU).
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Diagnostics only (tests/diag/stamps.py): -DPNTF_DEBUG_STAMPS records s_memtime at phase
// boundaries into pntf_stamps[wave*64 + idx] (each tile overwrites: the last tile remains).
#ifdef PNTF_DEBUG_STAMPS
__device__ unsigned long long* pntf_stamps;
#define PNTF_STAMP(idx)                                                                  \
  do {                                                                                   \
    unsigned long long _t = __builtin_amdgcn_s_memtime();                                \
    if ((threadIdx.x & 63) == 0)                                                         \
      pntf_stamps[(blockIdx.x * 4 + (threadIdx.x >> 6)) * 64 + (idx)] = _t;              \
  } while (0)
#else
#define PNTF_STAMP(idx)
#endif

// Out tiles per MFMA group: PNTF_NO1 for single-column layers, capped at the layer's out
// tiles (the out-tile-split kernels of pntf_split.h run layers of 2 local out tiles).
template <int NC, int OT = 16>
constexpr int out_group() { return NC == 1 ? (OT < PNTF_NO1 ? OT : PNTF_NO1) : 1; }

// "No previous layer tail" hook.
struct NoPre {
  template <class ST>
  __device__ void operator()(ST) const {}
};

// ---------------------------------------------------------------- generic layer
// Epilogue units per out tile: a tile's epilogue runs as EP_SPLIT units of 4/EP_SPLIT rows,
// one unit per step, so no step carries more VALU work than its MFMAs can shadow.
#ifndef PNTF_EP_SPLIT
#define PNTF_EP_SPLIT 2
#endif
constexpr int EP_SPLIT = PNTF_EP_SPLIT;
// k tiles per step in the encoder layers (2: 16 MFMAs and 2 weight fragments per step; 4: 32
// MFMAs and 4 fragments, so the 4-step ring runs twice as far ahead in time) and the
// matching epilogue units per out tile.
#ifndef PNTF_ENC_KS
#define PNTF_ENC_KS 2
#endif
constexpr int EKS = PNTF_ENC_KS;
constexpr int EEPS = EKS == 4 ? 1 : EP_SPLIT;
constexpr int EGS = 8 / EKS;                 // steps per encoder group (1 out tile x 2 cols)

// One Linear layer as out-tile groups of NO tiles x NC columns (NO*NC >= 2 independent MFMA
// chains); a step consumes KS k-tiles (NO*KS weight fragments), KT/KS steps per group.  The
// layer object ly supplies
//   ly.init(ot, acc)      at the first step of the group starting at out tile ot
//   ly.epi(t, c, h, v)    unit h (rows h*4/EPS ..) of the epilogue of out tile t, column c,
//                         from v[NC] = that tile's accumulators; runs deferred, one unit per
//                         step in the first NO*NC*EPS steps of the next group
//   ly.pend[NO][NC]       holds the last group's accumulators on return: its epilogue is
//                         still pending (run it with flush(), or as the next layer's pre hook)
// pre(st) runs at every step (the previous layer's pending tail; a no-op past its length).
template <int OT, int KT, int NC, int KS, int SITE, int NLN, int NIN, class L, class PreF,
          class NextF>
__device__ __forceinline__ void layer(Ring& ring, Rsrc W, int wbase, const f32x4 (&in)[NIN],
                                      int lane, L& ly, PreF pre, NextF naddr) {
  constexpr int NO = L::NO;
  static_assert(L::OT == OT && L::NC == NC, "layer object shape");
  constexpr int GS = KT / KS;                 // steps per group
  constexpr int STEPS = (OT / NO) * GS;
  constexpr int EPS = L::EPS;                 // epilogue units per out tile
  constexpr int UNITS = NO * NC * EPS;        // deferred epilogue units per group
  static_assert(KT % KS == 0 && UNITS <= GS, "a group's epilogue must fit in the next group");
  f32x4 acc[NO][NC];
  run_steps<STEPS, NO * KS, NLN, SITE>(
      ring, W, lane * 16,
      [&](int st, int l) {
        return frag<KT>(wbase, (st / GS) * NO + l / KS, (st % GS) * KS + l % KS);
      },
      naddr,
      [&](auto st, const f32x4 (&a)[NO * KS]) {
        constexpr int S = decltype(st)::value;
        constexpr int ot = (S / GS) * NO, ks0 = (S % GS) * KS;
        pre(st);
        if constexpr (S % GS == 0) ly.init(ot, acc);
        auto deferred = [&]() {
          if constexpr (ot > 0 && S % GS < UNITS) {
            constexpr int u = S % GS;
            ly.epi(ot - NO + u / (NC * EPS), (u / EPS) % NC, u % EPS,
                   ly.pend[u / (NC * EPS)]);
          }
        };
        if constexpr (!PNTF_EPI_LATE) deferred();
#pragma unroll
        for (int k = 0; k < KS; ++k)
#pragma unroll
          for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int o = 0; o < NO; ++o)
#pragma unroll
              for (int c = 0; c < NC; ++c)
                acc[o][c] = mfma(a[o * KS + k][s], in[c * KT + ks0 + k][s], acc[o][c]);
        if constexpr (PNTF_EPI_LATE) deferred();
        if constexpr (S % GS == GS - 1) {
#pragma unroll
          for (int o = 0; o < NO; ++o)
#pragma unroll
            for (int c = 0; c < NC; ++c) ly.pend[o][c] = acc[o][c];
        }
      });
}

// The pending epilogue of a layer's last group as a pre hook for the next layer (unit j at
// its step j; safe while that layer reads the pending tiles only at those or later steps) ...
template <class L>
struct Tail {
  L& ly;
  template <class ST>
  __device__ __forceinline__ void operator()(ST) const {
    constexpr int j = ST::value;
    if constexpr (j < L::NO * L::NC * L::EPS)
      ly.epi(L::OT - L::NO + j / (L::NC * L::EPS), (j / L::EPS) % L::NC, j % L::EPS,
             ly.pend[j / (L::NC * L::EPS)]);
  }
};
// ... or run at once.
template <class L>
__device__ __forceinline__ void flush(L& ly) {
#ifdef PNTF_DIAG_EPINOP   // diagnostics only (tests/diag split variants)
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#endif
  Tail<L> t{ly};
  static_for<0, L::NO * L::NC * L::EPS>([&](auto j) { t(j); });
}

// ---------------------------------------------------------------- layer kinds
// Forward: out[c*OT+t] = softplus(A·in + bias (+ out[c*OT+t] if RES)); σ10(pre) saved to
// scratch tile sc0 + c*OT + t when SAVE, and kept in keep[t] when KEEP (single column).
template <int OT_, int KT_, int NC_, bool RES, bool SAVE, bool KEEP = false, int EPS_ = EP_SPLIT>
struct FwdAct {
  static constexpr int OT = OT_, KT = KT_, NC = NC_, NO = out_group<NC_, OT_>();
  static constexpr int EPS = EPS_, ROWS = 4 / EPS_;
  Rsrc W;
  int bias;
  f32x4 (&out)[16];
  Scratch sc;
  int sc0, lane;
  f32x4 (&keep)[8];
  f32x4 bb[2][NO];
  f32x4 pend[NO][NC];
  __device__ __forceinline__ void init(int ot, f32x4 (&acc)[NO][NC]) {
    const int par = (ot / NO) & 1;
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      bb[par][o] = bload(W, (lane >> 4) * 16, bias + (16 * (ot + o)) * 4);
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[o][c] = RES ? out[c * OT + ot + o] : zero4();
    }
  }
  f32x4 sgp;   // σ rows of the tile being finished (units of one tile are consecutive)
  __device__ __forceinline__ void epi(int t, int c, int h, const f32x4 (&v)[NC]) {
    const f32x4 b = bb[(t / NO) & 1][t % NO];
#pragma unroll
    for (int r = h * ROWS; r < (h + 1) * ROWS; ++r) {
      SpSig q = sp_sig(v[c][r] + b[r]);
      out[c * OT + t][r] = q.sp;
      sgp[r] = q.sg;
    }
    if (h == EPS - 1) {
      if (SAVE) store_tile(sc, sc0 + c * OT + t, lane, sgp);
      if (KEEP) keep[t] = sgp;
    }
  }
};

// out[c*OT+t] = A·in + bias, no activation (encoder[-1], :234).
template <int OT_, int KT_, int NC_, int EPS_ = EP_SPLIT>
struct FwdLin {
  static constexpr int OT = OT_, KT = KT_, NC = NC_, NO = out_group<NC_, OT_>();
  static constexpr int EPS = EPS_, ROWS = 4 / EPS_;
  Rsrc W;
  int bias;
  f32x4 (&out)[16];
  int lane;
  f32x4 bb[2][NO];
  f32x4 pend[NO][NC];
  __device__ __forceinline__ void init(int ot, f32x4 (&acc)[NO][NC]) {
    const int par = (ot / NO) & 1;
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      bb[par][o] = bload(W, (lane >> 4) * 16, bias + (16 * (ot + o)) * 4);
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[o][c] = zero4();
    }
  }
  __device__ __forceinline__ void epi(int t, int c, int h, const f32x4 (&v)[NC]) {
    const f32x4 b = bb[(t / NO) & 1][t % NO];
#pragma unroll
    for (int r = h * ROWS; r < (h + 1) * ROWS; ++r) out[c * OT + t][r] = v[c][r] + b[r];
  }
};

// Reverse: out[c*OT+t] = (A^T·in (+ out[c*OT+t] if RES)) ⊙ scratch[mul0 + c*OT + t] (if MUL)
// The saved-σ tiles of group gi are loaded AH groups before its deferred epilogue runs: at
// the start of group gi - AH + 1 (AH = 1: when the group itself starts).  With AH > 1 the
// first AH - 1 groups are loaded by preload(), which the caller runs inside the previous
// layer (Preload / At hooks), so even the layer's first group gets the full lead.
template <int OT_, int KT_, int NC_, bool RES, bool MUL, int AH = 1, int EPS_ = EP_SPLIT>
struct Bwd {
  static constexpr int OT = OT_, KT = KT_, NC = NC_, NO = out_group<NC_, OT_>();
  static constexpr int EPS = EPS_, ROWS = 4 / EPS_;
  static constexpr int NG = OT / NO, NB = AH + 1;
  f32x4 (&out)[16];
  Scratch sc;
  int mul0, lane;
  f32x4 m[NB][NO][NC];
  f32x4 pend[NO][NC];
  __device__ __forceinline__ void load_group(int gi) {
#pragma unroll
    for (int o = 0; o < NO; ++o)
#pragma unroll
      for (int c = 0; c < NC; ++c)
        m[gi % NB][o][c] = load_tile(sc, mul0 + c * OT + gi * NO + o, lane);
  }
  __device__ __forceinline__ void preload() {
    if (MUL)
#pragma unroll
      for (int gi = 0; gi < AH - 1; ++gi) load_group(gi);
  }
  __device__ __forceinline__ void init(int ot, f32x4 (&acc)[NO][NC]) {
    const int gi = ot / NO;
    if (MUL && gi + AH - 1 < NG) load_group(gi + AH - 1);
#pragma unroll
    for (int o = 0; o < NO; ++o)
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[o][c] = RES ? out[c * OT + ot + o] : zero4();
  }
  __device__ __forceinline__ void epi(int t, int c, int h, const f32x4 (&v)[NC]) {
    const f32x4 mm = m[(t / NO) % NB][t % NO][c];
#pragma unroll
    for (int r = h * ROWS; r < (h + 1) * ROWS; ++r)
      out[c * OT + t][r] = MUL ? v[c][r] * mm[r] : v[c][r];
  }
};

// Pre hooks: run f() at step N of the layer; run two hooks.
template <int N, class F>
struct At {
  F f;
  template <class ST>
  __device__ __forceinline__ void operator()(ST) const {
    if constexpr (ST::value == N) f();
  }
};
template <int N, class F>
__device__ __forceinline__ At<N, F> at(F f) {
  return At<N, F>{f};
}
template <class A, class B>
struct Both {
  A a;
  B b;
  template <class ST>
  __device__ __forceinline__ void operator()(ST st) const {
    a(st);
    b(st);
  }
};
template <class A, class B>
__device__ __forceinline__ Both<A, B> both(A a, B b) {
  return Both<A, B>{a, b};
}

// ---------------------------------------------------------------- one pair tile
struct PairIO {
  float x[2][6];    // [start|goal][dim]
  const float* Bw;  // this lane's env B (dim x 128), un-scaled
};

// Registers a pair tile carries from the forward pass into the reverse sweep.
struct Carry {
  f32x4 sg3[8];   // σ10 of generator[-2] (:251-252)
  f32x4 g4w[8];   // generator[-1].weight rows of this lane
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

// Ring head of the forward pass (encoder[0] on Fourier features): step j reads fragments
// (out tile j % 8, k tile j / 8 + 8 l).
struct E0Head {
  __device__ int operator()(int j, int l) const {
    return frag<16>((OFF_FWD + OFF_E0) * 4, j % 8, j / 8 + 8 * l);
  }
};
// Ring head of the reverse sweep (generator[-2]^T, 256 x 128: OT 16, KT 8).
__device__ __forceinline__ Head<8> bwd_head() { return Head<8>{(OFF_BWD + OFF_G3) * 4}; }
// Ring head of the Fourier fold (encoder[0]^T, 256 x 128: KT 8): fragments (kf, kt) and
// (kf + 8, kt) for step (kf, kt).
struct FoldHead {
  __device__ int operator()(int j, int l) const {
    return frag<8>((OFF_BWD + OFF_E0) * 4, j / 8 + 8 * l, j % 8);
  }
};

// Forward pass (NN.out).  GRAD: also save σ tiles for the reverse sweep.  On entry the ring
// holds E0Head; on return it holds the first PF steps of `after` (NLA fragments per step).
// Returns τ for the lane's pair (identical in all four lane groups).
template <int DIM, bool GRAD, int NLA, class AfterF>
__device__ __forceinline__ float forward_pass(Ring& ring, const float* __restrict__ P,
                                              const PairIO& io, f32x4 (&X)[16], f32x4 (&Y)[16],
                                              Carry& cy, Scratch sc, int compat, int lane,
                                              AfterF after) {
  const int g = lane >> 4;
  const Rsrc W = make_rsrc(P, PACKED_FLOATS * 4);
  constexpr int BB = OFF_BIAS * 4;  // byte base of biases / head
  constexpr int F = OFF_FWD * 4;   // byte base of the forward fragments

  const float cm = compat ? 1.f : 0.f;   // branch-free mode blend

  // ---- encoder[0] on Fourier features computed on the fly (:186-190, :227).
  // E0 is (128 x 256): OT = 8, KT = 16; input tiles 0..7 = sin q, 8..15 = cos q.
  // Step (kt, ot) uses fragments (ot, kt) and (ot, kt + 8); out tile ot is complete after
  // step (7, ot), and its epilogue runs in step (7, ot + 1) (tile 7's in the next layer).
  PNTF_STAMP(0);
  f32x4 eb[8];
  // encoder[0] epilogue of out tile i (columns 0, 1): bias, softplus, σ; in compat mode the
  // out_backgrad quirk (:435-438) stores σ10(softplus(y)) = 1 / (2 - σ10(y)).
  auto e0epi = [&](int i) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int t = c * 8 + i;
      f32x4 s, sg;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        SpSig v = sp_sig(X[t][r] + eb[i][r]);
        s[r] = v.sp;
        sg[r] = fmaf(cm, __builtin_amdgcn_rcpf(2.f - v.sg) - v.sg, v.sg);
      }
      X[t] = s;
      if (GRAD) store_tile(sc, T_E0 + t, lane, sg);
    }
  };
#pragma unroll
  for (int i = 0; i < 16; ++i) X[i] = zero4();
  {
    f32x4 sn[2], cs[2];
    f32x4 bw[2][DIM];   // B rows of the lane's features, one Fourier tile ahead
#pragma unroll
    for (int d = 0; d < DIM; ++d) bw[0][d] = ld4(io.Bw + d * H + 4 * g);
    run_steps<64, 2, EKS, SITE_FWD_E0>(
        ring, W, lane * 16,
        [&](int st, int l) { return frag<16>(F + OFF_E0 * 4, st % 8, st / 8 + 8 * l); },
        Head<8, EKS>{F + OFF_EBLK * 4},
        [&](auto st, const f32x4 (&a)[2]) {
          constexpr int S = decltype(st)::value;
          constexpr int kt = S / 8, ot = S % 8;
          if constexpr (S == 1) {
#pragma unroll
            for (int t = 0; t < 8; ++t) eb[t] = bload(W, g * 16, BB + (B_E0 + 16 * t) * 4);
          }
          if constexpr (ot == 1 && kt < 7) {
#pragma unroll
            for (int d = 0; d < DIM; ++d) bw[(kt + 1) & 1][d] = ld4(io.Bw + d * H + 16 * (kt + 1) + 4 * g);
          }
          if constexpr (ot == 0) {
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
          if constexpr (kt == 7 && ot > 0 && !PNTF_EPI_LATE) e0epi(ot - 1);
#pragma unroll
          for (int s = 0; s < 4; ++s) {
#pragma unroll
            for (int c = 0; c < 2; ++c) X[c * 8 + ot] = mfma(a[0][s], sn[c][s], X[c * 8 + ot]);
#pragma unroll
            for (int c = 0; c < 2; ++c) X[c * 8 + ot] = mfma(a[1][s], cs[c][s], X[c * 8 + ot]);
          }
          if constexpr (kt == 7 && ot > 0 && PNTF_EPI_LATE) e0epi(ot - 1);
        });
  }
  PNTF_STAMP(1);

  // ---- encoder residual blocks (:228-232), unrolled; X = h (2 cols x 8 tiles)
  const int BE = BB + B_EBLK * 4;
  const int WE = F + OFF_EBLK * 4;
  FwdAct<8, 8, 2, false, GRAD, false, EEPS> a0{W, BE, Y, sc, T_EBLK, lane, cy.sg3};
  layer<8, 8, 2, EKS, SITE_FWD_ENC, EKS>(
      ring, W, WE, X, lane, a0,
      [&](auto st) {
        if constexpr (decltype(st)::value == 0) e0epi(7);
      },
      Head<8, EKS>{WE + SZ_E * 4});
  PNTF_STAMP(2);
  FwdAct<8, 8, 2, true, GRAD, false, EEPS> b0{W, BE + 128 * 4, X, sc, T_EBLK + 16, lane, cy.sg3};
  layer<8, 8, 2, EKS, SITE_FWD_ENC, EKS>(ring, W, WE + SZ_E * 4, Y, lane, b0,
                                      Tail<decltype(a0)>{a0}, Head<8, EKS>{WE + 2 * SZ_E * 4});
  PNTF_STAMP(3);
  FwdAct<8, 8, 2, false, GRAD, false, EEPS> a1{W, BE + 256 * 4, Y, sc, T_EBLK + 32, lane, cy.sg3};
  layer<8, 8, 2, EKS, SITE_FWD_ENC, EKS>(ring, W, WE + 2 * SZ_E * 4, X, lane, a1,
                                      Tail<decltype(b0)>{b0}, Head<8, EKS>{WE + 3 * SZ_E * 4});
  PNTF_STAMP(4);
  FwdAct<8, 8, 2, true, GRAD, false, EEPS> b1{W, BE + 384 * 4, X, sc, T_EBLK + 48, lane, cy.sg3};
  layer<8, 8, 2, EKS, SITE_FWD_ENC, EKS>(ring, W, WE + 3 * SZ_E * 4, Y, lane, b1,
                                      Tail<decltype(a1)>{a1}, Head<8, EKS>{F + OFF_E3 * 4});
  PNTF_STAMP(5);
  // ---- encoder[-1] (:234) -> Y (zs = Y[0..7], zg = Y[8..15])
  FwdLin<8, 8, 2, EEPS> e3{W, BB + B_E3 * 4, Y, lane};
  layer<8, 8, 2, EKS, SITE_FWD_ENC, 4>(ring, W, F + OFF_E3 * 4, X, lane, e3,
                                    Tail<decltype(b1)>{b1}, Head<16>{F + OFF_GBLK * 4});
  flush(e3);
  PNTF_STAMP(6);

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
  PNTF_STAMP(7);

  // ---- generator residual blocks (:246-249); X = u (16 tiles)
#pragma unroll 1
  for (int i = 0; i < 3; ++i) {
    const int wa = opaque(F + (OFF_GBLK + (2 * i) * SZ_G) * 4);
    const int wb = opaque(F + (OFF_GBLK + (2 * i + 1) * SZ_G) * 4);
    const int wn = opaque(i < 2 ? F + (OFF_GBLK + (2 * i + 2) * SZ_G) * 4 : F + OFF_G3 * 4);
    FwdAct<16, 16, 1, false, GRAD> ga{W, BB + (B_GBLK + (2 * i) * 256) * 4, Y, sc,
                                      T_GBLK + 32 * i, lane, cy.sg3};
    layer<16, 16, 1, 1, SITE_FWD_GEN, 4>(ring, W, wa, X, lane, ga, NoPre{}, Head<16>{wb});
    FwdAct<16, 16, 1, true, GRAD> gb{W, BB + (B_GBLK + (2 * i + 1) * 256) * 4, X, sc,
                                     T_GBLK + 32 * i + 16, lane, cy.sg3};
    layer<16, 16, 1, 1, SITE_FWD_GEN, 4>(ring, W, wb, Y, lane, gb, Tail<decltype(ga)>{ga},
                                      Head<16>{wn});
    flush(gb);
  }
  PNTF_STAMP(13);
  // ---- generator[-2] + act (:251-252) -> Y[0..7]; its σ tiles stay in registers for the
  // reverse sweep, and the head row is fetched while it runs.
#pragma unroll
  for (int t = 0; t < 8; ++t) cy.g4w[t] = bload(W, g * 16, BB + (B_G4W + 16 * t) * 4);
  const float g4b = bload(W, 0, BB + B_G4B * 4)[0];
  FwdAct<8, 16, 1, false, GRAD, GRAD> g3{W, BB + B_G3 * 4, Y, sc, T_G3, lane, cy.sg3};
  layer<8, 16, 1, 1, SITE_FWD_GEN, NLA>(ring, W, F + OFF_G3 * 4, X, lane, g3, NoPre{}, after);
  flush(g3);
  PNTF_STAMP(14);

  // ---- head generator[-1] + sigmoid(0.1 y) (:254-255)
  float part = 0.f;
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int s = 0; s < 4; ++s) part = fmaf(cy.g4w[t][s], Y[t][s], part);
  part += __shfl_xor(part, 16);
  part += __shfl_xor(part, 32);
  float y4 = part + g4b;
  PNTF_STAMP(15);
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-0.144269504088896341f * y4));
}

// Reverse sweep: exact reverse mode, or NN.out_backgrad when the forward stored the quirk.
// On entry the ring holds bwd_head(); on return the first PF steps of `after`.  Produces
// dτ/dxs (ds) and dτ/dxg (dg), identical in all four lane groups.
template <int DIM, int NLA, class AfterF>
__device__ __forceinline__ void backward_pass(Ring& ring, const float* __restrict__ P,
                                              const PairIO& io, float tau, f32x4 (&X)[16],
                                              f32x4 (&Y)[16], const Carry& cy, Scratch sc,
                                              int lane, float (&ds)[DIM], float (&dg)[DIM],
                                              AfterF after) {
  const int g = lane >> 4;
  const Rsrc W = make_rsrc(P, PACKED_FLOATS * 4);
  constexpr int Bk = OFF_BWD * 4;  // byte base of the transposed fragments

  // ---- head and generator[-2] (:592-613): Y[t] = d * G4 ⊙ σ10(y3)
  const float dd = 0.1f * tau * (1.f - tau);
#pragma unroll
  for (int t = 0; t < 8; ++t) Y[t] = (dd * cy.g4w[t]) * cy.sg3[t];
  PNTF_STAMP(17);
  // du = G3^T dv ⊙ σ10(y2 of generator block 2) -> X  (G3^T is 256 x 128: OT 16, KT 8)
  {
    Bwd<16, 8, 1, false, true> l{X, sc, T_GBLK + 32 * 2 + 16, lane};
    layer<16, 8, 1, 1, SITE_BWD_GEN, 4>(ring, W, Bk + OFF_G3 * 4, Y, lane, l, NoPre{},
                                     Head<16>{Bk + (OFF_GBLK + 5 * SZ_G) * 4});
    flush(l);
  }
  PNTF_STAMP(18);
#ifdef PNTF_S0_EARLY
  // the merge switch tiles, fetched now and held through the generator sweep
  f32x4 s0t[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) s0t[t] = load_tile(sc, T_S0 + t, lane);
#endif

  // encoder reverse layers (constructed here: each one's first σ groups are preloaded inside
  // the layer before it, PNTF_ENC_AH groups ahead of their use)
  const int WE = Bk + OFF_EBLK * 4;
  constexpr int EAH = PNTF_ENC_AH;
  Bwd<8, 8, 2, false, true, EAH, EEPS> e3{Y, sc, T_EBLK + 32 * 1 + 16, lane};
  Bwd<8, 8, 2, false, true, EAH, EEPS> b1{X, sc, T_EBLK + 32, lane};
  Bwd<8, 8, 2, true, true, EAH, EEPS> a1{Y, sc, T_EBLK + 16, lane};
  Bwd<8, 8, 2, false, true, EAH, EEPS> b0{X, sc, T_EBLK, lane};
  Bwd<8, 8, 2, true, true, EAH, EEPS> a0{Y, sc, T_E0, lane};
  constexpr int ELAST = 7 * EGS;   // first step of an encoder layer's last group (of 8)

  // ---- generator blocks, reverse (:615-618)
#pragma unroll 1
  for (int i = 2; i >= 0; --i) {
    const int wa = opaque(Bk + (OFF_GBLK + (2 * i) * SZ_G) * 4);
    const int wb = opaque(Bk + (OFF_GBLK + (2 * i + 1) * SZ_G) * 4);
    // da = (G1_i^T dr) ⊙ σ10(y1_i) -> Y
    Bwd<16, 16, 1, false, true> lb{Y, sc, T_GBLK + 32 * i, lane};
    layer<16, 16, 1, 1, SITE_BWD_GEN, 4>(ring, W, wb, X, lane, lb, NoPre{}, Head<16>{wa});
    // du = G_i^T da + dr, then ⊙ σ10(y2_{i-1}) for the next block (none after block 0)
    if (i > 0) {
      const int wn = opaque(Bk + (OFF_GBLK + (2 * i - 1) * SZ_G) * 4);
      Bwd<16, 16, 1, true, true> la{X, sc, T_GBLK + 32 * (i - 1) + 16, lane};
      layer<16, 16, 1, 1, SITE_BWD_GEN, 4>(ring, W, wa, Y, lane, la, Tail<decltype(lb)>{lb},
                                        Head<16>{wn});
      flush(la);
    } else {
      Bwd<16, 16, 1, true, false> la{X, sc, 0, lane};
      // its last group (4 out tiles x 16 steps) starts at step 48: preload e3's first σ there
      layer<16, 16, 1, 1, SITE_BWD_GEN, EKS>(ring, W, wa, Y, lane, la,
                                          both(Tail<decltype(lb)>{lb},
                                               at<48>([&] { e3.preload(); })),
                                          Head<8, EKS>{Bk + OFF_E3 * 4});
      flush(la);
    }
  }
  PNTF_STAMP(24);

  // ---- merge Jacobian (:620-627): X[0..7] = dzs, X[8..15] = dzg
#pragma unroll
  for (int t = 0; t < 8; ++t) {
#ifdef PNTF_S0_EARLY
    f32x4 s0 = s0t[t];
#else
    f32x4 s0 = load_tile(sc, T_S0 + t, lane);
#endif
    f32x4 s1 = 1.f - s0;
    f32x4 dM = X[t], dm = X[8 + t];
    X[t] = s0 * dM + s1 * dm;
    X[8 + t] = s1 * dM + s0 * dm;
  }
  PNTF_STAMP(25);
  // ---- encoder[-1]^T, then ⊙ σ10(y2 of encoder block 1) -> Y
  layer<8, 8, 2, EKS, SITE_BWD_ENC, EKS>(ring, W, Bk + OFF_E3 * 4, X, lane, e3,
                                      at<ELAST>([&] { b1.preload(); }),
                                      Head<8, EKS>{WE + 3 * SZ_E * 4});
  PNTF_STAMP(26);
  // ---- encoder blocks, reverse (:633-636), unrolled
  // da = (E1_b^T dr) ⊙ σ10(y1_b)
  layer<8, 8, 2, EKS, SITE_BWD_ENC, EKS>(
      ring, W, WE + 3 * SZ_E * 4, Y, lane, b1,
      both(Tail<decltype(e3)>{e3}, at<ELAST>([&] { a1.preload(); })),
      Head<8, EKS>{WE + 2 * SZ_E * 4});
  PNTF_STAMP(27);
  // dh = E_b^T da + dr, then ⊙ σ10 of the layer below (block 0's y2, or encoder[0])
  layer<8, 8, 2, EKS, SITE_BWD_ENC, EKS>(
      ring, W, WE + 2 * SZ_E * 4, X, lane, a1,
      both(Tail<decltype(b1)>{b1}, at<ELAST>([&] { b0.preload(); })),
      Head<8, EKS>{WE + 1 * SZ_E * 4});
  PNTF_STAMP(28);
  layer<8, 8, 2, EKS, SITE_BWD_ENC, EKS>(
      ring, W, WE + 1 * SZ_E * 4, Y, lane, b0,
      both(Tail<decltype(a1)>{a1}, at<ELAST>([&] { a0.preload(); })), Head<8, EKS>{WE});
  PNTF_STAMP(29);
  layer<8, 8, 2, EKS, SITE_BWD_ENC, 2>(ring, W, WE, X, lane, a0, Tail<decltype(b0)>{b0},
                                    FoldHead{});
  PNTF_STAMP(30);

  // ---- encoder[0]^T (256 x 128: OT 16, KT 8) fused with the Fourier Jacobian (:639-645)
  // Step (kf, kt) uses fragments (kf, kt) [dφ_sin rows] and (kf + 8, kt) [dφ_cos rows].  The
  // Fourier fold of feature tile kf runs deferred in the first steps of feature tile kf + 1.
  float acc[2][DIM];
#pragma unroll
  for (int d = 0; d < DIM; ++d) acc[0][d] = acc[1][d] = 0.f;
  f32x4 ph[2][2][2];   // [kf parity][sin|cos rows][column]
  f32x4 bw[2][DIM];    // B rows of the lane's features of tile kf (fetched in step (kf, 2))
  auto fold = [&](int kf, int c) {
    const int p = kf & 1;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float q = 0.f;
#pragma unroll
      for (int d = 0; d < DIM; ++d) q = fmaf(io.x[c][d], TWO_PI * bw[p][d][s], q);
      float sn, cs;
      sincos_fast(q, sn, cs);
      float gg = ph[p][0][c][s] * cs - ph[p][1][c][s] * sn;
#pragma unroll
      for (int d = 0; d < DIM; ++d) acc[c][d] = fmaf(TWO_PI * bw[p][d][s], gg, acc[c][d]);
    }
  };
  Tail<decltype(a0)> a0tail{a0};
  run_steps<64, 2, NLA, SITE_FOLD>(
      ring, W, lane * 16,
      [&](int st, int l) { return frag<8>(Bk + OFF_E0 * 4, st / 8 + 8 * l, st % 8); }, after,
      [&](auto st, const f32x4 (&a)[2]) {
        constexpr int S = decltype(st)::value;
        constexpr int kf = S / 8, kt = S % 8, p = kf & 1;
        a0tail(st);
        if constexpr (kt == 0) {
#pragma unroll
          for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int c = 0; c < 2; ++c) ph[p][u][c] = zero4();
        }
        if constexpr (kt == 2) {
#pragma unroll
          for (int d = 0; d < DIM; ++d) bw[p][d] = ld4(io.Bw + d * H + 16 * kf + 4 * g);
        }
        if constexpr (kf > 0 && kt < 2 && !PNTF_EPI_LATE) fold(kf - 1, kt);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            ph[p][0][c] = mfma(a[0][s], Y[c * 8 + kt][s], ph[p][0][c]);
            ph[p][1][c] = mfma(a[1][s], Y[c * 8 + kt][s], ph[p][1][c]);
          }
        if constexpr (kf > 0 && kt < 2 && PNTF_EPI_LATE) fold(kf - 1, kt);
      });
  fold(7, 0);
  fold(7, 1);
#pragma unroll
  for (int d = 0; d < DIM; ++d) {
    float a0v = acc[0][d], a1v = acc[1][d];
    a0v += __shfl_xor(a0v, 16);
    a1v += __shfl_xor(a1v, 16);
    a0v += __shfl_xor(a0v, 32);
    a1v += __shfl_xor(a1v, 32);
    ds[d] = a0v;
    dg[d] = a1v;
  }
  PNTF_STAMP(31);
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
// Per-kind outputs of one pair (lanes 0..15 store: `store`).
template <int DIM, int KIND>
__device__ __forceinline__ void store_field(const FieldArgs& a, int64_t pair, bool ok,
                                            bool store, float tau, const PairIO& io,
                                            const float (&ds)[DIM], const float (&dg)[DIM]) {
  const float nan = __builtin_nanf("");
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
  } else if (KIND == K_TAU_GRAD) {
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

// Persistent body: wave `slot` of `nslots` takes tiles slot, slot + nslots, ...
template <int DIM, int KIND>
__device__ __forceinline__ void field_body(const FieldArgs& a, int slot, int nslots) {
  constexpr bool GRAD = KIND != K_TAU && KIND != K_TRAVEL;
  const int lane = threadIdx.x & 63;
  const int64_t ntiles = (a.n + TILE - 1) / TILE;
  const Scratch sc = make_scratch(GRAD ? a.ws + (int64_t)slot * SCRATCH_FLOATS_PER_WAVE : nullptr);
  const Rsrc W = make_rsrc(a.P, PACKED_FLOATS * 4);
  Ring ring;
  ring_fill<2>(ring, W, lane * 16, E0Head{});
  for (int64_t tile = slot; tile < ntiles; tile += nslots) {
    f32x4 X[16], Y[16];
    Carry cy;
    const int64_t pair = tile * TILE + (lane & 15);
    PairIO io;
    const bool ok = load_pair<DIM>(a.xp, a.Btab, a.env, a.n, a.n_env, pair, io);
    float tau;
    if constexpr (GRAD)
      tau = forward_pass<DIM, true, 4>(ring, a.P, io, X, Y, cy, sc, a.compat, lane, bwd_head());
    else
      tau = forward_pass<DIM, false, 2>(ring, a.P, io, X, Y, cy, sc, a.compat, lane, E0Head{});
    if (GRAD) drain_stores();
    PNTF_STAMP(16);
    const bool store = (lane < 16) && pair < a.n;
    float ds[DIM], dg[DIM];
    if constexpr (GRAD)
      backward_pass<DIM, 2>(ring, a.P, io, tau, X, Y, cy, sc, lane, ds, dg, E0Head{});
    store_field<DIM, KIND>(a, pair, ok, store, tau, io, ds, dg);
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
  const Rsrc W = make_rsrc(a.P, PACKED_FLOATS * 4);
  const int cap = a.max_iter + 1;
  const int64_t rows = (int64_t)cap + 1;
  Ring ring;
  ring_fill<2>(ring, W, lane * 16, E0Head{});
  for (int64_t tile = slot; tile < ntiles; tile += nslots) {
    f32x4 X[16], Y[16];
    Carry cy;
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
      float tau = forward_pass<DIM, true, 4>(ring, a.P, io, X, Y, cy, sc, a.compat, lane,
                                             bwd_head());
      drain_stores();
      float ds[DIM], dg[DIM], vs[DIM], vg[DIM];
      backward_pass<DIM, 2>(ring, a.P, io, tau, X, Y, cy, sc, lane, ds, dg, E0Head{});
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
