#pragma once
// Quad-tile τ / ∇τ / planner kernels for batches of a few queries.
//
// A planner step streams both weight directions (4.33 MB) through the CU that owns the query
// tile, so its time is bounded below by one CU's weight-stream rate (tests/diag/stream_probe:
// ≈42 µs per step at ≈103 GB/s per CU) and by the tile's MFMA work.  On 16-pair tiles the
// MFMA work alone is ≈68 µs per step on one CU (16x16x4: 16 pairs per instruction), and a
// 1024-query plan (BASELINE C5) keeps only 64 CUs busy.  Here a tile is 4 pairs and the
// matrix op is v_mfma_f32_4x4x1_16b_f32 (16 independent 4x4x1 blocks per instruction):
//   * blocks b = 4·og + kb: og picks 4 of the instruction's 16 out rows, kb one of its 4 k;
//     A lane l = W[r0 + 4·og + ((l + kb) & 3)][k0 + kb], B lane l = act[k0 + kb][pair l & 3],
//     so one instruction is 16 out rows x 4 k x 4 pairs and accumulator element i of block
//     (og, kb) holds row 4·og + ((i + kb) & 3) summed over k sub-block kb.  The rows are
//     rotated by kb so that after the layer the four sub-blocks of a row sit on a diagonal:
//     three DPP row_ror adds (a pairwise tree) leave row 4·og + kb in lane (og, kb, j), with
//     no per-lane select (qring_sum);
//   * the Q_WAVES = 8 waves of the workgroup (two per SIMD) own an eighth of every layer's
//     out rows; after the sum each lane keeps one (row, pair) value ("compact": row
//     r0 + 4·og + kb, pair l & 3), runs the epilogue on it and writes it to an LDS
//     activation buffer laid out for the next layer's B reads (one ds_read_b128 per 4 k and
//     column, conflict-free), then one workgroup barrier per layer.  Eight waves, not four:
//     a planner step is bound by the CU's weight stream, and one CU reads L2/MALL at
//     ~130 GB/s with eight waves loading against ~103 GB/s with four
//     (tests/diag/stream_probe2.hip: 33 vs 42 µs per 4.33 MB step);
//   * the saved σ10 values stay in LDS (compact, per wave), so there is no global scratch;
//   * each wave's weight fragments are packed in consumption order (pntf_common.h Q_LAYERS),
//     so the prefetch ring is one linear stream of 1 KiB fragments, 16 in flight per wave
//     (128 KiB per CU), that wraps from the last reverse layer into the next step's
//     encoder[0].
// 1024 queries are 256 tiles: every CU of the chip has one.  Reductions whose result every
// lane consumes (τ, ∇τ) use xor butterflies and a fixed wave order, so all lanes of a pair
// hold bitwise identical values and the planner's freeze/exit decisions agree in all waves.
#include "pntf_split.h"
#include "pntf_stamp.h"

namespace pntf {

constexpr int QPAIRS = 4;
// independent accumulator chains per column (k steps alternate between them)
#ifndef PNTF_Q_CHAINS
#define PNTF_Q_CHAINS 2
#endif
constexpr int QCH = PNTF_Q_CHAINS;
#ifndef PNTF_QKEEPB
#define PNTF_QKEEPB 1
#endif
// Fragments in flight per wave: the ∇τ kernels (4224 / Q_WAVES fragments per step) run
// PNTF_QRING of them; the τ-only kernels wrap after the forward half and run half as many.
// (128 KiB in flight per CU at either wave count)
#ifndef PNTF_QRING
#define PNTF_QRING (128 / PNTF_QWAVES)
#endif
constexpr int QRING = PNTF_QRING;
// the SOLO planner layers (one query per workgroup, VALU) hold their own accumulators beside
// the ring: a unit may give them a different depth
#ifndef PNTF_QRING_SOLO
#define PNTF_QRING_SOLO PNTF_QRING
#endif
constexpr int QRING_SOLO = PNTF_QRING_SOLO;
constexpr int QRING_TAU = 64 / Q_WAVES;
#ifndef PNTF_QPIN
#define PNTF_QPIN 1
#endif
// cache policy of the weight-stream loads (every CU reads the same fragments from L2 once per
// step; the CU's L1 never sees a fragment twice)
#ifndef PNTF_QLOAD_AUX
#define PNTF_QLOAD_AUX 0
#endif
// stream position (mod the ring) of a layer that follows a 128 x 128 one: the first ring slot
// of every other encoder layer
constexpr int QH = 64 / Q_WAVES;
// groups of 16 out rows per wave of a layer with OUT rows
constexpr int qg(int out) { return out / (16 * Q_WAVES); }
// ring slot of layer L's first fragment: its position in the wave's stream mod the ring depth
// (compile-time for every layer, so any ring depth that divides the per-step stream works)
template <int L, int QR>
constexpr int qslot() { return (q_layer_off(L) / 256) % QR; }
// layer L prefetches QR fragments ahead: past the end of the NF-fragment stream those loads
// wrap to the next step's first layer (qfetch WRAP), which only the stream's last layers reach
template <int L, int NF, int QR>
constexpr bool qwrap() { return q_layer_off(L + 1) / 256 + QR > NF; }
constexpr int Q_NF_ALL = 2 * Q_NF_FWD;
static_assert(Q_NF_ALL % QRING == 0 && Q_NF_ALL % QRING_SOLO == 0 && Q_NF_FWD % QRING_TAU == 0,
              "the ring depth must divide the per-step stream (its slots repeat every step)");
constexpr int QBUF = 2 * 16 * 68;           // activation buffer: 2 columns x 16 lane rows x 68
constexpr int QNSIG = 48;                   // saved σ10 slots per wave (64 floats each)
constexpr int Q_RED = 3 * QBUF + Q_WAVES * QNSIG * 64;
constexpr int Q_BW = Q_RED + Q_WAVES * 12 * 4;   // 2π·B of the tile's 4 pairs: [pair][dim][128]
// 96 KiB (4 waves) / 135 KiB (8 waves): more than half the CU's LDS, so one workgroup per CU
// (a second one would stream the weights through the same CU a second time per step)
constexpr int Q_LDS_FLOATS = (Q_BW + QPAIRS * 6 * H + 64 + 1023) / 1024 * 1024;
static_assert(Q_LDS_FLOATS >= 24576 && Q_LDS_FLOATS <= 40960, "quad LDS budget");
// σ slots (forward order): encoder[0] 0-3, encoder blocks a0 4-7, b0 8-11, a1 12-15,
// b1 16-19 (group·2 + column), merge switch 20-21, generator a_i 22 + 8i + g, b_i 26 + 8i + g,
// generator[-2] 46-47.
constexpr int QS_E0 = 0, QS_EBLK = 4, QS_S0 = 20, QS_GBLK = 22, QS_G3 = 46;

__device__ __forceinline__ void qsync() {
#ifndef PNTF_QABL_NOBAR   // diagnostics only (tests/diag timing ablations; wrong results)
  wg_sync();
#endif
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}
// v of the lane CTRL selects (DPP row_ror:N = 0x120 + N: lane i of a 16-lane row reads
// lane (i - N) mod 16; quad_perm 0x00: lane 4m reads lane 4m)
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                       0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
// Sum of the four k sub-blocks of a layer's rows.  t[i] of lane (og, kb, j) is row
// (i + kb) & 3 over sub-block kb (pack_quad_kernel rotates the rows by kb), so S_k, row kb's
// partial over sub-block k, is t[kb - k] of lane (og, k, j).  A pairwise tree in three DPP adds
// with no per-lane select:
//   B = t[0] + ror4(t[1])   in lane kb: S_kb + S_kb-1 of row kb
//   A = t[2] + ror4(t[3])   in lane m: S_m + S_m-1 of row m + 2, so lane kb - 2 holds
//                           S_kb-2 + S_kb-3 of row kb
//   v = B + ror8(A)         (S_kb + S_kb-1) + (S_kb-2 + S_kb-3) = row kb, pair j
// (the association of the unrotated layout's two full-row butterflies, so results do not
// depend on the rotation).
__device__ __forceinline__ float qring_sum(const f32x4& t) {
  const float b = t[0] + dpp<0x124>(t[1]);
  const float a = t[2] + dpp<0x124>(t[3]);
  return b + dpp<0x128>(a);
}
// The same sum for a SOLO layer, whose lane (og, kb, r) holds one partial: row (r + kb) & 3
// over sub-block kb, so S_k of row kb sits in lane (og, k, kb - k).  row_ror:3 reads lane
// (k - 1, r + 1) from (k, r < 3): B = t + ror3(t) is S_kb + S_kb-1 in lane (kb, 0) and
// S_kb-2 + S_kb-3 in lane (kb - 2, 2), six lanes below, so B + ror6(B) in lane (og, kb, 0) is
// qring_sum's value bit for bit; a quad_perm broadcast gives it to the lane's other pair slots.
__device__ __forceinline__ float qring_sum_solo(float t) {
  const float b = t + dpp<0x123>(t);
  return dpp<0x00>(b + dpp<0x126>(b));
}

// x ^ mask lane exchange inside 32-lane halves (ds_swizzle bit mode)
template <int MASK>
__device__ __forceinline__ float swz_xor(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_swizzle(__builtin_bit_cast(int, v),
                                                                0x1f | (MASK << 10)));
}
// Sum over the 16 lanes of the same pair (lane bits 2-5), identical in all of them: xor
// butterflies (a + b == b + a bitwise).
__device__ __forceinline__ float pair_sum(float v) {
  v += swz_xor<4>(v);
  v += swz_xor<8>(v);
  v += swz_xor<16>(v);
  v += __shfl_xor(v, 32);
  return v;
}

// Bias vectors per layer: one value per group of 16 out rows the wave owns (qg(256) of them at
// most: 2 with 8 waves), so 14 of them take 28 VGPRs, not the 56 of a 4-group vector.  The
// head bias generator.4.bias rides in aux[13][qg(128)], a slot generator[-2] does not use.
constexpr int QAUXW = 256 / (16 * Q_WAVES);
static_assert(QAUXW == 2 || QAUXW == 4, "quad bias vector width");
typedef float qaux_t __attribute__((ext_vector_type(QAUXW)));
constexpr int QAUX_G4B = 128 / (16 * Q_WAVES);
// pack_quad_aux_kernel stores 4 groups per lane (16 bytes); the first QAUXW are the used ones
__device__ __forceinline__ qaux_t qaux_load(Rsrc AX, int lane, int i) {
  qaux_t r;
  if constexpr (QAUXW == 4) {
    const f32x4 t = bload(AX, lane * 16, i * 1024);
#pragma unroll
    for (int k = 0; k < QAUXW; ++k) r[k] = t[k % 4];
  } else {
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const f32x2 t = __builtin_bit_cast(
        f32x2, __builtin_amdgcn_raw_buffer_load_b64(AX, lane * 16, i * 1024, 0));
#pragma unroll
    for (int k = 0; k < QAUXW; ++k) r[k] = t[k % 2];
  }
  return r;
}
// v[g] for a runtime group index (explicit selects: a dynamic vector index would put the
// vector on the stack)
template <int N = QAUXW>
__device__ __forceinline__ float pick(const qaux_t& v, int g) {
  if constexpr (N == 2) return g == 0 ? v[0] : v[1];
  else return g == 0 ? v[0] : g == 1 ? v[1] : g == 2 ? v[2] : v[3];
}

struct QCx {
  lds_f* lds;
  int w, lane, og, kb, l16;
  int sp;   // the pair a SOLO layer reads (0: the single query)
  __device__ lds_f* buf(int b) const { return lds + b * QBUF; }
  __device__ lds_f* sig(int slot) const { return lds + 3 * QBUF + (w * QNSIG + slot) * 64 + lane; }
  __device__ lds_f* red(int wave, int v) const { return lds + Q_RED + (wave * 12 + v) * 4; }
  // 2π·B[d][f] of pair j of the tile (staged once per tile by quad_stage_b)
  __device__ lds_f* bw(int j, int d) const { return lds + Q_BW + (j * 6 + d) * H; }
  // compact (row, pair) slot of a layer with OUT rows, group g, column c in a buffer read by
  // the next layer (its in features = BUF, default OUT: row stride BUF/4 + 4)
  template <int OUT, int BUF = OUT>
  __device__ lds_f* at(lds_f* b, int c, int g) const {
    return b + (c * 16 + l16) * (BUF / 4 + 4) + w * (OUT / (4 * Q_WAVES)) + 4 * g + og;
  }
};

template <int QR>
struct QRing {
  f32x4 r[QR];
  int off;   // byte offset of the next fragment to load (wave-uniform)
};
// Load the next stream fragment into ring slot `slot`: one scalar add per load.  Only the
// stream's last layer (WRAP) prefetches past the end of the stream, into the next step's first
// layer: there the offset is wrapped before the load (two more scalar ops, that layer alone;
// the layer before it leaves the offset at the end of the stream).
template <int NF, int QR, bool WRAP>
__device__ __forceinline__ void qfetch(QRing<QR>& ring, Rsrc W, int lane, int slot) {
  if constexpr (WRAP) ring.off = ring.off == NF * 1024 ? 0 : ring.off;
#ifdef PNTF_QABL_NOLOAD   // diagnostics only (tests/diag timing ablations; wrong results)
  ring.r[slot] = ring.r[slot] * 1.0001f;
#else
  ring.r[slot] = __builtin_bit_cast(
      f32x4, __builtin_amdgcn_raw_buffer_load_b128(W, lane * 16, ring.off, PNTF_QLOAD_AUX));
#endif
  ring.off += 1024;
#if PNTF_QPIN
  // keep the load where it is: under register pressure the scheduler otherwise sinks it to
  // just before its use QR fragments later, and the ring drains to vmcnt(0) every layer
  __builtin_amdgcn_sched_barrier(0);
#endif
}

// One layer: G groups of 16 out rows; per group IN/16 fragments of 4 k steps x NC columns;
// B operands read from `in` (IN features, row stride IN/4 + 4).  The layer's first fragment
// sits in ring slot S0.  epi(g, v[NC]) gets the compact sums of group g.
template <int NC, int IN, int NF, int G, int S0, int QR, bool SOLO, bool WRAP = false,
          class Epi>
__device__ __forceinline__ void qlayer(QRing<QR>& ring, Rsrc W, const QCx& cx, const lds_f* in,
                                       Epi&& epi) {
  constexpr int SP = IN / 4 + 4, NQ = IN / 16;
  // B operands kept in registers for all groups of the layer when they fit (64 VGPRs):
  // one LDS read per fragment instead of one per fragment and group
  // (not in the SOLO layers at 8 waves: beside the VALU accumulators they spilled)
  constexpr bool KEEP = PNTF_QKEEPB && G > 1 && NC * NQ <= 16 && !(SOLO && Q_WAVES == 8);
  // SOLO: every lane reads the one active pair's B operands (row kb, pair cx.sp)
  const lds_f* src = in + (SOLO ? ((cx.l16 & ~3) | cx.sp) : cx.l16) * SP;
  f32x4 xb[KEEP ? NC : 1][KEEP ? NQ : 1];
  if constexpr (KEEP) {
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        xb[c][q] = *reinterpret_cast<const lds_f4*>(src + c * 16 * SP + 4 * q);
  }
  if constexpr (SOLO) {
  // one active query in the tile (planner): the fragment runs on the VALU for that pair
  // (4 FMAs per column instead of 4 MFMAs of which 3 columns are idle); each lane's sum is
  // row r0 + 4·og + ((l + kb) & 3) over its k sub-block kb, and every pair slot carries the
  // values
  static_for<0, G>([&](auto gg) {
    constexpr int g = decltype(gg)::value;
    const lds_f* src0 = src;
    float acc[NC][QCH];
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int h = 0; h < QCH; ++h) acc[c][h] = 0.f;
    static_for<0, NQ>([&](auto qq) {
      constexpr int q = decltype(qq)::value, slot = (S0 + g * NQ + q) % QR;
      f32x4 b[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if constexpr (KEEP) b[c] = xb[c][q];
        else b[c] = *reinterpret_cast<const lds_f4*>(src0 + c * 16 * SP + 4 * q);
      }
      const f32x4 a = ring.r[slot];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[c][e % QCH] = fmaf(a[e], b[c][e], acc[c][e % QCH]);
      qfetch<NF, QR, WRAP>(ring, W, cx.lane, slot);
    });
    float v[NC];
    // the compact value of lane l is row r0 + 4·og + kb (the MFMA path's layout), summed in
    // the MFMA path's order, so SOLO and the MFMA layers give bit-identical results (the
    // planner's tail hand-off switches a query from one to the other mid-plan)
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      float t = acc[c][0];
#pragma unroll
      for (int h = 1; h < QCH; ++h) t += acc[c][h];
      v[c] = qring_sum_solo(t);
    }
    epi(g, v);
  });
  return;
  }
  static_for<0, G>([&](auto gg) {
    constexpr int g = decltype(gg)::value;
    f32x4 acc[NC][QCH];
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int h = 0; h < QCH; ++h) acc[c][h] = zero4();
    static_for<0, NQ>([&](auto qq) {
      constexpr int q = decltype(qq)::value, slot = (S0 + g * NQ + q) % QR;
      f32x4 b[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
#ifdef PNTF_QABL_NOLDS   // diagnostics only (tests/diag timing ablations; wrong results)
        b[c] = f32x4{0.1f * q, 0.2f * c, 0.3f, 0.4f} + (float)cx.lane;
#else
        if constexpr (KEEP) b[c] = xb[c][q];
        else b[c] = *reinterpret_cast<const lds_f4*>(src + c * 16 * SP + 4 * q);
#endif
      }
      const f32x4 a = ring.r[slot];
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[c][e % QCH] = mfma4(a[e], b[c][e], acc[c][e % QCH]);
      qfetch<NF, QR, WRAP>(ring, W, cx.lane, slot);
    });
    float v[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      f32x4 t = acc[c][0];
#pragma unroll
      for (int h = 1; h < QCH; ++h) t += acc[c][h];
      v[c] = qring_sum(t);
    }
    epi(g, v);
  });
}

// Sum of NV per-lane values over the pair's 16 lanes and the 4 waves (fixed order); the
// result is identical in every lane of the pair in every wave.
template <int NV>
__device__ __forceinline__ void qreduce(const QCx& cx, float (&v)[NV]) {
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = pair_sum(v[i]);
  if (cx.lane < QPAIRS)
#pragma unroll
    for (int i = 0; i < NV; ++i) cx.red(cx.w, i)[cx.lane] = v[i];
  qsync();
  const int j = cx.lane & 3;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float s = cx.red(0, i)[j];
#pragma unroll
    for (int q = 1; q < Q_WAVES; ++q) s += cx.red(q, i)[j];
    v[i] = s;
  }
}

// Forward pass (NN.out, :215-259) for the 4 pairs of the tile; returns τ of the lane's pair.
// GRAD: save σ10 for the reverse sweep.  Buffers: 0 = features / dz, 1 = A, 2 = B.
template <int DIM, bool GRAD, int NF, int QR, bool SOLO = false>
__device__ __forceinline__ float quad_forward(QRing<QR>& ring, Rsrc W, const QCx& cx,
                                              const PairIO& io, const qaux_t (&aux)[Q_NAUX],
                                              int compat) {
  const float cm = compat ? 1.f : 0.f;
  lds_f *F = cx.buf(0), *A = cx.buf(1), *B = cx.buf(2);
  const int t = cx.w * 64 + cx.lane;
  // ---- Fourier features (:186-190): thread t computes column (t >> 2) & 1 of its lane's
  // pair for features t >> 3 + 32 m; sin f -> k = f, cos f -> k = f + 128
  {
    const int c = (t >> 2) & 1, j = t & 3, fb = t >> 3;
    float xc[DIM];
#pragma unroll
    for (int d = 0; d < DIM; ++d) xc[d] = c ? io.x[1][d] : io.x[0][d];
#pragma unroll
    for (int m = 0; m < 128 / (8 * Q_WAVES); ++m) {
      const int f = fb + 8 * Q_WAVES * m;
      float q = 0.f;
#pragma unroll
      for (int d = 0; d < DIM; ++d) q = fmaf(xc[d], cx.bw(j, d)[f], q);
      float sn, cs;
      sincos_fast(q, sn, cs);
      lds_f* p = F + (c * 16 + 4 * (f & 3) + j) * 68 + (f >> 2);
      p[0] = sn;
      p[32] = cs;
    }
  }
  qsync();
  // ---- encoder[0] (:227); compat: the out_backgrad quirk (:435-438) stores σ10(softplus(y))
  qlayer<2, 256, NF, qg(128), qslot<0, QR>(), QR, SOLO, qwrap<0, NF, QR>()>(ring, W, cx, F, [&](int g, const float (&v)[2]) {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      SpSig q = sp_sig(v[c] + pick(aux[0], g));
      *cx.at<128>(A, c, g) = q.sp;
      if (GRAD) *cx.sig(QS_E0 + 2 * g + c) = fmaf(cm, __builtin_amdgcn_rcpf(2.f - q.sg) - q.sg, q.sg);
    }
  });
  qsync();
  // ---- encoder residual blocks (:228-232): a: A -> B, b: B (+ A residual) -> A
  static_for<0, 2>([&](auto bb) {
    constexpr int blk = decltype(bb)::value;
    constexpr int la = 1 + 2 * blk, sa = QS_EBLK + 8 * blk;
    qlayer<2, 128, NF, qg(128), qslot<la, QR>(), QR, SOLO, qwrap<la, NF, QR>()>(ring, W, cx, A, [&](int g, const float (&v)[2]) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        SpSig q = sp_sig(v[c] + pick(aux[la], g));
        *cx.at<128>(B, c, g) = q.sp;
        if (GRAD) *cx.sig(sa + 2 * g + c) = q.sg;
      }
    });
    qsync();
    qlayer<2, 128, NF, qg(128), qslot<la + 1, QR>(), QR, SOLO, qwrap<la + 1, NF, QR>()>(ring, W, cx, B, [&](int g, const float (&v)[2]) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        lds_f* o = cx.at<128>(A, c, g);
        SpSig q = sp_sig(v[c] + pick(aux[la + 1], g) + *o);
        *o = q.sp;
        if (GRAD) *cx.sig(sa + 4 + 2 * g + c) = q.sg;
      }
    });
    qsync();
  });
  // ---- encoder[-1] (:234) and the smooth max / min merge (:236-244): u = [M | m] -> B
  qlayer<2, 128, NF, qg(128), qslot<5, QR>(), QR, SOLO, qwrap<5, NF, QR>()>(ring, W, cx, A, [&](int g, const float (&v)[2]) {
    const float zs = v[0] + pick(aux[5], g), zg = v[1] + pick(aux[5], g);
    const float d = zs - zg;
    const float e = exp_neg10abs(d);
    const float cc = 0.1f * log1p_small(e);
    lds_f* o = cx.at<128, 256>(B, 0, g);   // row r of a 128-row layer in a 256-row buffer
    o[0] = fmaxf(zs, zg) + cc;
    o[32] = fminf(zs, zg) - cc;
    if (GRAD) {
      const float rr = __builtin_amdgcn_rcpf(1.f + e);
      *cx.sig(QS_S0 + g) = (d >= 0.f) ? rr : e * rr;
    }
  });
  qsync();
  // ---- generator residual blocks (:246-249): a: B -> A, b: A (+ B residual) -> B
  // a generator block is 2 x 256 x 256 / Q_WAVES / 256 fragments; when the ring depth divides
  // that, every block starts on the same slot and the loop stays rolled (code size).  (The
  // body is a macro: as a lambda called with a runtime block index it put `aux` on the stack.)
#define PNTF_QGEN_FWD(i, S0A, S0B, WA, WB)                                                                 \
  {                                                                                                \
    const qaux_t ba = (i) == 0 ? aux[6] : (i) == 1 ? aux[8] : aux[10];                              \
    const qaux_t bb = (i) == 0 ? aux[7] : (i) == 1 ? aux[9] : aux[11];                              \
    qlayer<1, 256, NF, qg(256), S0A, QR, SOLO, WA>(ring, W, cx, B, [&](int g, const float (&v)[1]) {   \
      SpSig q = sp_sig(v[0] + pick(ba, g));                                                        \
      *cx.at<256>(A, 0, g) = q.sp;                                                                 \
      if (GRAD) *cx.sig(QS_GBLK + 8 * (i) + g) = q.sg;                                             \
    });                                                                                            \
    qsync();                                                                                       \
    qlayer<1, 256, NF, qg(256), S0B, QR, SOLO, WB>(ring, W, cx, A, [&](int g, const float (&v)[1]) {   \
      lds_f* o = cx.at<256>(B, 0, g);                                                              \
      SpSig q = sp_sig(v[0] + pick(bb, g) + *o);                                                   \
      *o = q.sp;                                                                                   \
      if (GRAD) *cx.sig(QS_GBLK + 8 * (i) + 4 + g) = q.sg;                                         \
    });                                                                                            \
    qsync();                                                                                       \
  }
  if constexpr ((2 * 256 * 256 / Q_WAVES / 256) % QR == 0) {
#pragma unroll 1
    for (int i = 0; i < 3; ++i)
      PNTF_QGEN_FWD(i, (qslot<6, QR>()), (qslot<7, QR>()), (qwrap<10, NF, QR>()), (qwrap<11, NF, QR>()))
  } else {
    static_for<0, 3>([&](auto ii) {
      constexpr int i = decltype(ii)::value;
      PNTF_QGEN_FWD(i, (qslot<6 + 2 * i, QR>()), (qslot<7 + 2 * i, QR>()), (qwrap<6 + 2 * i, NF, QR>()),
                    (qwrap<7 + 2 * i, NF, QR>()))
    });
  }
#undef PNTF_QGEN_FWD
  // ---- generator[-2] + act (:251-252) and the head generator[-1] (:254-255)
  float part[1] = {0.f};
  qlayer<1, 256, NF, qg(128), qslot<12, QR>(), QR, SOLO, qwrap<12, NF, QR>()>(ring, W, cx, B, [&](int g, const float (&v)[1]) {
    SpSig q = sp_sig(v[0] + pick(aux[12], g));
    part[0] = fmaf(pick(aux[13], g), q.sp, part[0]);
    if (GRAD) *cx.sig(QS_G3 + g) = q.sg;
  });
  qreduce<1>(cx, part);
  const float y4 = part[0] + aux[13][QAUX_G4B];
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-0.144269504088896341f * y4));
}

// Reverse sweep (exact, or out_backgrad when the forward stored the quirk): dτ/dxs, dτ/dxg of
// the lane's pair, identical in all lanes of the pair.
template <int DIM, int NF, int QR, bool SOLO = false>
__device__ __forceinline__ void quad_backward(QRing<QR>& ring, Rsrc W, const QCx& cx,
                                              const PairIO& io, float tau,
                                              const qaux_t (&aux)[Q_NAUX], float (&ds)[DIM],
                                              float (&dg)[DIM]) {
  lds_f *F = cx.buf(0), *A = cx.buf(1), *B = cx.buf(2);
  // ---- head and generator[-2] (:592-613): dv = d · G4 ⊙ σ10(y3) -> A (128 rows)
  const float dd = 0.1f * tau * (1.f - tau);
#pragma unroll
  for (int g = 0; g < qg(128); ++g) *cx.at<128>(A, 0, g) = dd * pick(aux[13], g) * *cx.sig(QS_G3 + g);
  qsync();
  // du = G3^T dv ⊙ σ10(y2 of generator block 2) -> B
  qlayer<1, 128, NF, qg(256), qslot<13, QR>(), QR, SOLO, qwrap<13, NF, QR>()>(ring, W, cx, A, [&](int g, const float (&v)[1]) {
    *cx.at<256>(B, 0, g) = v[0] * *cx.sig(QS_GBLK + 16 + 4 + g);
  });
  qsync();
  // ---- generator blocks, reverse (:615-618): lb: B -> A, la: A (+ B residual) -> B
#define PNTF_QGEN_BWD(i, S0B, S0A, WB, WA)                                                                 \
  {                                                                                                \
    qlayer<1, 256, NF, qg(256), S0B, QR, SOLO, WB>(ring, W, cx, B, [&](int g, const float (&v)[1]) {   \
      *cx.at<256>(A, 0, g) = v[0] * *cx.sig(QS_GBLK + 8 * (i) + g);                                \
    });                                                                                            \
    qsync();                                                                                       \
    const int sb = QS_GBLK + 8 * ((i) - 1) + 4;   /* σ10(y2) of block i - 1 (none for i = 0) */   \
    qlayer<1, 256, NF, qg(256), S0A, QR, SOLO, WA>(ring, W, cx, A, [&](int g, const float (&v)[1]) {   \
      lds_f* o = cx.at<256>(B, 0, g);                                                              \
      const float y = v[0] + *o;                                                                   \
      *o = (i) > 0 ? y * *cx.sig(sb + g) : y;                                                      \
    });                                                                                            \
    qsync();                                                                                       \
  }
  if constexpr ((2 * 256 * 256 / Q_WAVES / 256) % QR == 0) {
#pragma unroll 1
    for (int i = 2; i >= 0; --i)
      PNTF_QGEN_BWD(i, (qslot<14, QR>()), (qslot<15, QR>()), (qwrap<18, NF, QR>()), (qwrap<19, NF, QR>()))
  } else {
    static_for<0, 3>([&](auto jj) {
      constexpr int j = decltype(jj)::value, i = 2 - j;
      PNTF_QGEN_BWD(i, (qslot<14 + 2 * j, QR>()), (qslot<15 + 2 * j, QR>()), (qwrap<14 + 2 * j, NF, QR>()),
                    (qwrap<15 + 2 * j, NF, QR>()))
    });
  }
#undef PNTF_QGEN_BWD
  // ---- merge Jacobian (:620-627) on the wave's 128-row share: dz -> F (2 columns)
#pragma unroll
  for (int g = 0; g < qg(128); ++g) {
    const lds_f* u = cx.at<128, 256>(B, 0, g);   // row r of the 128-row map
    const float dM = u[0], dm = u[32];
    const float s0 = *cx.sig(QS_S0 + g), s1 = 1.f - s0;
    *cx.at<128>(F, 0, g) = s0 * dM + s1 * dm;
    *cx.at<128>(F, 1, g) = s1 * dM + s0 * dm;
  }
  qsync();
  // ---- encoder[-1]^T, then ⊙ σ10(y2 of encoder block 1): F -> A
  qlayer<2, 128, NF, qg(128), qslot<20, QR>(), QR, SOLO, qwrap<20, NF, QR>()>(ring, W, cx, F, [&](int g, const float (&v)[2]) {
#pragma unroll
    for (int c = 0; c < 2; ++c) *cx.at<128>(A, c, g) = v[c] * *cx.sig(QS_EBLK + 12 + 2 * g + c);
  });
  qsync();
  // ---- encoder blocks, reverse (:633-636): b^T: A -> B (⊙ σ10(y1)), a^T: B (+ A) -> A
  // (⊙ σ10 of the layer below: block 0's y2, or encoder[0])
  static_for<0, 2>([&](auto jj) {
    constexpr int blk = 1 - decltype(jj)::value;
    constexpr int sa = QS_EBLK + 8 * blk, sbelow = blk ? QS_EBLK + 4 : QS_E0;
    qlayer<2, 128, NF, qg(128), qslot<21 + 2 * (1 - blk), QR>(), QR, SOLO, qwrap<21 + 2 * (1 - blk), NF, QR>()>(ring, W, cx, A, [&](int g, const float (&v)[2]) {
#pragma unroll
      for (int c = 0; c < 2; ++c) *cx.at<128>(B, c, g) = v[c] * *cx.sig(sa + 2 * g + c);
    });
    qsync();
    qlayer<2, 128, NF, qg(128), qslot<22 + 2 * (1 - blk), QR>(), QR, SOLO, qwrap<22 + 2 * (1 - blk), NF, QR>()>(ring, W, cx, B, [&](int g, const float (&v)[2]) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        lds_f* o = cx.at<128>(A, c, g);
        *o = (v[c] + *o) * *cx.sig(sbelow + 2 * g + c);
      }
    });
    qsync();
  });
  // ---- encoder[0]^T fused with the Fourier Jacobian (:639-645): the wave's 256/Q_WAVES
  // feature rows f (sin rows f < 128 in the first half of the waves, cos rows in the second),
  // both columns
  float acc[2 * DIM];
#pragma unroll
  for (int i = 0; i < 2 * DIM; ++i) acc[i] = 0.f;
  qlayer<2, 128, NF, qg(256), qslot<25, QR>(), QR, SOLO, qwrap<25, NF, QR>()>(ring, W, cx, A, [&](int g, const float (&v)[2]) {
    const int f = cx.w * (256 / Q_WAVES) + 16 * g + 4 * cx.og + cx.kb;
    const int fb = f & 127;
    float bw[DIM];
#pragma unroll
    for (int d = 0; d < DIM; ++d) bw[d] = cx.bw(cx.lane & 3, d)[fb];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      float q = 0.f;
#pragma unroll
      for (int d = 0; d < DIM; ++d) q = fmaf(io.x[c][d], bw[d], q);
      float sn, cs;
      sincos_fast(q, sn, cs);
      const float gg = f < 128 ? v[c] * cs : -(v[c] * sn);
#pragma unroll
      for (int d = 0; d < DIM; ++d) acc[c * DIM + d] = fmaf(bw[d], gg, acc[c * DIM + d]);
    }
  });
  qreduce<2 * DIM>(cx, acc);
#pragma unroll
  for (int d = 0; d < DIM; ++d) {
    ds[d] = acc[d];
    dg[d] = acc[DIM + d];
  }
}

// The tile's Fourier matrices (2π·B of each pair's env) into LDS, once per tile: the per-step
// feature and fold reads then never wait on vmcnt, which would drain the weight ring.  The
// caller's next barrier (the one after the features) orders the writes before any read; the
// previous tile's last reads (its fold) precede the qreduce barrier.
template <int DIM>
__device__ __forceinline__ void quad_stage_b(const QCx& cx, const PairIO& io) {
  // thread (w, lane): pair j = lane & 3 (its own io), rows d, features (lane >> 2) + 16 i
  const int j = cx.lane & 3, f0 = (cx.lane >> 2) + 16 * cx.w;
#pragma unroll
  for (int d = 0; d < DIM; ++d)
#pragma unroll
    for (int i = 0; i < H / (16 * Q_WAVES); ++i)
      cx.bw(j, d)[f0 + 16 * Q_WAVES * i] = TWO_PI * io.Bw[d * H + f0 + 16 * Q_WAVES * i];
}

__device__ __forceinline__ QCx quad_cx(lds_f* lds) {
  QCx cx;
  cx.lds = lds;
  cx.lane = threadIdx.x & 63;
  cx.w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  cx.og = cx.lane >> 4;
  cx.kb = (cx.lane >> 2) & 3;
  cx.l16 = cx.lane & 15;
  cx.sp = 0;
#if defined(PNTF_QPRIO) && PNTF_QPRIO   // diagnostics: static priority for the second wave half
  if (cx.w >= Q_WAVES / 2) __builtin_amdgcn_s_setprio(1);
#endif
  return cx;
}

// τ / ∇τ / epilogues on quad tiles: one workgroup per 4-pair tile (grid-stride), same
// outputs as field_kernel<DIM, KIND>.
template <int DIM, int KIND>
__global__ __launch_bounds__(64 * Q_WAVES, 1) void field_quad_kernel(FieldArgs a) {
  constexpr bool GRAD = KIND != K_TAU && KIND != K_TRAVEL;
  constexpr int NF = GRAD ? Q_NF_ALL : Q_NF_FWD;
  constexpr int QR = GRAD ? QRING : QRING_TAU;
  __shared__ float smem[Q_LDS_FLOATS];
  const QCx cx = quad_cx((lds_f*)smem);
  const Rsrc W = make_rsrc(a.P + OFF_QUAD + cx.w * Q_STREAM, Q_STREAM * 4);
  const Rsrc AX = make_rsrc(a.P + OFF_QUAD + Q_OFF_AUX + cx.w * Q_NAUX * 256, Q_NAUX * 1024);
  qaux_t aux[Q_NAUX];
#pragma unroll
  for (int i = 0; i < Q_NAUX; ++i) aux[i] = qaux_load(AX, cx.lane, i);
  aux[13][QAUX_G4B] = a.P[OFF_BIAS + B_G4B];
  QRing<QR> ring;
  ring.off = 0;
#pragma unroll
  for (int s = 0; s < QR; ++s) qfetch<NF, QR, false>(ring, W, cx.lane, s);
  const int64_t ntiles = (a.n + QPAIRS - 1) / QPAIRS;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t pair = tile * QPAIRS + (cx.lane & 3);
    PairIO io;
    const bool ok = load_pair<DIM>(a.xp, a.Btab, a.env, a.n, a.n_env, pair, io);
    quad_stage_b<DIM>(cx, io);
    qsync();
    const float tau = quad_forward<DIM, GRAD, NF, QR>(ring, W, cx, io, aux, a.compat);
    float ds[DIM], dg[DIM];
    if constexpr (GRAD) quad_backward<DIM, NF, QR>(ring, W, cx, io, tau, aux, ds, dg);
    const bool store = cx.w == 0 && cx.lane < QPAIRS && pair < a.n;
    store_field<DIM, KIND>(a, pair, ok, store, tau, io, ds, dg);
  }
}

// Batched planner on quad tiles: one workgroup per 4-query tile (grid-stride), the loop of
// plan_kernel (test/gib_plan.py:74-86, test/arm_plan.py:140-152) with per-query freeze.
// SOLO (one query per workgroup: the reference's Q = 1 loop, and any batch of at most one
// query per CU): the tile is a single query, loaded into all four pair slots; the layers run
// as VALU dot products for pair slot 0 (qlayer), the other slots carry the same values, and
// only slot 0 stores.
//
// Tail hand-off (a.tail != NULL): a 4-query tile costs ~57 µs per step on its
// CU whatever number of its queries are still active, a SOLO query ~43 µs (the per-CU weight
// stream).  The MFMA tiles count converged queries in tail[0] (device-scope atomics); once at
// most a.yield_at queries of the batch remain (one per CU), every tile that still has active
// queries hands them off — index and resume iteration into tail[] — and exits; the SOLO
// launch that follows resumes each from its path row, one query per workgroup.  The layers
// are bit-identical in both forms (qlayer), so the plan does not depend on when the hand-off
// happens.
constexpr int Q_YIELD_FLAG = Q_BW + QPAIRS * 6 * H;   // LDS word: this tile yields
#ifndef PNTF_Q_YIELD_EVERY
#define PNTF_Q_YIELD_EVERY 4
#endif
constexpr int Q_YIELD_EVERY = PNTF_Q_YIELD_EVERY;     // steps between hand-off checks (2^k)
static_assert(Q_YIELD_FLAG < Q_LDS_FLOATS, "quad LDS budget");

template <int DIM, bool SOLO>
__global__ __launch_bounds__(64 * Q_WAVES, 1) void plan_quad_kernel(PlanArgs a) {
  PNTF_CLOCK_SCOPE;
  __shared__ float smem[Q_LDS_FLOATS];
  const QCx cx = quad_cx((lds_f*)smem);
  int32_t* const tail = a.tail;
  const bool resume = SOLO && tail != nullptr;    // second launch: the handed-off queries
  const bool can_yield = !SOLO && tail != nullptr;
  int32_t* const tail_q = tail ? tail + 2 : nullptr;
  int32_t* const tail_it = tail ? tail + 2 + a.q : nullptr;
  const Rsrc W = make_rsrc(a.P + OFF_QUAD + cx.w * Q_STREAM, Q_STREAM * 4);
  const Rsrc AX = make_rsrc(a.P + OFF_QUAD + Q_OFF_AUX + cx.w * Q_NAUX * 256, Q_NAUX * 1024);
  qaux_t aux[Q_NAUX];
#pragma unroll
  for (int i = 0; i < Q_NAUX; ++i) aux[i] = qaux_load(AX, cx.lane, i);
  aux[13][QAUX_G4B] = a.P[OFF_BIAS + B_G4B];
  constexpr int QR = SOLO ? QRING_SOLO : QRING;
  QRing<QR> ring;
  ring.off = 0;
#pragma unroll
  for (int s = 0; s < QR; ++s) qfetch<Q_NF_ALL, QR, false>(ring, W, cx.lane, s);
  const int cap = a.max_iter + 1;
  const int64_t rows = (int64_t)cap + 1;
  constexpr int TQ = SOLO ? 1 : QPAIRS;   // queries per tile
  const int64_t ntiles = resume ? (int64_t)tail[1] : (a.q + TQ - 1) / TQ;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t qi = resume ? (int64_t)tail_q[tile] : SOLO ? tile : tile * QPAIRS + (cx.lane & 3);
    PairIO io;
    const bool ok = load_pair<DIM>(a.xp0, a.Btab, a.env, a.q, a.n_env, qi, io);
    quad_stage_b<DIM>(cx, io);
    qsync();
    const bool store = cx.w == 0 && cx.lane < TQ && qi < a.q;
    float* prow = a.path + (qi < a.q ? qi : 0) * rows * 2 * DIM;
    auto dist = [&]() {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < DIM; ++d) {
        float D = io.x[1][d] - io.x[0][d];
        s = fmaf(D, D, s);
      }
      return sqrtf(s);
    };
    int nsteps = 0;
    int it = 0;
    bool active;
    if (resume) {   // continue from the state the MFMA tile left in the path
      it = tail_it[qi];
      nsteps = a.steps[qi];
      const float* pr = prow + (int64_t)it * 2 * DIM;
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int d = 0; d < DIM; ++d) io.x[c][d] = pr[c * DIM + d];
      active = true;
    } else {
      active = ok && dist() > a.tol;
      if (store) {
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int d = 0; d < DIM; ++d) prow[c * DIM + d] = io.x[c][d];
      }
    }
    // queries of the batch this tile retires (done from the start: converged, invalid env)
    auto retire = [&](bool now_done) {
      const unsigned long long b = __ballot(now_done) & 0xfull;
      if (cx.w == 0 && cx.lane == 0 && b)
        __hip_atomic_fetch_add(tail, (int32_t)__builtin_popcountll(b), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    };
    if (can_yield) retire(qi < a.q && !active);
    bool yielded = false;
    for (; it < cap; ++it) {
      if (!__any(active) || yielded) break;
      const float tau =
          quad_forward<DIM, true, Q_NF_ALL, QR, SOLO>(ring, W, cx, io, aux, a.compat);
      float ds[DIM], dg[DIM], vs[DIM], vg[DIM];
      quad_backward<DIM, Q_NF_ALL, QR, SOLO>(ring, W, cx, io, tau, aux, ds, dg);
      path_velocity<DIM>(io.x, tau, ds, dg, vs, vg);
      bool converged = false;
      if (active) {
#pragma unroll
        for (int d = 0; d < DIM; ++d) {
          io.x[0][d] = io.x[0][d] + a.step * vs[d];
          io.x[1][d] = io.x[1][d] + a.step * vg[d];
        }
        ++nsteps;
        if (!(dist() > a.tol)) {
          active = false;
          converged = true;
        }
      }
      if (store) {
        float* pr = prow + (int64_t)(it + 1) * 2 * DIM;
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int d = 0; d < DIM; ++d) pr[c * DIM + d] = io.x[c][d];
      }
      if (can_yield) retire(qi < a.q && converged);
      if (can_yield && (it & (Q_YIELD_EVERY - 1)) == Q_YIELD_EVERY - 1) {
        // every Q_YIELD_EVERY steps one lane reads the batch's done count (device scope,
        // bypasses L1; its wait drains the weight ring once); the decision goes through LDS so
        // all four waves agree; a yield takes effect at the top of the next iteration (the
        // state is then path row it + 1)
        if (cx.w == 0 && cx.lane == 0) {
          const int32_t done = __hip_atomic_load(tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          cx.lds[Q_YIELD_FLAG] = a.q - done <= a.yield_at ? 1.f : 0.f;
        }
        qsync();
        yielded = cx.lds[Q_YIELD_FLAG] != 0.f;
      }
    }
    if (yielded && store && active) {
      // hand the query off: its state is path row `it`, its step count goes to steps[]
      const int32_t slot = __hip_atomic_fetch_add(tail + 1, 1, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      tail_q[slot] = (int32_t)qi;
      tail_it[qi] = it;
      a.steps[qi] = nsteps;
    } else if (store) {
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
// ---------------------------------------------------------------- quad weight packing
// Layer L of wave w: dst[w·Q_STREAM + r], r = ((g·IN/16 + q)·64 + l)·4 + e holds
// A[w·OUT/Q_WAVES + 16 g + 4 (l >> 4) + ((l + kb) & 3)][16 q + 4 e + kb], kb = (l >> 2) & 3,
// A = M (dir 0) or M^T (dir 1) of the rows x cols matrix M (rows rotated by kb: qring_sum).
__global__ void pack_quad_kernel(const float* __restrict__ src, int rows, int cols, int dir,
                                 float* __restrict__ dst) {
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= (int64_t)rows * cols) return;
  const int OUT = dir ? cols : rows, IN = dir ? rows : cols;
  const int per = OUT / Q_WAVES * IN;
  const int w = (int)(o / per), r = (int)(o % per);
  const int e = r & 3, l = (r >> 2) & 63, fq = r >> 8;
  const int g = fq / (IN / 16), q = fq % (IN / 16);
  const int kb = (l >> 2) & 3;
  const int row = w * (OUT / Q_WAVES) + 16 * g + 4 * (l >> 4) + ((l + kb) & 3);
  const int k = 16 * q + 4 * e + kb;
  dst[(int64_t)w * Q_STREAM + r] = dir ? src[(int64_t)k * cols + row] : src[(int64_t)row * cols + k];
}
// Bias vectors: aux[w][L][l][g] = bias_L[w·OUT/4 + 16 g + 4 (l >> 4) + ((l >> 2) & 3)] for the
// 13 forward layers, and the head row generator.4.weight (L = 13) for the 128 rows of
// generator[-2]; unused groups are 0.
__global__ void pack_quad_aux_kernel(const float* __restrict__ plain, float* __restrict__ quad) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= Q_WAVES * Q_NAUX * 256) return;
  const int g = o & 3, l = (o >> 2) & 63, L = (o >> 8) % Q_NAUX, w = o / (Q_NAUX * 256);
  constexpr int outs[Q_NAUX] = {128, 128, 128, 128, 128, 128, 256, 256, 256, 256, 256, 256, 128,
                                128};
  constexpr int offs[Q_NAUX] = {Q_LAYERS[0].bias,  Q_LAYERS[1].bias,  Q_LAYERS[2].bias,
                                Q_LAYERS[3].bias,  Q_LAYERS[4].bias,  Q_LAYERS[5].bias,
                                Q_LAYERS[6].bias,  Q_LAYERS[7].bias,  Q_LAYERS[8].bias,
                                Q_LAYERS[9].bias,  Q_LAYERS[10].bias, Q_LAYERS[11].bias,
                                Q_LAYERS[12].bias, B_G4W};
  const int out = outs[L], off = offs[L];
  float v = 0.f;
  if (g < qg(out))
    v = plain[off + w * (out / Q_WAVES) + 16 * g + 4 * (l >> 4) + ((l >> 2) & 3)];
  quad[Q_OFF_AUX + o] = v;
}
#endif  // PNTF_UTIL

}  // namespace pntf
