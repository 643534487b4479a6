// fp32 GEMMs of the training step (pntf/train.py) on v_mfma_f32_32x32x2_f32, replacing the
// library GEMMs the Taylor tape used: per Linear of NN.out_laplace (model_res_sigmoid_multi.py
// :710-848, differentiated by loss.backward() at :1048)
//   forward          Y (rows x N)  = X (rows x K) · Wᵀ          (A row-major, B = Wᵀ)
//   input gradient   gX (rows x K) (+)= gY (rows x N) · W       (A row-major, B row-major)
//   weight gradient  gW (N x K)    = gYᵀ · X  over all rows     (A = gYᵀ, B row-major, split-K)
// C = beta·C + A·B with A(m, k) = TA ? A[k·lda + m] : A[m·lda + k] and
// B(k, n) = TB ? B[n·ldb + k] : B[k·ldb + n].
// Three kernels serve them: the LDS panel kernel (forward and input gradient, K, N ∈ {128,
// 256}), the register-streamed wgrad kernel (weight gradients, M, N ∈ {128, 256}) and, for
// every other shape / operand, the LDS-tiled kernel described next.
//
// LDS-tiled kernel: workgroup tile 128 x 128, K chunks of 8 staged through LDS (double-buffered, one barrier per
// chunk, the next chunk's global loads in flight during the current chunk's MFMAs); 4 waves,
// each a 64 x 64 block = 2 x 2 MFMA tiles of 32 x 32 (64 accumulators).  Per chunk and wave:
// 16 MFMAs of 64 cycles; the chunk's LDS operands are read before its MFMAs (one latency per
// chunk), and interior chunks load without predication (a wave-uniform test).  Small LDS
// (20 KiB) lets 3 workgroups share a CU, so one's barrier hides behind the others' MFMAs
// (tools/gemm_probe.py, tests/diag/gemm_variants.py: chunks of 8 beat 16 and 32).  N must be a multiple of 128 (the layer widths 128 / 256); M and
// K are arbitrary (zero-filled / predicated edges).  Split-K (blockIdx.z) writes partial tiles
// to `work` and a second kernel sums them in split order: deterministic, no atomics.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#include <atomic>

#include "pntf.h"
#include "pntf_stamp.h"

namespace pntf_gemm {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#ifndef PNTF_GEMM_BK
#define PNTF_GEMM_BK 8
#endif
#ifndef PNTF_GEMM_SPLITS
#define PNTF_GEMM_SPLITS 512
#endif
#ifndef PNTF_GEMM_BM
#define PNTF_GEMM_BM 128
#endif
constexpr int BM = PNTF_GEMM_BM, BN = 128, BK = PNTF_GEMM_BK;   // BN: the narrowest tile
constexpr int RB = BM / 64;          // 32-row MFMA blocks per wave (waves are 2 x 2)
constexpr int GLA = BM * BK / 1024;  // float4 global loads per lane per chunk: A
constexpr int LSA = BM + 32;         // LDS row strides (≡ 32 mod 64: conflict-free halves)

struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  float* work;
  int64_t M, N, K, lda, ldb, ldc, kper;
  float beta;
};

template <bool TA, bool TB, int BNT>
__global__ __launch_bounds__(256, 1) void gemm_kernel(GemmArgs g) {
  constexpr int GLB = BNT * BK / 1024;   // float4 global loads per lane per chunk: B
  constexpr int LSB = BNT + 32;          // ≡ 32 mod 64, like LSA
  constexpr int CB = BNT / 64;           // 32-column MFMA blocks per wave
  __shared__ float As[2][BK * LSA];
  __shared__ float Bs[2][BK * LSB];
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wm = w & 1, wn = w >> 1;
  const int64_t m0 = (int64_t)blockIdx.y * BM;
  const int64_t n0 = (int64_t)blockIdx.x * BNT;
  const int64_t kb = (int64_t)blockIdx.z * g.kper;
  const int64_t ke = kb + g.kper < g.K ? kb + g.kper : g.K;
  const int nchunks = (int)((ke - kb + BK - 1) / BK);

  // global -> registers: 2 float4 per lane for A and for B
  f32x4 ra[GLA], rb[GLB];
  // interior chunks (the whole tile in range: a wave-uniform test) load without predication
  auto gload_fast = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < GLA; ++i) {
      const int idx = t + 256 * i;
      if (TA) {
        const int k = idx / (BM / 4), m = 4 * (idx % (BM / 4));
        ra[i] = *reinterpret_cast<const f32x4*>(g.A + (k0 + k) * g.lda + m0 + m);
      } else {
        const int m = idx % BM, k = 4 * (idx / BM);
        ra[i] = *reinterpret_cast<const f32x4*>(g.A + (m0 + m) * g.lda + k0 + k);
      }
    }
#pragma unroll
    for (int i = 0; i < GLB; ++i) {
      const int idx = t + 256 * i;
      if (TB) {
        const int n = idx % BNT, k = 4 * (idx / BNT);
        rb[i] = *reinterpret_cast<const f32x4*>(g.B + (n0 + n) * g.ldb + k0 + k);
      } else {
        const int k = idx / (BNT / 4), n = 4 * (idx % (BNT / 4));
        rb[i] = *reinterpret_cast<const f32x4*>(g.B + (k0 + k) * g.ldb + n0 + n);
      }
    }
  };
  auto gload_edge = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < GLA; ++i) {
      const int idx = t + 256 * i;
      if (TA) {   // rows k (BK) x m (BM) contiguous: float4 along m
        const int k = idx / (BM / 4), m = 4 * (idx % (BM / 4));
        const int64_t gk = k0 + k, gm = m0 + m;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (gk < ke) {
          if (gm + 3 < g.M) {
            v = *reinterpret_cast<const f32x4*>(g.A + gk * g.lda + gm);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = gm + e < g.M ? g.A[gk * g.lda + gm + e] : 0.f;
          }
        }
        ra[i] = v;
      } else {    // rows m (BM) x k (BK): float4 along k, consecutive lanes on consecutive m
                  // (so the transposed LDS writes below are bank-conflict-free)
        const int m = idx % BM, k = 4 * (idx / BM);
        const int64_t gk = k0 + k, gm = m0 + m;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (gm < g.M) {
          if (gk + 3 < ke) {
            v = *reinterpret_cast<const f32x4*>(g.A + gm * g.lda + gk);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = gk + e < ke ? g.A[gm * g.lda + gk + e] : 0.f;
          }
        }
        ra[i] = v;
      }
    }
#pragma unroll
    for (int i = 0; i < GLB; ++i) {
      const int idx = t + 256 * i;
      if (TB) {   // B(k, n) = B[n·ldb + k]: float4 along k, consecutive lanes on consecutive n
        const int n = idx % BNT, k = 4 * (idx / BNT);
        const int64_t gk = k0 + k, gn = n0 + n;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (gk + 3 < ke) {
          v = *reinterpret_cast<const f32x4*>(g.B + gn * g.ldb + gk);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = gk + e < ke ? g.B[gn * g.ldb + gk + e] : 0.f;
        }
        rb[i] = v;
      } else {    // B(k, n) = B[k·ldb + n]: float4 along n
        const int k = idx / (BNT / 4), n = 4 * (idx % (BNT / 4));
        const int64_t gk = k0 + k;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (gk < ke) v = *reinterpret_cast<const f32x4*>(g.B + gk * g.ldb + n0 + n);
        rb[i] = v;
      }
    }
  };
  const bool m_in = m0 + BM <= g.M;
  auto gload = [&](int64_t k0) {
    if (m_in && k0 + BK <= ke) gload_fast(k0);
    else gload_edge(k0);
  };
  // registers -> LDS image [k][m] / [k][n]
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < GLA; ++i) {
      const int idx = t + 256 * i;
      if (TA) {
        const int k = idx / (BM / 4), m = 4 * (idx % (BM / 4));
        *reinterpret_cast<f32x4*>(&As[buf][k * LSA + m]) = ra[i];
      } else {
        const int m = idx % BM, k = 4 * (idx / BM);
#pragma unroll
        for (int e = 0; e < 4; ++e) As[buf][(k + e) * LSA + m] = ra[i][e];
      }
    }
#pragma unroll
    for (int i = 0; i < GLB; ++i) {
      const int idx = t + 256 * i;
      if (TB) {
        const int n = idx % BNT, k = 4 * (idx / BNT);
#pragma unroll
        for (int e = 0; e < 4; ++e) Bs[buf][(k + e) * LSB + n] = rb[i][e];
      } else {
        const int k = idx / (BNT / 4), n = 4 * (idx % (BNT / 4));
        *reinterpret_cast<f32x4*>(&Bs[buf][k * LSB + n]) = rb[i];
      }
    }
  };

  f32x16 acc[RB][CB];
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int j = 0; j < CB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nchunks > 0) {
    gload(kb);
    lstore(0);
  }
  __syncthreads();
  const int am = wm * (BM / 2) + (lane & 31), bn = wn * (BNT / 2) + (lane & 31), kh = lane >> 5;
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
    const bool more = c + 1 < nchunks;
    if (more) gload(kb + (int64_t)(c + 1) * BK);
    const float* as = As[buf];
    const float* bs = Bs[buf];
    // all LDS operands of the chunk first (one latency exposed per chunk, not per k step)
    float a[BK / 2][RB], b[BK / 2][CB];
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      const int kr = 2 * kk + kh;
#pragma unroll
      for (int i = 0; i < RB; ++i) a[kk][i] = as[kr * LSA + am + 32 * i];
#pragma unroll
      for (int j = 0; j < CB; ++j) b[kk][j] = bs[kr * LSB + bn + 32 * j];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk)
#pragma unroll
      for (int i = 0; i < RB; ++i)
#pragma unroll
        for (int j = 0; j < CB; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[kk][i], b[kk][j], acc[i][j], 0, 0, 0);
    if (more) lstore(buf ^ 1);
    __syncthreads();
  }

  // D row of register r in lane half h: (r & 3) + 8·(r >> 2) + 4·h, column lane & 31
  const bool split = gridDim.z > 1;
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int j = 0; j < CB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t row = m0 + wm * (BM / 2) + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * kh;
        const int64_t col = n0 + wn * (BNT / 2) + 32 * j + (lane & 31);
        if (row < g.M) {
          if (split) {
            g.work[((int64_t)blockIdx.z * g.M + row) * g.N + col] = acc[i][j][r];
          } else {
            float* cp = g.C + row * g.ldc + col;
            *cp = g.beta != 0.f ? fmaf(g.beta, *cp, acc[i][j][r]) : acc[i][j][r];
          }
        }
      }
}

// Split-K reduction, two passes, fixed order (deterministic):
//   pass 1: group zg (blockIdx.y) sums splits [RG·zg, RG·zg + RG) into work[RG·zg] (in place;
//           that slot is read first by the same thread), 4 independent loads in flight;
//   pass 2: C = beta·C + Σ_zg work[RG·zg].
constexpr int RG = 32;
__global__ void gemm_reduce1_kernel(float* __restrict__ work, int splits, int64_t MN) {
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= MN) return;
  const int z0 = blockIdx.y * RG, z1 = z0 + RG < splits ? z0 + RG : splits;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  int z = z0;
  for (; z + 4 <= z1; z += 4)
#pragma unroll
    for (int u = 0; u < 4; ++u) s[u] += work[(int64_t)(z + u) * MN + o];
  for (; z < z1; ++z) s[0] += work[(int64_t)z * MN + o];
  work[(int64_t)z0 * MN + o] = (s[0] + s[1]) + (s[2] + s[3]);
}
__global__ void gemm_reduce2_kernel(const float* __restrict__ work, int splits, int64_t M,
                                    int64_t N, float* __restrict__ C, int64_t ldc, float beta) {
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= M * N) return;
  const int64_t row = o / N, col = o % N;
  float s = 0.f;
  for (int z = 0; z < splits; z += RG) s += work[(int64_t)z * M * N + o];
  float* cp = C + row * ldc + col;
  *cp = beta != 0.f ? fmaf(beta, *cp, s) : s;
}

// ---------------------------------------------------------------------------------------
// Panel GEMM: the forward X·Wᵀ and the input gradient gY·W of every Linear (K, N ∈ {128, 256}).
//   C (M x NC) = (C +) A (M x KC) · B,   B (KC x NC) = the layer weight, Wᵀ or W.
// The field kernels' transposed formulation (pntf_wide.h) applied to the tape: one wave owns a
// 32-row panel of A held in registers (KC/8 float4 per lane, read from HBM once), and the
// weight is the streamed MFMA A operand, pre-packed in fragment order (1 KiB per wave load,
// L2-resident), so there is no LDS, no barrier and no B-tile re-read:
//   D (32 out cols x 32 rows) += Bᵀfrag (32 x 2) · panelᵀ (2 x 32) per v_mfma_f32_32x32x2_f32.
// MFMA step s = 4q + e, lane half h, uses K index k = 8q + 4h + e: lane (row j, half h) holds
// A[row j][8q + 4h .. +3] as one float4 (x[q]) and the packed fragment
//   P[((nt·QK + q)·64 + lane)·4 + e] = B(8q + 4h + e, 32·nt + (lane & 31))
// supplies out column 32·nt + (lane & 31).  D register r of lane (j, h) is C[row j][32·nt +
// 8·(r >> 2) + 4h + (r & 3)]: four float4 stores per 32-column tile.
// Per tile: NC/128 groups of 4 out tiles (64 accumulators) x KC/8 iterations of 16 MFMAs; a
// 4-slot register ring prefetches fragments 3 iterations ahead and wraps into the next tile
// (the stream is the same for every tile).  The next panel's float4 q is loaded right after
// its last use in the last group, so the panel double-buffers in place.  Persistent waves,
// one per SIMD (≤ 512 VGPRs), grid-stride over 32-row tiles.  ACC adds C (the residual
// branch's gradient, beta = 1), loaded 4 iterations before the group's store.
#ifndef PNTF_PANEL_PF
#define PNTF_PANEL_PF 3
#endif
// diagnostic builds only (tests/diag/panel_variants.py): bit 1 = no next-panel loads (every
// tile reuses the first panel), bit 2 = no C stores, bit 4 = no fragment loads (ring reuse)
// waves per SIMD (workgroups per CU): 1 keeps ≤ 512 registers per wave
#ifndef PNTF_PANEL_WPS
#define PNTF_PANEL_WPS 1
#endif
#ifndef PNTF_PANEL_DIAG
#define PNTF_PANEL_DIAG 0
#endif
template <int B, int E, class F>
__device__ __forceinline__ void pg_static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    pg_static_for<B + 1, E>(f);
  }
}

struct PanelArgs {
  const float* A;
  const f32x4* P;
  float* C;
  int64_t M, lda, ldc;
  const float* Cin;   // ACC: the added matrix (C itself, or another one of C's layout)
  const float* bias;  // LDS kernel, ACC: bias[col] added to rows < brows first (else null)
  int64_t brows;
};

__global__ void panel_pack_kernel(const float* __restrict__ W, int64_t ldb, int tb, int KC,
                                  int NC, f32x4* __restrict__ P) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int QK = KC / 8;
  if (i >= (int64_t)(NC / 32) * QK * 64) return;
  const int lane = (int)(i & 63), q = (int)((i >> 6) % QK), nt = (int)((i >> 6) / QK);
  const int n = 32 * nt + (lane & 31), k0 = 8 * q + 4 * (lane >> 5);
  f32x4 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = tb ? W[(int64_t)n * ldb + k0 + e] : W[(int64_t)(k0 + e) * ldb + n];
  P[i] = v;
}

typedef __amdgpu_buffer_rsrc_t Rsrc;
// Buffer resources keep the per-load address math on the SALU (scalar fragment / column
// offsets) and clip the M edge: loads past num_records return 0, stores there are dropped.
__device__ __forceinline__ Rsrc pg_rsrc(const float* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f32x4 pg_load(Rsrc r, int voff, int soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}
__device__ __forceinline__ void pg_store(Rsrc r, f32x4 v, int voff, int soff) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                         r, voff, soff, 0);
  asm volatile("s_nop 0" ::"v"(v));   // store-data hazard guard (pntf_field.h bstore)
}

template <int KC, int NC, bool ACC>
__global__ __launch_bounds__(256, PNTF_PANEL_WPS) void panel_gemm_kernel(PanelArgs g) {
  constexpr int QK = KC / 8, NG = NC / 128, NQ = NG * QK, PF = PNTF_PANEL_PF, NS = PF + 1;
  static_assert(NQ % NS == 0, "ring slots must divide the per-tile fragment stream");
  static_assert(QK >= 8, "C prefetch distance");
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int64_t ntiles = (g.M + 31) / 32;
  const int64_t stride = (int64_t)gridDim.x * 4;
  int64_t tile = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (tile >= ntiles) return;   // wave-uniform
  // the 32-row window of tile t in A / C (rows past M are outside the resource)
  auto win = [&](const float* base, int64_t ld, int64_t t) {
    const int64_t rows = g.M - 32 * t;
    return pg_rsrc(base + 32 * t * ld, (rows < 32 ? rows : 32) * ld * 4);
  };
  const int va = (int)((j * g.lda + 4 * h) * 4), vc = (int)((j * g.ldc + 4 * h) * 4);
  const Rsrc rp = pg_rsrc(reinterpret_cast<const float*>(g.P), (int64_t)KC * NC * 4);
  const int vp = lane * 16;
  f32x4 x[QK];
  {
    const Rsrc ra = win(g.A, g.lda, tile);
#pragma unroll
    for (int q = 0; q < QK; ++q) x[q] = pg_load(ra, va, 32 * q);
  }
  f32x4 ring[NS][4];
  pg_static_for<0, PF>([&](auto I) {
    constexpr int it = decltype(I)::value;
#pragma unroll
    for (int t = 0; t < 4; ++t) ring[it][t] = pg_load(rp, vp, ((4 * (it / QK) + t) * QK + it % QK) * 1024);
  });
  for (;;) {
    const int64_t next = tile + stride;
    const bool more = next < ntiles;
    const Rsrc rn = win(g.A, g.lda, more ? next : tile);
    const Rsrc rc = win(g.C, g.ldc, tile), rci = win(g.Cin, g.ldc, tile);
    f32x16 acc[4];
    f32x4 cb[4][4];
    pg_static_for<0, NQ>([&](auto I) {
      constexpr int it = decltype(I)::value, G = it / QK, q = it % QK;
      if constexpr (q == 0) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
      }
      if constexpr (ACC && q == QK - 4) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int R = 0; R < 4; ++R) cb[t][R] = pg_load(rci, vc, (32 * (4 * G + t) + 8 * R) * 4);
      }
      // prefetch PF iterations ahead; past the tile's end the stream wraps to the next tile
      constexpr int pit = (it + PF) % NQ;
      if constexpr (!(PNTF_PANEL_DIAG & 4)) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          ring[(it + PF) % NS][t] = pg_load(rp, vp, ((4 * (pit / QK) + t) * QK + pit % QK) * 1024);
      }
      // four independent accumulator chains per k step; the fence keeps the scheduler from
      // regrouping them into back-to-back dependent MFMAs (it orders by load arrival)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(ring[it % NS][t][e], x[q][e], acc[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (G == NG - 1 && !(PNTF_PANEL_DIAG & 1)) {
        if (more) x[q] = pg_load(rn, va, 32 * q);   // x[q] is dead for this tile: next panel
      }
      if constexpr (q == QK - 1 && !(PNTF_PANEL_DIAG & 2)) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int R = 0; R < 4; ++R) {
            f32x4 v = {acc[t][4 * R], acc[t][4 * R + 1], acc[t][4 * R + 2], acc[t][4 * R + 3]};
            if (ACC) v += cb[t][R];
            pg_store(rc, v, vc, (32 * (4 * G + t) + 8 * R) * 4);
          }
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    if (!more) break;
    tile = next;
  }
}

// ---------------------------------------------------------------------------------------
// LDS panel GEMM: the same per-wave formulation with the weight held in LDS.  Workgroup b
// serves one 128-column group of C (4 out tiles); it copies that group's packed fragments
// (KC/2 KiB: 128 KiB at KC = 256) from P into LDS once, then its 4 waves stride over the
// 32-row tiles.  Per iteration a wave reads its 4 fragments with ds_read_b128 (one iteration
// ahead), so the only vector-memory loads in the loop are the A panels: a panel's float4 q is
// reloaded for the next tile right after its MFMAs, a whole tile (QK iterations, ~15 µs at
// KC = 256) before it is needed, and the in-order vmcnt never couples a weight read to an HBM
// panel read (the register-stream kernel above waits on both).  With two groups (NC = 256)
// the workgroups of a tile's two groups sit on the same XCD (block ids 8 apart), so the second
// panel read of a tile hits that XCD's L2.
template <int KC, int NC, bool ACC>
__global__ __launch_bounds__(256, 1) void panel_lds_kernel(PanelArgs g) {
  PNTF_CLOCK_SCOPE;
  constexpr int QK = KC / 8, NG = NC / 128, FR = 4 * QK;
  static_assert(QK >= 8, "C prefetch distance");
  __shared__ f32x4 lw[FR * 64];
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // block b -> (group, workgroup index): XCD = b % 8 (dispatch order); within an XCD's
  // blocks, consecutive pairs are the two groups of one set of tiles
  int grp = 0, wg = blockIdx.x, nwg = gridDim.x;
  if constexpr (NG == 2) {
    const int x = blockIdx.x & 7, s = blockIdx.x >> 3;
    grp = s & 1;
    wg = (s >> 1) * 8 + x;
    nwg = gridDim.x / 2;
  }
  __shared__ f32x4 lb[ACC ? 32 : 1];   // the group's 128 bias columns (ACC with a bias)
  {   // stage the group's fragments (contiguous in P: out tiles 4·grp .. 4·grp + 3)
    const f32x4* src = g.P + (int64_t)grp * FR * 64;
#pragma unroll 8
    for (int i = threadIdx.x; i < FR * 64; i += 256) lw[i] = src[i];
    if (ACC && g.bias && threadIdx.x < 32)
      lb[threadIdx.x] = *reinterpret_cast<const f32x4*>(g.bias + 128 * grp + 4 * threadIdx.x);
  }
  __syncthreads();
  const int64_t ntiles = (g.M + 31) / 32;
  const int64_t stride = (int64_t)nwg * 4;
  int64_t tile = (int64_t)wg * 4 + w;
  if (tile >= ntiles) return;   // wave-uniform; no barrier follows
  auto win = [&](const float* base, int64_t ld, int64_t t) {
    const int64_t rows = g.M - 32 * t;
    return pg_rsrc(base + 32 * t * ld, (rows < 32 ? rows : 32) * ld * 4);
  };
  const int va = (int)((j * g.lda + 4 * h) * 4), vc = (int)((j * g.ldc + 4 * h) * 4);
  const int c0 = 128 * grp;   // first out column of the group
  f32x4 x[QK];
  {
    const Rsrc ra = win(g.A, g.lda, tile);
#pragma unroll
    for (int q = 0; q < QK; ++q) x[q] = pg_load(ra, va, 32 * q);
  }
  const f32x4* lf = lw + lane;
  f32x4 fr[2][4];
#pragma unroll
  for (int t = 0; t < 4; ++t) fr[0][t] = lf[(t * QK) * 64];
  for (;;) {
    const int64_t next = tile + stride;
    const bool more = next < ntiles;
    const Rsrc rn = win(g.A, g.lda, more ? next : tile);
    const Rsrc rc = win(g.C, g.ldc, tile), rci = win(g.Cin, g.ldc, tile);
    f32x16 acc[4];
    f32x4 cb[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    pg_static_for<0, QK>([&](auto I) {
      constexpr int q = decltype(I)::value, cur = q & 1;
      if constexpr (ACC && q == QK - 4) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int R = 0; R < 4; ++R) cb[t][R] = pg_load(rci, vc, (c0 + 32 * t + 8 * R) * 4);
      }
      // next iteration's fragments (past the tile's end: the next tile's first ones)
      constexpr int qn = (q + 1) % QK;
#pragma unroll
      for (int t = 0; t < 4; ++t) fr[cur ^ 1][t] = lf[(t * QK + qn) * 64];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(fr[cur][t][e], x[q][e], acc[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (more) x[q] = pg_load(rn, va, 32 * q);   // x[q] is dead for this tile: next panel
      if constexpr (q == QK - 1) {
        // (acc + bias) + C: the order of nn.Linear's addmm and the residual add after it
        const bool brow = ACC && g.bias && 32 * tile + j < g.brows;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int R = 0; R < 4; ++R) {
            f32x4 v = {acc[t][4 * R], acc[t][4 * R + 1], acc[t][4 * R + 2], acc[t][4 * R + 3]};
            if (ACC) {
              if (brow) v += lb[8 * t + 2 * R + h];
              v += cb[t][R];
            }
            pg_store(rc, v, vc, (c0 + 32 * t + 8 * R) * 4);
          }
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    if (!more) break;
    tile = next;
  }
}

// ---------------------------------------------------------------------------------------
// Split-bf16 panel GEMM (round 5, `panel_x6_kernel`): the LDS panel GEMM above on the bf16
// matrix cores.  gfx950's fp32-input MFMA runs at 1/16 of the bf16 rate, so an fp32 product is
// cheaper as six bf16 products: every operand splits into three bf16 terms, RNE each,
//   x = x0 + x1 + x2,  x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1),
// |x1| <= 2^-8 |x|, |x2| <= 2^-16 |x|, |x - x0 - x1 - x2| <= 2^-25 |x| (the subtractions are
// exact).  Of the nine partial products a·b keeps the six of order >= 2^-16:
//   a0b0 + (a0b1 + a1b0) + (a0b2 + a1b1 + a2b0);
// the three dropped ones are <= 2^-23 |ab| together, about one fp32 rounding of the product.
// Each bf16 product is exact in the MFMA's fp32 accumulator; the terms go in smallest first.
// 6 x v_mfma_f32_32x32x16_bf16 (32 cycles each) do the work of 8 x v_mfma_f32_32x32x2_f32
// (64 cycles each): 2.67x the fp32 MFMA rate (the fp32 VALU rate is no higher).  Accuracy vs
// fp64 beside the fp32-MFMA kernel: tests/test_train.py (test_x6_gemm_vs_fp64).
// Layout: MFMA A = the weight (32 out columns x 16 k), pre-split by x6_pack_kernel into three
// 1 KiB bf16 fragments per (out tile, k block); MFMA B = the A panel's 32 rows: lane (row j,
// half h) holds A[row j][16 kb + 8h .. +7] as two float4 of the fp32 panel (KC/8 float4 per
// lane in registers, read from HBM once) and splits them per k block (VALU beside the MFMAs).
// D register r of lane (j, h) is C[row j][c0 + 32t + 8(r >> 2) + 4h + (r & 3)] as in the fp32
// kernels.  The pre-split weight is 1.5x the fp32 bytes, so a workgroup's LDS holds a 64-column
// group at K = 256 (96 KiB; 128 columns at K = 128) and a 256-column layer has four groups,
// whose workgroups take block ids 8 apart (one XCD: the panel's later reads hit its L2).
// C leaves through a per-wave LDS block so that its stores are row-contiguous (1; 0: straight
// from the MFMA layout, 32 half-filled lines per store)
#ifndef PNTF_X6_TSTORE
#define PNTF_X6_TSTORE 1
#endif
// Diagnostic variant (1): the A panel arrives row-contiguously (4 lanes per 64-byte row segment,
// 16 rows per load) and reaches the MFMA layout through a per-wave LDS block two k blocks ahead
// of its split.  Same-box A/B against the direct loads (0, shipped; one lane per row, 32 cache
// lines per load): no difference (generator forward 175.1 vs 173.8 TFLOP/s,
// profiles/r05_x6_gemm.txt), so the half-filled-line loads are not what binds.
#ifndef PNTF_X6_LSTAGE
#define PNTF_X6_LSTAGE 0
#endif
// 1: reload a panel block's registers in the block that splits them (one k block more lead
// for the next tile's loads); 0: one block later
#ifndef PNTF_X6_EARLY
#define PNTF_X6_EARLY 0
#endif
// diagnostics only (tests/diag/gemm_variants.py ablations; wrong results): bit 1 no operand
// split, 2 no LDS fragment reads in the loop, 4 no next-panel loads, 8 no C stores, 16 every
// panel load from the first tile (L2-resident), 32 the panel's bytes read row-contiguously
#ifndef PNTF_X6_ABL
#define PNTF_X6_ABL 0
#endif
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// PNTF_X6_DOT = 1: each split stage's residual v - bf16(v) is one v_dot2c_f32_bf16 per
// element (v + p.lo·(-1) + p.hi·0, exact), not an unpack and a subtract (pntf_common.h)
#ifndef PNTF_X6_DOT
#define PNTF_X6_DOT 0
#endif
__device__ __forceinline__ f32x2 x6_resid(f32x2 v, bf16x2 p) {
  // (-1, -0) and (-0, -1) as 32-bit literals: the plain (-1, 0) would be encoded as the inline
  // constant -1.0, which the hardware does not read as the bf16 pair (-1, 0)
  const bf16x2 nlo = __builtin_bit_cast(bf16x2, 0x8000bf80u), nhi = __builtin_bit_cast(bf16x2, 0xbf808000u);
  f32x2 r;
  r[0] = __builtin_amdgcn_fdot2_f32_bf16(p, nlo, v[0], false);
  r[1] = __builtin_amdgcn_fdot2_f32_bf16(p, nhi, v[1], false);
  return r;
}
// three-term RNE split of 8 fp32 (k order of the bf16 operand lane: 8 consecutive k)
__device__ __forceinline__ void x6_split(const f32x4& a, const f32x4& b, bf16x8 (&s)[3]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x2 v = i < 2 ? f32x2{a[2 * i], a[2 * i + 1]} : f32x2{b[2 * i - 4], b[2 * i - 3]};
    const bf16x2 p0 = __builtin_convertvector(v, bf16x2);
#if PNTF_X6_DOT
    const f32x2 r1 = x6_resid(v, p0);
    const bf16x2 p1 = __builtin_convertvector(r1, bf16x2);
    const f32x2 r2 = x6_resid(r1, p1);
#else
    const f32x2 r1 = v - __builtin_convertvector(p0, f32x2);
    const bf16x2 p1 = __builtin_convertvector(r1, bf16x2);
    const f32x2 r2 = r1 - __builtin_convertvector(p1, f32x2);
#endif
    const bf16x2 p2 = __builtin_convertvector(r2, bf16x2);
    s[0][2 * i] = p0[0]; s[0][2 * i + 1] = p0[1];
    s[1][2 * i] = p1[0]; s[1][2 * i + 1] = p1[1];
    s[2][2 * i] = p2[0]; s[2][2 * i + 1] = p2[1];
  }
}
// products of order 2^-8 and 2^-16 (variant V = 3 of panel_x6_kernel keeps them apart)
__device__ __forceinline__ f32x16 x6_mid(const bf16x8 (&w)[3], const bf16x8 (&x)[3], f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], x[0], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[1], acc, 0, 0, 0);
}
__device__ __forceinline__ f32x16 x6_low(const bf16x8 (&w)[3], const bf16x8 (&x)[3], f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[2], x[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], x[1], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[2], acc, 0, 0, 0);
}
// the five small products (variant V = 1 keeps them in their own accumulator)
__device__ __forceinline__ f32x16 x6_small(const bf16x8 (&w)[3], const bf16x8 (&x)[3], f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[2], x[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], x[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], x[0], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[1], acc, 0, 0, 0);
}
// a·b on one 32 x 32 x 16 block from the split operands (w: weight terms, x: panel terms),
// the small terms first
__device__ __forceinline__ f32x16 x6_mma(const bf16x8 (&w)[3], const bf16x8 (&x)[3], f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[2], x[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], x[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], x[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[1], acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], x[0], acc, 0, 0, 0);
}

// Pre-split weight fragments: P[((nt·KB + kb)·3 + p)·64 + lane] = term p of
// B(16 kb + 8h + j, 32 nt + r), j = 0..7 (lane = 32h + r); B = Wᵀ (tb) or W.
__global__ void x6_pack_kernel(const float* __restrict__ W, int64_t ldb, int tb, int KC, int NC,
                               bf16x8* __restrict__ P) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int KB = KC / 16;
  if (i >= (int64_t)(NC / 32) * KB * 64) return;
  const int lane = (int)(i & 63), kb = (int)((i >> 6) % KB), nt = (int)((i >> 6) / KB);
  const int n = 32 * nt + (lane & 31), k0 = 16 * kb + 8 * (lane >> 5);
  f32x4 a, b;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    a[e] = tb ? W[(int64_t)n * ldb + k0 + e] : W[(int64_t)(k0 + e) * ldb + n];
    b[e] = tb ? W[(int64_t)n * ldb + k0 + 4 + e] : W[(int64_t)(k0 + 4 + e) * ldb + n];
  }
  bf16x8 s[3];
  x6_split(a, b, s);
#pragma unroll
  for (int p = 0; p < 3; ++p) P[((int64_t)(nt * KB + kb) * 3 + p) * 64 + lane] = s[p];
}

// workgroups (so waves) per CU of the split kernel: 1 holds a 64-column group at K = 256 (128 at
// K = 128) in 96 KiB of LDS; 2 halves the group (48 KiB) so that two workgroups share a CU and
// each SIMD runs two waves (<= 256 registers each)
#ifndef PNTF_X6_WPS
#define PNTF_X6_WPS 1
#endif
constexpr int x6_cg1(int KC) { return (KC == 256 ? 64 : 128) / PNTF_X6_WPS; }
constexpr int x6_cg(int KC, int NC) { return x6_cg1(KC) < NC ? x6_cg1(KC) : NC; }

// V: how the six products accumulate.  0: one accumulator, small products first (x6_mma);
// 1: a0b0 in one accumulator and the five smaller products in a second, added at the store;
// 3 (the default): three accumulators, one per order (a0b0 | a0b1 + a1b0 | the three of order
// 2^-16), summed smallest first at the store.  On the reference's trained-weight training
// fixtures the single accumulator gave 3.6x the fp32-MFMA kernel's step-1 gradient error
// (every small product is rounded at the running sum's ulp); per-order accumulators bring it
// to the fp32 level or below, at the same speed (tests/diag/x6_train_acc.py, x6_probe.py;
// profiles/r05_x6_accuracy.txt).
template <int KC, int NC, bool ACC, int V = 3>
__global__ __launch_bounds__(256, PNTF_X6_WPS) void panel_x6_kernel(PanelArgs g) {
  PNTF_CLOCK_SCOPE;
  constexpr int KB = KC / 16, QK = KC / 8, CG = x6_cg(KC, NC), TG = CG / 32, NG = NC / CG;
  // the LDS-transposed store flushes a block after every odd tile
  static_assert(!PNTF_X6_TSTORE || TG % 2 == 0, "PNTF_X6_TSTORE needs an even tile count per group");
  constexpr int FR = TG * KB * 3;   // 1 KiB fragments per group
  static_assert(KB >= 4, "C prefetch distance");
  __shared__ bf16x8 lw[FR * 64];
  __shared__ f32x4 lb[ACC ? CG / 4 : 1];
#if PNTF_X6_TSTORE
  // per wave: a 32-row x 64-column block of C on its way out (row stride 17 float4: the MFMA
  // layout writes and the row-contiguous reads are both conflict-free)
  __shared__ f32x4 lt[4][32 * 17];
#endif
#if PNTF_X6_LSTAGE && PNTF_X6_EARLY
#error "PNTF_X6_EARLY applies to the direct panel loads"
#endif
#if PNTF_X6_LSTAGE
  // per wave: one k block of the panel (32 rows x 64 bytes, row stride 5 float4: conflict-free)
  __shared__ f32x4 lst[4][32 * 5];
#endif
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // block b -> (group, workgroup index): the NG workgroups of a set of tiles on one XCD
  int grp = 0, wg = blockIdx.x, nwg = gridDim.x;
  if constexpr (NG > 1) {
    const int x = blockIdx.x & 7, s = blockIdx.x >> 3;
    grp = s % NG;
    wg = (s / NG) * 8 + x;
    nwg = gridDim.x / NG;
  }
  {
    const bf16x8* src = reinterpret_cast<const bf16x8*>(g.P) + (int64_t)grp * FR * 64;
#pragma unroll 8
    for (int i = threadIdx.x; i < FR * 64; i += 256) lw[i] = src[i];
    if (ACC && g.bias && threadIdx.x < CG / 4)
      lb[threadIdx.x] = *reinterpret_cast<const f32x4*>(g.bias + CG * grp + 4 * threadIdx.x);
  }
  __syncthreads();
  const int64_t ntiles = (g.M + 31) / 32;
  const int64_t stride = (int64_t)nwg * 4;
  int64_t tile = (int64_t)wg * 4 + w;
  if (tile >= ntiles) return;   // wave-uniform; no barrier follows
  auto win = [&](const float* base, int64_t ld, int64_t t) {
    const int64_t rows = g.M - 32 * t;
    return pg_rsrc(base + 32 * t * ld, (rows < 32 ? rows : 32) * ld * 4);
  };
  const int va = (int)((j * g.lda + 8 * h) * 4), vc = (int)((j * g.ldc + 4 * h) * 4);
#if PNTF_X6_TSTORE
  const int vt = (int)(((lane >> 4) * g.ldc + 4 * (lane & 15)) * 4);
#endif
#if PNTF_X6_ABL & 32
  const int vco = (int)(((lane >> 3) * g.lda) * 4 + 16 * (lane & 7));
#endif
  const int c0 = CG * grp;
  f32x4 x[QK];
#if PNTF_X6_LSTAGE
  // raw panel registers: x[2b + q] = rows 16q + (lane >> 2), bytes 64b + 16 (lane & 3) ..
  // of the tile (k block b), staged through lst into the MFMA layout two blocks ahead
  const int vr = (int)(((lane >> 2) * g.lda) * 4 + 16 * (lane & 3));
  const int sq = __builtin_amdgcn_readfirstlane((int)(64 * g.lda));   // 16 rows, in bytes
  auto raw = [&](Rsrc r, int b, int q) { return pg_load(r, vr, 64 * b + q * sq); };
  auto stage = [&](int b, f32x4& y0, f32x4& y1) {
    lst[w][(lane >> 2) * 5 + (lane & 3)] = x[2 * b];
    lst[w][(16 + (lane >> 2)) * 5 + (lane & 3)] = x[2 * b + 1];
    asm volatile("" ::: "memory");     // (compiler order; LDS itself is in order per wave)
    y0 = lst[w][j * 5 + 2 * h];
    y1 = lst[w][j * 5 + 2 * h + 1];
  };
  auto tile_win = [&](int64_t t) { return win(g.A, g.lda, t < ntiles ? t : tile); };
  f32x4 y[2];
  bf16x8 s[3];
  {
    const Rsrc ra = win(g.A, g.lda, tile);
#pragma unroll
    for (int q = 0; q < QK; ++q) x[q] = raw(ra, q >> 1, q & 1);
    stage(0, y[0], y[1]);
    x6_split(y[0], y[1], s);
    stage(1, y[0], y[1]);
    // blocks 0 and 1 of the next tile: staged at this tile's blocks KB - 2, KB - 1
    const Rsrc rn = tile_win(tile + stride);
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = raw(rn, q >> 1, q & 1);
  }
#else
  {
    const Rsrc ra = win(g.A, g.lda, tile);
#pragma unroll
    for (int q = 0; q < QK; ++q) x[q] = pg_load(ra, va, 64 * (q >> 1) + 16 * (q & 1));
  }
  // the split terms of the current k block; the next block's are computed beside this
  // block's MFMAs (software pipeline, wrapping into the next tile's first block)
  bf16x8 s[3];
  x6_split(x[0], x[1], s);
#if PNTF_X6_EARLY
  {   // block 0 of the next tile (split at this tile's last block)
    const int64_t t1 = tile + stride;
    const Rsrc r1 = win(g.A, g.lda, t1 < ntiles ? t1 : tile);
    x[0] = pg_load(r1, va, 0);
    x[1] = pg_load(r1, va, 16);
  }
#endif
#endif
  const bf16x8* lf = lw + lane;
  bf16x8 fr[2][TG][3];
#pragma unroll
  for (int t = 0; t < TG; ++t)
#pragma unroll
    for (int p = 0; p < 3; ++p) fr[0][t][p] = lf[((t * KB) * 3 + p) * 64];
  for (;;) {
    const int64_t next = tile + stride;
    const bool more = next < ntiles;
#if PNTF_X6_ABL & 16
    const Rsrc rn = win(g.A, g.lda, 0);   // every panel load hits the first tile (L2)
#else
    const Rsrc rn = win(g.A, g.lda, more ? next : tile);
#endif
    const Rsrc rc = win(g.C, g.ldc, tile), rci = win(g.Cin, g.ldc, tile);
    f32x16 acc[TG], accl[V == 1 || V == 3 ? TG : 1], accm[V == 3 ? TG : 1];
    f32x4 cb[TG][4];
#pragma unroll
    for (int t = 0; t < TG; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    if constexpr (V == 1 || V == 3) {
#pragma unroll
      for (int t = 0; t < TG; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) accl[t][r] = 0.f;
    }
    if constexpr (V == 3) {
#pragma unroll
      for (int t = 0; t < TG; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) accm[t][r] = 0.f;
    }
    pg_static_for<0, KB>([&](auto I) {
      constexpr int kb = decltype(I)::value, cur = kb & 1;
      if constexpr (ACC && kb == KB - 4) {
#pragma unroll
        for (int t = 0; t < TG; ++t)
#pragma unroll
          for (int R = 0; R < 4; ++R) cb[t][R] = pg_load(rci, vc, (c0 + 32 * t + 8 * R) * 4);
      }
      // next k block's fragments (past the tile's end: the next tile's first ones)
      constexpr int kn = (kb + 1) % KB;
#if !(PNTF_X6_ABL & 2)
#pragma unroll
      for (int t = 0; t < TG; ++t)
#pragma unroll
        for (int p = 0; p < 3; ++p) fr[cur ^ 1][t][p] = lf[((t * KB + kn) * 3 + p) * 64];
#else
#pragma unroll
      for (int t = 0; t < TG; ++t)
#pragma unroll
        for (int p = 0; p < 3; ++p) fr[cur ^ 1][t][p] = fr[cur][t][p];
#endif
      // next block's terms (past the tile's end: the next panel's first block, loaded at
      // this tile's block 0)
      bf16x8 sn[3];
#if PNTF_X6_LSTAGE
      // stage block kb + 2 (the next tile's 0 / 1 past the end), reload its raw registers
      // with the tile one further, and split block kb + 1 (staged one block ago)
      f32x4 yn[2];
      {
        constexpr int b2 = (kb + 2) % KB;
        stage(b2, yn[0], yn[1]);
        const Rsrc rr = kb + 2 < KB ? rn : tile_win(tile + 2 * stride);
        x[2 * b2] = raw(rr, b2, 0);
        x[2 * b2 + 1] = raw(rr, b2, 1);
      }
      x6_split(y[0], y[1], sn);
#elif !(PNTF_X6_ABL & 1)
      x6_split(x[2 * kn], x[2 * kn + 1], sn);
#if PNTF_X6_EARLY
      {   // x[2kn], x[2kn + 1] are dead now: the next tile's block kn (the one after for kn = 0)
        const int64_t t2 = tile + 2 * stride;
        const Rsrc rr = kn != 0 ? rn : win(g.A, g.lda, t2 < ntiles ? t2 : tile);
        x[2 * kn] = pg_load(rr, va, 64 * kn);
        x[2 * kn + 1] = pg_load(rr, va, 64 * kn + 16);
      }
#endif
#else
      sn[0] = __builtin_bit_cast(bf16x8, x[2 * kn]);
      sn[1] = __builtin_bit_cast(bf16x8, x[2 * kn + 1]);
      sn[2] = sn[0];
#endif
#pragma unroll
      for (int t = 0; t < TG; ++t) {
        if constexpr (V == 1) {
          accl[t] = x6_small(fr[cur][t], s, accl[t]);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[cur][t][0], s[0], acc[t], 0, 0, 0);
        } else if constexpr (V == 3) {
          accl[t] = x6_low(fr[cur][t], s, accl[t]);
          accm[t] = x6_mid(fr[cur][t], s, accm[t]);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[cur][t][0], s[0], acc[t], 0, 0, 0);
        } else {
          acc[t] = x6_mma(fr[cur][t], s, acc[t]);
        }
      }
      // x[2kb], x[2kb + 1] were split one block ago: reload them with the next panel's (the
      // last tile reloads its own: no branch in the MFMA stream)
#if PNTF_X6_LSTAGE
      y[0] = yn[0];
      y[1] = yn[1];
#elif PNTF_X6_ABL & 32
      // (the same bytes per tile read row-contiguously: 8 lanes per 128-byte line, 8 rows per
      // instruction; wrong operands)
      x[2 * kb] = pg_load(rn, vco, 4096 * (kb & 3) + 128 * (kb >> 2));
      x[2 * kb + 1] = pg_load(rn, vco, 4096 * (kb & 3) + 128 * (kb >> 2) + 64);
#elif !(PNTF_X6_ABL & 4) && !PNTF_X6_EARLY
      x[2 * kb] = pg_load(rn, va, 64 * kb);
      x[2 * kb + 1] = pg_load(rn, va, 64 * kb + 16);
#endif
#pragma unroll
      for (int p = 0; p < 3; ++p) s[p] = sn[p];
      if constexpr (kb == KB - 1) {
        // (acc + bias) + C: the order of nn.Linear's addmm and the residual add after it
        const bool brow = ACC && g.bias && 32 * tile + j < g.brows;
#pragma unroll
        for (int t = 0; t < TG; ++t) {
#pragma unroll
          for (int R = 0; R < 4; ++R) {
            f32x4 v = {acc[t][4 * R], acc[t][4 * R + 1], acc[t][4 * R + 2], acc[t][4 * R + 3]};
            if constexpr (V == 3)
              v += f32x4{accl[t][4 * R], accl[t][4 * R + 1], accl[t][4 * R + 2], accl[t][4 * R + 3]} +
                   f32x4{accm[t][4 * R], accm[t][4 * R + 1], accm[t][4 * R + 2], accm[t][4 * R + 3]};
            if constexpr (V == 1)
              v += f32x4{accl[t][4 * R], accl[t][4 * R + 1], accl[t][4 * R + 2], accl[t][4 * R + 3]};
            if (ACC) {
              if (brow) v += lb[8 * t + 2 * R + h];
              v += cb[t][R];
            }
#if PNTF_X6_TSTORE
            // lane (j, h) holds row j's columns 32t + 8R + 4h .. +3 of the 64-column block
            lt[w][j * 17 + 8 * (t & 1) + 2 * R + h] = v;
#elif !(PNTF_X6_ABL & 8)
            pg_store(rc, v, vc, (c0 + 32 * t + 8 * R) * 4);
#else
            if (v[0] == 1.2345f) pg_store(rc, v, vc, (c0 + 32 * t + 8 * R) * 4);
#endif
          }
#if PNTF_X6_TSTORE
          if (t & 1) {
            // the block's rows go out row-contiguously: 16 lanes x 16 B per 256-byte row,
            // four rows per store (8 cache lines instead of 32 half-filled ones).  LDS is in
            // order within the wave; the wait is for the reads of the lanes' own data.
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const f32x4 v = lt[w][(4 * i + (lane >> 4)) * 17 + (lane & 15)];
#if !(PNTF_X6_ABL & 8)
              pg_store(rc, v, vt, (4 * i * (int)g.ldc + c0 + 32 * (t - 1)) * 4);
#else
              if (v[0] == 1.2345f) pg_store(rc, v, vt, (4 * i * (int)g.ldc + c0 + 32 * (t - 1)) * 4);
#endif
            }
          }
#endif
        }
      }
      // keep each block's loads where they are issued (the scheduler otherwise sinks the next
      // panel's loads to the tile's end and hoists later blocks' splits onto them)
      __builtin_amdgcn_sched_barrier(0);
    });
    if (!more) break;
    tile = next;
  }
}

// ---------------------------------------------------------------------------------------
// Split-bf16 panel GEMM on 16 x 16 x 32 tiles, two waves per SIMD (`panel_x6s_kernel`).
// panel_x6_kernel runs one wave per SIMD: its 32-row panel (128 VGPRs at K = 256) and the
// per-order accumulators leave no room for a second wave, so each next-panel load's latency is
// hidden only by the wave's own MFMAs.  Here a wave owns 16 rows (the B operand of
// v_mfma_f32_16x16x32_bf16: lane l holds panel row l & 15, k = 8(l >> 4) .. +7 of the 32-k
// block), so the panel takes 64 VGPRs and eight waves (two per SIMD) share the workgroup's
// weight group in LDS.  A operand: lane l holds W(out col 16t + (l & 15), k = 8(l >> 4) + j),
// three bf16 terms per 1 KiB fragment (x6s_pack_kernel).  D register i of lane l is out col
// c0 + 16t + 4(l >> 4) + i of row l & 15.  Each panel load covers 16 rows x 128 contiguous
// bytes (one cache line per row).  Same splits, products and per-order accumulation
// (V = 1: a0b0 | the five smaller products) as panel_x6_kernel.  Selected by panel mode 8
// (PNTF_GEMM_PANEL=8 / pntf_tt_set_panel_mode).  Same-box A/B (tests/diag/gemm_variants.py,
// profiles/r05_x6_gemm.txt): the generator GEMMs within noise of panel_x6_kernel (172-175 vs
// 165-172 TFLOP/s), some encoder shapes slower, so mode 3 stays the default: latency hiding is
// not what binds these kernels (the split-bf16 GEMMs also run at 1.77-1.88 GHz against the
// fp32-MFMA kernels' 2.3, profiles/r05_clock_probe.txt).
constexpr int X6S_CG = 64;   // columns per workgroup (4 out tiles of 16)

// P[((t·KB + kb)·3 + p)·64 + lane] = term p of B(32 kb + 8 (lane >> 4) + j, 16 t + (lane & 15))
__global__ void x6s_pack_kernel(const float* __restrict__ W, int64_t ldb, int tb, int KC, int NC,
                                bf16x8* __restrict__ P) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int KB = KC / 32;
  if (i >= (int64_t)(NC / 16) * KB * 64) return;
  const int lane = (int)(i & 63), kb = (int)((i >> 6) % KB), nt = (int)((i >> 6) / KB);
  const int n = 16 * nt + (lane & 15), k0 = 32 * kb + 8 * (lane >> 4);
  f32x4 a, b;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    a[e] = tb ? W[(int64_t)n * ldb + k0 + e] : W[(int64_t)(k0 + e) * ldb + n];
    b[e] = tb ? W[(int64_t)n * ldb + k0 + 4 + e] : W[(int64_t)(k0 + 4 + e) * ldb + n];
  }
  bf16x8 sp[3];
  x6_split(a, b, sp);
#pragma unroll
  for (int p = 0; p < 3; ++p) P[((int64_t)(nt * KB + kb) * 3 + p) * 64 + lane] = sp[p];
}

__device__ __forceinline__ f32x4 mfma16bf(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <int KC, int NC, bool ACC>
__global__ __launch_bounds__(512, 1) void panel_x6s_kernel(PanelArgs g) {
  PNTF_CLOCK_SCOPE;
  constexpr int KB = KC / 32, QK = KC / 8, CG = X6S_CG, TG = CG / 16, NG = NC / CG;
  constexpr int FR = TG * KB * 3;   // 1 KiB fragments per group
  constexpr int NW = 8;             // waves per workgroup
  static_assert(KB >= 4, "C prefetch distance");
  __shared__ bf16x8 lw[FR * 64];
  __shared__ f32x4 lb[ACC ? CG / 4 : 1];
  const int lane = threadIdx.x & 63, r = lane & 15, q4 = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int grp = 0, wg = blockIdx.x, nwg = gridDim.x;
  if constexpr (NG > 1) {   // the NG workgroups of a set of tiles on one XCD
    const int x = blockIdx.x & 7, sb = blockIdx.x >> 3;
    grp = sb % NG;
    wg = (sb / NG) * 8 + x;
    nwg = gridDim.x / NG;
  }
  {
    const bf16x8* src = reinterpret_cast<const bf16x8*>(g.P) + (int64_t)grp * FR * 64;
#pragma unroll 4
    for (int i = threadIdx.x; i < FR * 64; i += 64 * NW) lw[i] = src[i];
    if (ACC && g.bias && threadIdx.x < CG / 4)
      lb[threadIdx.x] = *reinterpret_cast<const f32x4*>(g.bias + CG * grp + 4 * threadIdx.x);
  }
  __syncthreads();
  const int64_t ntiles = (g.M + 15) / 16;
  const int64_t stride = (int64_t)nwg * NW;
  int64_t tile = (int64_t)wg * NW + w;
  if (tile >= ntiles) return;   // wave-uniform; no barrier follows
  auto win = [&](const float* base, int64_t ld, int64_t t) {
    const int64_t rows = g.M - 16 * t;
    return pg_rsrc(base + 16 * t * ld, (rows < 16 ? rows : 16) * ld * 4);
  };
  const int va = (int)((r * g.lda + 8 * q4) * 4), vc = (int)((r * g.ldc + 4 * q4) * 4);
  const int c0 = CG * grp;
  // panel: x[2kb], x[2kb + 1] = row r, k = 32 kb + 8 q4 .. +7
  f32x4 x[KB * 2];
  {
    const Rsrc ra = win(g.A, g.lda, tile);
#pragma unroll
    for (int q = 0; q < 2 * KB; ++q) x[q] = pg_load(ra, va, 128 * (q >> 1) + 16 * (q & 1));
  }
  const bf16x8* lf = lw + lane;
  bf16x8 fr[2][TG][3];
#pragma unroll
  for (int t = 0; t < TG; ++t)
#pragma unroll
    for (int p = 0; p < 3; ++p) fr[0][t][p] = lf[((t * KB) * 3 + p) * 64];
  bf16x8 s[3];
  x6_split(x[0], x[1], s);
  for (;;) {
    const int64_t next = tile + stride;
    const bool more = next < ntiles;
    const Rsrc rn = win(g.A, g.lda, more ? next : tile);
    const Rsrc rc = win(g.C, g.ldc, tile), rci = win(g.Cin, g.ldc, tile);
    f32x4 acc[TG], accl[TG], cb[TG];
#pragma unroll
    for (int t = 0; t < TG; ++t) {
      acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      accl[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    pg_static_for<0, KB>([&](auto I) {
      constexpr int kb = decltype(I)::value, cur = kb & 1;
      if constexpr (ACC && kb == KB - 4) {
#pragma unroll
        for (int t = 0; t < TG; ++t) cb[t] = pg_load(rci, vc, (c0 + 16 * t) * 4);
      }
      constexpr int kn = (kb + 1) % KB;
#pragma unroll
      for (int t = 0; t < TG; ++t)
#pragma unroll
        for (int p = 0; p < 3; ++p) fr[cur ^ 1][t][p] = lf[((t * KB + kn) * 3 + p) * 64];
      bf16x8 sn[3];
      x6_split(x[2 * kn], x[2 * kn + 1], sn);
#pragma unroll
      for (int t = 0; t < TG; ++t) {
        const bf16x8 (&a)[3] = fr[cur][t];
        f32x4 l = accl[t];
        l = mfma16bf(a[2], s[0], l);
        l = mfma16bf(a[1], s[1], l);
        l = mfma16bf(a[0], s[2], l);
        l = mfma16bf(a[1], s[0], l);
        l = mfma16bf(a[0], s[1], l);
        accl[t] = l;
        acc[t] = mfma16bf(a[0], s[0], acc[t]);
      }
      // x[2kb], x[2kb + 1] were split one block ago: the next panel's
      x[2 * kb] = pg_load(rn, va, 128 * kb);
      x[2 * kb + 1] = pg_load(rn, va, 128 * kb + 16);
#pragma unroll
      for (int p = 0; p < 3; ++p) s[p] = sn[p];
      if constexpr (kb == KB - 1) {
        const bool brow = ACC && g.bias && 16 * tile + r < g.brows;
#pragma unroll
        for (int t = 0; t < TG; ++t) {
          f32x4 v = acc[t] + accl[t];
          if (ACC) {
            if (brow) v += lb[4 * t + q4];
            v += cb[t];
          }
          pg_store(rc, v, vc, (c0 + 16 * t) * 4);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    if (!more) break;
    tile = next;
  }
}

// ---------------------------------------------------------------------------------------
// Linear + act_laplace of the Taylor tape in one pass (pntf_tt_linear_act; the forward of one
// Linear of NN.out_laplace, model_res_sigmoid_multi.py:710-848 with act_laplace :675-691).
// The LDS panel GEMM above with the tape's elementwise stage as its epilogue, so the
// pre-activation never round-trips HBM between the GEMM and a separate act kernel.  A wave
// owns a 32-POINT block and runs the block's R planes one after the other, in the order
//   value, then per endpoint group l: its GK = ndir/nl first-derivative (J) planes, its
//   summed second-derivative (L) plane,
// so everything the act of a plane needs is already in the wave: lane (j, h) holds point j's
// 64 features of the group (D register 4R + e of out tile t = column 32t + 8R + 4h + e), and
// keeps per feature σ(10 y₀) from the value plane and Σ_{k∈l} J_k² over the group's J planes:
//   value  y₀ = acc + bias (+ res)   h = softplus₁₀(y₀)          s = σ(10 y₀)
//   J_k    y  = acc (+ res)          h = s·y                      jj += y²
//   L_l    y  = acc (+ res)          h = 10 s(1 - s)·jj + s·y
// y (the tape) and h are both stored; the residual planes are loaded 4 iterations before the
// store, like the ACC path's C.  Same formulas as tt_act_fwd_kernel (pntf_train.hip).
struct ActArgs {
  const float* A;      // x planes (R·M, KC)
  const f32x4* P;      // packed weight fragments (panel_pack_kernel)
  float* Y;            // pre-activation planes (R·M, NC)
  float* H;            // activation planes (R·M, NC), act only
  const float* bias;   // (NC)
  const float* res;    // residual planes (R·M, NC) or null
  int64_t M;           // points per plane
  int R, ndir, nl, act;
};

__device__ __forceinline__ float pa_sig10(float y) { return 1.f / (1.f + expf(-10.f * y)); }
__device__ __forceinline__ float pa_softplus10(float y) {
  return 10.f * y > 20.f ? y : log1pf(expf(10.f * y)) / 10.f;
}

template <int KC, int NC>
__global__ __launch_bounds__(256, 1) void panel_act_kernel(ActArgs g) {
  constexpr int QK = KC / 8, NG = NC / 128, FR = 4 * QK;
  static_assert(QK >= 8, "residual prefetch distance");
  __shared__ f32x4 lw[FR * 64];
  __shared__ f32x4 lb[32];   // the group's 128 biases
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int grp = 0, wg = blockIdx.x, nwg = gridDim.x;
  if constexpr (NG == 2) {   // a block's two groups on one XCD (panel_lds_kernel)
    const int x = blockIdx.x & 7, s = blockIdx.x >> 3;
    grp = s & 1;
    wg = (s >> 1) * 8 + x;
    nwg = gridDim.x / 2;
  }
  {
    const f32x4* src = g.P + (int64_t)grp * FR * 64;
#pragma unroll 8
    for (int i = threadIdx.x; i < FR * 64; i += 256) lw[i] = src[i];
    if (threadIdx.x < 32)
      lb[threadIdx.x] = reinterpret_cast<const f32x4*>(g.bias)[grp * 32 + threadIdx.x];
  }
  __syncthreads();
  const int64_t nblk = (g.M + 31) / 32;
  const int64_t stride = (int64_t)nwg * 4;
  int64_t blk = (int64_t)wg * 4 + w;
  if (blk >= nblk) return;   // wave-uniform; no barrier follows
  const int R = g.R, ndir = g.ndir, GK = g.nl ? g.ndir / g.nl : 1;
  const bool has_res = g.res != nullptr, act = g.act != 0;
  // plane at sequence position i: 0, then per group l its GK J planes and its L plane
  auto plane_of = [&](int i) {
    if (i == 0) return 0;
    const int l = (i - 1) / (GK + 1), k = (i - 1) % (GK + 1);
    return k < GK ? 1 + l * GK + k : 1 + ndir + l;
  };
  // the 32-row window of (block b, plane r); rows past the plane's M are outside it
  auto win = [&](const float* base, int ld, int64_t b, int r) {
    const int64_t rows = g.M - 32 * b;
    return pg_rsrc(base + ((int64_t)r * g.M + 32 * b) * ld, (rows < 32 ? rows : 32) * ld * 4);
  };
  const int va = (j * KC + 4 * h) * 4, vc = (j * NC + 4 * h) * 4;
  const int c0 = 128 * grp;
  f32x4 x[QK];
  {
    const Rsrc ra = win(g.A, KC, blk, 0);
#pragma unroll
    for (int q = 0; q < QK; ++q) x[q] = pg_load(ra, va, 32 * q);
  }
  const f32x4* lf = lw + lane;
  f32x4 fr[2][4];
#pragma unroll
  for (int t = 0; t < 4; ++t) fr[0][t] = lf[(t * QK) * 64];
  f32x4 s[4][4], jj[4][4];   // per feature of point j: σ(10 y₀), Σ J² of the current group
  int i = 0;
  for (;;) {
    const int r = plane_of(i);
    int ni = i + 1;
    int64_t nb = blk;
    if (ni == R) {
      ni = 0;
      nb = blk + stride;
    }
    const bool more = nb < nblk;
    const Rsrc rn = win(g.A, KC, more ? nb : blk, more ? plane_of(ni) : r);
    const Rsrc ry = win(g.Y, NC, blk, r), rh = win(g.H, NC, blk, r);
    const Rsrc rr = win(has_res ? g.res : g.Y, NC, blk, r);
    // plane kind: 0 value, 1 J (first of its group: 2), 3 L
    const int kind = r == 0 ? 0 : r <= ndir ? ((r - 1) % GK == 0 ? 2 : 1) : 3;
    f32x16 acc[4];
    f32x4 cb[4][4];
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[t][e] = 0.f;
    pg_static_for<0, QK>([&](auto I) {
      constexpr int q = decltype(I)::value, cur = q & 1;
      if constexpr (q == QK - 4) {
        if (has_res) {
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int Q = 0; Q < 4; ++Q) cb[t][Q] = pg_load(rr, vc, (c0 + 32 * t + 8 * Q) * 4);
        }
      }
      constexpr int qn = (q + 1) % QK;
#pragma unroll
      for (int t = 0; t < 4; ++t) fr[cur ^ 1][t] = lf[(t * QK + qn) * 64];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(fr[cur][t][e], x[q][e], acc[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (more) x[q] = pg_load(rn, va, 32 * q);
      if constexpr (q == QK - 1) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int Q = 0; Q < 4; ++Q) {
            f32x4 v = {acc[t][4 * Q], acc[t][4 * Q + 1], acc[t][4 * Q + 2], acc[t][4 * Q + 3]};
            if (kind == 0) v += lb[8 * t + 2 * Q + h];   // (acc + bias) + res, as tt_act_fwd
            if (has_res) v += cb[t][Q];
            const int off = (c0 + 32 * t + 8 * Q) * 4;
            pg_store(ry, v, vc, off);
            if (act) {
              f32x4 hv;
              if (kind == 0) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  s[t][Q][e] = pa_sig10(v[e]);
                  hv[e] = pa_softplus10(v[e]);
                }
              } else if (kind == 3) {
                hv = 10.f * s[t][Q] * (1.f - s[t][Q]) * jj[t][Q] + v * s[t][Q];
              } else {
                hv = v * s[t][Q];
                jj[t][Q] = kind == 2 ? v * v : jj[t][Q] + v * v;
              }
              pg_store(rh, hv, vc, off);
            }
          }
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    if (!more) break;
    i = ni;
    blk = nb;
  }
}

// Cooperative form of the same fused Linear + act_laplace (schedule 3): the four waves of a
// workgroup share one 32-point block, wave w computing out tile w (32 columns) of the
// workgroup's 128-column group for every plane of the block, so the balance unit is a block
// per WORKGROUP: at the reference batch 625 generator blocks over 128 workgroups per column
// group (4.9 rounds, 98 % full) where panel_act_kernel gave 625 blocks to 512 waves (1.2
// rounds: 61 %).  Per wave and plane: KC/2 MFMAs on one accumulator tile, its A panel (the
// block's x rows of that plane, the same for the four waves: L1/L2 shared) loaded one plane
// ahead, its fragments from LDS.  The act of a column needs only that column's σ(10 y₀) and
// Σ J², so every wave keeps 16 of each and nothing crosses waves (no barrier in the loop).
template <int KC, int NC>
__global__ __launch_bounds__(256, 1) void panel_act_coop_kernel(ActArgs g) {
  constexpr int QK = KC / 8, NG = NC / 128, FR = 4 * QK;
  __shared__ f32x4 lw[FR * 64];
  __shared__ f32x4 lb[32];   // the group's 128 biases
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int grp = 0, wg = blockIdx.x, nwg = gridDim.x;
  if constexpr (NG == 2) {   // a block's two groups on one XCD (panel_lds_kernel)
    const int x = blockIdx.x & 7, s = blockIdx.x >> 3;
    grp = s & 1;
    wg = (s >> 1) * 8 + x;
    nwg = gridDim.x / 2;
  }
  {
    const f32x4* src = g.P + (int64_t)grp * FR * 64;
#pragma unroll 8
    for (int i = threadIdx.x; i < FR * 64; i += 256) lw[i] = src[i];
    if (threadIdx.x < 32)
      lb[threadIdx.x] = reinterpret_cast<const f32x4*>(g.bias)[grp * 32 + threadIdx.x];
  }
  __syncthreads();
  const int64_t nblk = (g.M + 31) / 32;
  int64_t blk = wg;
  if (blk >= nblk) return;   // workgroup-uniform; no barrier follows
  const int R = g.R, ndir = g.ndir, GK = g.nl ? g.ndir / g.nl : 1;
  const bool has_res = g.res != nullptr, act = g.act != 0;
  auto plane_of = [&](int i) {
    if (i == 0) return 0;
    const int l = (i - 1) / (GK + 1), k = (i - 1) % (GK + 1);
    return k < GK ? 1 + l * GK + k : 1 + ndir + l;
  };
  auto win = [&](const float* base, int ld, int64_t b, int r) {
    const int64_t rows = g.M - 32 * b;
    return pg_rsrc(base + ((int64_t)r * g.M + 32 * b) * ld, (rows < 32 ? rows : 32) * ld * 4);
  };
  const int va = (j * KC + 4 * h) * 4, vc = (j * NC + 4 * h) * 4;
  const int c0 = 128 * grp + 32 * w;   // the wave's 32 out columns
  f32x4 x[QK];
  {
    const Rsrc ra = win(g.A, KC, blk, 0);
#pragma unroll
    for (int q = 0; q < QK; ++q) x[q] = pg_load(ra, va, 32 * q);
  }
  const f32x4* lf = lw + w * QK * 64 + lane;
  f32x4 fr[2];
  fr[0] = lf[0];
  f32x4 s[4], jj[4];   // per feature of point j: σ(10 y₀), Σ J² of the current group
  int i = 0;
  for (;;) {
    const int r = plane_of(i);
    int ni = i + 1;
    int64_t nb = blk;
    if (ni == R) {
      ni = 0;
      nb = blk + nwg;
    }
    const bool more = nb < nblk;
    const Rsrc rn = win(g.A, KC, more ? nb : blk, more ? plane_of(ni) : r);
    const Rsrc ry = win(g.Y, NC, blk, r), rh = win(g.H, NC, blk, r);
    const Rsrc rr = win(has_res ? g.res : g.Y, NC, blk, r);
    const int kind = r == 0 ? 0 : r <= ndir ? ((r - 1) % GK == 0 ? 2 : 1) : 3;
    f32x16 acc;
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = 0.f;
    f32x4 cb[4];
    pg_static_for<0, QK>([&](auto I) {
      constexpr int q = decltype(I)::value, cur = q & 1;
      // the residual planes come from HBM: load them a whole plane (QK·4 MFMAs) ahead of the
      // epilogue (3 iterations of lead, as the one-wave kernel has, left ~2k cycles exposed)
      if constexpr (q == 0) {
        if (has_res) {
#pragma unroll
          for (int Q = 0; Q < 4; ++Q) cb[Q] = pg_load(rr, vc, (c0 + 8 * Q) * 4);
        }
      }
      constexpr int qn = (q + 1) % QK;
      fr[cur ^ 1] = lf[qn * 64];
#pragma unroll
      for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fr[cur][e], x[q][e], acc, 0, 0, 0);
      if (more) x[q] = pg_load(rn, va, 32 * q);
      if constexpr (q == QK - 1) {
#pragma unroll
        for (int Q = 0; Q < 4; ++Q) {
          f32x4 v = {acc[4 * Q], acc[4 * Q + 1], acc[4 * Q + 2], acc[4 * Q + 3]};
          if (kind == 0) v += lb[8 * w + 2 * Q + h];   // (acc + bias) + res, as tt_act_fwd
          if (has_res) v += cb[Q];
          const int off = (c0 + 8 * Q) * 4;
          pg_store(ry, v, vc, off);
          if (act) {
            f32x4 hv;
            if (kind == 0) {
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                s[Q][e] = pa_sig10(v[e]);
                hv[e] = pa_softplus10(v[e]);
              }
            } else if (kind == 3) {
              hv = 10.f * s[Q] * (1.f - s[Q]) * jj[Q] + v * s[Q];
            } else {
              hv = v * s[Q];
              jj[Q] = kind == 2 ? v * v : jj[Q] + v * v;
            }
            pg_store(rh, hv, vc, off);
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    if (!more) break;
    i = ni;
    blk = nb;
  }
}

// Input gradient of one Linear with the previous layer's act_laplace adjoint as its epilogue
// (pntf_tt_linear_bwd; the reverse of a Linear of NN.out_laplace and the act before it, what
// loss.backward() does at model_res_sigmoid_multi.py:1048 through :663-691): per plane
//   g_h = gY·W (+ res, the residual branch's gradient),   then, with s = σ(10 y₀) of the
//   previous layer's value plane, ds = 10 s (1 - s), dds = 10 ds (1 - 2 s):
//   L_l:  g_yL = gL s                  acc₀ += gL (L ds)          (gL kept)
//   J_k:  g_yJ = gJ s + 2 gL J ds      acc₀ += gJ J ds + gL dds J²
//   value g_y₀ = g_h₀ s + acc₀         bias partial += g_y₀
// (the formulas of tt_act_bwd_kernel, pntf_train.hip), so the g_h planes never round-trip
// HBM between the GEMM and the act adjoint.  Same cooperative layout as
// panel_act_coop_kernel: the four waves of a workgroup share a 32-point block, wave w owns out
// tile w of the workgroup's 128-column group; a block's planes run L_l, its J planes, ..., the
// value plane last.  The bias partials of a wave (its 32 columns, summed over its blocks and
// then over the block's 32 points) go to partial[workgroup][NC] in a fixed order.
struct BwdArgs {
  const float* A;      // gY planes (R·M, KC)
  const f32x4* P;      // packed W (panel_pack_kernel, tb = 0)
  const float* Y;      // previous layer's pre-activation planes (R·M, NC)
  const float* res;    // residual-branch gradient planes (R·M, NC) or null
  float* G;            // out: g_y planes of the previous layer (R·M, NC); may alias res
  float* partial;      // bias partials [workgroups per group][NC]
  int64_t M;
  int R, ndir, nl;
};

#ifndef PNTF_BWD_EARLY
#define PNTF_BWD_EARLY (QK / 2)
#endif
template <int KC, int NC>
__global__ __launch_bounds__(256, 1) void panel_bwd_coop_kernel(BwdArgs g) {
  constexpr int QK = KC / 8, NG = NC / 128, FR = 4 * QK;
  __shared__ f32x4 lw[FR * 64];
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int grp = 0, wg = blockIdx.x, nwg = gridDim.x;
  if constexpr (NG == 2) {
    const int x = blockIdx.x & 7, s = blockIdx.x >> 3;
    grp = s & 1;
    wg = (s >> 1) * 8 + x;
    nwg = gridDim.x / 2;
  }
  {
    const f32x4* src = g.P + (int64_t)grp * FR * 64;
#pragma unroll 8
    for (int i = threadIdx.x; i < FR * 64; i += 256) lw[i] = src[i];
  }
  __syncthreads();
  const int c0 = 128 * grp + 32 * w;   // the wave's 32 out columns
  f32x4 bsum[4];
#pragma unroll
  for (int Q = 0; Q < 4; ++Q) bsum[Q] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t nblk = (g.M + 31) / 32;
  int64_t blk = wg;
  if (blk < nblk) {
    const int R = g.R, ndir = g.ndir, nl = g.nl, GK = nl ? ndir / nl : 1;
    const bool has_res = g.res != nullptr;
    // plane at sequence position i: per group l its L plane then its GK J planes; value last
    auto plane_of = [&](int i) {
      if (i == R - 1) return 0;
      const int l = i / (GK + 1), k = i % (GK + 1);
      return k == 0 ? 1 + ndir + l : 1 + l * GK + (k - 1);
    };
    auto win = [&](const float* base, int ld, int64_t b, int r) {
      const int64_t rows = g.M - 32 * b;
      return pg_rsrc(base + ((int64_t)r * g.M + 32 * b) * ld, (rows < 32 ? rows : 32) * ld * 4);
    };
    const int va = (j * KC + 4 * h) * 4, vc = (j * NC + 4 * h) * 4;
    f32x4 x[QK];
    {
      const Rsrc ra = win(g.A, KC, blk, plane_of(0));
#pragma unroll
      for (int q = 0; q < QK; ++q) x[q] = pg_load(ra, va, 32 * q);
    }
    const f32x4* lf = lw + w * QK * 64 + lane;
    f32x4 fr[2];
    fr[0] = lf[0];
    f32x4 s[4], gL[4], a0[4];
    int i = 0;
    for (;;) {
      const int r = plane_of(i);
      int ni = i + 1;
      int64_t nb = blk;
      if (ni == R) {
        ni = 0;
        nb = blk + nwg;
      }
      const bool more = nb < nblk;
      const Rsrc rn = win(g.A, KC, more ? nb : blk, plane_of(more ? ni : i));
      const Rsrc ry = win(g.Y, NC, blk, r), rg = win(g.G, NC, blk, r);
      const Rsrc rr = win(has_res ? g.res : g.Y, NC, blk, r);
      const Rsrc ry0 = win(g.Y, NC, blk, 0);
      // 0 value, 1 J, 3 L
      const int kind = r == 0 ? 0 : r <= ndir ? 1 : 3;
      f32x16 acc;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = 0.f;
      f32x4 cb[4], yt[4];
      pg_static_for<0, QK>([&](auto I) {
        constexpr int q = decltype(I)::value, cur = q & 1;
        if constexpr (q == 0) {
          if (i == 0) {   // block start: σ of the previous layer's value plane
#pragma unroll
            for (int Q = 0; Q < 4; ++Q) s[Q] = pg_load(ry0, vc, (c0 + 8 * Q) * 4);
          }
        }
        if constexpr (q == PNTF_BWD_EARLY) {   // HBM planes: half a plane of lead or more
#pragma unroll
          for (int Q = 0; Q < 4; ++Q) {
            if (has_res) cb[Q] = pg_load(rr, vc, (c0 + 8 * Q) * 4);
            if (kind != 0) yt[Q] = pg_load(ry, vc, (c0 + 8 * Q) * 4);
          }
        }
        constexpr int qn = (q + 1) % QK;
        fr[cur ^ 1] = lf[qn * 64];
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(fr[cur][e], x[q][e], acc, 0, 0, 0);
        if (more) x[q] = pg_load(rn, va, 32 * q);
        if constexpr (q == QK / 2) {
          if (i == 0) {   // the loads above have had half a plane: σ from y₀, once per block
#pragma unroll
            for (int Q = 0; Q < 4; ++Q) {
#pragma unroll
              for (int e = 0; e < 4; ++e) s[Q][e] = pa_sig10(s[Q][e]);
              a0[Q] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
          }
        }
        if constexpr (q == QK - 1) {
#pragma unroll
          for (int Q = 0; Q < 4; ++Q) {
            f32x4 v = {acc[4 * Q], acc[4 * Q + 1], acc[4 * Q + 2], acc[4 * Q + 3]};
            if (has_res) v += cb[Q];
            const f32x4 sq = s[Q], ds = 10.f * sq * (1.f - sq);
            f32x4 o;
            if (kind == 3) {            // L_l: opens its group
              gL[Q] = v;
              o = v * sq;
              a0[Q] += v * (yt[Q] * ds);
            } else if (kind == 1) {     // J_k of the current group
              const f32x4 J = yt[Q], dds = 10.f * ds * (1.f - 2.f * sq);
              o = v * sq + 2.f * gL[Q] * J * ds;
              a0[Q] += v * J * ds + gL[Q] * dds * (J * J);
            } else {                    // value plane, last of the block
              o = v * sq + a0[Q];
              bsum[Q] += o;
            }
            pg_store(rg, o, vc, (c0 + 8 * Q) * 4);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      if (!more) break;
      i = ni;
      blk = nb;
    }
  }
  // bias partials: sum the block's 32 points (lanes j of each half) for the wave's 16 columns
  // per lane half, in a fixed butterfly order; lane (0, h) writes 16 columns
#pragma unroll
  for (int Q = 0; Q < 4; ++Q)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = bsum[Q][e];
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
      bsum[Q][e] = v;
    }
  if (j == 0) {   // row wg: the waves (and the groups' workgroups) fill disjoint columns
#pragma unroll
    for (int Q = 0; Q < 4; ++Q)
      *reinterpret_cast<f32x4*>(g.partial + (int64_t)wg * NC + c0 + 8 * Q + 4 * h) = bsum[Q];
  }
}

// The same fused input gradient + act adjoint on the split-bf16 MFMA (round 6,
// `panel_bwd_x6_kernel`, bwd mode 1): gY·W as panel_x6_kernel computes it (three-term splits of
// both operands, six v_mfma_f32_32x32x16_bf16 per 32 x 32 x 16 block, per-order accumulators
// summed smallest first), then the epilogue of panel_bwd_coop_kernel above.  A workgroup holds
// the pre-split W of a 64-column group in LDS (96 KiB at KC = 256); wave w owns out tile w & 1
// of the group and point blocks 2·wg + (w >> 1) + 2·nwg·i, so two waves share each block's panel
// rows (the second read hits the CU's caches).  Per wave: the 32-row panel of one plane (QK
// float4 registers, the next plane's loaded behind the current one's MFMAs, as in
// panel_x6_kernel), three accumulators and the epilogue state (σ, g_L, acc₀) of one out tile.
// Bias partials: row 2·wg + (w >> 1) of `partial`, the wave's 32 columns.
template <int KC, int NC>
__global__ __launch_bounds__(256, 1) void panel_bwd_x6_kernel(BwdArgs g) {
  constexpr int KB = KC / 16, QK = KC / 8, CG = 64, NG = NC / CG, FR = 2 * KB * 3;
  __shared__ bf16x8 lw[FR * 64];
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int grp = 0, wg = blockIdx.x, nwg = gridDim.x;
  if constexpr (NG > 1) {
    const int x = blockIdx.x & 7, s = blockIdx.x >> 3;
    grp = s % NG;
    wg = (s / NG) * 8 + x;
    nwg = gridDim.x / NG;
  }
  {
    const bf16x8* src = reinterpret_cast<const bf16x8*>(g.P) + (int64_t)grp * FR * 64;
#pragma unroll 8
    for (int i = threadIdx.x; i < FR * 64; i += 256) lw[i] = src[i];
  }
  __syncthreads();
  const int t = w & 1, pb = w >> 1;
  const int c0 = CG * grp + 32 * t;   // the wave's 32 out columns
  f32x4 bsum[4];
#pragma unroll
  for (int Q = 0; Q < 4; ++Q) bsum[Q] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t nblk = (g.M + 31) / 32, bstride = 2 * (int64_t)nwg;
  int64_t blk = 2 * (int64_t)wg + pb;
  if (blk < nblk) {
    const int R = g.R, ndir = g.ndir, nl = g.nl, GK = nl ? ndir / nl : 1;
    const bool has_res = g.res != nullptr;
    // plane at sequence position i: per group l its L plane then its GK J planes; value last
    auto plane_of = [&](int i) {
      if (i == R - 1) return 0;
      const int l = i / (GK + 1), k = i % (GK + 1);
      return k == 0 ? 1 + ndir + l : 1 + l * GK + (k - 1);
    };
    auto win = [&](const float* base, int ld, int64_t b, int r) {
      const int64_t rows = g.M - 32 * b;
      return pg_rsrc(base + ((int64_t)r * g.M + 32 * b) * ld, (rows < 32 ? rows : 32) * ld * 4);
    };
    // lane (j, h): panel row j, k = 16 kb + 8 h .. +7 as two float4 (x[2 kb], x[2 kb + 1]);
    // out row j, columns c0 + 8 Q + 4 h .. +3
    const int va = (j * KC + 8 * h) * 4, vc = (j * NC + 4 * h) * 4;
    f32x4 x[QK];
    {
      const Rsrc ra = win(g.A, KC, blk, plane_of(0));
#pragma unroll
      for (int q = 0; q < QK; ++q) x[q] = pg_load(ra, va, 64 * (q >> 1) + 16 * (q & 1));
    }
    bf16x8 xs[3];
    x6_split(x[0], x[1], xs);
    const bf16x8* lf = lw + (t * KB * 3) * 64 + lane;
    bf16x8 fr[2][3];
#pragma unroll
    for (int p = 0; p < 3; ++p) fr[0][p] = lf[p * 64];
    f32x4 s[4], gL[4], a0[4];
    int i = 0;
    for (;;) {
      const int r = plane_of(i);
      int ni = i + 1;
      int64_t nb = blk;
      if (ni == R) {
        ni = 0;
        nb = blk + bstride;
      }
      const bool more = nb < nblk;
      const Rsrc rn = win(g.A, KC, more ? nb : blk, plane_of(more ? ni : i));
      const Rsrc ry = win(g.Y, NC, blk, r), rg = win(g.G, NC, blk, r);
      const Rsrc rr = win(has_res ? g.res : g.Y, NC, blk, r);
      const Rsrc ry0 = win(g.Y, NC, blk, 0);
      // 0 value, 1 J, 3 L
      const int kind = r == 0 ? 0 : r <= ndir ? 1 : 3;
      f32x16 acc, accl, accm;
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[e] = accl[e] = accm[e] = 0.f;
      f32x4 cb[4], yt[4];
      pg_static_for<0, KB>([&](auto I) {
        constexpr int kb = decltype(I)::value, cur = kb & 1, kn = (kb + 1) % KB;
        if constexpr (kb == 0) {
          if (i == 0) {   // block start: the previous layer's value plane (σ at KB / 2)
#pragma unroll
            for (int Q = 0; Q < 4; ++Q) s[Q] = pg_load(ry0, vc, (c0 + 8 * Q) * 4);
          }
        }
        if constexpr (kb == KB / 2 - 1) {   // the plane's epilogue operands, half a plane ahead
#pragma unroll
          for (int Q = 0; Q < 4; ++Q) {
            if (has_res) cb[Q] = pg_load(rr, vc, (c0 + 8 * Q) * 4);
            if (kind != 0) yt[Q] = pg_load(ry, vc, (c0 + 8 * Q) * 4);
          }
        }
        // next k block's fragments (past the plane's end: block 0 again) and terms (past the
        // end: the next plane's block 0, loaded at this plane's block 0)
#pragma unroll
        for (int p = 0; p < 3; ++p) fr[cur ^ 1][p] = lf[(kn * 3 + p) * 64];
        bf16x8 sn[3];
        x6_split(x[2 * kn], x[2 * kn + 1], sn);
        accl = x6_low(fr[cur], xs, accl);
        accm = x6_mid(fr[cur], xs, accm);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fr[cur][0], xs[0], acc, 0, 0, 0);
        // block kb was split one block ago: its registers take the next plane's
        if (more) {
          x[2 * kb] = pg_load(rn, va, 64 * kb);
          x[2 * kb + 1] = pg_load(rn, va, 64 * kb + 16);
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) xs[p] = sn[p];
        if constexpr (kb == KB / 2) {
          if (i == 0) {
#pragma unroll
            for (int Q = 0; Q < 4; ++Q) {
#pragma unroll
              for (int e = 0; e < 4; ++e) s[Q][e] = pa_sig10(s[Q][e]);
              a0[Q] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
          }
        }
        if constexpr (kb == KB - 1) {
#pragma unroll
          for (int Q = 0; Q < 4; ++Q) {
            f32x4 v = {acc[4 * Q], acc[4 * Q + 1], acc[4 * Q + 2], acc[4 * Q + 3]};
            v += f32x4{accl[4 * Q], accl[4 * Q + 1], accl[4 * Q + 2], accl[4 * Q + 3]} +
                 f32x4{accm[4 * Q], accm[4 * Q + 1], accm[4 * Q + 2], accm[4 * Q + 3]};
            if (has_res) v += cb[Q];
            const f32x4 sq = s[Q], ds = 10.f * sq * (1.f - sq);
            f32x4 o;
            if (kind == 3) {            // L_l: opens its group
              gL[Q] = v;
              o = v * sq;
              a0[Q] += v * (yt[Q] * ds);
            } else if (kind == 1) {     // J_k of the current group
              const f32x4 J = yt[Q], dds = 10.f * ds * (1.f - 2.f * sq);
              o = v * sq + 2.f * gL[Q] * J * ds;
              a0[Q] += v * J * ds + gL[Q] * dds * (J * J);
            } else {                    // value plane, last of the block
              o = v * sq + a0[Q];
              bsum[Q] += o;
            }
            pg_store(rg, o, vc, (c0 + 8 * Q) * 4);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      if (!more) break;
      i = ni;
      blk = nb;
    }
  }
  // bias partials: the 32 points of each lane half summed in a fixed butterfly order
#pragma unroll
  for (int Q = 0; Q < 4; ++Q)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v = bsum[Q][e];
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
      bsum[Q][e] = v;
    }
  if (j == 0) {   // row 2·wg + pb: the waves and the groups' workgroups fill disjoint columns
#pragma unroll
    for (int Q = 0; Q < 4; ++Q)
      *reinterpret_cast<f32x4*>(g.partial + (2 * (int64_t)wg + pb) * NC + c0 + 8 * Q + 4 * h) =
          bsum[Q];
  }
}

// gbias[c] = Σ_b partial[b][c] in row order (deterministic); one thread per column
__global__ void colsum_kernel(const float* __restrict__ partial, int nb, int nc,
                              float* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nc) return;
  float a = 0.f, b = 0.f;
  int r = 0;
  for (; r + 1 < nb; r += 2) {
    a += partial[(int64_t)r * nc + c];
    b += partial[(int64_t)(r + 1) * nc + c];
  }
  if (r < nb) a += partial[(int64_t)r * nc + c];
  out[c] = a + b;
}

// ---------------------------------------------------------------------------------------
// Weight-gradient GEMM  gW (M x N) = gYᵀ (M x rows) · X (rows x N), M, N ∈ {128, 256}: the
// reduction runs over every Taylor row of the tape (10⁵-10⁶), the output is one or a few
// 128 x 128 tiles.  No LDS staging and no barrier in the loop: one wave owns a whole 128 x 128
// output tile (4 x 4 MFMA tiles = 256 accumulators) and streams its rows straight from HBM.
// Per row pair (k step of v_mfma_f32_32x32x2_f32, lane half h = row 2p + h) a lane loads ONE
// float4 of gY (out rows 4j .. 4j+3) and ONE float4 of X (out cols 4j .. 4j+3); component e of
// the first is the A operand of out rows {4i + e}, component d of the second the B operand of
// out cols {4j + d}, so the two 1 KiB wave loads feed all 16 MFMAs (1024 MFMA cycles per
// 2 KiB: the stream needs 8 B/clk per CU, far below L2 / HBM rates).  Three register buffers
// of one 16-row chunk each; a buffer is refilled in one burst right after its MFMAs, two
// chunks ahead of its use.  Workgroup b = (split s, tile): its 4 waves take the
// 16-row chunks of the split's row range round-robin (adjacent waves read adjacent rows), then
// sum their tiles through LDS in a fixed order (w0, + w1, + w2, + w3) and write one partial
// (M x N layout) per split; gemm_reduce1/2 sum the splits in order (deterministic).
// D register r of lane (j, h) for tile (e, d) is out row 4·((r & 3) + 8·(r >> 2) + 4h) + e,
// out col 4j + d: a float4 over d is one 16-byte store of consecutive columns.
struct WgradArgs {
  const float* A;   // gY (rows x M), row stride M
  const float* B;   // X (rows x N), row stride N
  float* work;      // splits x (M x N) partial sums
  int64_t rows, rps;  // reduction length; rows per split (a multiple of 128)
  int M, N;
  int xcd;            // splits a multiple of 8: XCD-aware block -> (split, tile) map
};
constexpr int WG_PF = 8;   // row pairs per chunk = ring slots

__device__ __forceinline__ void wg_store(float* p, f32x4 v) {
  *reinterpret_cast<f32x4*>(p) = v;
  asm volatile("s_nop 0" ::"v"(v));   // store-data hazard guard (pntf_field.h bstore)
}
__device__ __forceinline__ void wg_reduce_store(const WgradArgs& g, const f32x16 (&acc)[4][4],
                                                f32x4 (&red)[2][64 * 64], int s, int tm, int tn);

template <int T, int NB>
__global__ __launch_bounds__(256, 1) void wgrad_kernel(WgradArgs g) {
  PNTF_CLOCK_SCOPE;
  __shared__ f32x4 red[2][64 * 64];   // two 128 x 128 tiles (128 KiB)
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // block b runs on XCD b % 8 (dispatch order): with the split count a multiple of 8 the T
  // tiles of one split take blocks 8 apart, so they share an XCD and its L2 serves the second
  // read of each gY / X row segment
  const int b8 = blockIdx.x >> 3;
  const int tile = g.xcd ? b8 % T : blockIdx.x % T;
  const int s = g.xcd ? (blockIdx.x & 7) + 8 * (b8 / T) : blockIdx.x / T;
  const int tnn = g.N / 128, tm = tile / tnn, tn = tile % tnn;
  const int64_t r0 = (int64_t)s * g.rps;
  const int64_t left = g.rows - r0;
  const int64_t nrows = left <= 0 ? 0 : (left < g.rps ? left : g.rps);
  f32x16 acc[4][4];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[e][d][r] = 0.f;
  if (nrows > 0) {
    // rows past the split's end are outside the resources: their loads return 0
    const Rsrc ra = pg_rsrc(g.A + r0 * g.M, nrows * g.M * 4);
    const Rsrc rb = pg_rsrc(g.B + r0 * g.N, nrows * g.N * 4);
    const int va = (h * g.M + 128 * tm + 4 * j) * 4, vb = (h * g.N + 128 * tn + 4 * j) * 4;
    const int sa = __builtin_amdgcn_readfirstlane(2 * g.M * 4);
    const int sb = __builtin_amdgcn_readfirstlane(2 * g.N * 4);
    const int nchunks = (int)((nrows + 2 * WG_PF - 1) / (2 * WG_PF));
    int c = w;
    if constexpr (NB == 1) {
      // ring of WG_PF slots: slot p is refilled with the wave's next chunk right after its
      // MFMAs, WG_PF - 1 row pairs ahead of its use.  Loads past the range fall outside the
      // resources (zeros, no memory access), so they stay unconditional and vmcnt exact.
      f32x4 xa[WG_PF], xb[WG_PF];
      if (c < nchunks) {
#pragma unroll
        for (int p = 0; p < WG_PF; ++p) {
          xa[p] = pg_load(ra, va, (c * WG_PF + p) * sa);
          xb[p] = pg_load(rb, vb, (c * WG_PF + p) * sb);
        }
      }
      for (; c < nchunks; c += 4) {
        const int na = (c + 4) * WG_PF * sa, nb = (c + 4) * WG_PF * sb;
        pg_static_for<0, WG_PF>([&](auto I) {
          constexpr int p = decltype(I)::value;
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int d = 0; d < 4; ++d)
              acc[e][d] = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[p][e], xb[p][d], acc[e][d], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
          xa[p] = pg_load(ra, va, na + p * sa);
          xb[p] = pg_load(rb, vb, nb + p * sb);
          __builtin_amdgcn_sched_barrier(0);
        });
      }
    } else {
      // two chunk buffers, each refilled in one burst (16 rows of both operands) right after
      // its MFMAs, one chunk ahead of its use
      f32x4 xa[2][WG_PF], xb[2][WG_PF];
      // buffer indices are compile-time (a runtime index would put the arrays in scratch)
      auto fill = [&](auto B, int ch) {
        constexpr int buf = decltype(B)::value;
#pragma unroll
        for (int p = 0; p < WG_PF; ++p) {
          xa[buf][p] = pg_load(ra, va, (ch * WG_PF + p) * sa);
          xb[buf][p] = pg_load(rb, vb, (ch * WG_PF + p) * sb);
        }
      };
      auto run = [&](auto B) {
        constexpr int buf = decltype(B)::value;
        pg_static_for<0, WG_PF>([&](auto I) {
          constexpr int p = decltype(I)::value;
#pragma unroll
          for (int e = 0; e < 4; ++e)
#pragma unroll
            for (int d = 0; d < 4; ++d)
              acc[e][d] = __builtin_amdgcn_mfma_f32_32x32x2f32(xa[buf][p][e], xb[buf][p][d],
                                                               acc[e][d], 0, 0, 0);
          __builtin_amdgcn_sched_barrier(0);
        });
      };
      constexpr std::integral_constant<int, 0> b0{};
      constexpr std::integral_constant<int, 1> b1{};
      if (c < nchunks) {
        fill(b0, c);
        fill(b1, c + 4);
      }
      for (; c < nchunks; c += 8) {
        run(b0);
        fill(b0, c + 8);
        run(b1);   // unconditional (a branch here doubles the accumulators); the rows per
                   // split are a multiple of 128, so only the last split runs a zero chunk
        fill(b1, c + 12);
      }
    }
  }
  wg_reduce_store(g, acc, red, s, tm, tn);
}

// ---------------------------------------------------------------------------------------
// Split-bf16 weight-gradient GEMM (round 5): wgrad_kernel's workgroup / split / reduction
// scheme on v_mfma_f32_32x32x16_bf16 with the three-term operand split of panel_x6_kernel
// (x6_split, x6_mma: fp32 accuracy, 2.67x the fp32 MFMA rate).  A k block is 16 rows: lane
// (j, h) loads rows 16c + 8h + i (i = 0..7) of gY (out rows 4j .. 4j+3) and of X (out cols
// 4j .. 4j+3), one float4 each; component e of the eight gY float4 is the 8-k A operand of out
// rows {4i + e}, component d of the X ones the B operand of out cols {4j + d} (the fp32
// kernel's permutation, 8 rows deep), each split into three bf16 terms.  Same D layout, so
// the same LDS reduction and split partials.
__device__ __forceinline__ void x6_split8(const float (&v)[8], bf16x8 (&s)[3]) {
  x6_split(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}, s);
}

template <int T>
__global__ __launch_bounds__(256, 1) void wgrad_x6_kernel(WgradArgs g) {
  PNTF_CLOCK_SCOPE;
  __shared__ f32x4 red[2][64 * 64];   // two 128 x 128 tiles (128 KiB)
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b8 = blockIdx.x >> 3;
  const int tile = g.xcd ? b8 % T : blockIdx.x % T;
  const int s = g.xcd ? (blockIdx.x & 7) + 8 * (b8 / T) : blockIdx.x / T;
  const int tnn = g.N / 128, tm = tile / tnn, tn = tile % tnn;
  const int64_t r0 = (int64_t)s * g.rps;
  const int64_t left = g.rows - r0;
  const int64_t nrows = left <= 0 ? 0 : (left < g.rps ? left : g.rps);
  f32x16 acc[4][4];
#pragma unroll
  for (int e = 0; e < 4; ++e)
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[e][d][r] = 0.f;
  if (nrows > 0) {
    // rows past the split's end are outside the resources: their loads return 0
    const Rsrc ra = pg_rsrc(g.A + r0 * g.M, nrows * g.M * 4);
    const Rsrc rb = pg_rsrc(g.B + r0 * g.N, nrows * g.N * 4);
    const int va = (8 * h * g.M + 128 * tm + 4 * j) * 4, vb = (8 * h * g.N + 128 * tn + 4 * j) * 4;
    const int sa = __builtin_amdgcn_readfirstlane(g.M * 4);
    const int sb = __builtin_amdgcn_readfirstlane(g.N * 4);
    const int nchunks = (int)((nrows + 15) / 16);
    int c = w;
    f32x4 xa[2][8], xb[2][8];
    auto fill = [&](auto B, int ch) {
      constexpr int buf = decltype(B)::value;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        xa[buf][i] = pg_load(ra, va, (16 * ch + i) * sa);
        xb[buf][i] = pg_load(rb, vb, (16 * ch + i) * sb);
      }
    };
    auto run = [&](auto B) {
      constexpr int buf = decltype(B)::value;
      bf16x8 bs[4][3];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = xb[buf][i][d];
        x6_split8(v, bs[d]);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = xa[buf][i][e];
        bf16x8 as[3];
        x6_split8(v, as);
#pragma unroll
        for (int d = 0; d < 4; ++d) acc[e][d] = x6_mma(as, bs[d], acc[e][d]);
      }
    };
    constexpr std::integral_constant<int, 0> b0{};
    constexpr std::integral_constant<int, 1> b1{};
    if (c < nchunks) {
      fill(b0, c);
      fill(b1, c + 4);
    }
    // the fences keep each burst of loads right after the MFMAs that free its buffer
    for (; c < nchunks; c += 8) {
      run(b0);
      __builtin_amdgcn_sched_barrier(0);
      fill(b0, c + 8);
      __builtin_amdgcn_sched_barrier(0);
      run(b1);   // unconditional: the rows per split are a multiple of 128 (zero chunks past
                 // the end of the last split)
      __builtin_amdgcn_sched_barrier(0);
      fill(b1, c + 12);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  wg_reduce_store(g, acc, red, s, tm, tn);
}

// fixed-order sum of the four waves' tiles, (w0 + w2) + (w1 + w3), through LDS without
// writing the accumulators back (a read-modify-write of 256 of them spilled): w2, w3 store
// their tiles; w0, w1 add theirs into those in place; then wave w adds the two halves for
// out rows 4i + w and writes them to the split's partial
__device__ __forceinline__ void wg_reduce_store(const WgradArgs& g, const f32x16 (&acc)[4][4],
                                                f32x4 (&red)[2][64 * 64], int s, int tm, int tn) {
  const int lane = threadIdx.x & 63, h = lane >> 5, j = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  auto at = [&](int e, int r) { return (e * 16 + r) * 64 + lane; };
  auto quad = [&](int e, int r) {
    return f32x4{acc[e][0][r], acc[e][1][r], acc[e][2][r], acc[e][3][r]};
  };
  if (w >= 2) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[w - 2][at(e, r)] = quad(e, r);
  }
  __syncthreads();
  if (w < 2) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[w][at(e, r)] += quad(e, r);
  }
  __syncthreads();
  float* out = g.work + (int64_t)s * g.M * g.N + 128 * tn + 4 * j;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = 128 * tm + 4 * ((r & 3) + 8 * (r >> 2) + 4 * h) + w;
    wg_store(out + (int64_t)m * g.N, red[0][at(w, r)] + red[1][at(w, r)]);
  }
}

thread_local char g_err[512] = "";

// CU count of the current device, cached per device (queried on every GEMM otherwise).
int num_cus() {
  static int cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (dev >= 0 && dev < 64 && cache[dev] > 0) return cache[dev];
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    return 256;
  if (dev >= 0 && dev < 64) cache[dev] = cus;
  return cus;
}

// Split-K factor: enough workgroups for 2 per CU, chunks of at least 512 rows of K.
// Tile width: 128 columns.  256 (the A panel read once per row tile, PNTF_GEMM_WIDE=1) halves
// the occupancy and measured 10-20 % slower on the training shapes (tests/diag/gemm_variants.py).
#ifndef PNTF_GEMM_WIDE
#define PNTF_GEMM_WIDE 0
#endif
int tile_n(int64_t M, int64_t N) {
  return PNTF_GEMM_WIDE && N % 256 == 0 && (M + BM - 1) / BM >= 2 * (int64_t)num_cus() ? 256 : 128;
}

int64_t splits_for(int64_t M, int64_t N, int64_t K) {
  const int64_t tiles = ((M + BM - 1) / BM) * (N / tile_n(M, N));
  int64_t s = (2 * (int64_t)num_cus() + tiles - 1) / tiles;
  const int64_t kmax = (K + 511) / 512;
  if (s > kmax) s = kmax;
  if (s > PNTF_GEMM_SPLITS) s = PNTF_GEMM_SPLITS;
  // whole waves of workgroups: 273 splits of a 128x128 gradient put a second workgroup on 17
  // CUs and doubled the kernel's time; round the grid down to a multiple of the CU count
  const int64_t cus = num_cus();
  if (tiles * s > cus) s = (tiles * s / cus) * cus / tiles;
  return s < 1 ? 1 : s;
}

// The panel path serves the forward / input-gradient shapes: K, N ∈ {128, 256}, dense rows,
// beta 0 or 1, 16-byte aligned operands.  PNTF_GEMM_PANEL=0 in the environment turns it off
// (the LDS-tiled kernel then runs every shape; used to compare), 1 selects the register-stream
// panel kernel instead of the LDS one.
bool panel_shape(int64_t N, int64_t K) {
  return (K == 128 || K == 256) && (N == 128 || N == 256);
}
// PNTF_GEMM_PANEL: 0 = off, 1 = the register-stream panel kernel, 2 = the LDS one (fp32 MFMA),
// 3 (default) = the split-bf16 LDS one (panel_x6_kernel).
// pntf_tt_set_panel_mode overrides it (tests and A/B probes).
// (set once from the environment, thread-safely; then only by pntf_tt_set_panel_mode)
std::atomic<int> g_panel_mode{-1};
int mode_from_env(std::atomic<int>& m, const char* var, char hi, int dflt) {
  int v = m.load(std::memory_order_relaxed);
  if (v >= 0) return v;
  const char* e = getenv(var);
  int expect = -1;
  m.compare_exchange_strong(expect, e && e[0] >= '0' && e[0] <= hi ? e[0] - '0' : dflt);
  return m.load(std::memory_order_relaxed);
}
int panel_mode() { return mode_from_env(g_panel_mode, "PNTF_GEMM_PANEL", '8', 3); }
// work floats of the packed weight: fp32 fragments, or three bf16 terms (1.5x)
size_t panel_pack_floats(int64_t N, int64_t K) {
  return panel_mode() >= 3 ? (size_t)(K * N * 3 / 2) : (size_t)(K * N);
}

// The weight-gradient kernel serves gYᵀ·X with M, N ∈ {128, 256} (ta, not tb, beta 0, dense
// 16-byte aligned operands).  PNTF_GEMM_WGRAD=0 in the environment sends those shapes to the
// LDS-tiled split-K kernel instead (used to compare the two).
bool wgrad_shape(int64_t M, int64_t N) {
  return (M == 128 || M == 256) && (N == 128 || N == 256);
}
// PNTF_GEMM_WGRAD: 0 = the LDS-tiled kernel, 1 = wgrad_kernel (fp32 MFMA), 2 (default) =
// wgrad_x6_kernel (split bf16); pntf_tt_set_wgrad_mode overrides it.
std::atomic<int> g_wgrad_mode{-1};
int wgrad_mode() { return mode_from_env(g_wgrad_mode, "PNTF_GEMM_WGRAD", '2', 2); }
bool wgrad_enabled() { return wgrad_mode() != 0; }
// PNTF_GEMM_BWD: the kernel of pntf_tt_linear_bwd: 0 = panel_bwd_coop_kernel (fp32 MFMA), 1
// (default) = panel_bwd_x6_kernel (split bf16)
std::atomic<int> g_bwd_mode{-1};
int bwd_mode() { return mode_from_env(g_bwd_mode, "PNTF_GEMM_BWD", '1', 1); }
// Refill scheme per tile count: the two-buffer burst for the 256 x 256 gradients (T = 4:
// 206 vs 215 µs at 9 x 20 000 rows), the per-slot ring for T = 1, 2 (64 vs 67, 103 vs 106 µs;
// tools/wgrad_prof.sh).  PNTF_WGRAD_RING=1 or 2 forces one of them (to compare).
int wgrad_ring(int T) {
  static const int force = [] {
    const char* e = getenv("PNTF_WGRAD_RING");
    return e && (e[0] == '1' || e[0] == '2') ? e[0] - '0' : 0;
  }();
  return force ? force : (T == 4 ? 2 : 1);
}
// one workgroup per CU over all tiles, at least 256 rows per split
int64_t wgrad_splits(int64_t M, int64_t N, int64_t K) {
  const int64_t T = (M / 128) * (N / 128);
  int64_t s = num_cus() / T;
  const int64_t kmax = (K + 255) / 256;
  if (s > kmax) s = kmax;
  return s < 1 ? 1 : s;
}

}  // namespace pntf_gemm

using namespace pntf_gemm;

extern "C" {

size_t pntf_tt_gemm_work_floats(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const int64_t s = splits_for(M, N, K);
  const size_t split = s > 1 ? (size_t)(s * M * N) : 0;
  // the largest packed layout (the split-bf16 one, 1.5 K·N) whatever the current panel mode,
  // so a buffer sized here stays large enough after pntf_tt_set_panel_mode
  const size_t packed = panel_shape(N, K) ? (size_t)(K * N * 3 / 2) : 0;
  const size_t wgrad = wgrad_shape(M, N) ? (size_t)((wgrad_splits(M, N, K) + 7) * M * N) : 0;
  const size_t big = split > packed ? split : packed;
  return big > wgrad ? big : wgrad;
}

// The panel GEMMs' conditions (C = A·op(B) (+ Cin) on the register-panel / LDS-panel kernels)
static bool panel_path(int ta, int64_t N, int64_t K, int64_t lda, int64_t ldc, float beta,
                       const float* A, const float* C, const float* work, size_t work_floats) {
  return !ta && (beta == 0.f || beta == 1.f) && panel_shape(N, K) && panel_mode() != 0 &&
         lda == K && ldc == N && work && work_floats >= panel_pack_floats(N, K) &&
         ((uintptr_t)A & 15) == 0 && ((uintptr_t)C & 15) == 0 && ((uintptr_t)work & 15) == 0;
}

static int tt_gemm(int ta, int tb, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                   const float* B, int64_t ldb, float* C, int64_t ldc, float beta, float* work,
                   size_t work_floats, hipStream_t stream, const float* Cin,
                   const float* bias = nullptr, int64_t brows = 0);

int pntf_tt_gemm(int ta, int tb, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                 const float* B, int64_t ldb, float* C, int64_t ldc, float beta, float* work,
                 size_t work_floats, hipStream_t stream) {
  return tt_gemm(ta, tb, M, N, K, A, lda, B, ldb, C, ldc, beta, work, work_floats, stream, C);
}

int pntf_tt_set_panel_mode(int mode) {
  const int prev = panel_mode();
  if (mode >= 0 && mode <= 8) g_panel_mode = mode;
  return prev;
}

int pntf_tt_set_wgrad_mode(int mode) {
  const int prev = wgrad_mode();
  if (mode >= 0 && mode <= 2) g_wgrad_mode = mode;
  return prev;
}

int pntf_tt_set_bwd_mode(int mode) {
  const int prev = bwd_mode();
  if (mode >= 0 && mode <= 1) g_bwd_mode = mode;
  return prev;
}

extern "C" int pntf_tt_act_fwd_biased(int ndir, int nl, const float* y, float* h, int64_t m,
                                      int w, hipStream_t stream);

// Cin != C (and a bias) only on the LDS panel path (the caller checks panel_path and
// panel_mode): C = A·op(B) (+ bias on rows < brows) + Cin
static int tt_gemm(int ta, int tb, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                   const float* B, int64_t ldb, float* C, int64_t ldc, float beta, float* work,
                   size_t work_floats, hipStream_t stream, const float* Cin, const float* bias,
                   int64_t brows) {
  if (M < 0 || N < 0 || K < 0 || N % BN != 0) {
    snprintf(g_err, sizeof(g_err), "pntf_tt_gemm: need M, K >= 0 and N a multiple of %d", BN);
    return PNTF_ERR_ARG;
  }
  if (M == 0 || N == 0) return PNTF_OK;
  if (!A || !B || !C) {
    snprintf(g_err, sizeof(g_err), "pntf_tt_gemm: null pointer");
    return PNTF_ERR_ARG;
  }
  const int pm = panel_mode();
  if (panel_path(ta, N, K, lda, ldc, beta, A, C, work, work_floats) && pm == 8) {
    // the 16 x 16 x 32 split-bf16 panel kernel, eight waves per workgroup
    const int64_t nf = (N / 16) * (K / 32) * 64;
    hipLaunchKernelGGL(x6s_pack_kernel, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, stream,
                       B, ldb, tb, (int)K, (int)N, reinterpret_cast<bf16x8*>(work));
    PanelArgs p{A, reinterpret_cast<const f32x4*>(work), C, M, lda, ldc, Cin, bias, brows};
    const int64_t tiles = (M + 15) / 16, wgs = (tiles + 7) / 8;
    const int64_t ng = N / X6S_CG, cap = num_cus() / ng;
    int64_t nwg = wgs < cap ? wgs : cap;
    if (ng > 1) nwg = (nwg + 7) / 8 * 8;
    const dim3 grid((unsigned)(nwg * ng));
#define PNTF_PANEL(KC, NC)                                                                      \
  if (beta != 0.f) hipLaunchKernelGGL((panel_x6s_kernel<KC, NC, true>), grid, dim3(512), 0,      \
                                      stream, p);                                               \
  else hipLaunchKernelGGL((panel_x6s_kernel<KC, NC, false>), grid, dim3(512), 0, stream, p);
    if (K == 128 && N == 128) { PNTF_PANEL(128, 128) }
    else if (K == 128) { PNTF_PANEL(128, 256) }
    else if (N == 128) { PNTF_PANEL(256, 128) }
    else { PNTF_PANEL(256, 256) }
#undef PNTF_PANEL
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      snprintf(g_err, sizeof(g_err), "pntf_tt_gemm: %s", hipGetErrorString(e));
      return PNTF_ERR_HIP;
    }
    return PNTF_OK;
  }
  // modes 4 / 5 (diagnostics): the split kernel for the forward (tb) / input-gradient (!tb)
  // GEMMs only; 6 / 7: its accumulation variants V = 0 / 1
  const bool x6 = pm == 3 || pm == 6 || pm == 7 || (pm == 4 && tb) || (pm == 5 && !tb);
  if (panel_path(ta, N, K, lda, ldc, beta, A, C, work, work_floats) && x6) {
    const int64_t nf = (N / 32) * (K / 16) * 64;
    hipLaunchKernelGGL(x6_pack_kernel, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, stream,
                       B, ldb, tb, (int)K, (int)N, reinterpret_cast<bf16x8*>(work));
    PanelArgs p{A, reinterpret_cast<const f32x4*>(work), C, M, lda, ldc, Cin, bias, brows};
    // one workgroup per CU (96 KiB of LDS); per group at most CUs / NG of them, a multiple of
    // 8 with several groups so that a tile's group workgroups share an XCD
    const int64_t tiles = (M + 31) / 32, wgs = (tiles + 3) / 4;
    const int64_t cg = K == 256 ? x6_cg1(256) : x6_cg1(128);
    const int64_t ng = N / cg > 1 ? N / cg : 1;
    const int64_t cap = PNTF_X6_WPS * num_cus() / ng;
    int64_t nwg = wgs < cap ? wgs : cap;
    if (ng > 1) nwg = (nwg + 7) / 8 * 8;
    const dim3 grid((unsigned)(nwg * ng));
#define PNTF_PANEL(KC, NC)                                                                      \
  if (pm == 6) {                                                                                \
    if (beta != 0.f) hipLaunchKernelGGL((panel_x6_kernel<KC, NC, true, 0>), grid, dim3(256), 0,  \
                                        stream, p);                                             \
    else hipLaunchKernelGGL((panel_x6_kernel<KC, NC, false, 0>), grid, dim3(256), 0, stream, p); \
  } else if (pm == 7) {                                                                         \
    if (beta != 0.f) hipLaunchKernelGGL((panel_x6_kernel<KC, NC, true, 1>), grid, dim3(256), 0,  \
                                        stream, p);                                             \
    else hipLaunchKernelGGL((panel_x6_kernel<KC, NC, false, 1>), grid, dim3(256), 0, stream, p); \
  } else if (beta != 0.f) hipLaunchKernelGGL((panel_x6_kernel<KC, NC, true>), grid, dim3(256), 0, \
                                             stream, p);                                        \
  else hipLaunchKernelGGL((panel_x6_kernel<KC, NC, false>), grid, dim3(256), 0, stream, p);
    if (K == 128 && N == 128) { PNTF_PANEL(128, 128) }
    else if (K == 128) { PNTF_PANEL(128, 256) }
    else if (N == 128) { PNTF_PANEL(256, 128) }
    else { PNTF_PANEL(256, 256) }
#undef PNTF_PANEL
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      snprintf(g_err, sizeof(g_err), "pntf_tt_gemm: %s", hipGetErrorString(e));
      return PNTF_ERR_HIP;
    }
    return PNTF_OK;
  }
  if (panel_path(ta, N, K, lda, ldc, beta, A, C, work, work_floats)) {
    const int64_t nf = (N / 32) * (K / 8) * 64;
    hipLaunchKernelGGL(panel_pack_kernel, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0,
                       stream, B, ldb, tb, (int)K, (int)N, reinterpret_cast<f32x4*>(work));
    PanelArgs p{A, reinterpret_cast<const f32x4*>(work), C, M, lda, ldc, Cin, bias, brows};
    const int64_t tiles = (M + 31) / 32, wgs = (tiles + 3) / 4;
    if (panel_mode() >= 2) {
      // one workgroup per CU (128 KiB of LDS at K = 256); per group at most CUs / NG of them
      // a multiple of 8 so that a tile's two group workgroups share an XCD (N = 256)
      // (K = 128 without C: 64 KiB of LDS and ≤ 256 registers, so two per CU)
      const int64_t ng = N / 128, cap = (K == 128 && beta == 0.f ? 2 : 1) * num_cus() / ng;
      int64_t nwg = wgs < cap ? wgs : cap;
      if (ng == 2) nwg = (nwg + 7) / 8 * 8;
      const dim3 grid((unsigned)(nwg * ng));
#define PNTF_PANEL(KC, NC)                                                                      \
  if (beta != 0.f) hipLaunchKernelGGL((panel_lds_kernel<KC, NC, true>), grid, dim3(256), 0,      \
                                      stream, p);                                               \
  else hipLaunchKernelGGL((panel_lds_kernel<KC, NC, false>), grid, dim3(256), 0, stream, p);
      if (K == 128 && N == 128) { PNTF_PANEL(128, 128) }
      else if (K == 128) { PNTF_PANEL(128, 256) }
      else if (N == 128) { PNTF_PANEL(256, 128) }
      else { PNTF_PANEL(256, 256) }
#undef PNTF_PANEL
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "pntf_tt_gemm: %s", hipGetErrorString(e));
        return PNTF_ERR_HIP;
      }
      return PNTF_OK;
    }
    const int64_t slots = (int64_t)PNTF_PANEL_WPS * num_cus();
    const unsigned grid = (unsigned)(wgs < slots ? wgs : slots);
#define PNTF_PANEL(KC, NC)                                                                     \
  if (beta != 0.f) hipLaunchKernelGGL((panel_gemm_kernel<KC, NC, true>), dim3(grid), dim3(256), \
                                      0, stream, p);                                           \
  else hipLaunchKernelGGL((panel_gemm_kernel<KC, NC, false>), dim3(grid), dim3(256), 0, stream, p);
    if (K == 128 && N == 128) { PNTF_PANEL(128, 128) }
    else if (K == 128) { PNTF_PANEL(128, 256) }
    else if (N == 128) { PNTF_PANEL(256, 128) }
    else { PNTF_PANEL(256, 256) }
#undef PNTF_PANEL
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      snprintf(g_err, sizeof(g_err), "pntf_tt_gemm: %s", hipGetErrorString(e));
      return PNTF_ERR_HIP;
    }
    return PNTF_OK;
  }
  if (ta && !tb && beta == 0.f && K > 0 && wgrad_shape(M, N) && wgrad_enabled() && lda == M &&
      ldb == N && work && ((uintptr_t)A & 15) == 0 && ((uintptr_t)B & 15) == 0 &&
      ((uintptr_t)work & 15) == 0) {
    // rows per split: a multiple of 128 (4 waves x two 16-row chunks); the buffer offsets are
    // 32-bit, so a split must stay below 2 GiB of either operand
    const int64_t s0 = wgrad_splits(M, N, K);
    int64_t rps = ((K + s0 - 1) / s0 + 127) / 128 * 128;
    int64_t s = (K + rps - 1) / rps;
    // XCD-aware map: pad the split count to a multiple of 8 (empty splits write zeros)
    const bool xcd = (M / 128) * (N / 128) > 1 && s >= 8;
    if (xcd) s = (s + 7) / 8 * 8;
    if (rps * (M > N ? M : N) * 4 < ((int64_t)1 << 31) - ((int64_t)1 << 20) &&
        work_floats >= (size_t)(s * M * N)) {
      const int T = (int)((M / 128) * (N / 128));
      WgradArgs wa{A, B, work, K, rps, (int)M, (int)N, (int)xcd};
      const dim3 grid((unsigned)(s * T));
#define PNTF_WGRAD(NB)                                                                          \
  if (T == 1) hipLaunchKernelGGL((wgrad_kernel<1, NB>), grid, dim3(256), 0, stream, wa);         \
  else if (T == 2) hipLaunchKernelGGL((wgrad_kernel<2, NB>), grid, dim3(256), 0, stream, wa);    \
  else hipLaunchKernelGGL((wgrad_kernel<4, NB>), grid, dim3(256), 0, stream, wa);
      if (wgrad_mode() == 2) {
        if (T == 1) hipLaunchKernelGGL((wgrad_x6_kernel<1>), grid, dim3(256), 0, stream, wa);
        else if (T == 2) hipLaunchKernelGGL((wgrad_x6_kernel<2>), grid, dim3(256), 0, stream, wa);
        else hipLaunchKernelGGL((wgrad_x6_kernel<4>), grid, dim3(256), 0, stream, wa);
      } else if (wgrad_ring(T) == 2) { PNTF_WGRAD(2) } else { PNTF_WGRAD(1) }
#undef PNTF_WGRAD
      const int64_t n = M * N;
      const unsigned nb = (unsigned)((n + 255) / 256);
      hipLaunchKernelGGL(gemm_reduce1_kernel, dim3(nb, (unsigned)((s + RG - 1) / RG)),
                         dim3(256), 0, stream, work, (int)s, n);
      hipLaunchKernelGGL(gemm_reduce2_kernel, dim3(nb), dim3(256), 0, stream, work, (int)s, M,
                         N, C, ldc, beta);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) {
        snprintf(g_err, sizeof(g_err), "pntf_tt_gemm: %s", hipGetErrorString(e));
        return PNTF_ERR_HIP;
      }
      return PNTF_OK;
    }
  }
  // the LDS-tiled kernel puts the row tiles on grid.y (HIP limit 65535): M above
  // 65535 * 128 ≈ 8.4M rows cannot launch there (the panel path above has no such limit)
  if ((M + BM - 1) / BM > 65535) {
    snprintf(g_err, sizeof(g_err),
             "pntf_tt_gemm: M = %lld rows exceeds the LDS-tiled kernel's grid (65535 x %d); "
             "use the panel path (ta = 0, K, N in {128, 256}, beta 0 or 1, aligned operands)",
             (long long)M, BM);
    return PNTF_ERR_ARG;
  }
  const int64_t s = K > 0 ? splits_for(M, N, K) : 1;
  if (s > 1 && (!work || work_floats < (size_t)(s * M * N))) {
    snprintf(g_err, sizeof(g_err), "pntf_tt_gemm: work buffer too small");
    return PNTF_ERR_WORKSPACE;
  }
  GemmArgs g{A, B, C, work, M, N, K, lda, ldb, ldc, 0, beta};
  g.kper = ((K + s - 1) / s + BK - 1) / BK * BK;
  if (g.kper < BK) g.kper = BK;
  const int bn = tile_n(M, N);
  dim3 grid((unsigned)(N / bn), (unsigned)((M + BM - 1) / BM), (unsigned)s), block(256);
  if (bn == 256) {
    if (ta && tb) hipLaunchKernelGGL((gemm_kernel<true, true, 256>), grid, block, 0, stream, g);
    else if (ta) hipLaunchKernelGGL((gemm_kernel<true, false, 256>), grid, block, 0, stream, g);
    else if (tb) hipLaunchKernelGGL((gemm_kernel<false, true, 256>), grid, block, 0, stream, g);
    else hipLaunchKernelGGL((gemm_kernel<false, false, 256>), grid, block, 0, stream, g);
  } else {
    if (ta && tb) hipLaunchKernelGGL((gemm_kernel<true, true, 128>), grid, block, 0, stream, g);
    else if (ta) hipLaunchKernelGGL((gemm_kernel<true, false, 128>), grid, block, 0, stream, g);
    else if (tb) hipLaunchKernelGGL((gemm_kernel<false, true, 128>), grid, block, 0, stream, g);
    else hipLaunchKernelGGL((gemm_kernel<false, false, 128>), grid, block, 0, stream, g);
  }
  if (s > 1) {
    const int64_t n = M * N;
    const unsigned nb = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(gemm_reduce1_kernel, dim3(nb, (unsigned)((s + RG - 1) / RG)), dim3(256),
                       0, stream, work, (int)s, n);
    hipLaunchKernelGGL(gemm_reduce2_kernel, dim3(nb), dim3(256), 0, stream, work, (int)s, M, N,
                       C, ldc, beta);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "pntf_tt_gemm: %s", hipGetErrorString(e));
    return PNTF_ERR_HIP;
  }
  return PNTF_OK;
}

// pntf_train.hip defines the plane check (its with_planes list); this weak copy of the list
// only serves a standalone build of this file (tests/diag/build_gemm.sh)
extern "C" __attribute__((weak, visibility("hidden"))) int pntf_tt_planes_ok(int ndir, int nl) {
  const int ok[][2] = {{0, 0}, {3, 1}, {6, 1}, {6, 2}, {12, 2}, {3, 0},
                       {6, 0}, {12, 0}, {3, 3}, {6, 6}, {12, 12}};
  for (const auto& p : ok)
    if (p[0] == ndir && p[1] == nl) return 1;
  return 0;
}

int pntf_tt_linear_act(int ndir, int nl, const float* x, int64_t m, int k, const float* W,
                       int n, const float* bias, const float* res, float* y, float* h, int act,
                       int schedule, float* work, size_t work_floats, hipStream_t stream) {
  // the fused kernels take the Loss / value tapes' layouts; the first-order and per-direction
  // layouts of the general VJP tape (and act = 2, the out_backgrad quirk) run the GEMM + act pair
  const bool basic = ((nl == 0 && ndir == 0) || (nl == 1 && (ndir == 3 || ndir == 6)) ||
                      (nl == 2 && (ndir == 6 || ndir == 12))) && act != 2;
  const bool planes = pntf_tt_planes_ok(ndir, nl) && act >= 0 && act <= 2;
  const auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!planes || m < 0 || !panel_shape(n, k) || (m > 0 && (!x || !W || !bias || !y || !work ||
      (act && !h))) || (res && !act) || work_floats < (size_t)k * n ||
      !al(x) || !al(bias) || !al(res) || !al(y) || !al(h) || !al(work)) {
    snprintf(g_err, sizeof(g_err), "pntf_tt_linear_act: bad arguments");
    return PNTF_ERR_ARG;
  }
  if (schedule < 0 || schedule > 3) {
    snprintf(g_err, sizeof(g_err), "pntf_tt_linear_act: unknown schedule");
    return PNTF_ERR_ARG;
  }
  if (m == 0) return PNTF_OK;
  const int R = 1 + ndir + nl;
  // A wave of the fused kernel owns whole 32-point blocks (all R planes), so it balances only
  // when every wave gets about the same number of blocks: at the reference batch (625 blocks
  // of the generator's 20 000 points on 512 waves per column group) a fifth of the waves
  // would run two blocks and the rest one.  AUTO takes the fused kernel when the blocks fill
  // their rounds to >= 90 %, otherwise the GEMM (32-row tiles of every plane, balanced) and
  // the act kernel.
  const int64_t blocks = (m + 31) / 32, wgs = (blocks + 3) / 4;
  const int64_t ng = n / 128, cap = num_cus() / ng;
  int64_t nwg = wgs < cap ? wgs : cap;
  if (ng == 2) nwg = (nwg + 7) / 8 * 8;
  const int64_t waves = 4 * nwg, rounds = (blocks + waves - 1) / waves;
  // (and only with several rounds per wave: at one round, generator[3] of the reference batch,
  // the fused kernel measured 227 µs against 132 + 56 for the pair, profiles/r04_train_*)
  // (AUTO keeps the pair whenever the split-bf16 GEMM runs: the fused kernels are fp32 MFMA;
  // 2 x 100 000 pairs 57.6 ms with the pair vs 60.7 fused, profiles/r05_train_sched.txt)
  const bool fused = basic && (schedule == 1 || schedule == 3 ||
                     (schedule == 0 && panel_mode() < 3 && rounds >= 3 &&
                      10 * blocks >= 9 * rounds * waves));
  if (!fused) {
    // the residual enters the GEMM's epilogue (y = x·Wᵀ + res, its C read 4 iterations ahead),
    // so the act pass reads y and writes h instead of reading y and res and writing both back
    if (res && (nl > 0 || ndir > 0) && panel_mode() >= 2 &&
        panel_path(0, n, k, k, n, 1.f, x, y, work, work_floats)) {
      int st = tt_gemm(0, 1, R * m, n, k, x, k, W, k, y, n, 1.f, work, work_floats, stream, res,
                       bias, m);
      if (st) return st;
      return pntf_tt_act_fwd_biased(ndir, nl, y, h, m, n, stream);
    }
    int st = pntf_tt_gemm(0, 1, R * m, n, k, x, k, W, k, y, n, 0.f, work, work_floats, stream);
    if (st) return st;
    return pntf_tt_act_fwd(ndir, nl, y, h, bias, res, m, n, act, stream);
  }
  const int64_t nf = (int64_t)(n / 32) * (k / 8) * 64;
  hipLaunchKernelGGL(panel_pack_kernel, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0,
                     stream, W, (int64_t)k, 1, k, n, reinterpret_cast<f32x4*>(work));
  ActArgs a{x, reinterpret_cast<const f32x4*>(work), y, h, bias, res, m, R, ndir, nl, act};
  if (schedule == 3) {
    // cooperative blocks: one workgroup per CU and column group, each striding over blocks
    int64_t cw = blocks < cap ? blocks : cap;
    if (ng == 2) cw = (cw + 7) / 8 * 8;
    const dim3 cg((unsigned)(cw * ng));
    if (k == 128 && n == 128) hipLaunchKernelGGL((panel_act_coop_kernel<128, 128>), cg, dim3(256), 0, stream, a);
    else if (k == 128) hipLaunchKernelGGL((panel_act_coop_kernel<128, 256>), cg, dim3(256), 0, stream, a);
    else if (n == 128) hipLaunchKernelGGL((panel_act_coop_kernel<256, 128>), cg, dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((panel_act_coop_kernel<256, 256>), cg, dim3(256), 0, stream, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      snprintf(g_err, sizeof(g_err), "pntf_tt_linear_act: %s", hipGetErrorString(e));
      return PNTF_ERR_HIP;
    }
    return PNTF_OK;
  }
  // as the LDS panel GEMM: one workgroup per CU per column group (a multiple of 8 workgroups
  // per group for two groups); each wave strides over 32-point blocks
  const dim3 grid((unsigned)(nwg * ng));
  if (k == 128 && n == 128) hipLaunchKernelGGL((panel_act_kernel<128, 128>), grid, dim3(256), 0, stream, a);
  else if (k == 128) hipLaunchKernelGGL((panel_act_kernel<128, 256>), grid, dim3(256), 0, stream, a);
  else if (n == 128) hipLaunchKernelGGL((panel_act_kernel<256, 128>), grid, dim3(256), 0, stream, a);
  else hipLaunchKernelGGL((panel_act_kernel<256, 256>), grid, dim3(256), 0, stream, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "pntf_tt_linear_act: %s", hipGetErrorString(e));
    return PNTF_ERR_HIP;
  }
  return PNTF_OK;
}

size_t pntf_tt_linear_bwd_work_floats(int kc, int nc) {
  // either kernel: the packed weight (fp32, or three bf16 terms = 1.5x) and the bias partials
  // (one row per workgroup, or per point-block pair of a split-bf16 workgroup: <= 2 CUs + 16)
  return (size_t)kc * nc * 3 / 2 + (2 * (size_t)num_cus() + 16) * nc;
}

int pntf_tt_linear_bwd(int ndir, int nl, const float* gy, int64_t m, int kc, const float* W,
                       int nc, const float* yprev, const float* res, float* out, float* gbias,
                       float* work, size_t work_floats, hipStream_t stream) {
  const bool planes = (nl == 0 && ndir == 0) || (nl == 1 && (ndir == 3 || ndir == 6)) ||
                      (nl == 2 && (ndir == 6 || ndir == 12));
  const auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!planes || m < 0 || !panel_shape(nc, kc) || !gbias ||
      (m > 0 && (!gy || !W || !yprev || !out || !work)) ||
      work_floats < pntf_tt_linear_bwd_work_floats(kc, nc) || !al(gy) || !al(yprev) ||
      !al(res) || !al(out) || !al(work)) {
    snprintf(g_err, sizeof(g_err), "pntf_tt_linear_bwd: bad arguments");
    return PNTF_ERR_ARG;
  }
  if (m == 0) {
    hipMemsetAsync(gbias, 0, nc * sizeof(float), stream);
    return PNTF_OK;
  }
  const int R = 1 + ndir + nl;
  if (bwd_mode() == 1) {
    const int64_t nf = (int64_t)(nc / 32) * (kc / 16) * 64;
    hipLaunchKernelGGL(x6_pack_kernel, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0, stream,
                       W, (int64_t)nc, 0, kc, nc, reinterpret_cast<bf16x8*>(work));
    float* partial = work + (size_t)kc * nc * 3 / 2;
    // one workgroup per CU (96 KiB of LDS), each on two 32-point blocks at a time; per 64-column
    // group at most CUs / NG of them, a multiple of 8 so a block's group workgroups share an XCD
    const int64_t pairs = ((m + 31) / 32 + 1) / 2, ng = nc / 64, cap = num_cus() / ng;
    int64_t cw = pairs < cap ? pairs : cap;
    cw = (cw + 7) / 8 * 8;
    BwdArgs a{gy, reinterpret_cast<const f32x4*>(work), yprev, res, out, partial, m, R, ndir, nl};
    const dim3 cg((unsigned)(cw * ng));
    if (kc == 128 && nc == 128) hipLaunchKernelGGL((panel_bwd_x6_kernel<128, 128>), cg, dim3(256), 0, stream, a);
    else if (kc == 128) hipLaunchKernelGGL((panel_bwd_x6_kernel<128, 256>), cg, dim3(256), 0, stream, a);
    else if (nc == 128) hipLaunchKernelGGL((panel_bwd_x6_kernel<256, 128>), cg, dim3(256), 0, stream, a);
    else hipLaunchKernelGGL((panel_bwd_x6_kernel<256, 256>), cg, dim3(256), 0, stream, a);
    hipLaunchKernelGGL(colsum_kernel, dim3((nc + 255) / 256), dim3(256), 0, stream, partial,
                       (int)(2 * cw), nc, gbias);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      snprintf(g_err, sizeof(g_err), "pntf_tt_linear_bwd: %s", hipGetErrorString(e));
      return PNTF_ERR_HIP;
    }
    return PNTF_OK;
  }
  const int64_t nf = (int64_t)(nc / 32) * (kc / 8) * 64;
  hipLaunchKernelGGL(panel_pack_kernel, dim3((unsigned)((nf + 255) / 256)), dim3(256), 0,
                     stream, W, (int64_t)nc, 0, kc, nc, reinterpret_cast<f32x4*>(work));
  float* partial = work + (size_t)kc * nc;
  const int64_t blocks = (m + 31) / 32, ng = nc / 128, cap = num_cus() / ng;
  int64_t cw = blocks < cap ? blocks : cap;
  if (ng == 2) cw = (cw + 7) / 8 * 8;
  BwdArgs a{gy, reinterpret_cast<const f32x4*>(work), yprev, res, out, partial, m, R, ndir, nl};
  const dim3 cg((unsigned)(cw * ng));
  if (kc == 128 && nc == 128) hipLaunchKernelGGL((panel_bwd_coop_kernel<128, 128>), cg, dim3(256), 0, stream, a);
  else if (kc == 128) hipLaunchKernelGGL((panel_bwd_coop_kernel<128, 256>), cg, dim3(256), 0, stream, a);
  else if (nc == 128) hipLaunchKernelGGL((panel_bwd_coop_kernel<256, 128>), cg, dim3(256), 0, stream, a);
  else hipLaunchKernelGGL((panel_bwd_coop_kernel<256, 256>), cg, dim3(256), 0, stream, a);
  hipLaunchKernelGGL(colsum_kernel, dim3((nc + 255) / 256), dim3(256), 0, stream, partial,
                     (int)cw, nc, gbias);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "pntf_tt_linear_bwd: %s", hipGetErrorString(e));
    return PNTF_ERR_HIP;
  }
  return PNTF_OK;
}

const char* pntf_tt_gemm_last_error(void) { return g_err; }

}  // extern "C"
