// fp32 GEMMs of the training step (pntf/train.py) on v_mfma_f32_32x32x2_f32, replacing the
// library GEMMs the Taylor tape used: per Linear of NN.out_laplace (model_res_sigmoid_multi.py
// :710-848, differentiated by loss.backward() at :1048)
//   forward          Y (rows x N)  = X (rows x K) · Wᵀ          (A row-major, B = Wᵀ)
//   input gradient   gX (rows x K) (+)= gY (rows x N) · W       (A row-major, B row-major)
//   weight gradient  gW (N x K)    = gYᵀ · X  over all rows     (A = gYᵀ, B row-major, split-K)
// C = beta·C + A·B with A(m, k) = TA ? A[k·lda + m] : A[m·lda + k] and
// B(k, n) = TB ? B[n·ldb + k] : B[k·ldb + n].
//
// Workgroup tile 128 x 128, K chunks of 8 staged through LDS (double-buffered, one barrier per
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

#include "pntf.h"

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
// Forward Linear of the Taylor tape fused with its epilogue (pntf_tt_linear_act): per point
// and feature, y planes = x planes · Wᵀ, y₀ += bias, (+ residual planes), then act_laplace
// (:675-691) h₀ = softplus₁₀(y₀), h_J = σ·J, h_L = σ'·J² + σ·L — the work of pntf_tt_gemm +
// pntf_tt_act_fwd without the round trip of y through HBM between them.
// The workgroup's row tile is 32 points × all R planes (R = 1 + 2·ndir ≤ 13), one 32 x 32
// MFMA row block per plane, so every plane of a (point, feature) lands in the same lane and
// register of R different accumulators and the cross-plane epilogue runs in registers.
// 4 waves × 32 features = 128 columns per workgroup; K chunks of 16 through LDS (A stored
// [k][plane][point]: R odd makes the row stride ≡ 32 mod 64, conflict-free).
constexpr float TT_SCALE = 10.f;   // Softplus beta (model_res_sigmoid_multi.py:140)
__device__ __forceinline__ float tt_sig10(float y) { return 1.f / (1.f + expf(-TT_SCALE * y)); }
__device__ __forceinline__ float tt_softplus10(float y) {
  return TT_SCALE * y > 20.f ? y : log1pf(expf(TT_SCALE * y)) / TT_SCALE;
}

struct LinArgs {
  const float* x;      // (R, M, K)
  const float* w;      // (N, K)
  const float* bias;   // (N)
  const float* res;    // (R, M, N) or null
  float* y;            // (R, M, N): pre-activation (the tape)
  float* h;            // (R, M, N): activation (ACT)
  int64_t M;
  int N, K;
};

template <int NDIR, bool ACT, bool RES>
__global__ __launch_bounds__(256, 1) void tt_linear_act_kernel(LinArgs a) {
  constexpr int R = 1 + 2 * NDIR, LK = 16;
  constexpr int AS = R * 32, BS = 160;   // LDS row strides per k (floats)
  static_assert(R % 2 == 1, "plane count odd: conflict-free A rows");
  __shared__ float As[2][LK * AS];
  __shared__ float Bs[2][LK * BS];
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int64_t p0 = (int64_t)blockIdx.x * 32;
  const int n0 = blockIdx.y * 128;
  const int64_t plane_x = a.M * a.K, plane_y = a.M * a.N;
  constexpr int NA = (R * 32 * LK / 4 + 255) / 256;   // float4 loads per thread: A
  f32x4 ra[NA], rb[2];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = t + 256 * i;   // (plane b, k4, point p), p fastest
      const int p = idx & 31, k4 = (idx >> 5) & 3, b = idx >> 7;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (b < R && p0 + p < a.M)
        v = *reinterpret_cast<const f32x4*>(a.x + b * plane_x + (p0 + p) * a.K + k0 + 4 * k4);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = t + 256 * i;   // (k4, column n), n fastest
      const int n = idx & 127, k4 = idx >> 7;
      rb[i] = *reinterpret_cast<const f32x4*>(a.w + (int64_t)(n0 + n) * a.K + k0 + 4 * k4);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int idx = t + 256 * i;
      const int p = idx & 31, k4 = (idx >> 5) & 3, b = idx >> 7;
      if (b < R)
#pragma unroll
        for (int e = 0; e < 4; ++e) As[buf][(4 * k4 + e) * AS + b * 32 + p] = ra[i][e];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int idx = t + 256 * i;
      const int n = idx & 127, k4 = idx >> 7;
#pragma unroll
      for (int e = 0; e < 4; ++e) Bs[buf][(4 * k4 + e) * BS + n] = rb[i][e];
    }
  };

  f32x16 acc[R];
#pragma unroll
  for (int b = 0; b < R; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[b][r] = 0.f;
  const int nchunks = a.K / LK;
  gload(0);
  lstore(0);
  __syncthreads();
  const int m = lane & 31, kh = lane >> 5, bn = 32 * w + m;
  for (int c = 0; c < nchunks; ++c) {
    const int buf = c & 1;
    const bool more = c + 1 < nchunks;
    if (more) gload((c + 1) * LK);
    float av[LK / 2][R], bv[LK / 2];
#pragma unroll
    for (int kk = 0; kk < LK / 2; ++kk) {
      const int kr = 2 * kk + kh;
#pragma unroll
      for (int b = 0; b < R; ++b) av[kk][b] = As[buf][kr * AS + b * 32 + m];
      bv[kk] = Bs[buf][kr * BS + bn];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < LK / 2; ++kk)
#pragma unroll
      for (int b = 0; b < R; ++b)
        acc[b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[kk][b], bv[kk], acc[b], 0, 0, 0);
    if (more) lstore(buf ^ 1);
    __syncthreads();
  }

  // epilogue: lane (point row of register r, feature n)
  const int n = n0 + bn;
  const float bias = a.bias[n];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t p = p0 + (r & 3) + 8 * (r >> 2) + 4 * kh;
    if (p >= a.M) continue;
    const int64_t o = p * a.N + n;
    float v0 = acc[0][r] + bias;
    if (RES) v0 += a.res[o];
    a.y[o] = v0;
    if (!ACT) {
#pragma unroll
      for (int b = 1; b < R; ++b) a.y[b * plane_y + o] = acc[b][r];
      continue;
    }
    const float s = tt_sig10(v0), ds = TT_SCALE * s * (1.f - s);
    a.h[o] = tt_softplus10(v0);
#pragma unroll
    for (int k = 0; k < NDIR; ++k) {
      const int64_t oJ = (1 + k) * plane_y + o, oL = (1 + NDIR + k) * plane_y + o;
      float J = acc[1 + k][r], L = acc[1 + NDIR + k][r];
      if (RES) {
        J += a.res[oJ];
        L += a.res[oL];
      }
      a.y[oJ] = J;
      a.y[oL] = L;
      a.h[oJ] = J * s;
      a.h[oL] = J * J * ds + L * s;
    }
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

// Split-K factor: enough workgroups for 2 per CU, chunks of at least 1024 rows of K.
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
  const int64_t kmax = (K + 1023) / 1024;
  if (s > kmax) s = kmax;
  if (s > PNTF_GEMM_SPLITS) s = PNTF_GEMM_SPLITS;
  return s < 1 ? 1 : s;
}

}  // namespace pntf_gemm

using namespace pntf_gemm;

extern "C" {

size_t pntf_tt_gemm_work_floats(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const int64_t s = splits_for(M, N, K);
  return s > 1 ? (size_t)(s * M * N) : 0;
}

int pntf_tt_gemm(int ta, int tb, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                 const float* B, int64_t ldb, float* C, int64_t ldc, float beta, float* work,
                 size_t work_floats, hipStream_t stream) {
  if (M < 0 || N < 0 || K < 0 || N % BN != 0) {
    snprintf(g_err, sizeof(g_err), "pntf_tt_gemm: need M, K >= 0 and N a multiple of %d", BN);
    return PNTF_ERR_ARG;
  }
  if (M == 0 || N == 0) return PNTF_OK;
  if (!A || !B || !C) {
    snprintf(g_err, sizeof(g_err), "pntf_tt_gemm: null pointer");
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

const char* pntf_tt_gemm_last_error(void) { return g_err; }

int pntf_tt_linear_act(int ndir, const float* x, int64_t m, int k, const float* w, int n,
                       const float* bias, const float* res, int act, float* y, float* h,
                       hipStream_t stream) {
  if ((ndir != 3 && ndir != 6) || m < 0 || k % 16 != 0 || k <= 0 || n % 128 != 0 || n <= 0 ||
      (res && !act) || (m > 0 && (!x || !w || !bias || !y || (act && !h)))) {
    snprintf(g_err, sizeof(g_err), "pntf_tt_linear_act: bad arguments");
    return PNTF_ERR_ARG;
  }
  if (m == 0) return PNTF_OK;
  LinArgs a{x, w, bias, res, y, h, m, n, k};
  dim3 grid((unsigned)((m + 31) / 32), (unsigned)(n / 128)), block(256);
#define PNTF_LIN(ND)                                                                         \
  if (res) hipLaunchKernelGGL((tt_linear_act_kernel<ND, true, true>), grid, block, 0, stream, a); \
  else if (act) hipLaunchKernelGGL((tt_linear_act_kernel<ND, true, false>), grid, block, 0,   \
                                   stream, a);                                                \
  else hipLaunchKernelGGL((tt_linear_act_kernel<ND, false, false>), grid, block, 0, stream, a);
  if (ndir == 3) { PNTF_LIN(3) }
  else { PNTF_LIN(6) }
#undef PNTF_LIN
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "pntf_tt_linear_act: %s", hipGetErrorString(e));
    return PNTF_ERR_HIP;
  }
  return PNTF_OK;
}

}  // extern "C"
