// Training step of P-NTFields on MI355X: the weight gradient of the
// Eikonal residual loss, i.e. what `loss.backward()` computes inside Model.train
// (models/model_res_sigmoid_multi.py:1040-1052; arm models/model_res_sigmoid.py:1062-1075),
// plus the AdamW update of the reference's optimizer (:959-961).
//
// Design ("Taylor tape"): the Taylor-mode forward of NN.out_laplace (:710-848)
// is run layer by layer and every pre-activation is kept in HBM, then the reverse sweep
// walks the tape back.  The loss only needs each endpoint's Laplacian Δ_eτ = Σ_{d∈e} ∂²τ/∂x_d²
// (Model.Loss :919-920), and the diagonal second-derivative rows enter every layer linearly
// (Linear: L' = A L; act: L' = σ'J² + σL; merge: L_M = s0 L + c J², ...), so the tape carries
// their SUM per endpoint instead of one row per direction: a Taylor tensor of M points and
// width W is R = 1 + ndir + nl planes (R, M, W) = [value | ndir first-derivative rows | nl
// summed second-derivative rows], (ndir, nl) = (dim, 1) in the encoder and (2·dim, 2) after the
// start/goal merge ([∂x_start (dim) | ∂x_goal (dim) | Σ∂²x_start | Σ∂²x_goal]).  The loss
// and its gradient are those of the reference's per-direction rows (the sums commute with
// every operation); the Linear layers do 9 instead of 13 row GEMMs per pair (dim 3).  With
// that layout every Linear of the graph is ONE plain fp32 GEMM over R·M rows (pntf_gemm.hip),
// the bias touching plane 0 only, and everything between the GEMMs is a fused elementwise
// kernel here — one HBM pass per layer where the reference issues ~10 torch ops:
//   tt_fourier_kernel   input_mapping_laplace (:199-213)           Φ planes
//   tt_act_fwd_kernel   bias + act_laplace (:675-691)              y (saved), h planes
//   tt_act_bwd_kernel   adjoint of act_laplace + bias gradient     g_y planes
//   tt_merge_fwd/bwd    logsumexp merge of start/goal (:761-811) and its adjoint
//   tt_head_loss_kernel generator[4] + actout_laplace (:693-708) + Model.Loss (:897-946)
//                       forward AND backward per pair: diff, g of generator[3]'s output
//   reduce_kernel       deterministic column sums of per-block partials (bias gradients)
//   adamw_kernel        torch.optim.AdamW single-tensor update
// All kernels are HBM-bound; they are written for coalesced 1-float-per-lane plane access
// (consecutive lanes = consecutive features of one point) with grid-stride loops.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>

#include <type_traits>

#include "pntf.h"

namespace {

template <int V>
using IC = std::integral_constant<int, V>;

// The Taylor layouts (ndir, nl) of the tapes, R = 1 + ndir + nl planes per point:
//   (0, 0)                  value only (the weight gradient of a loss on NN.out's τ)
//   (dim, 0) / (2dim, 0)    + first derivatives (NN.out_grad / out_backgrad, Model.gradient
//                           with create_graph: a loss on ∇τ)
//   (dim, 1) / (2dim, 2)    + the per-endpoint SUM of the second derivatives (Model.Loss)
//   (dim, dim) / (2dim, 2dim) + one second-derivative row per direction (NN.out_laplace's
//                           diagonal ∇²τ under a general upstream gradient)
// encoder / after the start-goal merge.  with_planes calls f(IC<ndir>, IC<nl>).
template <class F>
bool with_planes(int ndir, int nl, F&& f) {
#define PNTF_PL(N, L)              \
  if (ndir == N && nl == L) {      \
    f(IC<N>{}, IC<L>{});           \
    return true;                   \
  }
  PNTF_PL(0, 0) PNTF_PL(3, 1) PNTF_PL(6, 1) PNTF_PL(6, 2) PNTF_PL(12, 2)
  PNTF_PL(3, 0) PNTF_PL(6, 0) PNTF_PL(12, 0) PNTF_PL(3, 3) PNTF_PL(6, 6) PNTF_PL(12, 12)
#undef PNTF_PL
  return false;
}

constexpr int H = 128;
constexpr float SCALE = 10.f;               // Softplus beta (model_res_sigmoid_multi.py:140)
constexpr float TWO_PI = 6.283185307179586f;
constexpr int NB_MAX = 512;                 // partial-sum blocks of the reductions (2/CU)

thread_local char g_err[512] = "";

int fail(const char* what) {
  snprintf(g_err, sizeof(g_err), "%s", what);
  return PNTF_ERR_ARG;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return PNTF_ERR_HIP;
  }
  return PNTF_OK;
}

unsigned grid_1d(int64_t total, int64_t cap = 16384) {
  int64_t g = (total + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > cap ? cap : g));
}

__device__ __forceinline__ float sig10(float y) { return 1.f / (1.f + expf(-SCALE * y)); }

// torch.nn.Softplus(beta=10) with its default threshold 20 (linear above)
__device__ __forceinline__ float softplus10(float y) {
  return SCALE * y > 20.f ? y : log1pf(expf(SCALE * y)) / SCALE;
}

// ---------------------------------------------------------------- Φ planes (:199-213)
// phi (1 + NJ + NL, 2n, 256): point m < n is x_start of pair m, m >= n the x_goal of pair
// m - n; planes [value | ∂x_d (NJ = DIM, or none) | second derivatives: Σ_d ∂²x_d (NL = 1) or
// ∂²x_d per direction (NL = DIM)].  (NJ, NL) = (0, 0): the value plane only (input_mapping
// :186-190, the first-order tape of NN.out's weight gradient); (DIM, 0): input_mapping_grad
// (:192-197).
template <int DIM, int NJ, int NL>
__global__ __launch_bounds__(256) void tt_fourier_kernel(const float* __restrict__ xp, int64_t n,
                                  const float* __restrict__ Btab, const int32_t* __restrict__ env,
                                  int32_t n_env, float* __restrict__ phi) {
  static_assert((NJ == 0 && NL == 0) || (NJ == DIM && (NL == 0 || NL == 1 || NL == DIM)), "planes");
  const int64_t M = 2 * n, plane = M * 256;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < M * H;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / H;
    const int j = (int)(i % H);
    const int64_t p = m < n ? m : m - n;
    const float* x = xp + p * 2 * DIM + (m < n ? 0 : DIM);
    const int e = env ? env[p] : 0;
    float* o = phi + m * 256 + j;
    if (e < 0 || e >= n_env) {
      for (int r = 0; r < 1 + NJ + NL; ++r) o[r * plane] = o[r * plane + H] = NAN;
      continue;
    }
    const float* B = Btab + (int64_t)e * DIM * H + j;
    float w[DIM], q = 0.f, w2 = 0.f;
#pragma unroll
    for (int k = 0; k < DIM; ++k) {
      w[k] = TWO_PI * B[k * H];
      q = fmaf(x[k], w[k], q);
      w2 = fmaf(w[k], w[k], w2);
    }
    float s, c;
    sincosf(q, &s, &c);
    o[0] = s;
    o[H] = c;
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      o[(1 + k) * plane] = w[k] * c;
      o[(1 + k) * plane + H] = -w[k] * s;
    }
    if (NL == 1) {
      o[(1 + NJ) * plane] = -w2 * s;
      o[(1 + NJ) * plane + H] = -w2 * c;
    } else if (NL == DIM) {
#pragma unroll
      for (int k = 0; k < NL; ++k) {
        const float wk2 = w[k] * w[k];
        o[(1 + NJ + k) * plane] = -wk2 * s;
        o[(1 + NJ + k) * plane + H] = -wk2 * c;
      }
    }
  }
}

__device__ __forceinline__ float wave_sum(float v);

// Fourier adjoint (the coords gradient of every tape): gphi (1 + NJ + NL, 2n, 256) = dL/dΦ
// planes -> gx (n, 2 DIM) = dL/dxp.  With q_j = x·w_j: Φ = [sin q | cos q],
// J_k = w_k [cos q | -sin q], L = -w²[sin q | cos q] (summed, w² = Σ_k w_k²) or -w_k²[...] per
// direction, so dL/dq_j = G_j sums the planes' q-derivatives and dL/dx_d = Σ_j G_j w_dj.  One
// wave per point (two features per lane, wave sums in a fixed order).
template <int DIM, int NJ, int NL>
__global__ __launch_bounds__(256) void tt_fourier_bwd_kernel(
    const float* __restrict__ gphi, const float* __restrict__ xp, int64_t n,
    const float* __restrict__ Btab, const int32_t* __restrict__ env, int32_t n_env,
    float* __restrict__ gx) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t M = 2 * n, plane = M * 256;
  for (int64_t m = blockIdx.x * 4 + wave; m < M; m += (int64_t)gridDim.x * 4) {
    const int64_t p = m < n ? m : m - n;
    const float* x = xp + p * 2 * DIM + (m < n ? 0 : DIM);
    float* o = gx + p * 2 * DIM + (m < n ? 0 : DIM);
    const int e = env ? env[p] : 0;
    if (e < 0 || e >= n_env) {               // wave-uniform
      if (lane < DIM) o[lane] = NAN;
      continue;
    }
    const float* B = Btab + (int64_t)e * DIM * H;
    float acc[DIM];
#pragma unroll
    for (int k = 0; k < DIM; ++k) acc[k] = 0.f;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int j = lane + 64 * half;
      float w[DIM], q = 0.f, w2 = 0.f;
#pragma unroll
      for (int k = 0; k < DIM; ++k) {
        w[k] = TWO_PI * B[k * H + j];
        q = fmaf(x[k], w[k], q);
        w2 = fmaf(w[k], w[k], w2);
      }
      float s, c;
      sincosf(q, &s, &c);
      const float* g = gphi + m * 256 + j;
      float G = g[0] * c - g[H] * s;
#pragma unroll
      for (int k = 0; k < NJ; ++k) G -= w[k] * (g[(1 + k) * plane] * s + g[(1 + k) * plane + H] * c);
      if (NL == 1) {
        G += w2 * (g[(1 + NJ) * plane + H] * s - g[(1 + NJ) * plane] * c);
      } else if (NL == DIM) {
#pragma unroll
        for (int k = 0; k < NL; ++k)
          G += w[k] * w[k] * (g[(1 + NJ + k) * plane + H] * s - g[(1 + NJ + k) * plane] * c);
      }
#pragma unroll
      for (int k = 0; k < DIM; ++k) acc[k] = fmaf(G, w[k], acc[k]);
    }
#pragma unroll
    for (int k = 0; k < DIM; ++k) {
      const float v = wave_sum(acc[k]);
      if (lane == 0) o[k] = v;
    }
  }
}

// ---------------------------------------------------------------- act_laplace (:675-691)
// Elementwise over planes with 16-byte accesses: a thread owns 4 consecutive features of one
// point (W is 128 or 256, a multiple of 4), so every plane access is one dwordx4 per lane.
typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }
__device__ __forceinline__ void st4(float* p, f4 v) { *reinterpret_cast<f4*>(p) = v; }

// y (R, M, W), R = 1 + NDIR + NL: GEMM output; plane 0 gets the bias (kept in place as the
// saved pre-activation).  ACT: h = softplus10(y), J' = σJ, L'_l = σ' Σ_{k∈l} J_k² + σ L_l
// (σ = σ(10y), σ' = 10σ(1-σ); summed row l covers the J rows k of its endpoint group,
// l·NDIR/NL <= k < (l+1)·NDIR/NL; NL = 0: first derivatives only).  RES: the residual branch
// (:744, :828) res (R, M, W) is added to every plane first (and the sum kept in y).
// BIAS = false: y already holds bias + residual (the panel GEMM's epilogue added them,
// pntf_gemm.hip tt_linear_res); only h is written.
// QUIRK (NL = 0): encoder[0] of NN.out_backgrad, whose derivative row is multiplied by
// σ(10·softplus(y)) instead of σ(10y) (models/model_res_sigmoid_multi.py:435-438).
template <int NDIR, int NL, bool ACT, bool RES, bool BIAS = true, bool QUIRK = false>
__global__ __launch_bounds__(256) void tt_act_fwd_kernel(float* __restrict__ y, float* __restrict__ h,
                                  const float* __restrict__ bias, const float* __restrict__ res,
                                  int64_t M, int W) {
  static_assert(!QUIRK || NL == 0, "the out_backgrad quirk is first order");
  constexpr int GK = NL ? NDIR / (NL ? NL : 1) : 0;
  const int64_t plane = M * W;
  for (int64_t i = 4 * (blockIdx.x * (int64_t)blockDim.x + threadIdx.x); i < plane;
       i += 4 * (int64_t)gridDim.x * blockDim.x) {
    f4 v = ld4(y + i);
    if (BIAS) {
      v += ld4(bias + i % W);
      if (RES) v += ld4(res + i);
      st4(y + i, v);
    }
    if (!ACT) continue;
    f4 s, ds, hv;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      s[c] = sig10(v[c]);
      ds[c] = SCALE * s[c] * (1.f - s[c]);
      hv[c] = softplus10(v[c]);
    }
    st4(h + i, hv);
    if (NL == 0) {
      f4 sJ = s;
      if (QUIRK) {
#pragma unroll
        for (int c = 0; c < 4; ++c) sJ[c] = sig10(hv[c]);
      }
#pragma unroll
      for (int k = 0; k < NDIR; ++k) {
        const int64_t iJ = (1 + k) * plane + i;
        f4 J = ld4(y + iJ);
        if (RES) {
          J += ld4(res + iJ);
          st4(y + iJ, J);
        }
        st4(h + iJ, J * sJ);
      }
    }
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      f4 jj = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = l * GK; k < (l + 1) * GK; ++k) {
        const int64_t iJ = (1 + k) * plane + i;
        f4 J = ld4(y + iJ);
        if (RES) {
          J += ld4(res + iJ);
          st4(y + iJ, J);
        }
        st4(h + iJ, J * s);
        jj += J * J;
      }
      const int64_t iL = (1 + NDIR + l) * plane + i;
      f4 L = ld4(y + iL);
      if (RES) {
        L += ld4(res + iL);
        st4(y + iL, L);
      }
      st4(h + iL, jj * ds + L * s);
    }
  }
}

// Per-block column partial sums of a (rows, W) value -> partial[blockIdx][W]: the thread owns
// columns 4·(tid % (W/4)) .. +3 and rows tid / (W/4) + k·RB; the RB row groups are folded
// through LDS in fixed order.
template <int W>
__device__ __forceinline__ void block_colsum(f4 acc, float* __restrict__ partial) {
  constexpr int TPR = W / 4, RB = 256 / TPR;
  __shared__ f4 red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x < TPR) {
    f4 s = red[threadIdx.x];
#pragma unroll
    for (int r = 1; r < RB; ++r) s += red[r * TPR + threadIdx.x];
    st4(partial + blockIdx.x * W + 4 * threadIdx.x, s);
  }
}

// Adjoint of act_laplace, in place on g (dL/dh planes in, dL/dy planes out):
//   g_y = g_h σ + Σ_k g_Jk J_k σ' + Σ_l g_Ll (σ'' Σ_{k∈l} J_k² + L_l σ')   σ'' = 10 σ' (1 - 2σ)
//   g_Jk = g_Jk σ + 2 g_L(k) J_k σ'      g_Ll = g_Ll σ
// ACT=false (a Linear with no activation) only forms the bias partials.  QUIRK: the adjoint of
// tt_act_fwd_kernel's out_backgrad encoder[0] (J' = σq J, σq = σ(10 softplus(y)),
// dσq/dy = 10 σq (1 - σq) σ).
template <int NDIR, int NL, int W, bool ACT, bool QUIRK = false>
__global__ __launch_bounds__(256) void tt_act_bwd_kernel(const float* __restrict__ y,
                                                         float* __restrict__ g, int64_t M,
                                                         float* __restrict__ partial) {
  static_assert(!QUIRK || NL == 0, "the out_backgrad quirk is first order");
  constexpr int TPR = W / 4, RB = 256 / TPR, GK = NL ? NDIR / (NL ? NL : 1) : 0;
  const int64_t plane = M * W;
  const int j = 4 * (threadIdx.x % TPR);
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int64_t m = blockIdx.x * RB + threadIdx.x / TPR; m < M; m += (int64_t)gridDim.x * RB) {
    const int64_t i = m * W + j;
    if (!ACT) {
      acc += ld4(g + i);
      continue;
    }
    const f4 v = ld4(y + i);
    f4 s, ds, dds;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      s[c] = sig10(v[c]);
      ds[c] = SCALE * s[c] * (1.f - s[c]);
      dds[c] = SCALE * ds[c] * (1.f - 2.f * s[c]);
    }
    f4 gy = ld4(g + i) * s;
    if (NL == 0) {
      f4 sJ = s, dJ = ds;
      if (QUIRK) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float q = sig10(softplus10(v[c]));
          sJ[c] = q;
          dJ[c] = SCALE * q * (1.f - q) * s[c];
        }
      }
#pragma unroll
      for (int k = 0; k < NDIR; ++k) {
        const int64_t iJ = (1 + k) * plane + i;
        const f4 J = ld4(y + iJ), gJ = ld4(g + iJ);
        gy += gJ * J * dJ;
        st4(g + iJ, gJ * sJ);
      }
    }
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int64_t iL = (1 + NDIR + l) * plane + i;
      const f4 L = ld4(y + iL), gL = ld4(g + iL);
      f4 jj = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = l * GK; k < (l + 1) * GK; ++k) {
        const int64_t iJ = (1 + k) * plane + i;
        const f4 J = ld4(y + iJ), gJ = ld4(g + iJ);
        gy += gJ * J * ds;
        jj += J * J;
        st4(g + iJ, gJ * s + 2.f * gL * J * ds);
      }
      gy += gL * (jj * dds + L * ds);
      st4(g + iL, gL * s);
    }
    st4(g + i, gy);
    acc += gy;
  }
  block_colsum<W>(acc, partial);
}

// out[j] (+)= Σ_b partial[b][j], deterministic: workgroup x owns columns 64x..64x+63 (one per
// lane, coalesced rows); wave w of RW sums the rows b ≡ w (mod RW) in order, 4 loads in
// flight; the wave sums are combined in fixed order through LDS.  RW = 16 waves: a 512-row
// partial is 8 rounds of 4 loads per wave (the 4-wave version ran 11 µs, latency-bound).
constexpr int RW = 16;
__global__ __launch_bounds__(64 * RW) void reduce_kernel(const float* __restrict__ partial,
                                                         int nb, int W, float* __restrict__ out,
                                                         int accumulate) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (j < W) {
    int b = w;
    for (; b + 3 * RW < nb; b += 4 * RW) {
      s0 += partial[(int64_t)b * W + j];
      s1 += partial[(int64_t)(b + RW) * W + j];
      s2 += partial[(int64_t)(b + 2 * RW) * W + j];
      s3 += partial[(int64_t)(b + 3 * RW) * W + j];
    }
    for (; b < nb; b += RW) s0 += partial[(int64_t)b * W + j];
  }
  __shared__ float red[RW][64];
  red[w][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (w == 0 && j < W) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < RW; k += 2) s += red[k][lane] + red[k + 1][lane];
    out[j] = accumulate ? out[j] + s : s;
  }
}

void launch_reduce(const float* partial, int nb, int W, float* out, int accumulate,
                   hipStream_t stream) {
  hipLaunchKernelGGL(reduce_kernel, dim3((W + 63) / 64), dim3(64 * RW), 0, stream, partial, nb,
                     W, out, accumulate);
}

// ---------------------------------------------------------------- start/goal merge (:761-811)
// z (1 + DIM + NLE, 2n, 128) encoder output planes [value | ∂ (DIM) | NLE second-derivative
// rows] -> u (1 + 2 DIM + 2 NLE, n, 256) generator planes [value | ∂xs (DIM) | ∂xg (DIM) |
// L_s (NLE) | L_g (NLE)], features [max-part | min-part]; c = 10 s0 s1 is the merge curvature
// (:768-813).  NLE = 1: the per-endpoint sums Σ∂²; NLE = DIM: one row per direction; NLE = 0:
// first derivatives only (out_grad :338-358).  Row l of an endpoint covers its ∂ rows
// l·DIM/NLE .. (l+1)·DIM/NLE - 1.
template <int DIM, int NLE>
__global__ __launch_bounds__(256) void tt_merge_fwd_kernel(const float* __restrict__ z, int64_t n,
                                    float* __restrict__ u) {
  static_assert(NLE == 0 || NLE == 1 || NLE == DIM, "merge planes");
  constexpr int GK = NLE ? DIM / (NLE ? NLE : 1) : 0;
  const int64_t pz = 2 * n * H, pu = n * 256;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * H;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i / H;
    const int j = (int)(i % H);
    const int64_t is = p * H + j, ig = (n + p) * H + j, o = p * 256 + j;
    const float zs = z[is], zg = z[ig], d = zs - zg;
    const float lse = log1pf(expf(-SCALE * fabsf(d))) / SCALE;
    u[o] = fmaxf(zs, zg) + lse;
    u[o + H] = fminf(zs, zg) - lse;
    const float s0 = sig10(d), s1 = 1.f - s0, c = SCALE * s0 * s1;
#pragma unroll
    for (int k = 0; k < DIM; ++k) {
      const float Js = z[(1 + k) * pz + is], Jg = z[(1 + k) * pz + ig];
      u[(1 + k) * pu + o] = Js * s0;
      u[(1 + k) * pu + o + H] = Js * s1;
      u[(1 + DIM + k) * pu + o] = Jg * s1;
      u[(1 + DIM + k) * pu + o + H] = Jg * s0;
    }
#pragma unroll
    for (int l = 0; l < NLE; ++l) {
      float jjs = 0.f, jjg = 0.f;
#pragma unroll
      for (int k = l * GK; k < (l + 1) * GK; ++k) {
        const float Js = z[(1 + k) * pz + is], Jg = z[(1 + k) * pz + ig];
        jjs = fmaf(Js, Js, jjs);
        jjg = fmaf(Jg, Jg, jjg);
      }
      const float Ls = z[(1 + DIM + l) * pz + is], Lg = z[(1 + DIM + l) * pz + ig];
      const float cs = c * jjs, cg = c * jjg;
      u[(1 + 2 * DIM + l) * pu + o] = cs + Ls * s0;
      u[(1 + 2 * DIM + l) * pu + o + H] = -cs + Ls * s1;
      u[(1 + 2 * DIM + NLE + l) * pu + o] = cg + Lg * s1;
      u[(1 + 2 * DIM + NLE + l) * pu + o + H] = -cg + Lg * s0;
    }
  }
}

// Adjoint of the merge: gu (1 + 2 DIM + 2 NLE, n, 256) -> gz (1 + DIM + NLE, 2n, 128).
template <int DIM, int NLE>
__global__ __launch_bounds__(256) void tt_merge_bwd_kernel(const float* __restrict__ z, const float* __restrict__ gu,
                                    int64_t n, float* __restrict__ gz) {
  constexpr int GK = NLE ? DIM / (NLE ? NLE : 1) : 1, NA = NLE ? NLE : 1;
  const int64_t pz = 2 * n * H, pu = n * 256;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * H;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i / H;
    const int j = (int)(i % H);
    const int64_t is = p * H + j, ig = (n + p) * H + j, o = p * 256 + j;
    const float d = z[is] - z[ig];
    const float s0 = sig10(d), s1 = 1.f - s0, c = SCALE * s0 * s1;
    float dLs[NA], dLg[NA], jjs[NA], jjg[NA], g_s0 = 0.f;
#pragma unroll
    for (int l = 0; l < NLE; ++l) {
      const float Ls = z[(1 + DIM + l) * pz + is], Lg = z[(1 + DIM + l) * pz + ig];
      const float gLsM = gu[(1 + 2 * DIM + l) * pu + o], gLsm = gu[(1 + 2 * DIM + l) * pu + o + H];
      const float gLgM = gu[(1 + 2 * DIM + NLE + l) * pu + o];
      const float gLgm = gu[(1 + 2 * DIM + NLE + l) * pu + o + H];
      dLs[l] = gLsM - gLsm;
      dLg[l] = gLgM - gLgm;
      g_s0 += dLs[l] * Ls - dLg[l] * Lg;
      jjs[l] = jjg[l] = 0.f;
      gz[(1 + DIM + l) * pz + is] = gLsM * s0 + gLsm * s1;
      gz[(1 + DIM + l) * pz + ig] = gLgM * s1 + gLgm * s0;
    }
#pragma unroll
    for (int k = 0; k < DIM; ++k) {
      const float Js = z[(1 + k) * pz + is], Jg = z[(1 + k) * pz + ig];
      const float gJsM = gu[(1 + k) * pu + o], gJsm = gu[(1 + k) * pu + o + H];
      const float gJgM = gu[(1 + DIM + k) * pu + o], gJgm = gu[(1 + DIM + k) * pu + o + H];
      g_s0 += (gJsM - gJsm) * Js - (gJgM - gJgm) * Jg;
      float gs = gJsM * s0 + gJsm * s1, gg = gJgM * s1 + gJgm * s0;
      if (NLE) {
        const int l = k / GK;
        jjs[l] = fmaf(Js, Js, jjs[l]);
        jjg[l] = fmaf(Jg, Jg, jjg[l]);
        gs += 2.f * c * Js * dLs[l];
        gg += 2.f * c * Jg * dLg[l];
      }
      gz[(1 + k) * pz + is] = gs;
      gz[(1 + k) * pz + ig] = gg;
    }
    float g_c = 0.f;
#pragma unroll
    for (int l = 0; l < NLE; ++l) g_c += dLs[l] * jjs[l] + dLg[l] * jjg[l];
    const float kk = (g_s0 + g_c * SCALE * (1.f - 2.f * s0)) * c;
    const float gM = gu[o], gm = gu[o + H];
    gz[is] = gM * s0 + gm * s1 + kk;
    gz[ig] = gM * s1 + gm * s0 - kk;
  }
}

// Value plane only (the first-order tape of NN.out, :236-244): z (2n, 128) -> u (n, 256) and
// the adjoint gu (n, 256) -> gz (2n, 128) with s0 = σ(10 (zs - zg)) (:620-627).
__global__ __launch_bounds__(256) void tt_merge_value_fwd_kernel(const float* __restrict__ z,
                                                                 int64_t n, float* __restrict__ u) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * H;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i / H;
    const int j = (int)(i % H);
    const float zs = z[p * H + j], zg = z[(n + p) * H + j];
    const float lse = log1pf(expf(-SCALE * fabsf(zs - zg))) / SCALE;
    u[p * 256 + j] = fmaxf(zs, zg) + lse;
    u[p * 256 + j + H] = fminf(zs, zg) - lse;
  }
}

__global__ __launch_bounds__(256) void tt_merge_value_bwd_kernel(const float* __restrict__ z,
                                                                 const float* __restrict__ gu,
                                                                 int64_t n, float* __restrict__ gz) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n * H;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t p = i / H;
    const int j = (int)(i % H);
    const int64_t is = p * H + j, ig = (n + p) * H + j;
    const float s0 = sig10(z[is] - z[ig]), s1 = 1.f - s0;
    const float gM = gu[p * 256 + j], gm = gu[p * 256 + j + H];
    gz[is] = gM * s0 + gm * s1;
    gz[ig] = gM * s1 + gm * s0;
  }
}

// ---------------------------------------------------------------- head + loss, fwd and bwd
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// τ head of the first-order tape, one wave per pair: τ = σ(0.1 (w4·v + b4)) (:254-255) from
// generator[3]'s output v (n, 128).  With gtau (the incoming dL/dτ per pair): g = gtau·τ'
// (τ' = 0.1 τ (1 - τ), :295), gv = g·w4 and per-block partials of g_w4 = Σ g v, g_b4 = Σ g.
__global__ __launch_bounds__(256) void tt_head_tau_kernel(
    const float* __restrict__ v, const float* __restrict__ w4, const float* __restrict__ b4,
    int64_t n, const float* __restrict__ gtau, float* __restrict__ tau, float* __restrict__ gv,
    float* __restrict__ partial) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float wa = w4[lane], wb = w4[lane + 64], bias = b4[0];
  float gwa = 0.f, gwb = 0.f, gb = 0.f;
  for (int64_t p = blockIdx.x * 4 + wave; p < n; p += (int64_t)gridDim.x * 4) {
    const float* row = v + p * H;
    const float va = row[lane], vb = row[lane + 64];
    const float y = wave_sum(fmaf(va, wa, vb * wb)) + bias;
    const float t = 1.f / (1.f + expf(-0.1f * y));
    if (tau && lane == 0) tau[p] = t;
    if (!gtau) continue;
    const float g = gtau[p] * (0.1f * t * (1.f - t));
    gb += g;
    gwa = fmaf(g, va, gwa);
    gwb = fmaf(g, vb, gwb);
    gv[p * H + lane] = g * wa;
    gv[p * H + lane + 64] = g * wb;
  }
  if (!gtau) return;   // grid-uniform
  __shared__ float red[4][129];
  red[wave][lane] = gwa;
  red[wave][lane + 64] = gwb;
  if (lane == 0) red[wave][128] = gb;
  __syncthreads();
  if (threadIdx.x < 129) {
    const float s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                    red[3][threadIdx.x];
    if (threadIdx.x < 128) partial[blockIdx.x * 128 + threadIdx.x] = s;
    else partial[(int64_t)gridDim.x * 128 + blockIdx.x] = s;
  }
}

// One wave per pair.  v (R, n, 128) = generator[3]'s Taylor output, R = 3 + 2 DIM planes
// [value | ∂xs (DIM) | ∂xg (DIM) | Σ∂²xs | Σ∂²xg].
// Forward: y_r = w4·v_r (+ b4 on r = 0); τ = σ(0.1 y), ∇τ and the per-endpoint Laplacian
// Δ_eτ = Σ_{k∈e} (J_k² τ'' + L_e τ') (actout_laplace :693-708, summed as Model.Loss :919-920
// does); diff (Model.Loss :914-946, ARM: models/model_res_sigmoid.py:888-933).  Backward of
// scale·Σ diff: g_r per row, written as gv_r = g_r w4 (the input gradient of generator[4])
// and folded into per-block partials of g_w4 = Σ g_r v_r and g_b4 = Σ g_0.
template <int DIM, bool ARM>
__global__ __launch_bounds__(256) void tt_head_loss_kernel(
    const float* __restrict__ v, const float* __restrict__ w4, const float* __restrict__ b4,
    const float* __restrict__ xp, const float* __restrict__ yobs, int64_t n, float gamma,
    float scale, float* __restrict__ diff, float* __restrict__ gv, float* __restrict__ partial) {
  constexpr int ND = 2 * DIM, R = 3 + ND;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t plane = n * H;
  const float wa = w4[lane], wb = w4[lane + 64], bias = b4[0];
  float gwa = 0.f, gwb = 0.f, gb = 0.f;
  for (int64_t p = blockIdx.x * 4 + wave; p < n; p += (int64_t)gridDim.x * 4) {
    float yr[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float* row = v + r * plane + p * H;
      yr[r] = wave_sum(fmaf(row[lane], wa, row[lane + 64] * wb));
    }
    const float y = yr[0] + bias;
    const float t = 1.f / (1.f + expf(-0.1f * y));
    const float dt = 0.1f * t * (1.f - t), ddt = 0.1f * dt * (1.f - 2.f * t);
    const float dddt = 0.1f * (ddt * (1.f - 2.f * t) - 2.f * dt * dt);
    float dtau[ND], lap[2];
#pragma unroll
    for (int k = 0; k < ND; ++k) dtau[k] = yr[1 + k] * dt;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      float jj = 0.f;
#pragma unroll
      for (int k = 0; k < DIM; ++k) jj = fmaf(yr[1 + e * DIM + k], yr[1 + e * DIM + k], jj);
      lap[e] = fmaf(jj, ddt, yr[1 + ND + e] * dt);
    }
    // ---- Model.Loss and its adjoint
    const float* x = xp + p * 2 * DIM;
    float D[DIM], T0 = 0.f;
#pragma unroll
    for (int k = 0; k < DIM; ++k) {
      D[k] = x[DIM + k] - x[k];
      T0 = fmaf(D[k], D[k], T0);
    }
    float gt = 0.f, gd[ND], gl[2], df = -4.f;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float sgn = e == 0 ? 1.f : -1.f;
      float dd = 0.f, nn = 0.f;
#pragma unroll
      for (int k = 0; k < DIM; ++k) {
        dd = fmaf(dtau[e * DIM + k], D[k], dd);
        nn = fmaf(dtau[e * DIM + k], dtau[e * DIM + k], nn);
      }
      const float S = T0 * nn + sgn * 2.f * t * dd + t * t;
      const float rS = sqrtf(S);
      const float yp = 1.f / (rS / (t * t) + gamma * lap[e]);
      const float yo = yobs[p * 2 + e];
      float dfy;
      if (ARM) {
        const float a = sqrtf(yp), b = sqrtf(yo);
        df += a / b + b / a;
        dfy = (1.f / b - b / (a * a)) / (2.f * a);
      } else {
        df += yp / yo + yo / yp;
        dfy = 1.f / yo - yo / (yp * yp);
      }
      const float gQ = -scale * dfy * yp * yp;
      const float gS = gQ / (2.f * rS * t * t);
      gt += gQ * (-2.f * rS / (t * t * t)) + gS * (sgn * 2.f * dd + 2.f * t);
#pragma unroll
      for (int k = 0; k < DIM; ++k)
        gd[e * DIM + k] = gS * (2.f * T0 * dtau[e * DIM + k] + sgn * 2.f * t * D[k]);
      gl[e] = gQ * gamma;
    }
    if (lane == 0) diff[p] = df;
    // ---- actout_laplace adjoint -> g_r of generator[4]'s output rows
    float g0 = gt * dt;
#pragma unroll
    for (int k = 0; k < ND; ++k) {
      const float J = yr[1 + k];
      g0 += gd[k] * J * ddt + gl[k / DIM] * J * J * dddt;
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) g0 += gl[e] * yr[1 + ND + e] * ddt;
    gb += g0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float g;
      if (r == 0) g = g0;
      else if (r <= ND) g = gd[r - 1] * dt + 2.f * gl[(r - 1) / DIM] * yr[r] * ddt;
      else g = gl[r - 1 - ND] * dt;
      const float* row = v + r * plane + p * H;
      float* grow = gv + r * plane + p * H;
      gwa = fmaf(g, row[lane], gwa);
      gwb = fmaf(g, row[lane + 64], gwb);
      grow[lane] = g * wa;
      grow[lane + 64] = g * wb;
    }
  }
// per-block partials: [gridDim][128] for g_w4, then [gridDim] for g_b4
  __shared__ float red[4][129];
  red[wave][lane] = gwa;
  red[wave][lane + 64] = gwb;
  if (lane == 0) red[wave][128] = gb;
  __syncthreads();
  if (threadIdx.x < 129) {
    const float s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                    red[3][threadIdx.x];
    if (threadIdx.x < 128) partial[blockIdx.x * 128 + threadIdx.x] = s;
    else partial[(int64_t)gridDim.x * 128 + blockIdx.x] = s;
  }
}

// generator[4] + actout_laplace (:693-708) with a GENERAL upstream gradient: the backward of
// Σ_p (gtau_p τ_p + gdtau_p·∇τ_p + glap_p·Δ_p) for a loss a user writes on NN.out_laplace /
// out_grad / out_backgrad / Model.gradient outputs.  One wave per pair.  v (R, n, 128),
// R = 1 + 2 DIM + 2 NLE planes [value | ∂xs | ∂xg | L (2 NLE)]; row l of the second
// derivatives covers ∂ rows l·GK .. (l+1)·GK - 1, GK = DIM / NLE, so Δ_l = Σ_{k∈l} J_k² τ'' +
// L_l τ' is the per-direction ∇²τ (NLE = DIM) or the per-endpoint Laplacian (NLE = 1).
// Outputs (each optional): tau (n), dtau (n, 2 DIM), lap (n, 2 NLE); gv (R, n, 128) = dL/dv
// and per-block partials of g_w4, g_b4 as tt_head_loss_kernel.  A NULL upstream is zero.
template <int DIM, int NLE>
__global__ __launch_bounds__(256) void tt_head_vjp_kernel(
    const float* __restrict__ v, const float* __restrict__ w4, const float* __restrict__ b4,
    int64_t n, const float* __restrict__ gtau, const float* __restrict__ gdtau,
    const float* __restrict__ glap, float* __restrict__ tau, float* __restrict__ dtau,
    float* __restrict__ lap, float* __restrict__ gv, float* __restrict__ partial) {
  constexpr int ND = 2 * DIM, NLT = 2 * NLE, R = 1 + ND + NLT, GK = NLE ? DIM / (NLE ? NLE : 1) : 1;
  constexpr int NA = NLT ? NLT : 1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t plane = n * H;
  const float wa = w4[lane], wb = w4[lane + 64], bias = b4[0];
  float gwa = 0.f, gwb = 0.f, gb = 0.f;
  for (int64_t p = blockIdx.x * 4 + wave; p < n; p += (int64_t)gridDim.x * 4) {
    float yr[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float* row = v + r * plane + p * H;
      yr[r] = wave_sum(fmaf(row[lane], wa, row[lane + 64] * wb));
    }
    const float y = yr[0] + bias;
    const float t = 1.f / (1.f + expf(-0.1f * y));
    const float dt = 0.1f * t * (1.f - t), ddt = 0.1f * dt * (1.f - 2.f * t);
    const float dddt = 0.1f * (ddt * (1.f - 2.f * t) - 2.f * dt * dt);
    if (lane == 0) {
      if (tau) tau[p] = t;
      if (dtau) {
#pragma unroll
        for (int k = 0; k < ND; ++k) dtau[p * ND + k] = yr[1 + k] * dt;
      }
      if (lap) {
#pragma unroll
        for (int l = 0; l < NLT; ++l) {
          float jj = 0.f;
#pragma unroll
          for (int k = l * GK; k < (l + 1) * GK; ++k) jj = fmaf(yr[1 + k], yr[1 + k], jj);
          lap[p * NLT + l] = fmaf(jj, ddt, yr[1 + ND + l] * dt);
        }
      }
    }
    const float gt = gtau ? gtau[p] : 0.f;
    float gd[ND], gl[NA];
#pragma unroll
    for (int k = 0; k < ND; ++k) gd[k] = gdtau ? gdtau[p * ND + k] : 0.f;
#pragma unroll
    for (int l = 0; l < NA; ++l) gl[l] = (NLT && glap) ? glap[p * NLT + l] : 0.f;
    // actout_laplace adjoint -> g_r of generator[4]'s output rows
    float g0 = gt * dt;
#pragma unroll
    for (int k = 0; k < ND; ++k) {
      const float J = yr[1 + k];
      g0 += gd[k] * J * ddt;
      if (NLT) g0 += gl[k / GK] * J * J * dddt;
    }
#pragma unroll
    for (int l = 0; l < NLT; ++l) g0 += gl[l] * yr[1 + ND + l] * ddt;
    gb += g0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      float g;
      if (r == 0) g = g0;
      else if (r <= ND) g = gd[r - 1] * dt + (NLT ? 2.f * gl[(r - 1) / GK] * yr[r] * ddt : 0.f);
      else g = gl[r - 1 - ND] * dt;
      const float* row = v + r * plane + p * H;
      float* grow = gv + r * plane + p * H;
      gwa = fmaf(g, row[lane], gwa);
      gwb = fmaf(g, row[lane + 64], gwb);
      grow[lane] = g * wa;
      grow[lane + 64] = g * wb;
    }
  }
  __shared__ float red[4][129];
  red[wave][lane] = gwa;
  red[wave][lane + 64] = gwb;
  if (lane == 0) red[wave][128] = gb;
  __syncthreads();
  if (threadIdx.x < 129) {
    const float s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                    red[3][threadIdx.x];
    if (threadIdx.x < 128) partial[blockIdx.x * 128 + threadIdx.x] = s;
    else partial[(int64_t)gridDim.x * 128 + blockIdx.x] = s;
  }
}

// ---------------------------------------------------------------- AdamW (torch.optim.AdamW)
// Same operation order as torch's single-tensor AdamW: p *= 1 - lr·wd; m = lerp(m, g, 1-β1);
// v = β2 v + (1-β2) g²; p -= step_size · m / (sqrt(v)/sqrt(bc2) + eps).
__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                             float* __restrict__ m, float* __restrict__ v, int64_t n,
                             float decay, float one_minus_b1, float b2, float one_minus_b2,
                             float step_size, float bc2_sqrt, float eps) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i];
    float pi = p[i] * decay;
    float mi = m[i];
    mi = fmaf(one_minus_b1, gi - mi, mi);
    const float vi = fmaf(b2, v[i], one_minus_b2 * gi * gi);
    pi -= step_size * mi / (sqrtf(vi) / bc2_sqrt + eps);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

// Every tensor of a parameter group in one launch: blockIdx.y picks the tensor (the model has
// 28 trained tensors; one launch each cost ~2.3 us of kernel plus a launch boundary apiece).
constexpr int ADAMW_MAX_TENSORS = 64;
struct AdamwList {
  float* p[ADAMW_MAX_TENSORS];
  const float* g[ADAMW_MAX_TENSORS];
  float* m[ADAMW_MAX_TENSORS];
  float* v[ADAMW_MAX_TENSORS];
  int64_t n[ADAMW_MAX_TENSORS];
};

__global__ void adamw_multi_kernel(AdamwList t, float decay, float one_minus_b1, float b2,
                                   float one_minus_b2, float step_size, float bc2_sqrt, float eps) {
  const int k = blockIdx.y;
  float* __restrict__ p = t.p[k];
  const float* __restrict__ g = t.g[k];
  float* __restrict__ m = t.m[k];
  float* __restrict__ v = t.v[k];
  const int64_t n = t.n[k];
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i];
    float pi = p[i] * decay;
    float mi = m[i];
    mi = fmaf(one_minus_b1, gi - mi, mi);
    const float vi = fmaf(b2, v[i], one_minus_b2 * gi * gi);
    pi -= step_size * mi / (sqrtf(vi) / bc2_sqrt + eps);
    p[i] = pi;
    m[i] = mi;
    v[i] = vi;
  }
}

int nb_for(int64_t rows) {
  int64_t nb = rows < 1 ? 1 : rows;
  return (int)(nb > NB_MAX ? NB_MAX : nb);
}

// (ndir, nl) of the encoder's Fourier planes: (0, 0), (dim, 0), (dim, 1) or (dim, dim)
bool fourier_planes_ok(int dim, int ndir, int nl) {
  return (dim == 3 || dim == 6) &&
         ((ndir == 0 && nl == 0) || (ndir == dim && (nl == 0 || nl == 1 || nl == dim)));
}

template <class F>
void with_fourier(int dim, int ndir, int nl, F&& f) {
  if (dim == 3) {
    if (ndir == 0) f(IC<3>{}, IC<0>{}, IC<0>{});
    else if (nl == 0) f(IC<3>{}, IC<3>{}, IC<0>{});
    else if (nl == 1) f(IC<3>{}, IC<3>{}, IC<1>{});
    else f(IC<3>{}, IC<3>{}, IC<3>{});
  } else {
    if (ndir == 0) f(IC<6>{}, IC<0>{}, IC<0>{});
    else if (nl == 0) f(IC<6>{}, IC<6>{}, IC<0>{});
    else if (nl == 1) f(IC<6>{}, IC<6>{}, IC<1>{});
    else f(IC<6>{}, IC<6>{}, IC<6>{});
  }
}

template <class F>
void with_merge(int dim, int nle, F&& f) {
  if (dim == 3) {
    if (nle == 0) f(IC<3>{}, IC<0>{});
    else if (nle == 1) f(IC<3>{}, IC<1>{});
    else f(IC<3>{}, IC<3>{});
  } else {
    if (nle == 0) f(IC<6>{}, IC<0>{});
    else if (nle == 1) f(IC<6>{}, IC<1>{});
    else f(IC<6>{}, IC<6>{});
  }
}

}  // namespace

extern "C" {

size_t pntf_tt_partial_floats(void) { return (size_t)NB_MAX * 257; }

const char* pntf_tt_last_error(void) { return g_err; }

int pntf_tt_fourier_ex(int dim, int ndir, int nl, const float* xp, int64_t n, const float* Btab,
                       const int32_t* env, int32_t n_env, float* phi, hipStream_t stream) {
  if (!fourier_planes_ok(dim, ndir, nl) || n < 0 || n_env < 1 ||
      (n > 0 && (!xp || !Btab || !phi)))
    return fail("pntf_tt_fourier_ex: bad arguments");
  if (n == 0) return PNTF_OK;
  const unsigned g = grid_1d(2 * n * H);
  with_fourier(dim, ndir, nl, [&](auto D, auto NJ, auto NL) {
    hipLaunchKernelGGL((tt_fourier_kernel<decltype(D)::value, decltype(NJ)::value, decltype(NL)::value>), dim3(g), dim3(256), 0,
                       stream, xp, n, Btab, env, n_env, phi);
  });
  return check_launch("tt_fourier_kernel");
}

int pntf_tt_fourier(int dim, const float* xp, int64_t n, const float* Btab, const int32_t* env,
                    int32_t n_env, float* phi, hipStream_t stream) {
  return pntf_tt_fourier_ex(dim, dim, 1, xp, n, Btab, env, n_env, phi, stream);
}

int pntf_tt_fourier_bwd(int dim, int ndir, int nl, const float* gphi, const float* xp, int64_t n,
                        const float* Btab, const int32_t* env, int32_t n_env, float* gx,
                        hipStream_t stream) {
  if (!fourier_planes_ok(dim, ndir, nl) || n < 0 || n_env < 1 ||
      (n > 0 && (!gphi || !xp || !Btab || !gx)))
    return fail("pntf_tt_fourier_bwd: bad arguments");
  if (n == 0) return PNTF_OK;
  const unsigned g = grid_1d(2 * n * 64, 4096);   // one wave per point, 4 per workgroup
  with_fourier(dim, ndir, nl, [&](auto D, auto NJ, auto NL) {
    hipLaunchKernelGGL((tt_fourier_bwd_kernel<decltype(D)::value, decltype(NJ)::value, decltype(NL)::value>), dim3(g), dim3(256),
                       0, stream, gphi, xp, n, Btab, env, n_env, gx);
  });
  return check_launch("tt_fourier_bwd_kernel");
}

// every (ndir, nl) of with_planes (hidden: pntf_gemm.hip's pntf_tt_linear_act checks with it)
extern "C" __attribute__((visibility("hidden"))) int pntf_tt_planes_ok(int ndir, int nl) {
  return with_planes(ndir, nl, [](auto, auto) {}) ? 1 : 0;
}

int pntf_tt_act_fwd(int ndir, int nl, float* y, float* h, const float* bias, const float* res,
                    int64_t m, int w, int act, hipStream_t stream) {
  // act: 0 none, 1 softplus10 act_laplace, 2 the out_backgrad encoder[0] quirk (first order)
  const bool quirk = act == 2;
  if (!pntf_tt_planes_ok(ndir, nl) || act < 0 || act > 2 ||
      (quirk && (nl != 0 || (ndir != 3 && ndir != 6))) || m < 0 || (w != 128 && w != 256) ||
      (m > 0 && (!y || !bias || (act && !h))) || (res && !act))
    return fail("pntf_tt_act_fwd: bad arguments");
  if (m == 0) return PNTF_OK;
  const dim3 g(grid_1d(m * w / 4)), b(256);
  if (quirk) {
    if (ndir == 3) hipLaunchKernelGGL((tt_act_fwd_kernel<3, 0, true, false, true, true>), g, b, 0, stream, y, h, bias, res, m, w);
    else hipLaunchKernelGGL((tt_act_fwd_kernel<6, 0, true, false, true, true>), g, b, 0, stream, y, h, bias, res, m, w);
    return check_launch("tt_act_fwd_kernel<quirk>");
  }
  with_planes(ndir, nl, [&](auto N, auto L) {
    constexpr int ND = decltype(N)::value, NL = decltype(L)::value;
    if (res) hipLaunchKernelGGL((tt_act_fwd_kernel<ND, NL, true, true>), g, b, 0, stream, y, h, bias, res, m, w);
    else if (act) hipLaunchKernelGGL((tt_act_fwd_kernel<ND, NL, true, false>), g, b, 0, stream, y, h, bias, res, m, w);
    else hipLaunchKernelGGL((tt_act_fwd_kernel<ND, NL, false, false>), g, b, 0, stream, y, h, bias, res, m, w);
  });
  return check_launch("tt_act_fwd_kernel");
}

// act pass of a Linear whose panel GEMM already added bias and residual (pntf_gemm.hip):
// reads y, writes h.  Library-internal (not in include/pntf.h).
extern "C" __attribute__((visibility("hidden"))) int pntf_tt_act_fwd_biased(
    int ndir, int nl, const float* y, float* h, int64_t m, int w, hipStream_t stream) {
  if (!pntf_tt_planes_ok(ndir, nl) || m < 0 || (w != 128 && w != 256) || (m > 0 && (!y || !h)))
    return fail("pntf_tt_act_fwd_biased: bad arguments");
  if (m == 0) return PNTF_OK;
  const dim3 g(grid_1d(m * w / 4)), b(256);
  float* yy = const_cast<float*>(y);
  with_planes(ndir, nl, [&](auto N, auto L) {
    hipLaunchKernelGGL((tt_act_fwd_kernel<decltype(N)::value, decltype(L)::value, true, false, false>),
                       g, b, 0, stream, yy, h, nullptr, nullptr, m, w);
  });
  return check_launch("tt_act_fwd_kernel<biased>");
}

int pntf_tt_act_bwd(int ndir, int nl, const float* y, float* g, int64_t m, int w, int act,
                    float* gbias, int accumulate, float* partial, hipStream_t stream) {
  const bool quirk = act == 2;
  if (!pntf_tt_planes_ok(ndir, nl) || act < 0 || act > 2 ||
      (quirk && (nl != 0 || (ndir != 3 && ndir != 6) || w != 128)) || m < 0 ||
      (w != 128 && w != 256) || !gbias || !partial || (m > 0 && (!g || (act && !y))))
    return fail("pntf_tt_act_bwd: bad arguments");
  const int nb = nb_for(m / (1024 / w));
  const dim3 gr(nb), b(256);
  if (quirk) {
    if (ndir == 3) hipLaunchKernelGGL((tt_act_bwd_kernel<3, 0, 128, true, true>), gr, b, 0, stream, y, g, m, partial);
    else hipLaunchKernelGGL((tt_act_bwd_kernel<6, 0, 128, true, true>), gr, b, 0, stream, y, g, m, partial);
  } else {
    with_planes(ndir, nl, [&](auto N, auto L) {
      constexpr int ND = decltype(N)::value, NL = decltype(L)::value;
      if (w == 128) {
        if (act) hipLaunchKernelGGL((tt_act_bwd_kernel<ND, NL, 128, true>), gr, b, 0, stream, y, g, m, partial);
        else hipLaunchKernelGGL((tt_act_bwd_kernel<ND, NL, 128, false>), gr, b, 0, stream, y, g, m, partial);
      } else {
        if (act) hipLaunchKernelGGL((tt_act_bwd_kernel<ND, NL, 256, true>), gr, b, 0, stream, y, g, m, partial);
        else hipLaunchKernelGGL((tt_act_bwd_kernel<ND, NL, 256, false>), gr, b, 0, stream, y, g, m, partial);
      }
    });
  }
  launch_reduce(partial, nb, w, gbias, accumulate, stream);
  return check_launch("tt_act_bwd_kernel");
}

int pntf_tt_merge_fwd_ex(int dim, int nle, const float* z, int64_t n, float* u,
                         hipStream_t stream) {
  if ((dim != 3 && dim != 6) || (nle != 0 && nle != 1 && nle != dim) || n < 0 ||
      (n > 0 && (!z || !u)))
    return fail("pntf_tt_merge_fwd: bad arguments");
  if (n == 0) return PNTF_OK;
  const dim3 g(grid_1d(n * H)), b(256);
  with_merge(dim, nle, [&](auto D, auto L) {
    hipLaunchKernelGGL((tt_merge_fwd_kernel<decltype(D)::value, decltype(L)::value>), g, b, 0, stream, z, n, u);
  });
  return check_launch("tt_merge_fwd_kernel");
}

int pntf_tt_merge_bwd_ex(int dim, int nle, const float* z, const float* gu, int64_t n, float* gz,
                         hipStream_t stream) {
  if ((dim != 3 && dim != 6) || (nle != 0 && nle != 1 && nle != dim) || n < 0 ||
      (n > 0 && (!z || !gu || !gz)))
    return fail("pntf_tt_merge_bwd: bad arguments");
  if (n == 0) return PNTF_OK;
  const dim3 g(grid_1d(n * H)), b(256);
  with_merge(dim, nle, [&](auto D, auto L) {
    hipLaunchKernelGGL((tt_merge_bwd_kernel<decltype(D)::value, decltype(L)::value>), g, b, 0, stream, z, gu, n, gz);
  });
  return check_launch("tt_merge_bwd_kernel");
}

int pntf_tt_merge_fwd(int dim, const float* z, int64_t n, float* u, hipStream_t stream) {
  return pntf_tt_merge_fwd_ex(dim, 1, z, n, u, stream);
}

int pntf_tt_merge_bwd(int dim, const float* z, const float* gu, int64_t n, float* gz,
                      hipStream_t stream) {
  return pntf_tt_merge_bwd_ex(dim, 1, z, gu, n, gz, stream);
}

int pntf_tt_fourier_value(int dim, const float* xp, int64_t n, const float* Btab,
                          const int32_t* env, int32_t n_env, float* phi, hipStream_t stream) {
  return pntf_tt_fourier_ex(dim, 0, 0, xp, n, Btab, env, n_env, phi, stream);
}

int pntf_tt_merge_value_fwd(const float* z, int64_t n, float* u, hipStream_t stream) {
  if (n < 0 || (n > 0 && (!z || !u))) return fail("pntf_tt_merge_value_fwd: bad arguments");
  if (n == 0) return PNTF_OK;
  hipLaunchKernelGGL(tt_merge_value_fwd_kernel, dim3(grid_1d(n * H)), dim3(256), 0, stream, z, n,
                     u);
  return check_launch("tt_merge_value_fwd_kernel");
}

int pntf_tt_merge_value_bwd(const float* z, const float* gu, int64_t n, float* gz,
                            hipStream_t stream) {
  if (n < 0 || (n > 0 && (!z || !gu || !gz))) return fail("pntf_tt_merge_value_bwd: bad arguments");
  if (n == 0) return PNTF_OK;
  hipLaunchKernelGGL(tt_merge_value_bwd_kernel, dim3(grid_1d(n * H)), dim3(256), 0, stream, z, gu,
                     n, gz);
  return check_launch("tt_merge_value_bwd_kernel");
}

int pntf_tt_head_tau(const float* v, const float* w4, const float* b4, int64_t n,
                     const float* gtau, float* tau, float* gv, float* gw4, float* gb4,
                     float* partial, hipStream_t stream) {
  if (n < 0 || !w4 || !b4 || (n > 0 && !v) || (!gtau && !tau) ||
      (gtau && (!gv || !gw4 || !gb4 || !partial)))
    return fail("pntf_tt_head_tau: bad arguments");
  const int nb = nb_for((n + 3) / 4);
  if (n > 0)
    hipLaunchKernelGGL(tt_head_tau_kernel, dim3(nb), dim3(256), 0, stream, v, w4, b4, n, gtau, tau,
                       gv, partial);
  if (gtau) {
    if (n == 0) {   // an empty batch: zero gradients
      hipMemsetAsync(gw4, 0, 128 * sizeof(float), stream);
      hipMemsetAsync(gb4, 0, sizeof(float), stream);
      return check_launch("pntf_tt_head_tau");
    }
    launch_reduce(partial, nb, 128, gw4, 0, stream);
    launch_reduce(partial + (int64_t)nb * 128, nb, 1, gb4, 0, stream);
  }
  return check_launch("tt_head_tau_kernel");
}

int pntf_tt_head_loss(int dim, int arm, const float* v, const float* w4, const float* b4,
                      const float* xp, const float* yobs, int64_t n, float gamma, float scale,
                      float* diff, float* gv, float* gw4, float* gb4, float* partial,
                      hipStream_t stream) {
  if ((dim != 3 && dim != 6) || n < 0 || !w4 || !b4 || !gw4 || !gb4 || !partial ||
      (n > 0 && (!v || !xp || !yobs || !diff || !gv)))
    return fail("pntf_tt_head_loss: bad arguments");
  const int nb = nb_for((n + 3) / 4);
  const dim3 g(nb), b(256);
#define PNTF_HEAD(D, A)                                                                     \
  hipLaunchKernelGGL((tt_head_loss_kernel<D, A>), g, b, 0, stream, v, w4, b4, xp, yobs, n,   \
                     gamma, scale, diff, gv, partial)
  if (dim == 3) {
    if (arm) PNTF_HEAD(3, true);
    else PNTF_HEAD(3, false);
  } else {
    if (arm) PNTF_HEAD(6, true);
    else PNTF_HEAD(6, false);
  }
#undef PNTF_HEAD
  launch_reduce(partial, nb, 128, gw4, 0, stream);
  launch_reduce(partial + (int64_t)nb * 128, nb, 1, gb4, 0, stream);
  return check_launch("tt_head_loss_kernel");
}

int pntf_tt_head_vjp(int dim, int nle, const float* v, const float* w4, const float* b4,
                     int64_t n, const float* gtau, const float* gdtau, const float* glap,
                     float* tau, float* dtau, float* lap, float* gv, float* gw4, float* gb4,
                     float* partial, hipStream_t stream) {
  if ((dim != 3 && dim != 6) || (nle != 0 && nle != 1 && nle != dim) || n < 0 || !w4 || !b4 ||
      !gw4 || !gb4 || !partial || (glap && nle == 0) || (lap && nle == 0) ||
      (n > 0 && (!v || !gv)))
    return fail("pntf_tt_head_vjp: bad arguments");
  if (n == 0) {
    hipMemsetAsync(gw4, 0, 128 * sizeof(float), stream);
    hipMemsetAsync(gb4, 0, sizeof(float), stream);
    return check_launch("pntf_tt_head_vjp");
  }
  const int nb = nb_for((n + 3) / 4);
  with_merge(dim, nle, [&](auto D, auto L) {
    hipLaunchKernelGGL((tt_head_vjp_kernel<decltype(D)::value, decltype(L)::value>), dim3(nb), dim3(256), 0, stream, v,
                       w4, b4, n, gtau, gdtau, glap, tau, dtau, lap, gv, partial);
  });
  launch_reduce(partial, nb, 128, gw4, 0, stream);
  launch_reduce(partial + (int64_t)nb * 128, nb, 1, gb4, 0, stream);
  return check_launch("tt_head_vjp_kernel");
}

int pntf_adamw(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
               float beta2, float eps, float weight_decay, int64_t step, hipStream_t stream) {
  if (n < 0 || step < 1 || (n > 0 && (!p || !g || !m || !v)))
    return fail("pntf_adamw: bad arguments");
  if (n == 0) return PNTF_OK;
  // host-side scalars in double, as torch computes them in Python floats
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_1d(n, 4096)), dim3(256), 0, stream, p, g, m, v, n,
                     (float)(1.0 - (double)lr * weight_decay), (float)(1.0 - beta1), beta2,
                     (float)(1.0 - beta2), (float)(lr / bc1), (float)sqrt(bc2), eps);
  return check_launch("adamw_kernel");
}

int pntf_adamw_multi(int count, float* const* p, const float* const* g, float* const* m,
                     float* const* v, const int64_t* n, float lr, float beta1, float beta2,
                     float eps, float weight_decay, int64_t step, hipStream_t stream) {
  if (count < 0 || count > ADAMW_MAX_TENSORS || step < 1 || (count > 0 && (!p || !g || !m || !v || !n)))
    return fail("pntf_adamw_multi: bad arguments");
  AdamwList t{};
  int64_t most = 0;
  for (int k = 0; k < count; ++k) {
    if (n[k] < 0 || (n[k] > 0 && (!p[k] || !g[k] || !m[k] || !v[k])))
      return fail("pntf_adamw_multi: bad tensor");
    t.p[k] = p[k];
    t.g[k] = g[k];
    t.m[k] = m[k];
    t.v[k] = v[k];
    t.n[k] = n[k];
    most = n[k] > most ? n[k] : most;
  }
  if (count == 0 || most == 0) return PNTF_OK;
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  hipLaunchKernelGGL(adamw_multi_kernel, dim3(grid_1d(most, 4096), count), dim3(256), 0, stream, t,
                     (float)(1.0 - (double)lr * weight_decay), (float)(1.0 - beta1), beta2,
                     (float)(1.0 - beta2), (float)(lr / bc1), (float)sqrt(bc2), eps);
  return check_launch("adamw_multi_kernel");
}

}  // extern "C"
