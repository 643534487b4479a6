// Microprobe: how much VALU issue hides beside v_mfma_f32_32x32x2_f32 (64-cycle fp32 MFMA,
// the wide kernels' instruction) at one wave per SIMD.  Cycles per MFMA for NV independent
// VALU ops per MFMA placed in each gap (sched_group_barrier), VK = 0: v_fma_f32, 1: v_exp_f32,
// 2: v_mul_f32, 3: the softplus/σ epilogue of one
// element (exp, rcp, log + 5 plain ops) per gap; and the same work clustered after 16 MFMAs.
// Diagnostics only: hipcc -O3 --offload-arch=gfx950 coexec32_probe.hip -o coexec32_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void sp_sig(float y, float& sp, float& sg) {
  float t = __builtin_amdgcn_exp2f(-14.4269504f * fabsf(y));
  float u = 1.f + t;
  float r = __builtin_amdgcn_rcpf(u);
  bool pos = y >= 0.f;
  sp = fmaf(__builtin_amdgcn_logf(u), 0.0693147f, pos ? y : 0.f);
  sg = pos ? r : t * r;
}

template <int NV, int VK, bool CLUSTER>
__global__ __launch_bounds__(256, 1) void probe(float* out, long long* cyc, int iters) {
  f32x16 acc[2] = {};
  float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
  float v[16], w[16];
  for (int i = 0; i < 16; ++i) v[i] = 0.1f * i + a, w[i] = 0.2f * i;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      acc[m & 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[m & 1], 0, 0, 0);
      if (!CLUSTER) {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          float& x = v[(m * NV + j) & 15];
          if (VK == 0) x = fmaf(x, 0.999f, 1e-3f);
          else if (VK == 1) x = __builtin_amdgcn_exp2f(x * -0.5f);
          else if (VK == 2) x = x * w[(m * NV + j) & 15];
          else { float s, g; sp_sig(x, s, g); x = s; w[(m * NV + j) & 15] += g; }
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, NV * (VK == 1 ? 2 : VK == 3 ? 11 : 1), 0);
      }
    }
    if (CLUSTER) {
#pragma unroll
      for (int j = 0; j < 16 * NV; ++j) {
        float& x = v[j & 15];
        if (VK == 0) x = fmaf(x, 0.999f, 1e-3f);
        else if (VK == 1) x = __builtin_amdgcn_exp2f(x * -0.5f);
        else if (VK == 2) x = x * w[j & 15];
        else { float s, g; sp_sig(x, s, g); x = s; w[j & 15] += g; }
      }
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += v[i] + w[i];
  for (int i = 0; i < 2; ++i)
    for (int r = 0; r < 16; ++r) s += acc[i][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NV, int VK, bool CLUSTER>
void run(float* out, long long* cyc, int grid) {
  const int iters = 1000;
  probe<NV, VK, CLUSTER><<<grid, 256>>>(out, cyc, iters);
  hipDeviceSynchronize();
  probe<NV, VK, CLUSTER><<<grid, 256>>>(out, cyc, iters);
  hipDeviceSynchronize();
  long long h[1024];
  hipMemcpy(h, cyc, grid * sizeof(long long), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < grid; ++i) m += h[i];
  m /= grid;
  printf("%s NV=%d VK=%d  cycles/MFMA = %.2f\n", CLUSTER ? "cluster" : "spread ", NV, VK,
         m / (iters * 16.0));
}

int main() {
  float* out;
  long long* cyc;
  int grid = 256;
  hipMalloc(&out, grid * 256 * 4);
  hipMalloc(&cyc, grid * 8);
  run<0, 0, false>(out, cyc, grid);
  run<2, 0, false>(out, cyc, grid);
  run<4, 0, false>(out, cyc, grid);
  run<8, 0, false>(out, cyc, grid);
  run<12, 0, false>(out, cyc, grid);
  run<2, 1, false>(out, cyc, grid);
  run<4, 1, false>(out, cyc, grid);
  run<6, 1, false>(out, cyc, grid);
  run<4, 2, false>(out, cyc, grid);
  run<1, 3, false>(out, cyc, grid);
  run<2, 3, false>(out, cyc, grid);
  run<4, 0, true>(out, cyc, grid);
  run<4, 1, true>(out, cyc, grid);
  run<4, 2, true>(out, cyc, grid);
  run<1, 3, true>(out, cyc, grid);
  run<2, 3, true>(out, cyc, grid);
  return 0;
}
