// Microprobe: does VALU work between v_mfma_f32_16x16x4_f32 instructions co-issue with the
// MFMA pipe (one wave per SIMD)?  Cycles per MFMA for NV independent VALU ops (VK = 0:
// v_fma_f32, 1: v_exp_f32, 2: dependent exp->fma chain) per MFMA, 4 accumulator chains.
// Diagnostics only: hipcc -O3 --offload-arch=gfx950 coexec_probe.hip -o coexec_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NV, int VK>
__global__ __launch_bounds__(256, 1) void probe(float* out, long long* cyc, int iters) {
  f32x4 acc[4] = {};
  float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
  float v[8];
  for (int i = 0; i < 8; ++i) v[i] = 0.1f * i + a;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m & 3], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        float& x = v[(m * NV + j) & 7];
        if (VK == 0) x = fmaf(x, 0.999f, 1e-3f);
        else if (VK == 1) x = __builtin_amdgcn_exp2f(x * -0.5f);
        else x = fmaf(__builtin_amdgcn_exp2f(x * -0.5f), 0.5f, 0.25f);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, NV * (VK == 2 ? 3 : (VK == 1 ? 2 : 1)), 0);
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 8; ++i) s += v[i];
  for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// Clustered: 16 MFMAs, then all 16*NV VALU ops in one gap.
template <int NV, int VK>
__global__ __launch_bounds__(256, 1) void probe_cluster(float* out, long long* cyc, int iters) {
  f32x4 acc[4] = {};
  float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
  float v[16];
  for (int i = 0; i < 16; ++i) v[i] = 0.1f * i + a;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 16; ++m)
      acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m & 3], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 16 * NV; ++j) {
      float& x = v[j & 15];
      if (VK == 0) x = fmaf(x, 0.999f, 1e-3f);
      else x = __builtin_amdgcn_exp2f(x * -0.5f);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, 16 * NV * (VK == 1 ? 2 : 1), 0);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += v[i];
  for (int i = 0; i < 4; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NV, int VK>
void runc(float* out, long long* cyc, int grid) {
  const int iters = 2000;
  probe_cluster<NV, VK><<<grid, 256>>>(out, cyc, iters);
  hipDeviceSynchronize();
  probe_cluster<NV, VK><<<grid, 256>>>(out, cyc, iters);
  hipDeviceSynchronize();
  long long h[1024];
  hipMemcpy(h, cyc, grid * sizeof(long long), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < grid; ++i) m += h[i];
  m /= grid;
  printf("cluster NV=%d VK=%d  cycles/MFMA = %.2f\n", NV, VK, m / (iters * 16.0));
}

template <int NV, int VK>
void run(float* out, long long* cyc, int grid) {
  const int iters = 2000;
  probe<NV, VK><<<grid, 256>>>(out, cyc, iters);
  hipDeviceSynchronize();
  probe<NV, VK><<<grid, 256>>>(out, cyc, iters);
  hipDeviceSynchronize();
  long long h[1024];
  hipMemcpy(h, cyc, grid * sizeof(long long), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < grid; ++i) m += h[i];
  m /= grid;
  printf("NV=%d VK=%d  cycles/MFMA = %.2f\n", NV, VK, m / (iters * 16.0));
}

int main() {
  float* out;
  long long* cyc;
  int grid = 256;
  hipMalloc(&out, grid * 256 * 4);
  hipMalloc(&cyc, grid * 8);
  run<0, 0>(out, cyc, grid);
  run<1, 0>(out, cyc, grid);
  run<2, 0>(out, cyc, grid);
  run<4, 0>(out, cyc, grid);
  run<6, 0>(out, cyc, grid);
  run<8, 0>(out, cyc, grid);
  run<1, 1>(out, cyc, grid);
  run<2, 1>(out, cyc, grid);
  run<3, 1>(out, cyc, grid);
  run<4, 1>(out, cyc, grid);
  run<1, 2>(out, cyc, grid);
  run<2, 2>(out, cyc, grid);
  runc<1, 0>(out, cyc, grid);
  runc<2, 0>(out, cyc, grid);
  runc<4, 0>(out, cyc, grid);
  runc<1, 1>(out, cyc, grid);
  runc<2, 1>(out, cyc, grid);
  return 0;
}
