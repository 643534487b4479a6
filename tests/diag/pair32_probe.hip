// Microprobe: do two waves on one SIMD overlap fp32 MFMA (v_mfma_f32_32x32x2_f32) with
// VALU/transcendental work?  512-thread workgroups, one per CU: waves 0-3 (one per SIMD) run
// an MFMA-only loop, waves 4-7 (the partners on the same SIMDs) a VALU loop of the softplus /
// σ epilogue (exp, rcp, log + plain ops).  Each role is also timed alone (the partner idle).
// If the pipes overlap, the pair takes ~max(MFMA, VALU) cycles; if they share an issue or
// datapath resource, ~their sum.  Diagnostics only:
//   hipcc -O3 --offload-arch=gfx950 pair32_probe.hip -o pair32_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float sp_sig(float y, float& sg) {
  float t = __builtin_amdgcn_exp2f(-14.4269504f * fabsf(y));
  float u = 1.f + t;
  float r = __builtin_amdgcn_rcpf(u);
  bool pos = y >= 0.f;
  sg = pos ? r : t * r;
  return fmaf(__builtin_amdgcn_logf(u), 0.0693147f, pos ? y : 0.f);
}

// mode bit 0: MFMA waves active; bit 1: VALU waves active
__global__ __launch_bounds__(512, 1) void probe(float* out, long long* cyc, int iters, int mode,
                                                int valu_per_iter) {
  const int w = threadIdx.x >> 6;
  const bool mf = w < 4;
  long long t0 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  if (mf && (mode & 1)) {
    f32x16 acc[2] = {};
    float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int m = 0; m < 16; ++m)
        acc[m & 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[m & 1], 0, 0, 0);
    }
    for (int i = 0; i < 2; ++i)
      for (int r = 0; r < 16; ++r) s += acc[i][r];
  } else if (!mf && (mode & 2)) {
    float v[16], g[16];
    for (int i = 0; i < 16; ++i) v[i] = 0.01f * i + threadIdx.x * 1e-5f, g[i] = 0.f;
    for (int it = 0; it < iters; ++it) {
      for (int k = 0; k < valu_per_iter; ++k) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float sg;
          v[i] = sp_sig(v[i] - 0.05f, sg);
          g[i] += sg;
        }
      }
    }
    for (int i = 0; i < 16; ++i) s += v[i] + g[i];
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

int main() {
  float* out;
  long long* cyc;
  const int grid = 256, iters = 2000;
  hipMalloc(&out, grid * 512 * 4);
  hipMalloc(&cyc, grid * 8 * 8);
  long long h[256 * 8];
  for (int vpi : {1, 2}) {
    for (int mode : {1, 2, 3}) {
      for (int rep = 0; rep < 2; ++rep)
        hipLaunchKernelGGL(probe, dim3(grid), dim3(512), 0, 0, out, cyc, iters, mode, vpi);
      hipDeviceSynchronize();
      hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
      double mfc = 0, vc = 0;
      for (int b = 0; b < grid; ++b)
        for (int w = 0; w < 8; ++w) (w < 4 ? mfc : vc) += h[b * 8 + w];
      mfc /= grid * 4.0 * iters;
      vc /= grid * 4.0 * iters;
      printf("valu_per_iter=%d mode=%d (%s): MFMA waves %.1f cyc/iter (16 MFMAs), VALU waves %.1f "
             "cyc/iter (%d sp_sig x16)\n", vpi, mode,
             mode == 1 ? "MFMA alone" : mode == 2 ? "VALU alone" : "both", mfc, vc, vpi);
    }
  }
  return 0;
}
