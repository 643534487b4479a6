// Microprobe: with two waves per SIMD, does one wave's VALU (or LDS) work run while the other
// wave's v_mfma_f32_16x16x4_f32 / 32x32x2 stream issues?  Workgroup of 8 waves (2 per SIMD):
// waves 0-3 run MFMAs, waves 4-7 run VALU / LDS / nothing (MODE); cycles per MFMA of waves 0-3.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int MODE, bool BIG>
__global__ __launch_bounds__(512, 1) void probe(float* out, long long* cyc, int iters) {
  __shared__ float lds[8 * 1024];
  const int w = threadIdx.x >> 6;
  float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
  float s = 0.f;
  if (w < 4 || MODE == 3) {
    f32x4 acc[4] = {};
    f32x16 acc2[2] = {};
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        if (BIG) acc2[m & 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc2[m & 1], 0, 0, 0);
        else acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m & 3], 0, 0, 0);
      }
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < 4; ++i) s += acc[i][0] + acc2[i & 1][i];
    if ((threadIdx.x & 63) == 0 && w < 4) cyc[blockIdx.x * 4 + w] = t1 - t0;
  } else if (MODE == 1) {   // VALU: independent exp / fma chains
    float v[8];
    for (int i = 0; i < 8; ++i) v[i] = 0.1f * i + a;
    for (int it = 0; it < iters * 8; ++it)
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = fmaf(__builtin_amdgcn_exp2f(v[i] * -0.5f), 0.5f, 0.25f);
    for (int i = 0; i < 8; ++i) s += v[i];
  } else if (MODE == 2) {   // LDS reads
    typedef __attribute__((address_space(3))) f32x4 l4;
    l4* L = (l4*)lds;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int it = 0; it < iters * 4; ++it) {
      f32x4 x = L[((it + w) & 31) * 64 + (threadIdx.x & 63)];
      acc += x;
    }
    s = acc[0];
  }
  out[blockIdx.x * 512 + threadIdx.x] = s;
}

template <int MODE, bool BIG>
void run(float* out, long long* cyc, int grid, const char* what) {
  const int iters = 2000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float ms = 0.f;
  for (int r = 0; r < 2; ++r) {
    (void)hipEventRecord(e0);
    probe<MODE, BIG><<<grid, 512>>>(out, cyc, iters);
    (void)hipEventRecord(e1);
    (void)hipDeviceSynchronize();
    (void)hipEventElapsedTime(&ms, e0, e1);
  }
  long long h[1024];
  (void)hipMemcpy(h, cyc, grid * 4 * sizeof(long long), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < grid * 4; ++i) m += h[i];
  m /= grid * 4;
  const int nw = MODE == 3 ? 8 : 4;
  const double flop = (double)grid * nw * iters * 8 * (BIG ? 32768.0 : 2048.0);
  printf("%s %s: cycles/MFMA of the MFMA waves = %.2f, kernel %.3f ms = %.1f TF/s\n",
         BIG ? "32x32x2" : "16x16x4", what, m / (iters * 8.0), ms, flop / (ms * 1e-3) / 1e12);
}

int main() {
  float* out;
  long long* cyc;
  int grid = 256;
  (void)hipMalloc(&out, grid * 512 * 4);
  (void)hipMalloc(&cyc, grid * 4 * 8);
  run<0, false>(out, cyc, grid, "partner idle");
  run<1, false>(out, cyc, grid, "partner VALU");
  run<2, false>(out, cyc, grid, "partner LDS");
  run<3, false>(out, cyc, grid, "partner MFMA");
  run<0, true>(out, cyc, grid, "partner idle");
  run<1, true>(out, cyc, grid, "partner VALU");
  run<2, true>(out, cyc, grid, "partner LDS");
  return 0;
}
