// Microprobe: v_mfma_f32_4x4x1_16b_f32 (16 independent 4x4x1 blocks) on gfx950 — operand /
// result lane layout and issue rate against v_mfma_f32_16x16x4_f32, plus the cost of the
// row_ror DPP adds that sum partial products over k sub-blocks.
// Diagnostics only: hipcc -O3 --offload-arch=gfx950 quad_probe.hip -o quad_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void layout(float* out) {
  const int l = threadIdx.x;
  float a = 1000.f + l, b = 1.f + l;
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  f32x4 d = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) out[l * 4 + i] = d[i];
}

template <int KIND, int NDPP>
__global__ __launch_bounds__(256, 1) void rate(float* out, long long* cyc, int iters) {
  const int l = threadIdx.x & 63;
  float a = 1e-3f * l, b = 1.f + 1e-4f * l;
  f32x4 acc[4] = {};
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      if (KIND == 0) acc[m] = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc[m], 0, 0, 0);
      else acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m], 0, 0, 0);
    }
    if (NDPP) {
#pragma unroll
      for (int j = 0; j < NDPP; ++j) {
        // v += row_ror:4(v): dpp_ctrl 0x124
        float v = acc[j & 3][(j >> 2) & 3];
        float r = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
            0, __builtin_bit_cast(int, v), 0x124, 0xf, 0xf, false));
        a += r * 1e-9f;
      }
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = a;
  for (int m = 0; m < 4; ++m) s += acc[m][0] + acc[m][1] + acc[m][2] + acc[m][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND, int NDPP>
void run(float* out, long long* cyc, int grid) {
  const int iters = 4000;
  for (int rep = 0; rep < 2; ++rep) {
    rate<KIND, NDPP><<<grid, 256>>>(out, cyc, iters);
    (void)hipDeviceSynchronize();
  }
  long long h[1024];
  (void)hipMemcpy(h, cyc, grid * sizeof(long long), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < grid; ++i) m += h[i];
  m /= grid;
  printf("%s + %d dpp per 4 MFMA: cycles/MFMA = %.2f\n", KIND == 0 ? "4x4x1_16b" : "16x16x4",
         NDPP, m / (iters * 4.0));
}

int main() {
  float* out;
  long long* cyc;
  (void)hipMalloc(&out, 1 << 22);
  (void)hipMalloc(&cyc, 1 << 16);
  layout<<<1, 64>>>(out);
  float h[256];
  (void)hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
  // hypothesis: D[i] at lane l = A[4*(l/4) + i] * B[l]  (block l/4, row i, col l%4)
  int bad = 0;
  for (int l = 0; l < 64; ++l)
    for (int i = 0; i < 4; ++i) {
      float e = (1000.f + 4 * (l / 4) + i) * (1.f + l);
      if (std::fabs(h[l * 4 + i] - e) > 1e-3f * e) ++bad;
    }
  printf("layout hypothesis (block l/4, row i, col l%%4): %s\n", bad ? "WRONG" : "ok");
  if (bad)
    for (int l = 0; l < 8; ++l)
      printf("lane %d: %g %g %g %g\n", l, h[l * 4], h[l * 4 + 1], h[l * 4 + 2], h[l * 4 + 3]);
  run<0, 0>(out, cyc, 256);
  run<1, 0>(out, cyc, 256);
  run<0, 2>(out, cyc, 256);
  run<0, 4>(out, cyc, 256);
  run<0, 8>(out, cyc, 256);
  return 0;
}
