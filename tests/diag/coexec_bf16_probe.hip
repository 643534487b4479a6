// Microprobe: how much VALU issue hides beside v_mfma_f32_32x32x16_bf16,
// the instruction of the headline kernel's split-bf16 layers.
//
// Part 1, one wave per SIMD (256-thread workgroups, one per CU: 96 KiB of LDS reserved): cycles
// per MFMA with NV independent VALU instructions of kind VK placed in every MFMA gap
// (sched_group_barrier), against the same work clustered after 16 MFMAs:
//   VK 0 v_fma_f32, 1 v_exp_f32 (+ its v_mul), 2 one 2-element step of the three-term bf16 split
//   (v_cvt_pk_bf16_f32, unpack by v_lshlrev / v_and, v_sub: 11 instructions per 2 elements),
//   3 one softplus/σ element (exp, rcp, log + plain ops, ~11 instructions).
// Part 2, two waves per SIMD (512-thread workgroups): waves 0-3 bf16-MFMA only, waves 4-7 the
// split or the softplus only, alone and together (fp32 MFMA: tests/diag/pair32_probe.hip).
// Diagnostics only:  hipcc -O3 --offload-arch=gfx950 coexec_bf16_probe.hip -o coexec_bf16_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float sp_sig(float y, float& sg) {
  const float t = __builtin_amdgcn_exp2f(-fabsf(y));
  const float u = 1.f + t;
  const float r = __builtin_amdgcn_rcpf(u);
  const bool pos = y >= 0.f;
  sg = pos ? r : t * r;
  return (pos ? y : 0.f) + __builtin_amdgcn_logf(u);
}
// one 2-element step of the three-term split (the kernel's wx6_split, per pair of elements)
__device__ __forceinline__ void split2(f32x2& x, unsigned& acc) {
  asm volatile("" : "+v"(x));
  const bf16x2 p0 = __builtin_convertvector(x, bf16x2);
  const f32x2 r1 = x - __builtin_convertvector(p0, f32x2);
  const bf16x2 p1 = __builtin_convertvector(r1, bf16x2);
  const f32x2 r2 = r1 - __builtin_convertvector(p1, f32x2);
  const bf16x2 p2 = __builtin_convertvector(r2, bf16x2);
  acc ^= __builtin_bit_cast(unsigned, p0) ^ __builtin_bit_cast(unsigned, p1) ^
         __builtin_bit_cast(unsigned, p2);
}

template <int VK>
constexpr int valu_per_unit() { return VK == 1 ? 2 : VK == 2 ? 11 : VK == 3 ? 11 : 1; }

template <int NV, int VK, bool CLUSTER>
__global__ __launch_bounds__(256, 1) void probe(float* out, long long* cyc, int iters) {
  extern __shared__ float pad[];
  f32x16 acc[2] = {};
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) a[i] = (__bf16)(threadIdx.x * 1e-3f + i), b[i] = (__bf16)(1.f + i * 1e-2f);
  float v[16], w[16];
  f32x2 x2[8];
  unsigned sacc = 0;
  for (int i = 0; i < 16; ++i) v[i] = 0.1f * i + threadIdx.x * 1e-4f, w[i] = 0.2f * i;
  for (int i = 0; i < 8; ++i) x2[i] = f32x2{v[2 * i], v[2 * i + 1]};
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      acc[m & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[m & 1], 0, 0, 0);
      if (!CLUSTER) {
#pragma unroll
        for (int j = 0; j < NV; ++j) {
          const int q = (m * NV + j) & 15;
          if (VK == 0) v[q] = fmaf(v[q], 0.999f, 1e-3f);
          else if (VK == 1) v[q] = __builtin_amdgcn_exp2f(v[q] * -0.5f);
          else if (VK == 2) split2(x2[q & 7], sacc);
          else { float g; v[q] = sp_sig(v[q] - 0.05f, g); w[q] += g; }
        }
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, NV * valu_per_unit<VK>(), 0);
      }
    }
    if (CLUSTER) {
#pragma unroll
      for (int j = 0; j < 16 * NV; ++j) {
        const int q = j & 15;
        if (VK == 0) v[q] = fmaf(v[q], 0.999f, 1e-3f);
        else if (VK == 1) v[q] = __builtin_amdgcn_exp2f(v[q] * -0.5f);
        else if (VK == 2) split2(x2[q & 7], sacc);
        else { float g; v[q] = sp_sig(v[q] - 0.05f, g); w[q] += g; }
      }
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = (float)sacc;
  for (int i = 0; i < 16; ++i) s += v[i] + w[i];
  for (int i = 0; i < 8; ++i) s += x2[i][0] + x2[i][1];
  for (int i = 0; i < 2; ++i)
    for (int r = 0; r < 16; ++r) s += acc[i][r];
  if (iters < 0) pad[threadIdx.x] = s;
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NV, int VK, bool CLUSTER>
void run(float* out, long long* cyc, int grid) {
  const int iters = 1000;
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL((probe<NV, VK, CLUSTER>), dim3(grid), dim3(256), 96 * 1024, 0, out, cyc,
                       iters);
  hipDeviceSynchronize();
  long long h[1024];
  hipMemcpy(h, cyc, grid * sizeof(long long), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < grid; ++i) m += h[i];
  m /= grid;
  printf("%s NV=%2d VK=%d (%2d VALU/gap)  cycles/MFMA = %.2f\n", CLUSTER ? "cluster" : "spread ",
         NV, VK, NV * valu_per_unit<VK>(), m / (iters * 16.0));
}

// part 2: mode bit 0 MFMA waves (0-3) active, bit 1 VALU waves (4-7) active; vk 2 split, 3 sp
__global__ __launch_bounds__(512, 1) void pair(float* out, long long* cyc, int iters, int mode,
                                               int vk) {
  const int w = threadIdx.x >> 6;
  long long t0 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  if (w < 4 && (mode & 1)) {
    f32x16 acc[2] = {};
    bf16x8 a, b;
    for (int i = 0; i < 8; ++i) a[i] = (__bf16)(threadIdx.x * 1e-3f + i), b[i] = (__bf16)1.f;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int m = 0; m < 16; ++m)
        acc[m & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[m & 1], 0, 0, 0);
    }
    for (int i = 0; i < 2; ++i)
      for (int r = 0; r < 16; ++r) s += acc[i][r];
  } else if (w >= 4 && (mode & 2)) {
    float v[16], g[16];
    f32x2 x2[8];
    unsigned sacc = 0;
    for (int i = 0; i < 16; ++i) v[i] = 0.01f * i + threadIdx.x * 1e-5f, g[i] = 0.f;
    for (int i = 0; i < 8; ++i) x2[i] = f32x2{v[2 * i], v[2 * i + 1]};
    for (int it = 0; it < iters; ++it) {
      if (vk == 2) {
#pragma unroll
        for (int i = 0; i < 16; ++i) split2(x2[i & 7], sacc);
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          float sg;
          v[i] = sp_sig(v[i] - 0.05f, sg);
          g[i] += sg;
        }
      }
    }
    s = (float)sacc;
    for (int i = 0; i < 16; ++i) s += v[i] + g[i];
    for (int i = 0; i < 8; ++i) s += x2[i][0] + x2[i][1];
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

int main() {
  float* out;
  long long* cyc;
  const int grid = 256;
  hipMalloc(&out, grid * 512 * 4);
  hipMalloc(&cyc, grid * 8 * 8);
  run<0, 0, false>(out, cyc, grid);
  run<2, 0, false>(out, cyc, grid);
  run<4, 0, false>(out, cyc, grid);
  run<5, 0, false>(out, cyc, grid);
  run<6, 0, false>(out, cyc, grid);
  run<8, 0, false>(out, cyc, grid);
  run<12, 0, false>(out, cyc, grid);
  run<1, 1, false>(out, cyc, grid);
  run<2, 1, false>(out, cyc, grid);
  run<3, 1, false>(out, cyc, grid);
  run<1, 2, false>(out, cyc, grid);
  run<2, 2, false>(out, cyc, grid);
  run<1, 3, false>(out, cyc, grid);
  run<2, 3, false>(out, cyc, grid);
  run<4, 0, true>(out, cyc, grid);
  run<8, 0, true>(out, cyc, grid);
  run<1, 2, true>(out, cyc, grid);
  run<1, 3, true>(out, cyc, grid);
  const int iters = 2000;
  long long h[256 * 8];
  for (int vk : {2, 3})
    for (int mode : {1, 2, 3}) {
      for (int rep = 0; rep < 2; ++rep)
        hipLaunchKernelGGL(pair, dim3(grid), dim3(512), 0, 0, out, cyc, iters, mode, vk);
      hipDeviceSynchronize();
      hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
      double mfc = 0, vc = 0;
      for (int b = 0; b < grid; ++b)
        for (int w = 0; w < 8; ++w) (w < 4 ? mfc : vc) += h[b * 8 + w];
      mfc /= grid * 4.0 * iters;
      vc /= grid * 4.0 * iters;
      printf("pair vk=%d mode=%d (%s): MFMA waves %.1f cyc/iter (16 bf16 MFMAs), VALU waves %.1f "
             "cyc/iter (16 %s)\n", vk, mode,
             mode == 1 ? "MFMA alone" : mode == 2 ? "VALU alone" : "both", mfc, vc,
             vk == 2 ? "2-element split steps" : "softplus elements");
    }
  return 0;
}
