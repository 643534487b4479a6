// Microprobe: v_mfma_f32_32x32x2_f32 issue rate on 1 or 2 accumulator chains, with one
// buffer_load_dwordx4 per 4 MFMAs (the 32-pair weight-fragment rate), against
// v_mfma_f32_16x16x4_f32 with one load per 4 MFMAs (the 16-pair generator rate).
// Diagnostics only: hipcc -O3 --offload-arch=gfx950 mfma32_probe.hip -o mfma32_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __amdgpu_buffer_rsrc_t Rsrc;

template <int CH, int LD, bool BIG>
__device__ __forceinline__ void phase(Rsrc r, int lane, int base, f32x4& ld, const f32x4& use,
                                      f32x16 (&acc)[2], f32x4 (&acc4)[4], float b) {
  if (LD) ld = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16, base, 0));
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    float a = LD ? use[m] : b;
    if (BIG) acc[m % CH] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[m % CH], 0, 0, 0);
    else acc4[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc4[m], 0, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <int CH, int LD, bool BIG>
__global__ __launch_bounds__(256, 1) void probe(const float* w, float* out, long long* cyc,
                                                int iters) {
  Rsrc r = __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, 1 << 20, 0x00020000);
  const int lane = threadIdx.x & 63;
  f32x16 acc[2] = {};
  f32x4 acc4[4] = {};
  f32x4 rA = {0.f, 0.f, 0.f, 0.f}, rB = rA, rC = rA, rD = rA;
  float b = 1.0f + threadIdx.x * 1e-4f;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; it += 4) {
    const int base = (it & 255) * 1024;
    phase<CH, LD, BIG>(r, lane, base, rA, rC, acc, acc4, b);
    phase<CH, LD, BIG>(r, lane, base + 1024, rB, rD, acc, acc4, b);
    phase<CH, LD, BIG>(r, lane, base + 2048, rC, rA, acc, acc4, b);
    phase<CH, LD, BIG>(r, lane, base + 3072, rD, rB, acc, acc4, b);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float sum = rA[0] + rB[1] + rC[2] + rD[3];
  for (int i = 0; i < 16; ++i) sum += acc[0][i] + acc[1][i];
  for (int i = 0; i < 4; ++i) sum += acc4[i][0];
  out[blockIdx.x * 256 + threadIdx.x] = sum;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int CH, int LD, bool BIG>
void run(const float* w, float* out, long long* cyc, int grid) {
  const int iters = 4000;
  for (int rep = 0; rep < 2; ++rep) {
    probe<CH, LD, BIG><<<grid, 256>>>(w, out, cyc, iters);
    (void)hipDeviceSynchronize();
  }
  long long h[1024];
  (void)hipMemcpy(h, cyc, grid * sizeof(long long), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < grid; ++i) m += h[i];
  m /= grid;
  printf("%s chains=%d load/4mfma=%d  cycles/MFMA = %.2f\n", BIG ? "32x32x2" : "16x16x4", CH, LD,
         m / (iters * 4.0));
}

// VALU beside 32x32x2: NV independent ops per MFMA (VK 0: fma, 1: exp2)
template <int NV, int VK>
__global__ __launch_bounds__(256, 1) void vprobe(float* out, long long* cyc, int iters) {
  f32x16 acc[2] = {};
  float a = threadIdx.x * 1e-3f, b = 1.0f + threadIdx.x * 1e-4f;
  float v[16];
  for (int i = 0; i < 16; ++i) v[i] = 0.1f * i + a;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      acc[m & 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[m & 1], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        float& x = v[(m * NV + j) & 15];
        if (VK == 0) x = fmaf(x, x, 1e-3f);
        else x = __builtin_amdgcn_exp2f(x);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += v[i] + acc[0][i] + acc[1][i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NV, int VK>
void vrun(float* out, long long* cyc, int grid) {
  const int iters = 4000;
  for (int rep = 0; rep < 2; ++rep) {
    vprobe<NV, VK><<<grid, 256>>>(out, cyc, iters);
    (void)hipDeviceSynchronize();
  }
  long long h[1024];
  (void)hipMemcpy(h, cyc, grid * sizeof(long long), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < grid; ++i) m += h[i];
  m /= grid;
  printf("32x32x2 + %d %s per MFMA  cycles/MFMA = %.2f\n", NV, VK ? "exp" : "fma", m / (iters * 4.0));
}

// ds_read_b128 beside 32x32x2: NR LDS fragment reads per 4 MFMAs (operands consumed)
template <int NR>
__global__ __launch_bounds__(256, 1) void dprobe(float* out, long long* cyc, int iters) {
  __shared__ float lds[16 * 256];
  typedef __attribute__((address_space(3))) f32x4 l4;
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 16 * 256; i += 256) lds[i] = 0.001f * i;
  __syncthreads();
  f32x16 acc[2] = {};
  float b = 1.0f + threadIdx.x * 1e-4f;
  f32x4 r0 = {0.f, 0.f, 0.f, 0.f}, r1 = r0;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    l4* L = (l4*)lds;
    f32x4 n0 = r0, n1 = r1;
    if (NR >= 1) n0 = L[((it * 2) & 15) * 64 + lane];
    if (NR >= 2) n1 = L[((it * 2 + 1) & 15) * 64 + lane];
#pragma unroll
    for (int m = 0; m < 4; ++m)
      acc[m & 1] = __builtin_amdgcn_mfma_f32_32x32x2f32(NR ? (m < 2 ? r0[m] : r1[m]) : b, b, acc[m & 1], 0, 0, 0);
    r0 = n0;
    r1 = n1;
    __builtin_amdgcn_sched_barrier(0);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float sm = r0[0] + r1[1];
  for (int i = 0; i < 16; ++i) sm += acc[0][i] + acc[1][i];
  out[blockIdx.x * 256 + threadIdx.x] = sm;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NR>
void drun(float* out, long long* cyc, int grid) {
  const int iters = 4000;
  for (int rep = 0; rep < 2; ++rep) {
    dprobe<NR><<<grid, 256>>>(out, cyc, iters);
    (void)hipDeviceSynchronize();
  }
  long long h[1024];
  (void)hipMemcpy(h, cyc, grid * sizeof(long long), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < grid; ++i) m += h[i];
  m /= grid;
  printf("32x32x2 + %d ds_read_b128 per 4 MFMA  cycles/MFMA = %.2f\n", NR, m / (iters * 4.0));
}

int main() {
  float *w, *out;
  long long* cyc;
  int grid = 256;
  (void)hipMalloc(&w, 1 << 20);
  (void)hipMemset(w, 0, 1 << 20);
  (void)hipMalloc(&out, grid * 256 * 4);
  (void)hipMalloc(&cyc, grid * 8);
  run<1, 0, true>(w, out, cyc, grid);
  run<2, 0, true>(w, out, cyc, grid);
  run<1, 1, true>(w, out, cyc, grid);
  run<2, 1, true>(w, out, cyc, grid);
  run<1, 0, false>(w, out, cyc, grid);
  run<1, 1, false>(w, out, cyc, grid);
  vrun<1, 0>(out, cyc, grid);
  vrun<2, 0>(out, cyc, grid);
  vrun<4, 0>(out, cyc, grid);
  vrun<8, 0>(out, cyc, grid);
  vrun<12, 0>(out, cyc, grid);
  vrun<1, 1>(out, cyc, grid);
  vrun<2, 1>(out, cyc, grid);
  vrun<4, 1>(out, cyc, grid);
  vrun<6, 1>(out, cyc, grid);
  drun<0>(out, cyc, grid);
  drun<1>(out, cyc, grid);
  drun<2>(out, cyc, grid);
  return 0;
}
