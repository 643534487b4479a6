// Microprobe: issue cost of buffer_load_dwordx4 (L2/L1-resident weights) and of SALU offset
// moves beside v_mfma_f32_16x16x4_f32 (one wave per SIMD, 4 waves per CU, every CU busy).
// Diagnostics only: hipcc -O3 --offload-arch=gfx950 vmem_probe.hip -o vmem_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t Rsrc;

template <int NL, int NS>
__device__ __forceinline__ void phase(Rsrc r, int lane, int base, f32x4 (&ld)[4],
                                      const f32x4 (&use)[4], f32x4 (&acc)[4], float b, int& s) {
#pragma unroll
  for (int l = 0; l < NL; ++l)
    ld[l] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16,
                                                                           base + l * 1024, 0));
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    float a = NL ? use[(m / 4) % (NL ? NL : 1)][m & 3] : b;
    acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m & 3], 0, 0, 0);
    if (m % 4 == 3) {
#pragma unroll
      for (int k = 0; k < NS / 4; ++k) {
        s += k * 7 + m;
        asm volatile("" : "+s"(s));
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <int NL, int NS>
__global__ __launch_bounds__(256, 1) void probe(const float* w, float* out, long long* cyc,
                                                int iters) {
  Rsrc r = __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, 1 << 20, 0x00020000);
  const int lane = threadIdx.x & 63;
  f32x4 acc[4] = {};
  f32x4 rA[4], rB[4];
  for (int l = 0; l < 4; ++l) rA[l] = rB[l] = f32x4{0.f, 0.f, 0.f, 0.f};
  float b = 1.0f + threadIdx.x * 1e-4f;
  int s = 0;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; it += 2) {
    const int base = ((it * NL) & 127) * 1024;
    phase<NL, NS>(r, lane, base, rA, rB, acc, b, s);
    phase<NL, NS>(r, lane, base + NL * 1024, rB, rA, acc, b, s);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float sum = s;
  for (int i = 0; i < 4; ++i) sum += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  for (int l = 0; l < 4; ++l) sum += rA[l][0] + rB[l][1];
  out[blockIdx.x * 256 + threadIdx.x] = sum;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NL, int NS>
void run(const float* w, float* out, long long* cyc, int grid) {
  const int iters = 4000;
  for (int rep = 0; rep < 2; ++rep) {
    probe<NL, NS><<<grid, 256>>>(w, out, cyc, iters);
    (void)hipDeviceSynchronize();
  }
  long long h[1024];
  (void)hipMemcpy(h, cyc, grid * sizeof(long long), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < grid; ++i) m += h[i];
  m /= grid;
  printf("loads/16mfma=%d salu/16mfma=%d  cycles/MFMA = %.2f\n", NL, NS, m / (iters * 16.0));
}

// LDS variant: NR ds_read_b128 + NW ds_write_b128 per 16 MFMAs (fragments from a 16 KiB LDS
// buffer, read with the lane-contiguous 16 B layout of the weight fragments).
template <int NR, int NW>
__device__ __forceinline__ void lphase(float* lds, int lane, int base, f32x4 (&ld)[4],
                                       const f32x4 (&use)[4], f32x4 (&acc)[4], float b) {
  typedef __attribute__((address_space(3))) f32x4 l4;
  l4* L = (l4*)lds;
#pragma unroll
  for (int l = 0; l < NR; ++l) ld[l] = L[((base + l) & 15) * 64 + lane];
#pragma unroll
  for (int l = 0; l < NW; ++l) L[((base + 8 + l) & 15) * 64 + lane] = use[l];
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    float a = NR ? use[(m / 4) % (NR ? NR : 1)][m & 3] : b;
    acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[m & 3], 0, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <int NR, int NW>
__global__ __launch_bounds__(256, 1) void lprobe(float* out, long long* cyc, int iters) {
  __shared__ float lds[16 * 256 * 4];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < 16 * 256 * 4; i += 256) lds[i] = 0.f;
  __syncthreads();
  f32x4 acc[4] = {};
  f32x4 rA[4], rB[4];
  for (int l = 0; l < 4; ++l) rA[l] = rB[l] = f32x4{0.f, 0.f, 0.f, 0.f};
  float b = 1.0f + threadIdx.x * 1e-4f;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; it += 2) {
    lphase<NR, NW>(lds, lane, it, rA, rB, acc, b);
    lphase<NR, NW>(lds, lane, it + 4, rB, rA, acc, b);
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float sum = 0.f;
  for (int i = 0; i < 4; ++i) sum += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  for (int l = 0; l < 4; ++l) sum += rA[l][0] + rB[l][1];
  out[blockIdx.x * 256 + threadIdx.x] = sum;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NR, int NW>
void lrun(float* out, long long* cyc, int grid) {
  const int iters = 4000;
  for (int rep = 0; rep < 2; ++rep) {
    lprobe<NR, NW><<<grid, 256>>>(out, cyc, iters);
    (void)hipDeviceSynchronize();
  }
  long long h[1024];
  (void)hipMemcpy(h, cyc, grid * sizeof(long long), hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < grid; ++i) m += h[i];
  m /= grid;
  printf("ds_read/16mfma=%d ds_write/16mfma=%d  cycles/MFMA = %.2f\n", NR, NW, m / (iters * 16.0));
}

int main() {
  float *w, *out;
  long long* cyc;
  int grid = 256;
  (void)hipMalloc(&w, 1 << 20);
  (void)hipMemset(w, 0, 1 << 20);
  (void)hipMalloc(&out, grid * 256 * 4);
  (void)hipMalloc(&cyc, grid * 8);
  run<0, 0>(w, out, cyc, grid);
  run<1, 0>(w, out, cyc, grid);
  run<2, 0>(w, out, cyc, grid);
  run<4, 0>(w, out, cyc, grid);
  run<0, 4>(w, out, cyc, grid);
  run<0, 8>(w, out, cyc, grid);
  run<0, 16>(w, out, cyc, grid);
  run<4, 4>(w, out, cyc, grid);
  lrun<0, 0>(out, cyc, grid);
  lrun<1, 0>(out, cyc, grid);
  lrun<2, 0>(out, cyc, grid);
  lrun<4, 0>(out, cyc, grid);
  lrun<4, 1>(out, cyc, grid);
  lrun<0, 1>(out, cyc, grid);
  lrun<0, 2>(out, cyc, grid);
  return 0;
}
