// Microprobe: does the per-CU weight-stream rate of a planner step grow with the number of
// waves in the (single) workgroup on the CU?  Each workgroup streams the fwd + bwd packs
// (4.33 MB) once per "step", NW waves each a 1/NW share, DEPTH 1 KiB buffer_load_dwordx4 in
// flight per wave.  A 96 KiB dynamic LDS reservation keeps one workgroup per CU (as the quad
// planner's LDS does).  Diagnostics only:
//   hipcc -O3 --offload-arch=gfx950 stream_probe2.hip -o stream_probe2
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int FLOATS = 2 * 540672;
constexpr int FRAGS = FLOATS / 256;   // 1 KiB wave fragments (4224)

template <int NW, int DEPTH>
__global__ __launch_bounds__(NW * 64, 1) void stream(const float* w, float* out, int steps) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, FLOATS * 4, 0x00020000);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  constexpr int per = FRAGS / NW;
  for (int s = 0; s < steps; ++s) {
    f32x4 ring[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
      ring[d] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
          r, lane * 16, (wv * per + d) * 1024, 0));
    for (int f = 0; f < per; f += DEPTH) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        acc += ring[d];
        int nf = f + DEPTH + d;
        nf = nf < per ? nf : per - 1;
        ring[d] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
            r, lane * 16, (wv * per + nf) * 1024, 0));
      }
    }
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) acc += ring[d];
  }
  if (steps < 0) lds[threadIdx.x] = acc[0];
  out[blockIdx.x * 1024 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

template <int NW, int DEPTH>
void run(const float* w, float* out, int grid) {
  const int steps = 50;
  const size_t shm = 96 * 1024;
  (void)hipFuncSetAttribute((const void*)stream<NW, DEPTH>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  stream<NW, DEPTH><<<grid, NW * 64, shm>>>(w, out, 2);
  (void)hipEventRecord(a);
  stream<NW, DEPTH><<<grid, NW * 64, shm>>>(w, out, steps);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  double us = ms * 1e3 / steps;
  printf("grid %4d waves %2d depth %2d: %.1f us/step  (%.1f GB/s per CU)\n", grid, NW, DEPTH, us,
         FLOATS * 4.0 / (us * 1e3));
}

int main() {
  float *w, *out;
  (void)hipMalloc(&w, FLOATS * 4);
  (void)hipMemset(w, 0, FLOATS * 4);
  (void)hipMalloc(&out, 1024 * 1024 * 4);
  for (int g : {1, 256}) {
    run<4, 16>(w, out, g);
    run<4, 32>(w, out, g);
    run<8, 4>(w, out, g);
    run<8, 8>(w, out, g);
    run<8, 16>(w, out, g);
    run<12, 8>(w, out, g);
    run<16, 4>(w, out, g);
    run<16, 8>(w, out, g);
  }
  return 0;
}
