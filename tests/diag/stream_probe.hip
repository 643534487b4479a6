// Microprobe: per-CU weight-stream floor of a planner step.  Each workgroup (4 waves, one per
// SIMD) streams the fwd + bwd packs (2 x SZ_DIR floats, 4.33 MB) once per "step" through
// buffer_load_dwordx4 (1 KiB per wave-instruction, each wave a quarter), DEPTH loads in flight,
// one add per load; grid = tiles in flight.  Reports microseconds per step.
// Diagnostics only: hipcc -O3 --offload-arch=gfx950 stream_probe.hip -o stream_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int FLOATS = 2 * 540672;
constexpr int FRAGS = FLOATS / 256;   // 1 KiB wave fragments

template <int DEPTH>
__global__ __launch_bounds__(256, 1) void stream(const float* w, float* out, int steps) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, FLOATS * 4, 0x00020000);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const int per = FRAGS / 4;
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
  out[blockIdx.x * 256 + threadIdx.x] = acc[0] + acc[1] + acc[2] + acc[3];
}

template <int DEPTH>
void run(const float* w, float* out, int grid) {
  const int steps = 50;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  stream<DEPTH><<<grid, 256>>>(w, out, 2);
  (void)hipEventRecord(a);
  stream<DEPTH><<<grid, 256>>>(w, out, steps);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  double us = ms * 1e3 / steps;
  printf("grid %4d depth %2d: %.1f us/step  (%.1f GB/s per CU)\n", grid, DEPTH, us,
         FLOATS * 4.0 / (us * 1e3));
}

int main() {
  float *w, *out;
  (void)hipMalloc(&w, FLOATS * 4);
  (void)hipMemset(w, 0, FLOATS * 4);
  (void)hipMalloc(&out, 1024 * 256 * 4);
  for (int g : {1, 64, 256, 512}) {
    run<4>(w, out, g);
    run<8>(w, out, g);
    run<16>(w, out, g);
    run<32>(w, out, g);
    run<48>(w, out, g);
  }
  return 0;
}
