// Diagnostic: is pntf_common.h x6_resid (v_dot2c_f32_bf16 against a (-1, -0) / (-0, -1) pair)
// exactly x - bf16_rne(x) on gfx950?  Prints mismatches over random and edge-case inputs.
//   hipcc -O3 --offload-arch=gfx950 -Ip-ntfields_amd/csrc tests/diag/dot2_probe.hip -o /tmp/p
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include "pntf_common.h"
using namespace pntf;

__global__ void probe(const float* x, float* r1, float* r2, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  x6f32x2 v = {x[2 * i], x[2 * i + 1]};
  x6bf16x2 p = __builtin_convertvector(v, x6bf16x2);
  x6f32x2 a = x6_resid(v, p);                    // dot2 residual
  x6f32x2 b = v - __builtin_convertvector(p, x6f32x2);   // plain residual
  r1[2 * i] = a[0]; r1[2 * i + 1] = a[1];
  r2[2 * i] = b[0]; r2[2 * i + 1] = b[1];
}

int main() {
  const int n = 1 << 22;
  float* h = (float*)malloc(n * 4);
  srand(1);
  for (int i = 0; i < n; ++i) {
    float u = (rand() + 0.5f) / (RAND_MAX + 1.0f);
    float e = ldexpf(1.f, (rand() % 60) - 30);
    h[i] = (rand() & 1 ? -1.f : 1.f) * u * e;
  }
  const float edge[] = {0.f, -0.f, 1.f, -1.f, 1e-38f, -1e-38f, 1e-40f, 3e38f, -3e38f, 65504.f,
                        1.00390625f, 1.0078125f, 0.99609375f, 1.f + 1.f / 256 + 1.f / 65536};
  memcpy(h, edge, sizeof(edge));
  float *dx, *d1, *d2;
  hipMalloc(&dx, n * 4); hipMalloc(&d1, n * 4); hipMalloc(&d2, n * 4);
  hipMemcpy(dx, h, n * 4, hipMemcpyHostToDevice);
  probe<<<n / 2 / 256, 256>>>(dx, d1, d2, n);
  float* a = (float*)malloc(n * 4); float* b = (float*)malloc(n * 4);
  hipMemcpy(a, d1, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(b, d2, n * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i) {
    if (memcmp(&a[i], &b[i], 4) != 0 && !(a[i] == 0.f && b[i] == 0.f)) {
      if (bad < 12) printf("x=%a  dot2=%a  sub=%a  (elem %d)\n", h[i], a[i], b[i], i & 1);
      ++bad;
    }
  }
  printf("dot2 residual vs subtract: %d of %d differ\n", bad, n);
  return bad != 0;
}
