// Point -> triangle-mesh unsigned distance on MI355X: the query the
// speed-sample generator makes for every sampled start / goal point,
// `point_obstacle_distance` (dataprocessing/speed_sampling_gpu.py:325-336), which the
// reference answers with the un-vendored CUDA extension bvh_distance_queries
// (.gitmodules:1-3, github.com/YuliangXiu/bvh-distance-queries, no pinned commit): a BVH
// over the triangles, exact closest point per (point, triangle), squared distance out,
// `torch.sqrt` in the caller (:334).
//
// MI355X design: the meshes here are the scaled Gibson obstacle meshes (10^3..10^5
// triangles) and a sampling round queries 8·numsamples points, so the work is a dense
// (points x triangles) min-reduction, VALU-bound, not a pointer-chasing tree walk.  Each
// workgroup owns 256 points (one per lane, in registers) and a contiguous chunk of
// triangles, which it stages through LDS 256 at a time; every lane then reads the same
// triangle (LDS broadcast, conflict-free).  When the point grid alone cannot fill 256 CUs
// the triangle range is split over grid.y and the chunks combine with a global unsigned
// atomic min on the fp32 bit pattern of d^2 (order-preserving for d^2 >= 0, so the result
// is the exact minimum, independent of chunk order); a finalize pass takes the sqrt.
//
// Closest point on a triangle: the region test of Ericson, "Real-Time Collision Detection"
// §5.1.5 (the algorithm bvh_distance_queries' device code uses), restated in fp32.
// Degenerate (sin^2 of the angle at vertex a <= 1e-12) triangles whose closest point falls
// in the interior region fall back to the nearest of their three edges.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>

#include "pntf.h"

namespace {

constexpr int BLOCK = 256;       // points per workgroup = triangles per LDS tile
constexpr int TARGET_WG = 2048;  // 8 workgroups per CU on 256 CUs

thread_local char g_err[512] = "";

int fail(const char* what) {
  snprintf(g_err, sizeof(g_err), "%s", what);
  return PNTF_ERR_ARG;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
    return PNTF_ERR_HIP;
  }
  return PNTF_OK;
}

__device__ __forceinline__ float dot3(float ax, float ay, float az, float bx, float by,
                                      float bz) {
  return fmaf(ax, bx, fmaf(ay, by, az * bz));
}

// squared distance from p to segment [a, a + e]
__device__ __forceinline__ float seg_d2(float px, float py, float pz, float ax, float ay,
                                        float az, float ex, float ey, float ez) {
  const float qx = px - ax, qy = py - ay, qz = pz - az;
  const float ee = dot3(ex, ey, ez, ex, ey, ez);
  float t = ee > 0.f ? dot3(qx, qy, qz, ex, ey, ez) / ee : 0.f;
  t = fminf(fmaxf(t, 0.f), 1.f);
  const float rx = qx - t * ex, ry = qy - t * ey, rz = qz - t * ez;
  return dot3(rx, ry, rz, rx, ry, rz);
}

// Ericson §5.1.5 ClosestPtPointTriangle; returns |p - closest|^2.
__device__ __forceinline__ float tri_d2(float px, float py, float pz, const float* __restrict__ t) {
  const float ax = t[0], ay = t[1], az = t[2];
  const float bx = t[3], by = t[4], bz = t[5];
  const float cx = t[6], cy = t[7], cz = t[8];
  const float abx = bx - ax, aby = by - ay, abz = bz - az;
  const float acx = cx - ax, acy = cy - ay, acz = cz - az;
  const float apx = px - ax, apy = py - ay, apz = pz - az;
  const float d1 = dot3(abx, aby, abz, apx, apy, apz);
  const float d2 = dot3(acx, acy, acz, apx, apy, apz);
  float qx, qy, qz;
  if (d1 <= 0.f && d2 <= 0.f) {
    qx = ax; qy = ay; qz = az;
  } else {
    const float bpx = px - bx, bpy = py - by, bpz = pz - bz;
    const float d3 = dot3(abx, aby, abz, bpx, bpy, bpz);
    const float d4 = dot3(acx, acy, acz, bpx, bpy, bpz);
    const float cpx = px - cx, cpy = py - cy, cpz = pz - cz;
    const float d5 = dot3(abx, aby, abz, cpx, cpy, cpz);
    const float d6 = dot3(acx, acy, acz, cpx, cpy, cpz);
    const float vc = d1 * d4 - d3 * d2;
    const float vb = d5 * d2 - d1 * d6;
    const float va = d3 * d6 - d5 * d4;
    if (d3 >= 0.f && d4 <= d3) {
      qx = bx; qy = by; qz = bz;
    } else if (vc <= 0.f && d1 >= 0.f && d3 <= 0.f) {
      const float v = d1 / (d1 - d3);
      qx = ax + v * abx; qy = ay + v * aby; qz = az + v * abz;
    } else if (d6 >= 0.f && d5 <= d6) {
      qx = cx; qy = cy; qz = cz;
    } else if (vb <= 0.f && d2 >= 0.f && d6 <= 0.f) {
      const float w = d2 / (d2 - d6);
      qx = ax + w * acx; qy = ay + w * acy; qz = az + w * acz;
    } else if (va <= 0.f && (d4 - d3) >= 0.f && (d5 - d6) >= 0.f) {
      const float w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
      qx = bx + w * (cx - bx); qy = by + w * (cy - by); qz = bz + w * (cz - bz);
    } else {
      // interior region; a (near-)zero-area triangle, sin^2(angle at a) <= 1e-12, makes
      // va + vb + vc ill-conditioned: take its nearest edge instead
      const float nx = aby * acz - abz * acy, ny = abz * acx - abx * acz,
                  nz = abx * acy - aby * acx;
      const float s = va + vb + vc;
      if (!(s > 0.f) || dot3(nx, ny, nz, nx, ny, nz) <=
                            1e-12f * dot3(abx, aby, abz, abx, aby, abz) *
                                dot3(acx, acy, acz, acx, acy, acz)) {
        float m = seg_d2(px, py, pz, ax, ay, az, abx, aby, abz);
        m = fminf(m, seg_d2(px, py, pz, ax, ay, az, acx, acy, acz));
        return fminf(m, seg_d2(px, py, pz, bx, by, bz, cx - bx, cy - by, cz - bz));
      }
      const float denom = 1.f / s;
      const float v = vb * denom, w = vc * denom;
      qx = ax + abx * v + acx * w; qy = ay + aby * v + acy * w; qz = az + abz * v + acz * w;
    }
  }
  const float rx = px - qx, ry = py - qy, rz = pz - qz;
  return dot3(rx, ry, rz, rx, ry, rz);
}

// grid (ceil(n/256), n_chunks); chunk y covers triangles [y*per, min(t,(y+1)*per)).
// SPLIT: combine through atomicMin on d^2 bits in `acc`; else write sqrt(d^2) to `dist`.
template <bool SPLIT>
__global__ __launch_bounds__(BLOCK) void mesh_distance_kernel(
    const float* __restrict__ pts, int64_t n, const float* __restrict__ tris, int64_t t,
    int64_t per, float* __restrict__ dist, unsigned int* __restrict__ acc) {
  __shared__ float s_tri[BLOCK * 9];
  const int64_t i = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
  const bool live = i < n;
  float px = 0.f, py = 0.f, pz = 0.f;
  if (live) {
    px = pts[3 * i]; py = pts[3 * i + 1]; pz = pts[3 * i + 2];
  }
  const int64_t t0 = (int64_t)blockIdx.y * per;
  const int64_t t1 = t0 + per < t ? t0 + per : t;
  float best = INFINITY;
  for (int64_t base = t0; base < t1; base += BLOCK) {
    const int cnt = (int)(t1 - base < BLOCK ? t1 - base : BLOCK);
    __syncthreads();
    // coalesced: the tile is cnt*9 contiguous floats
    const float* src = tris + base * 9;
    for (int k = threadIdx.x; k < cnt * 9; k += BLOCK) s_tri[k] = src[k];
    __syncthreads();
    for (int j = 0; j < cnt; ++j) best = fminf(best, tri_d2(px, py, pz, s_tri + 9 * j));
  }
  if (!live) return;
  if (SPLIT)
    atomicMin(acc + i, __float_as_uint(best));
  else
    dist[i] = sqrtf(best);
}

__global__ void fill_inf_kernel(unsigned int* __restrict__ acc, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) acc[i] = 0x7f800000u;
}

__global__ void finalize_kernel(float* __restrict__ dist, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dist[i] = sqrtf(__uint_as_float(reinterpret_cast<unsigned int*>(dist)[i]));
}

}  // namespace

extern "C" {

const char* pntf_mesh_last_error(void) { return g_err; }

int pntf_mesh_chunks(int64_t n, int64_t t) {
  if (n <= 0 || t <= 0) return 1;
  const int64_t gx = (n + BLOCK - 1) / BLOCK;
  const int64_t tiles = (t + BLOCK - 1) / BLOCK;
  int64_t c = (TARGET_WG + gx - 1) / gx;
  if (c > tiles) c = tiles;
  if (c > 65535) c = 65535;
  return (int)(c < 1 ? 1 : c);
}

int pntf_point_mesh_distance(const float* pts, int64_t n, const float* tris, int64_t t,
                             float* dist, int chunks, hipStream_t stream) {
  if (n < 0 || t < 0 || (n > 0 && (!pts || !dist)) || (t > 0 && !tris))
    return fail("pntf_point_mesh_distance: bad arguments");
  if (n == 0) return PNTF_OK;
  if (t == 0) return fail("pntf_point_mesh_distance: empty mesh");
  if ((n + BLOCK - 1) / BLOCK > 0x7fffffff)
    return fail("pntf_point_mesh_distance: too many points");
  if (chunks <= 0) chunks = pntf_mesh_chunks(n, t);
  if (chunks > 65535) return fail("pntf_point_mesh_distance: chunks > 65535");
  // whole LDS tiles per chunk, so only the last chunk has a ragged tile
  int64_t per = (t + chunks - 1) / chunks;
  per = (per + BLOCK - 1) / BLOCK * BLOCK;
  const int64_t c = (t + per - 1) / per;
  const dim3 grid((unsigned)((n + BLOCK - 1) / BLOCK), (unsigned)c);
  if (c == 1) {
    hipLaunchKernelGGL(mesh_distance_kernel<false>, grid, dim3(BLOCK), 0, stream, pts, n, tris,
                       t, per, dist, nullptr);
    return check_launch("mesh_distance_kernel");
  }
  unsigned int* acc = reinterpret_cast<unsigned int*>(dist);
  const unsigned g1 = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(fill_inf_kernel, dim3(g1), dim3(256), 0, stream, acc, n);
  hipLaunchKernelGGL(mesh_distance_kernel<true>, grid, dim3(BLOCK), 0, stream, pts, n, tris, t,
                     per, dist, acc);
  hipLaunchKernelGGL(finalize_kernel, dim3(g1), dim3(256), 0, stream, dist, n);
  return check_launch("mesh_distance_kernel");
}

}  // extern "C"
